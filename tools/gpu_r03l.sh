# The bench's region with per-stream start/end events (no cross-stream waits): the driver's
# 20-step command three times, the default 200 steps once, and a rocprofv3 kernel trace of
# the 20-step command (the launch stagger at the region's start)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03l
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03l/bd_$rep.log 2>&1 || { tail -20 gpurun_out/r03l/bd_$rep.log; exit 1; }
  echo "20/5 #$rep $(grep '^{' gpurun_out/r03l/bd_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_ms_mean"], r["frac"], r["pipelined"]["interval_ms"])')"
done
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r03l/b200.log 2>&1 || { tail -20 gpurun_out/r03l/b200.log; exit 1; }
echo "200/20 $(grep '^{' gpurun_out/r03l/b200.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_ms_mean"], r["frac"], r["pipelined"]["interval_ms"])')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r03l/prof_B20 -o run --output-format csv \
    -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r03l/prof_B20.log 2>&1 || { tail -20 gpurun_out/r03l/prof_B20.log; exit 1; }
echo done
