# Full GPU suite on the single-pass routes, then single-pass (default) against two-pass
# (EMURX_OWNER_PASS=1) routes on config D, both variants (partitioned value, replicated
# alternative), then rocprofv3 kernel traces of the D step
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03k gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03k/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03k/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r03k/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03k/smoke.log 2>&1 || { tail -20 gpurun_out/r03k/smoke.log; exit 1; }
for rep in 1 2; do
  for v in single twopass; do
    op=0; [ $v = twopass ] && op=1
    EMURX_OWNER_PASS=$op timeout -k 10 300 python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline --no-check --no-replay > gpurun_out/ab/Dk_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/ab/Dk_${v}_$rep.log; exit 1; }
    echo "D $v #$rep $(grep '^{' gpurun_out/ab/Dk_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["exchange"]["phases"]; a=d["alternative"]; q=a["exchange"]["phases"]; print(d["value"], d["ms_per_step"], p["source_side_ms"], p["k_rx_ms"], p["owner_lookup_ms"], "| repl", a["value"], a["ms_per_step"], q["source_side_ms"], q["k_rx_ms"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r03k/prof_D -o run --output-format csv \
    -- python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r03k/prof_D.log 2>&1 || { tail -20 gpurun_out/r03k/prof_D.log; exit 1; }
echo done
