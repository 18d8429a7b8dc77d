# GPU suite (with the single-pass vs two-pass owner-offset test), then single-pass owner offsets
# (default) against the two-pass source (EMURX_OWNER_PASS=1) on partitioned D, then a
# rocprofv3 kernel trace of the single-pass D step
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03j gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_tables.py -x -v --timeout 120 --timeout-method thread -k "single_pass or partitioned" > gpurun_out/r03j/pytest_tables.log 2>&1 || { tail -40 gpurun_out/r03j/pytest_tables.log; exit 1; }
tail -3 gpurun_out/r03j/pytest_tables.log
for rep in 1 2; do
  for v in single twopass; do
    op=0; [ $v = twopass ] && op=1
    EMURX_OWNER_PASS=$op timeout -k 10 300 python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline --no-check --no-replay > gpurun_out/ab/D_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/ab/D_${v}_$rep.log; exit 1; }
    echo "D $v #$rep $(grep '^{' gpurun_out/ab/D_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["exchange"]["phases"]; print(d["value"], d["ms_per_step"], p["source_side_ms"], p["owner_count_scan_ms"], p["k_rx_ms"], p["owner_lookup_ms"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r03j/prof_D -o run --output-format csv \
    -- python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r03j/prof_D.log 2>&1 || { tail -20 gpurun_out/r03j/prof_D.log; exit 1; }
echo done
