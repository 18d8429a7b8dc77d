# k_owner_count with its frame bytes staged by LDS-DMA (libemurx_ocstage.so) against the per-lane
# gather (the default): the partitioned GPU tests, then partitioned D at N = 1, two rounds
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03n gpurun_out/ab
EMURX_LIB=$PWD/trex-emu_amd/lib/libemurx_ocstage.so timeout -k 10 400 python -u -m pytest tests/test_gpu_tables.py tests/test_bench_launch.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03n/pytest_tables.log 2>&1 || { tail -40 gpurun_out/r03n/pytest_tables.log; exit 1; }
tail -2 gpurun_out/r03n/pytest_tables.log
for rep in 1 2; do
  for v in default ocstage; do
    lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
    EMURX_LIB=$lib timeout -k 10 300 python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline --no-check --no-replay > gpurun_out/ab/Dn_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/ab/Dn_${v}_$rep.log; exit 1; }
    echo "D $v #$rep $(grep '^{' gpurun_out/ab/Dn_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["exchange"]["phases"]; print(d["value"], d["ms_per_step"], p["source_side_ms"], p["owner_count_scan_ms"], p["k_rx_ms"], p["owner_lookup_ms"])')"
  done
done
EMURX_LIB=$PWD/trex-emu_amd/lib/libemurx_ocstage.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r03n/prof_D -o run --output-format csv \
    -- python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r03n/prof_D.log 2>&1 || { tail -20 gpurun_out/r03n/prof_D.log; exit 1; }
echo done
