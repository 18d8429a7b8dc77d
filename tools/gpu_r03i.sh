# GPU suite, then coalesced lookup-record stores (default) against per-lane stores (libemurx_lkold.so) on partitioned D
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03i gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03i/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03i/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r03i/pytest_gpu.log
for rep in 1 2; do
  for v in default lkold; do
    lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
    EMURX_LIB=$lib timeout -k 10 300 python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline --no-check --no-replay > gpurun_out/ab/D_${v}_$rep.log 2>&1 || exit 1
    echo "D $v #$rep $(grep '^{' gpurun_out/ab/D_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["exchange"]["phases"]; print(d["value"], d["ms_per_step"], p["source_side_ms"], p["owner_count_scan_ms"], p["k_rx_ms"], p["owner_lookup_ms"], d["alternative"]["value"], d["alternative"]["exchange"]["phases"]["scan_pack_ms"])')"
  done
done
