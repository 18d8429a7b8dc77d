#!/bin/bash
# Round-6 check of the tree: the GPU suite, smoke, the driver's 20-step command, the default
# command (with the CPU baseline), and the default command at N = 2 over gloo on this one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/final_${1:-r06}; mkdir -p $out
step() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_driver 400 python -u bench.py --gpus 1 --steps 20 --warmup 5
step bench_default 500 python -u bench.py
step bench_N2_gloo 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29571 bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline
echo "done $(date +%T)"
# the driver's command under rocprofv3 kernel stats (the same bench, profiled)
if [ "${PROF:-0}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv \
    -- python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/prof_driver.log 2>&1 || exit $?
  f=$(ls $out/prof/*/run_kernel_stats.csv $out/prof/run_kernel_stats.csv 2>/dev/null | head -n 1)
  cp "$f" $out/prof_driver_kernel_stats.csv && rm -rf $out/prof
  echo "prof done $(date +%T)"
fi
