#!/bin/bash
# Round-5 verification on one MI355X: the GPU suite, smoke, the driver's default command, its
# rocprofv3 kernel trace, and the N = 2 (gloo, one GPU) exchange rehearsal of config D.
#   tools/gpu_r05_verify.sh <tag>   -> gpurun_out/verify_<tag>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/verify_${1:-r05}; mkdir -p $out
step() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 400 python -u bench.py
step prof_default 400 rocprofv3 --kernel-trace --stats -d $out/prof_default -o run --output-format csv -- python -u bench.py --no-cpu-baseline
t=$(ls $out/prof_default/*/run_kernel_trace.csv $out/prof_default/run_kernel_trace.csv 2>/dev/null | head -n 1)
[ -n "$t" ] && python tools/prof_interval.py "$t" 20 --kernel "k_rx<1" > $out/prof_default_interval.json 2>&1
step bench_D2_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 2 --config D --backend gloo --frames 262144 --exchange-frames 262144 --steps 10 --warmup 2 --no-cpu-baseline
echo "done $(date +%T)"
