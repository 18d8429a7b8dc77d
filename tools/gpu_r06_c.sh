#!/bin/bash
# Round 6 (c): the N > 1 rehearsals over gloo on this one GPU (the driver's torchrun form) with
# the measured transfer choice (--a2a auto), and the rocprofv3 kernel statistics of the
# driver's N = 1 command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r06c; mkdir -p $out
step() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step bench_N2_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29571 bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline
step bench_N8_gloo 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29581 bench.py --gpus 8 --backend gloo --steps 10 --warmup 3 --frames 262144 --exchange-frames 262144 \
  --batches 2 --no-cpu-baseline
step prof_driver 400 rocprofv3 --kernel-trace --stats -d $out/prof_driver -o run --output-format csv \
  -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
f=$(ls $out/prof_driver/*/run_kernel_stats.csv $out/prof_driver/run_kernel_stats.csv 2>/dev/null | head -n 1)
[ -n "$f" ] && cp "$f" $out/prof_driver_kernel_stats.csv && cut -d, -f1-4 "$f" | head -n 14
t=$(ls $out/prof_driver/*/run_kernel_trace.csv $out/prof_driver/run_kernel_trace.csv 2>/dev/null | head -n 1)
[ -n "$t" ] && python tools/prof_interval.py "$t" 20 > $out/prof_driver_interval.json && cat $out/prof_driver_interval.json
rm -rf $out/prof_driver
echo "done $(date +%T)"
