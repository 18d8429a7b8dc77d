#!/bin/bash
# The driver's default command shape at N = 8 rehearsed on one GPU: 8 ranks over gloo (the
# collectives through host copies), smaller batches so that the host all-to-alls stay short.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/n8; mkdir -p $out
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29551 bench.py --gpus 8 --backend gloo --steps 6 --warmup 2 --frames 262144 --exchange-frames 262144 \
  --batches 2 --no-cpu-baseline > $out/bench_N8_gloo.log 2>&1
rc=$?; echo "N8 gloo rc=$rc"; tail -c 1500 $out/bench_N8_gloo.log; exit $rc
