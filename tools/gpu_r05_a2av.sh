#!/bin/bash
# The payload-sized exchange (--a2a v) against whole regions (--a2a equal): the N = 2 GPU tests
# of the bench's exchange, then config D at N = 2 and the default command at N = 8, both over
# gloo on this one GPU (protocol and bytes; rates are the host copies').
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/a2av; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_bench_launch.py -m gpu -x -q -p no:cacheprovider --timeout 600 \
  --timeout-method thread > $out/pytest_launch.log 2>&1
rc=$?; echo "launch tests rc=$rc"; tail -n 2 $out/pytest_launch.log; [ $rc -eq 0 ] || exit $rc
for v in v equal; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 2956$([ $v = v ] && echo 1 || echo 2) bench.py --gpus 2 --config D --backend gloo --frames 262144 \
    --exchange-frames 262144 --steps 10 --warmup 2 --no-cpu-baseline --a2a $v > $out/D2_$v.log 2>&1 || { echo "D2 $v fail"; tail -5 $out/D2_$v.log; exit 1; }
  echo "D2 $v: $(python tools/exsum.py $out/D2_$v.log | tail -2 | head -1)"
done
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29563 bench.py --gpus 8 --backend gloo --steps 6 --warmup 2 --frames 262144 --exchange-frames 262144 \
  --batches 2 --no-cpu-baseline > $out/N8.log 2>&1 || { echo "N8 fail"; tail -5 $out/N8.log; exit 1; }
python tools/exsum.py $out/N8.log
echo done
