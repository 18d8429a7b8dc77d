#!/bin/bash
# The exchange's phase times measured as back-to-back groups: the bench's GPU tests, the
# driver's command, and the N = 2 gloo command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/phases; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_bench_launch.py -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $out/pytest_bench.log 2>&1 || { tail -n 40 $out/pytest_bench.log; exit 1; }
tail -n 2 $out/pytest_bench.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.log 2>&1 || exit $?
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29571 bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_N2_gloo.log 2>&1 || exit $?
for f in bench_driver bench_N2_gloo; do
python - $out/$f.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); x = d["namespace_exchange"]
        print(sys.argv[1], d["value"], x["value"], json.dumps(x["exchange"]["phases"])[:700])
PY
done
