#!/bin/bash
# Device-scope ordering / timing events: the comm GPU tests and the C++ exchange test, then the
# exchange step on a 1-rank communicator with the ordering events at device and at system scope
# (interleaved), with the own region by device copy and through RCCL, then the driver command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/fence; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_comm.py tests/test_host_mirror.py -m gpu -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $out/pytest_comm.log 2>&1 || { tail -n 40 $out/pytest_comm.log; exit 1; }
tail -n 2 $out/pytest_comm.log
for k in 1 2; do
  for f in device system; do
    for s in copy rccl; do
      EMURX_COMM_FENCE=$f EMURX_COMM_SELF=$s timeout -k 10 300 python tools/comm_fence_probe.py 50 \
        > $out/probe_${f}_${s}_$k.json 2> $out/probe_${f}_${s}_$k.err || exit $?
      cat $out/probe_${f}_${s}_$k.json
    done
  done
done
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.log 2>&1 || exit $?
python - $out/bench_driver.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); x = d["namespace_exchange"]
        print(d["value"], x["value"], x["k_rx_ms_mean"], json.dumps(x["exchange"]["phases"])[:300])
PY
