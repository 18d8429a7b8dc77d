#!/bin/bash
# (Record of a trial: emurx_ingest_stage and the staged pass were removed after this run.)
# emurx_ingest_stage: the ingest GPU tests, then the host-inclusive passes of config B with the
# receive staging every 1/parts of the batch (parts 4, 8, 16; two runs each, interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/stage; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k ingest -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $out/pytest_ingest.log 2>&1 || { tail -n 40 $out/pytest_ingest.log; exit 1; }
tail -n 2 $out/pytest_ingest.log
for k in 1 2; do
  for p in 4 8 16; do
    EMURX_BENCH_STAGE_PARTS=$p timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exchange-run \
      > $out/B_p${p}_$k.json 2> $out/B_p${p}_$k.err || exit $?
    python - $out/B_p${p}_$k.json $p <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
h = d["host_inclusive"]
print("parts", sys.argv[2], "copy", h["with_host_copy"]["mpkts"], "staged", h["with_host_copy_staged"]["mpkts"],
      "1thr", h["with_host_copy_1_thread"]["mpkts"], "prefilled", h["prefilled"]["mpkts"], flush=True)
PY
  done
done
