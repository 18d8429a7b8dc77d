#!/bin/bash
# The host-inclusive passes of config B with the runtime's copy engines (default: SDMA) and with
# copies as blit kernels (HSA_ENABLE_SDMA=0), interleaved, two runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/sdma; mkdir -p $out
for k in 1 2; do
  for m in default blit; do
    if [ $m = blit ]; then export HSA_ENABLE_SDMA=0; else unset HSA_ENABLE_SDMA; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exchange-run \
      > $out/B_${m}_$k.json 2> $out/B_${m}_$k.err || exit $?
    python - $out/B_${m}_$k.json $m <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
h = d["host_inclusive"]
print(sys.argv[2], "value", d["value"], "copy", h["with_host_copy"]["mpkts"], "1thr", h["with_host_copy_1_thread"]["mpkts"],
      "prefilled", h["prefilled"]["mpkts"], flush=True)
PY
  done
done
