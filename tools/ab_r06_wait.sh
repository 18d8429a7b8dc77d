#!/bin/bash
# The driver's 20-step command of config B (headline only) with the HIP runtime's default host
# wait (active for ROC_ACTIVE_WAIT_TIMEOUT us, then the completion interrupt) and with an active
# wait long enough to cover the whole region, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/ab_wait; mkdir -p $out
for k in 1 2 3 4; do
  for w in default 2000; do
    if [ $w = default ]; then unset ROC_ACTIVE_WAIT_TIMEOUT; else export ROC_ACTIVE_WAIT_TIMEOUT=$w; fi
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exchange-run --no-host-inclusive \
      > $out/run_${w}_$k.log 2>&1 || exit $?
    python - "$out/run_${w}_$k.log" "$w" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d["roofline"].get("pipelined", {})
print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_mean"], p.get("interval_ms"),
      d["host_submit_ms_per_step"], flush=True)
PY
  done
done
