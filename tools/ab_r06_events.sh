#!/bin/bash
# The driver's 20-step command of config B with the region's HIP events inside the wall-timed
# region (region) and without them (off), interleaved; plus 3 streams.  Headline only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/ab_events; mkdir -p $out
for k in 1 2 3 4; do
  for tr in "--kernel-timing region" "--kernel-timing off" "--kernel-timing region --streams 3"; do
    tag=$(echo "$tr" | tr -d ' -')
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exchange-run --no-host-inclusive \
      $tr > $out/run${tag}_$k.log 2>&1 || exit $?
    python - "$out/run${tag}_$k.log" "$tr" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d["roofline"].get("pipelined", {})
print(sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_mean"], p.get("interval_ms"),
      d["host_submit_ms_per_step"], flush=True)
PY
  done
done
