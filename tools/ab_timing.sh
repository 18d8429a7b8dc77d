#!/bin/bash
# k_rx timing modes side by side on one box (config B): one event pair around the timed region,
# events around single launches, none, then the rocprof kernel statistics of the same bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/ab_timing; mkdir -p $out
for k in 1 2; do
  for tr in "region" "launch" "off" "launch --time-stride 1"; do
    tag=$(echo "$tr" | tr -d ' -')
    timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --kernel-timing $tr > $out/run${tag}_$k.log 2>&1 || exit $?
    python - "$out/run${tag}_$k.log" "$tr" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("kernel-timing", sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_mean"], d["roofline"]["frac"],
      d["host_submit_ms_per_step"])
PY
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv \
  -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --kernel-timing off > $out/prof.log 2>&1 || exit $?
f=$(ls $out/prof/*/run_kernel_stats.csv $out/prof/run_kernel_stats.csv 2>/dev/null | head -n 1)
cut -d, -f1-8 "$f"
