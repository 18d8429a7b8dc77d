#!/bin/bash
# rocprofv3 kernel trace of config B's 20-step command (headline only): the per-launch timeline
# of the timed region (tools/trace_timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/trace20; mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $out/prof -o run \
  -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exchange-run --no-host-inclusive --no-replay \
  > $out/bench.log 2>&1 || exit $?
f=$(ls $out/prof/*/run_kernel_trace.csv $out/prof/run_kernel_trace.csv 2>/dev/null | head -n 1)
python tools/trace_timeline.py "$f" 20 --no-replay > $out/timeline.json || exit $?
gzip -c "$f" > $out/run_kernel_trace.csv.gz; rm -rf $out/prof
cat $out/timeline.json | head -c 3000
