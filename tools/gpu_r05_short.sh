#!/bin/bash
# The driver's 20-step command against longer regions, and a kernel trace of the 20-step run
# (per-launch start / end inside the timed region).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/short; mkdir -p $out
for s in 20 40 100; do
  timeout -k 10 300 python -u bench.py --steps $s --warmup 5 --no-cpu-baseline --no-exchange-run --no-host-inclusive > $out/steps_$s.log 2>&1 || { tail -5 $out/steps_$s.log; exit 1; }
  grep '^{' $out/steps_$s.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("'$s'", d["value"], d["ms_per_step"], r["pipelined"]["interval_ms"], d["host_submit_ms_per_step"])'
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 \
  --no-cpu-baseline --no-exchange-run --no-host-inclusive > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
echo done
