#!/bin/bash
# The driver's 20-step bench with 2 / 3 / 4 streams (pipelined batches), and 200 steps.
export TMPDIR=/tmp
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['kernel_ms_mean'], r['frac'], r['pipelined']['interval_ms'])"; }
for st in 2 3 4; do
  for steps in "20 5" "200 20"; do
    set -- $steps
    timeout -k 10 200 python -u bench.py --steps $1 --warmup $2 --streams $st --no-cpu-baseline > gpurun_out/bs.log 2>&1 || exit 1
    summ gpurun_out/bs.log "streams=$st steps=$1"
  done
done
