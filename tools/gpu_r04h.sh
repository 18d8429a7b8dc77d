#!/bin/bash
# Round 4: the tx paths timed (bench.py --tx-path: tx ZMQ framing and tx checksum generation)
# on configs B and E, and rocprofv3 kernel stats of the same.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04h; mkdir -p $out
for c in B E; do
  timeout -k 10 300 python -u bench.py --config $c --steps 50 --warmup 5 --tx-path --no-exchange-run --no-cpu-baseline \
    > $out/tx_$c.log 2>&1 || { tail -5 $out/tx_$c.log; exit 1; }
  grep '^{' $out/tx_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$c'", json.dumps(d["tx_zmq"]), json.dumps(d["tx_checksum"]))'
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$c -o run --output-format csv -- python bench.py --config $c \
    --steps 20 --warmup 5 --tx-path --no-exchange-run --no-cpu-baseline > $out/prof_$c.log 2>&1 || { tail -5 $out/prof_$c.log; exit 1; }
  f=$(ls $out/prof_$c/*/run_kernel_stats.csv $out/prof_$c/run_kernel_stats.csv 2>/dev/null | head -n 1)
  [ -n "$f" ] && grep -i "tx" "$f" | cut -d, -f1-4
done
echo done
