#!/bin/bash
# Table spreads (slots per entry: ns, mac, ip, ci; EMURX_TABLE_SPREAD) against config D's
# partitioned step at N = 1 (k_lookup's random probe lines), interleaved, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_spread
for rep in 1 2; do
  for sp in default 8,4,16,16 8,4,8,8 8,16,16,16; do
    log=gpurun_out/ab_spread/D_${sp//,/_}_$rep.log
    if [ $sp = default ]; then e=""; else e="EMURX_TABLE_SPREAD=$sp"; fi
    env $e timeout -k 10 300 python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline --no-check \
      --no-exchange-run > $log 2>&1 || { echo "fail $sp"; tail -3 $log; exit 1; }
    echo "$sp #$rep $(python tools/exsum.py $log | tail -1)"
  done
done
