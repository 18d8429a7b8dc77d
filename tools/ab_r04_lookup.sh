#!/bin/bash
# k_lookup register variants on config D's partitioned step (tools/build_variant.sh builds):
# the in-tree library against libemurx_<name>.so, interleaved, plus one rocprofv3 kernel-trace
# run each for k_lookup's mean duration.   tools/ab_r04_lookup.sh <name> [name...]
# AB_ARGS: extra bench.py arguments (e.g. --unkeyed); AB_TAG: a suffix for the output directory
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/ab_lookup${AB_TAG:-}; mkdir -p $out
lib_of() { [ $1 = default ] && echo $PWD/trex-emu_amd/lib/libemurx.so || echo $PWD/trex-emu_amd/lib/libemurx_$1.so; }
for rep in 1 2; do
  for v in default "$@"; do
    log=$out/D_${v}_$rep.log
    EMURX_LIB=$(lib_of $v) timeout -k 10 300 python bench.py --config D --steps 100 --warmup 10 --no-cpu-baseline ${AB_ARGS:-} \
      > $log 2>&1 || { echo "fail $v"; tail -3 $log; exit 1; }
    echo "D $v #$rep $(grep '^{' $log | python -c '
import json, sys
d = json.loads(sys.stdin.read()); x = d.get("namespace_exchange", d); e = x.get("exchange", {}); p = e.get("phases", {})
print(d["value"], d["ms_per_step"], "lookup_ms", p.get("owner_lookup_ms"), "k_rx_ms", p.get("k_rx_ms"))')"
  done
done
for v in default "$@"; do
  EMURX_LIB=$(lib_of $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$v -o run --output-format csv \
    -- python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline ${AB_ARGS:-} > $out/prof_$v.log 2>&1 \
    || { echo "prof fail $v"; tail -3 $out/prof_$v.log; exit 1; }
  f=$(ls $out/prof_$v/run_kernel_stats.csv $out/prof_$v/*/run_kernel_stats.csv 2>/dev/null | head -n 1)
  [ -n "$f" ] && echo "$v $(grep -E 'k_lookup|k_owner_count' "$f" | cut -d, -f1-4)"
done
echo done
