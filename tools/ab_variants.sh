#!/bin/bash
# Bench the in-tree libemurx.so and alternative builds (tools/build_variant.sh) on one box,
# interleaved, per config:   tools/ab_variants.sh "<configs>" <name> [name...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
configs=$1; shift
mkdir -p gpurun_out/ab
for cfg in $configs; do
  for rep in 1 2; do
    for v in default "$@"; do
      lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
      log=gpurun_out/ab/${cfg}_${v}_$rep.log
      EMURX_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline \
        --no-check --tables none ${AB_ARGS:-} > $log 2>&1 || { echo "fail $cfg $v"; tail -3 $log; exit 1; }
      echo "$cfg $v #$rep $(grep '^{' $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_mean"], d["roofline"]["frac"])')"
    done
  done
done
