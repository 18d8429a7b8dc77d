#!/bin/bash
# A/B of an alternative libemurx.so against the in-tree one under one environment setting:
#   tools/ab_lib_env.sh <alt.so> "<VAR=val ...>" [configs...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
alt=$1; e=$2; shift 2
mkdir -p gpurun_out/ab
for cfg in ${@:-B C E}; do
  for v in default alt; do
    lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v = alt ] && lib=$PWD/$alt
    env $e EMURX_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 200 --warmup 20 --no-cpu-baseline --no-check \
      > gpurun_out/ab/${cfg}_$v.log 2>&1 || { echo "fail $cfg $v"; tail -3 gpurun_out/ab/${cfg}_$v.log; exit 1; }
    echo "$cfg $v [$e] $(tail -1 gpurun_out/ab/${cfg}_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_mean"], d["roofline"]["frac"])')"
  done
done
