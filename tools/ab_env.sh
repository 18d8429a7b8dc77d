#!/bin/bash
# A/B of environment settings with the in-tree library: tools/ab_env.sh "<VAR=val ...>" "<VAR=val ...>" [configs...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
a=$1; b=$2; shift 2
mkdir -p gpurun_out/ab
for cfg in ${@:-B C E}; do
  for v in a b; do
    e=$a; [ $v = b ] && e=$b
    env $e timeout -k 10 300 python bench.py --config $cfg --steps 200 --warmup 20 --no-cpu-baseline --no-check \
      > gpurun_out/ab/${cfg}_$v.log 2>&1 || { echo "fail $cfg $v"; tail -3 gpurun_out/ab/${cfg}_$v.log; exit 1; }
    echo "$cfg [$e] $(tail -1 gpurun_out/ab/${cfg}_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "one", d["roofline"]["kernel_ms_mean"], d["roofline"]["frac"], "pipe", d["roofline"].get("pipelined",{}).get("interval_ms"))')"
  done
done
