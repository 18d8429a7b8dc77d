#!/bin/bash
# Config D's N = 1 exchange step (partitioned, pipelined over S streams with their own buffers):
# S = 2 (the default), 3, 4, interleaved, two runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/dstreams; mkdir -p $out
for k in 1 2; do
  for s in 2 3 4; do
    timeout -k 10 300 python bench.py --config D --steps 50 --warmup 10 --streams $s --no-cpu-baseline --no-exchange-run \
      > $out/D_s${s}_$k.json 2> $out/D_s${s}_$k.err || exit $?
    python - $out/D_s${s}_$k.json $s <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("streams", sys.argv[2], d["value"], d["ms_per_step"], d["exchange"].get("one_stream_steps", {}).get("value"), flush=True)
PY
  done
done
