#!/bin/bash
# The driver's 20-step command five times on one box: the spread of the headline and of
# namespace_exchange on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/driver5; mkdir -p $out
for k in 1 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/run_$k.log 2>&1 || exit $?
  python - $out/run_$k.log <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["namespace_exchange"]["value"],
      d["host_inclusive"]["with_host_copy"]["mpkts"], flush=True)
PY
done
