#!/bin/bash
# Round 4 final check on the committed tree: every GPU test, smoke, the default bench line and
# the driver's 20-step command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04v
mkdir -p $out
step() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python -u bench.py
step bench_driverlike 300 python -u bench.py --steps 20 --warmup 5
grep -h '^{' $out/bench_default.log $out/bench_driverlike.log | python -c '
import json, sys
for l in sys.stdin:
    d = json.loads(l); x = d.get("namespace_exchange", {})
    print(d["steps"], d["value"], d["roofline"]["frac"], d["roofline"].get("traffic"), x.get("value"), d.get("cpu_baseline", {}).get("value"))'
echo done
