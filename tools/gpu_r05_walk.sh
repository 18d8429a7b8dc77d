#!/bin/bash
# The framing walk: its GPU tests (walk, ingest, rx stream), then config D's exchange line
# (key_derivation: the walk with and without the owner keys).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/walk; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "walk or ingest or stream" \
  --timeout 300 --timeout-method thread > $out/pytest_walk.log 2>&1
rc=$?; echo "walk tests rc=$rc"; tail -n 2 $out/pytest_walk.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline --no-check --no-exchange-run \
    > $out/D_$r.log 2>&1 || { tail -5 $out/D_$r.log; exit 1; }
  grep '^{' $out/D_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["exchange"]; print(d["value"], json.dumps(e["key_derivation"])[:200])'
done
