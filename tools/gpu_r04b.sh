#!/bin/bash
# Round 4: the small-ingest latency path (host completion word) — its parity tests, then the
# default bench line with --host-path (latency by batch size, crossover).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04b
mkdir -p $out
step() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step pytest_ingest 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 \
  --timeout-method thread -k "ingest or stream or zmq"
step bench_B_host 600 python -u bench.py --host-path --no-exchange-run
grep '^{' $out/bench_B_host.log | python -c 'import json,sys; d=json.loads(sys.stdin.read())["host_inclusive"]; print(json.dumps({k: d[k] for k in ("batch_latency_by_msgs", "two_slot_rate_by_msgs", "crossover") if k in d}))'
echo done
