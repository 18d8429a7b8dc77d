#!/bin/bash
# GPU suite + the config-D exchange benches (partitioned and replicated, N = 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r03c; mkdir -p $out
run() { local name=$1 to=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$to" "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n ${TAILN:-3} $out/$name.log | cut -c1-3000; [ $rc -eq 0 ] || exit $rc; }
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 580 --timeout-method thread
run bench_D 600 python -u bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline
echo done
