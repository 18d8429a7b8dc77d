#!/bin/bash
# Round-3 check: GPU parity suite, smoke, timeline stamps (rotating vs replayed input) and SQ
# counters of config B on rotating input.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03b
run() { local name=$1 to=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$to" "$@" > gpurun_out/r03b/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n ${TAILN:-4} gpurun_out/r03b/$name.log; [ $rc -eq 0 ] || exit $rc; }
run pytest_gpu 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=16 run stamps_rot 300 env EMURX_LIB=$PWD/trex-emu_amd/lib/libemurx_stamp.so python tools/stamps.py B C
TAILN=16 run stamps_replay 300 env EMURX_LIB=$PWD/trex-emu_amd/lib/libemurx_stamp.so python tools/stamps.py --replay B
TAILN=30 run pmc_sq_B 600 bash tools/pmc_sq.sh sq --no-replay
echo done
