#!/bin/bash
# Round 4: the TransportCtx bit in the client slots (no client-info probe for the transport flow
# rule): GPU parity, then the in-tree build against the previous one (libemurx_ciprobe.so) on E / C / B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tables.py -m gpu -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/ab/pytest_ctxbit.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -n 2 gpurun_out/ab/pytest_ctxbit.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-exchange-run" bash tools/ab_variants.sh "E C B" ciprobe
