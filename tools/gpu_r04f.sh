#!/bin/bash
# Round 4: GPU parity after the one-D2H ingest result block, then the uniform-key scalar hashing
# variant (EMURX_UNIHASH=1) against the in-tree build on B / C / E / D classification.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04f
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_host_mirror.py -m gpu -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/r04f/pytest_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -n 2 gpurun_out/r04f/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-exchange-run" bash tools/ab_variants.sh "B C E" uhash
