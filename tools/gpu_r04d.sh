#!/bin/bash
# Round 4: every GPU test on the current default build (window-skip checksum now default).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04d
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -n 3 $out/pytest_gpu.log
exit $rc
