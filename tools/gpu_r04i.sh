#!/bin/bash
# Round 4: the LDS-staged / cooperative tx checksum kernel and the shared coop_span_sum: the tx and
# rx window-path GPU parity tests, then the tx timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04h
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_txzmq.py -m gpu -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "tx or long_spans or configs or corpus" > gpurun_out/r04h/pytest_tx.log 2>&1
rc=$?; echo "tx parity rc=$rc"; tail -n 2 gpurun_out/r04h/pytest_tx.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r04h.sh
