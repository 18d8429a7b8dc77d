#!/bin/bash
# Round 4: the early MAC-bucket touch variant (EMURX_EARLYPF=1): parity, then C / D (classify) / B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
EMURX_LIB=$PWD/trex-emu_amd/lib/libemurx_epf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "configs or corpus or fuzz or edge" > gpurun_out/ab/pytest_epf.log 2>&1
rc=$?; echo "epf parity rc=$rc"; tail -n 2 gpurun_out/ab/pytest_epf.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-exchange-run" bash tools/ab_variants.sh "C D B" epf
