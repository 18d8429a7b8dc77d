#!/bin/bash
# Round 4: config B's PMC passes without the namespace_exchange run in the same process, then
# the short-span checksum variant (EMURX_SHORTSUM=1): parity, then B / C / E interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/round_profile.sh r04f B pmc || exit 1
mkdir -p gpurun_out/ab
EMURX_LIB=$PWD/trex-emu_amd/lib/libemurx_ssum.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/ab/pytest_ssum.log 2>&1
rc=$?; echo "ssum parity rc=$rc"; tail -n 2 gpurun_out/ab/pytest_ssum.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_variants.sh "B C E" ssum
