#!/bin/bash
# round 6 (e): the C++ exchange test, then the k_rx<2> owner-offset prefetch A/B
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread -m gpu \
  "tests/test_host_mirror.py" > gpurun_out/te.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/te.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/ab_r06_tol.sh
