#!/bin/bash
# round 6: the full GPU suite, then the default bench line (only if the suite ended normally)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/gt.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gt.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 500 python -u bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err
