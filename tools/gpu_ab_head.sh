#!/bin/bash
# The in-tree library against the last commit's (lib/libemurx_head.so): GPU parity suite on the
# in-tree one, then interleaved bench A/B.   tools/gpu_ab_head.sh "<configs>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 580 --timeout-method thread > gpurun_out/ab/pytest_new.log 2>&1; rc=$?; tail -2 gpurun_out/ab/pytest_new.log; [ $rc -eq 0 ] || exit $rc
AB_ARGS="--no-replay" bash tools/ab_variants.sh "${1:-B C E}" head
