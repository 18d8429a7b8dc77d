#!/bin/bash
# The own region's copy on the caller's stream (whole regions): the comm GPU tests, the C++
# exchange test, the bench's GPU tests, and the 1-rank probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/selfcopy; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_comm.py tests/test_host_mirror.py tests/test_bench_launch.py -m gpu -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -n 40 $out/pytest.log; exit 1; }
tail -n 2 $out/pytest.log
for s in copy rccl; do
  EMURX_COMM_SELF=$s timeout -k 10 300 python tools/comm_fence_probe.py 50 > $out/probe_$s.json 2> $out/probe_$s.err || exit $?
  cat $out/probe_$s.json
done
