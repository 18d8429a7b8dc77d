#!/bin/bash
# PC sampling of k_rx on config B (rocprofv3 beta; hot instructions by sample count).
#   tools/pcsample.sh [method] [unit] [interval] [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pcs; mkdir -p $out
m=${1:-host_trap}; u=${2:-time}; iv=${3:-1}; shift 3 || true
timeout -k 10 120 rocprofv3 -L > $out/list.txt 2>&1; grep -i -A12 "pc" $out/list.txt | head -40
ROCPROFILER_PC_SAMPLING_BETA_ENABLED=1 timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $m \
  --pc-sampling-unit $u --pc-sampling-interval $iv -d $out/run -o run --output-format csv \
  -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-check --no-replay --no-exchange-run "$@" > $out/run.log 2>&1
rc=$?; echo "rc=$rc"; tail -5 $out/run.log; ls -R $out/run | head -20
exit $rc
