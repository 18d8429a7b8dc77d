#!/bin/bash
# Round 4 evidence, part A: the driver-like command, then bench lines and rocprofv3 kernel
# traces per config (tools/round_profile.sh r04f).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/round_r04f
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/round_r04f/driverlike_B.log 2>&1 || exit 1
grep '^{' gpurun_out/round_r04f/driverlike_B.log | cut -c1-400
bash tools/round_profile.sh r04f "B C D DN E" "bench prof"
