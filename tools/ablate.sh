#!/bin/bash
# Stage ablation (experiment only): build k_rx with stages skipped (EMURX_ABL bits: 1 checksum,
# 2 classify, 4 histogram, 8 queues, 16 records) and time each with bench.py + PMC counts.
#   tools/ablate.sh build            (here, CPU)       -> trex-emu_amd/lib/abl/libemurx_<bits>.so
#   tools/ablate.sh run [bench args] (GPU box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARIANTS="0 1 2 4 8 16 31"
if [ "${1:-run}" = build ]; then
  mkdir -p trex-emu_amd/lib/abl trex-emu_amd/build/abl
  for v in $VARIANTS; do
    H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DEMURX_ABL=$v"
    $H -c trex-emu_amd/csrc/emurx_kernels.hip -o trex-emu_amd/build/abl/k$v.o &&
    $H -c trex-emu_amd/csrc/emurx_route.hip -o trex-emu_amd/build/abl/r$v.o &&
    $H -shared -o trex-emu_amd/lib/abl/libemurx_$v.so trex-emu_amd/build/abl/k$v.o trex-emu_amd/build/abl/r$v.o \
       trex-emu_amd/build/emurx_ingest.o trex-emu_amd/build/emurx_tx.o trex-emu_amd/build/emurx_txzmq.o trex-emu_amd/build/emurx_api.o || exit 1
  done
  exit 0
fi
shift
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
for v in $VARIANTS; do
  EMURX_LIB=$PWD/trex-emu_amd/lib/abl/libemurx_$v.so timeout -k 10 300 \
    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -T --kernel-include-regex k_rx \
    -d gpurun_out/abl/p$v -o run --output-format csv \
    -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check "$@" > gpurun_out/abl/pmc_$v.log 2>&1 || { echo "pmc $v rc=$?"; exit 1; }
  EMURX_LIB=$PWD/trex-emu_amd/lib/abl/libemurx_$v.so timeout -k 10 300 \
    python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-check "$@" > gpurun_out/abl/bench_$v.log 2>&1 || { echo "bench $v rc=$?"; exit 1; }
  echo "abl $v: $(grep -o '"kernel_ms_mean": [0-9.]*' gpurun_out/abl/bench_$v.log)"
done
