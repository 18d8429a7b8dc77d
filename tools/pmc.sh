#!/bin/bash
# PMC passes for the bench workload (each --pmc set fits one hardware pass).
#   tools/pmc.sh <tag> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/pmc_$tag
[ -f gpurun_out/counters_list.txt ] || timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1))
  echo "== pass $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set -T --kernel-include-regex "k_rx" \
      -d gpurun_out/pmc_$tag/p$i -o run --output-format csv \
      -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/pmc_$tag/p$i.log 2>&1
  rc=$?; echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc_$tag/p$i.log; [ $rc -ne 1 ] && exit $rc; fi
done <<'SETS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
SETS
echo done
