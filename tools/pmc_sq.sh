#!/bin/bash
# Counter passes over the config-B bench (k_rx only), one rocprofv3 run per pass.
#   tools/pmc_sq.sh [sq|mem] [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmc_sq${PMC_TAG:-}; rm -rf $out; mkdir -p $out
timeout -s KILL 60 rocprofv3 -L > $out/counters_list.txt 2>&1
i=0
mode=${1:-sq}; shift || true
if [ "$mode" = icache ]; then
  SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE"
elif [ "$mode" = mem ]; then
  SETS="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE
TA_DATA_STALLED_BY_TC_CYCLES TA_ADDR_STALLED_BY_TD_CYCLES GRBM_GUI_ACTIVE
TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES GRBM_GUI_ACTIVE
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"
else
  SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA
SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_INT32 SQ_IFETCH GRBM_GUI_ACTIVE"
fi
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1)); echo "== pass $i: $set"
  timeout -s KILL 90 rocprofv3 --pmc $set -T --kernel-include-regex k_rx -d $out/p$i -o run --output-format csv \
      -- python bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-check "$@" > $out/p$i.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -3 $out/p$i.log; exit $rc; }
done <<< "$SETS"
OUT=$out python - <<'PY'
import csv, glob, collections, os
tot = collections.defaultdict(list)
for f in glob.glob(os.environ["OUT"] + "/p*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        tot[c].append((int(d), v))
for c, l in sorted(tot.items()):
    l.sort(); v = [x[1] for x in l][3:] or [x[1] for x in l]
    print(f"{c:28s} {sum(v)/len(v):14.1f}")
PY
