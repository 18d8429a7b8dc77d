#!/bin/bash
# Counter passes over the tx framing write of config E (bench.py --tx-path), k_txz_emit only,
# one rocprofv3 run per pass (tools/pmc_sq.sh's sets).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmc_tx; rm -rf $out; mkdir -p $out
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1)); echo "== pass $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set -T --kernel-include-regex k_txz -d $out/p$i -o run --output-format csv \
      -- python bench.py --config ${CFG:-E} --steps 5 --warmup 2 --tx-path --no-exchange-run --no-cpu-baseline --no-check > $out/p$i.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -3 $out/p$i.log; exit $rc; }
done <<'SETS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE
SETS
python - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("gpurun_out/pmc_tx/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_txz_emit" not in r.get("Kernel_Name", ""):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"], r.get("Dispatch_Id")] += 1
disp = {}
for (c, d) in n:
    disp.setdefault(c, set()).add(d)
for c in sorted(tot):
    k = len(disp[c])
    print(f"{c:32s} {tot[c] / k:16.1f} per dispatch ({k} dispatches)")
PY
