#!/bin/bash
# Ablation builds (EMURX_ABL bits, tools/build_variant.sh abl<N>) on one config: k_rx time and
# per-wave instruction counts.   [COUNTERS="..."] tools/abl_counts.sh <config> <variant>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
cfg=$1; shift
COUNTERS=${COUNTERS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU"}
out=gpurun_out/abl_$cfg; mkdir -p $out
for v in default "$@"; do
  lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
  EMURX_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-check \
    --tables none > $out/bench_$v.log 2>&1 || { tail -3 $out/bench_$v.log; exit 1; }
  EMURX_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $COUNTERS -T --kernel-include-regex k_rx -d $out/p_$v -o run \
    --output-format csv -- python bench.py --config $cfg --steps 20 --warmup 4 --no-cpu-baseline --no-check \
    --tables none > $out/pmc_$v.log 2>&1 || { tail -3 $out/pmc_$v.log; exit 1; }
  python - "$out" "$v" <<'PY'
import csv, glob, json, sys, collections
out, v = sys.argv[1], sys.argv[2]
d = json.loads([l for l in open(f"{out}/bench_{v}.log") if l.startswith("{")][-1])
tot = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob(f"{out}/p_{v}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
per = collections.defaultdict(list)
for (dsp, c), x in tot.items():
    per[c].append(x)
m = {c: sum(x) / len(x) for c, x in per.items()}
w = m.get("SQ_WAVES", 1)
print(v, "k_rx_ms", d["roofline"]["kernel_ms_mean"], "per wave:",
      " ".join(f"{c[8:] if c.startswith('SQ_INSTS') else c[3:]}={m[c] / w:.0f}" for c in sorted(m) if c != "SQ_WAVES"))
PY
done
