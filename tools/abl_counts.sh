#!/bin/bash
# Per-variant instruction counts (SQ_INSTS_* per wave, one rocprofv3 --pmc pass) and the one-launch
# k_rx time of ablation builds (tools/build_variant.sh abl<N> "-DEMURX_ABL=<N>", built from a
# temporarily patched tree; the knobs are not in the committed kernel).
#   tools/abl_counts.sh "<configs>" <variant> [variant ...]      (variant "default" = in-tree library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
configs=$1; shift
out=gpurun_out/abl; mkdir -p $out
for cfg in $configs; do
  args="--steps 30 --warmup 4"; [ $cfg != B ] && args="--config $cfg --steps 30 --warmup 4"
  for v in "$@"; do
    lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
    EMURX_LIB=$lib timeout -k 10 120 python bench.py $args --no-cpu-baseline --no-check --no-replay > $out/${cfg}_$v.log 2>&1 || { echo "fail $cfg $v"; tail -3 $out/${cfg}_$v.log; exit 1; }
    t=$(tail -1 $out/${cfg}_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["roofline"]["kernel_ms_mean"], d["roofline"]["pipelined"]["interval_ms"])')
    EMURX_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH \
      -T --kernel-include-regex k_rx -d $out/p_${cfg}_$v -o run --output-format csv -- python bench.py $args --no-cpu-baseline --no-check --no-replay > $out/p_${cfg}_$v.log 2>&1 || { echo "pmc fail $cfg $v"; tail -3 $out/p_${cfg}_$v.log; exit 1; }
    c=$(python - "$out/p_${cfg}_$v" <<'PY'
import csv, glob, sys, collections
per = collections.defaultdict(float)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        per[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
ds = sorted({d for d, _ in per})[3:]
tot = collections.defaultdict(float)
for d in ds:
    for (dd, c), v in per.items():
        if dd == d: tot[c] += v
w = tot["SQ_WAVES"] or 1
print(" ".join(f"{k[8:] if k.startswith('SQ_INSTS') else k[3:]}={tot[k]/w:.0f}" for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY")))
PY
)
    echo "$cfg $v one/pipe ms $t  per wave: $c"
  done
done
