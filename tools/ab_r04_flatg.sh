#!/bin/bash
# Round-4 A/B of the flat resolver with its views guarded by wave-uniform tests (EMURX_FLATRES=1
# after the hybrid runs) against the in-tree build: GPU parity of flat first, then configs
# C / B / D (replicated) interleaved, then SQ counts of k_rx on config C.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/ab4g
mkdir -p $out
L=$PWD/trex-emu_amd/lib
EMURX_LIB=$L/libemurx_flat.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tables.py \
  -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/pytest_flat.log 2>&1
rc=$?; echo "flat parity rc=$rc"; tail -n 3 $out/pytest_flat.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for cfg in "C" "B" "D --tables none"; do
    for v in default flat; do
      lib=$L/libemurx.so; [ $v != default ] && lib=$L/libemurx_$v.so
      tag=$(echo "$cfg" | tr -d ' -')_${v}_$rep
      EMURX_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline \
        --no-exchange-run > $out/$tag.log 2>&1 || { echo "fail $tag"; tail -3 $out/$tag.log; exit 1; }
      echo "$tag $(grep '^{' $out/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r.get("kernel_ms_mean"), r["frac"])')"
    done
  done
done
for v in default flat; do
  lib=$L/libemurx.so; [ $v != default ] && lib=$L/libemurx_$v.so
  EMURX_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES \
    -T --kernel-include-regex k_rx -d $out/sq_$v -o run --output-format csv \
    -- python bench.py --config C --steps 40 --warmup 8 --no-cpu-baseline --no-check --no-replay \
    > $out/sq_$v.log 2>&1 || { echo "sq fail $v"; tail -3 $out/sq_$v.log; exit 1; }
  f=$(ls $out/sq_$v/*/run_counter_collection.csv $out/sq_$v/run_counter_collection.csv 2>/dev/null | head -n 1)
  [ -n "$f" ] && python - "$f" "$v" <<'PY'
import csv, sys, statistics, collections
per = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_rx" in r.get("Kernel_Name", ""):
        per[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
by = collections.defaultdict(list)
for (d, c), v in sorted(per.items()):
    by[c].append(v)
med = {c: statistics.median(v[3:] or v) for c, v in by.items()}
w = med.get("SQ_WAVES", 1) or 1
print(sys.argv[2], " ".join(f"{c}={med[c]:.0f} ({med[c] / w:.1f}/wave)" for c in sorted(med)))
PY
done
echo done
