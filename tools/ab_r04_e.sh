#!/bin/bash
# Round-4 A/B of config E (IMIX, window path): the in-tree build against the window-skip
# variants (EMURX_WSKIP: the cooperative checksum reads only the span bytes past each lane's
# header window; + EMURX_WIN_NT: non-temporal window loads; + EMURX_COOP_NT: non-temporal
# cooperative loads), interleaved on one box, then FETCH_SIZE of k_rx for each.  Built by
# tools/build_variant.sh wskip "-DEMURX_WSKIP=1"; wskipnt "... -DEMURX_WIN_NT=1"; wskipnt2
# "... -DEMURX_WIN_NT=1 -DEMURX_COOP_NT=1".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab4e
L=$PWD/trex-emu_amd/lib
for rep in 1 2; do
  for v in default wskip wskipnt wskipnt2; do
    lib=$L/libemurx.so; [ $v != default ] && lib=$L/libemurx_$v.so
    EMURX_LIB=$lib timeout -k 10 300 python bench.py --config E --steps 100 --warmup 10 --no-cpu-baseline --no-check \
      > gpurun_out/ab4e/E_${v}_$rep.log 2>&1 || { echo "fail $v"; tail -3 gpurun_out/ab4e/E_${v}_$rep.log; exit 1; }
    echo "E $v #$rep $(grep '^{' gpurun_out/ab4e/E_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["kernel_ms_mean"], r["frac"])')"
  done
done
for v in default wskip wskipnt wskipnt2; do
  lib=$L/libemurx.so; [ $v != default ] && lib=$L/libemurx_$v.so
  EMURX_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --kernel-include-regex k_rx -d gpurun_out/ab4e/pmc_$v \
    -o run --output-format csv -- python bench.py --config E --steps 40 --warmup 8 --no-cpu-baseline --no-check --no-replay \
    > gpurun_out/ab4e/pmc_$v.log 2>&1 || { echo "pmc fail $v"; tail -3 gpurun_out/ab4e/pmc_$v.log; exit 1; }
  f=$(ls gpurun_out/ab4e/pmc_$v/*/run_counter_collection.csv gpurun_out/ab4e/pmc_$v/run_counter_collection.csv 2>/dev/null | head -n 1)
  [ -n "$f" ] && python - "$f" "$v" <<'PY'
import csv, sys, statistics
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_rx" in r.get("Kernel_Name", "")]
vals = [float(r["Counter_Value"]) for r in rows if r.get("Counter_Name") == "FETCH_SIZE"]
print(sys.argv[2], "FETCH_SIZE KB per k_rx launch: median", statistics.median(vals) if vals else None, "n", len(vals))
PY
done
echo done
