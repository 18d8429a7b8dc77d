#!/bin/bash
# k_owner_count with 1 (default), 2, 4, 8 tiles per workgroup (-DEMURX_OC_TPW): tools/krx_kinds.py
# under rocprofv3 kernel stats per library (config D, 2M frames, keyed descriptors), then the
# partitioned parity tests with each variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/octpw; mkdir -p $out
for k in 1 2; do
  for v in "" _oc2 _oc4 _oc8; do
    lib=$PWD/trex-emu_amd/lib/libemurx$v.so
    EMURX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p$v$k -o run --output-format csv \
      -- python tools/krx_kinds.py > $out/kinds${v}_$k.log 2>&1 || exit $?
    f=$(ls $out/p$v$k/*/run_kernel_stats.csv $out/p$v$k/run_kernel_stats.csv 2>/dev/null | head -n 1)
    cp "$f" $out/stats${v}_$k.csv; rm -rf $out/p$v$k
    python - $out/stats${v}_$k.csv "$v" $out/kinds${v}_$k.log <<'PY'
import csv, json, sys
r = {row[0][:22]: (row[1], row[3]) for row in csv.reader(open(sys.argv[1])) if "owner_count" in row[0] or "route_scan" in row[0]}
k = [json.loads(l) for l in open(sys.argv[3]) if l.startswith("{")][-1]
print(sys.argv[2] or "_oc1", r, k["parse_route_k_rx2_with_counts_us_1"], k["k_rx2_alone_us"], flush=True)
PY
  done
done
for v in _oc4 _oc8; do
  EMURX_LIB=$PWD/trex-emu_amd/lib/libemurx$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tables.py tests/test_gpu_comm.py -m gpu -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest$v.log 2>&1 || { tail -n 30 $out/pytest$v.log; exit 1; }
  echo "$v $(tail -n 1 $out/pytest$v.log)"
done
