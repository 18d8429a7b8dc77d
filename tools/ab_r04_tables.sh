#!/bin/bash
# Round-4 A/B on one box: the sparse single-line tables (in-tree libemurx.so) against the
# two-choice cuckoo tables (libemurx_cuckoo.so, built from branch exp-cuckoo), interleaved,
# and the partitioned exchange step with keyed / unkeyed descriptors.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab4
L=$PWD/trex-emu_amd/lib
one() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  EMURX_LIB=$L/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange-run "$@" > gpurun_out/ab4/$tag.log 2>&1
  local rc=$?
  [ $rc -eq 0 ] || { echo "fail $tag rc=$rc"; tail -3 gpurun_out/ab4/$tag.log; exit $rc; }
  grep '^{' gpurun_out/ab4/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; x=d.get("exchange",{}); ph=x.get("phases") or {}; print("'$tag'", d["value"], d["ms_per_step"], r["kernel_ms_mean"], r["frac"], x.get("one_stream_steps",{}).get("value",""), ph.get("owner_count_scan_ms",""), ph.get("owner_lookup_ms",""))'
}
for rep in 1 2; do
  for v in sparse cuckoo; do
    lib=libemurx.so; [ $v = cuckoo ] && lib=libemurx_cuckoo.so
    one B_${v}_$rep $lib --steps 200 --warmup 20
    one C_${v}_$rep $lib --config C --steps 100 --warmup 10
    one DN_${v}_$rep $lib --config D --tables none --steps 50 --warmup 5
    one DP_${v}_keyed_$rep $lib --config D --steps 50 --warmup 5
  done
  one DP_sparse_unkeyed_$rep libemurx.so --config D --steps 50 --warmup 5 --unkeyed
done
echo done
