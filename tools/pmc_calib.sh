#!/bin/bash
# FETCH_SIZE calibration on the GPU box (tools/pmc_calib.hip, built as trex-emu_amd/build/pmc_calib):
# per mode one timing run, one FETCH_SIZE pass and one pass of the TCC request counters.
#   tools/pmc_calib.sh [out]   -> <out>/calib_<mode>.json, <out>/pmc_<mode>_<pass>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=${1:-gpurun_out/calib}
mkdir -p $out
BIN=$PWD/trex-emu_amd/build/pmc_calib
# mode: stream_MB table_MB probes   (D: 2M frames stream about 279 MB and probe two buckets each)
modes="S:279:0:0 PH:0:1024:4194304 PC:0:32:4194304 M:279:32:4194304 MH:279:1024:4194304"
for m in $modes; do
  IFS=: read name s t p <<< "$m"
  timeout -k 10 60 $BIN $s $t $p 12 > $out/calib_$name.json || { echo "fail $name"; exit 1; }
  cat $out/calib_$name.json
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_${name}_fetch -o run --output-format csv \
    -- $BIN $s $t $p 12 > $out/pmc_${name}_fetch.log 2>&1 || { echo "pmc fetch fail $name"; tail -5 $out/pmc_${name}_fetch.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum \
    -d $out/pmc_${name}_req -o run --output-format csv \
    -- $BIN $s $t $p 12 > $out/pmc_${name}_req.log 2>&1 || { echo "pmc req fail $name"; tail -5 $out/pmc_${name}_req.log; exit 1; }
done
python tools/pmc_calib_summary.py $out | tee $out/summary.json
