#!/bin/bash
# k_rx<2> (config D's partitioned source, N = 1): the owner-offset loads issued before the
# staging wait (libemurx.so) against inside the tile body (libemurx_tolbase.so), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/ab_tol; mkdir -p $out
for rep in 1 2 3; do
  for v in tolbase default; do
    lib=$PWD/trex-emu_amd/lib/libemurx.so
    [ $v = tolbase ] && lib=$PWD/trex-emu_amd/lib/libemurx_tolbase.so
    log=$out/D_${v}_$rep.log
    EMURX_LIB=$lib timeout -k 10 300 python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline --no-check \
      --no-exchange-run > $log 2>&1 || { echo "fail $v"; tail -3 $log; exit 1; }
    echo "$v #$rep $(python tools/exsum.py $log | head -2 | tr '\n' ' ')"
  done
done
