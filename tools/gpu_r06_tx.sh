#!/bin/bash
# round 6: the tx long path split over waves -- parity (default choice, and every call forced
# onto the long path), then E / B framing time per batch size for 1, 2 (default) and 4 waves
# per tile, interleaved
cd "$(dirname "$0")/.." || exit 2
out=gpurun_out/tx; mkdir -p $out
timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_txzmq.py \
  > $out/pytest_default.log 2>&1; rc=$?; echo "default rc=$rc"; tail -2 $out/pytest_default.log
[ $rc -gt 1 ] && exit $rc
EMURX_TXZ=long timeout -k 10 600 python -u -m pytest -v --timeout 500 --timeout-method thread -m gpu \
  tests/test_gpu_txzmq.py -k "not write_choice" > $out/pytest_long.log 2>&1; rc2=$?; echo "long rc=$rc2"; tail -2 $out/pytest_long.log
[ $rc2 -gt 1 ] && exit $rc2
[ $rc -ne 0 ] || [ $rc2 -ne 0 ] && exit 1
for rep in 1 2; do
  for v in split1 default split4; do
    lib=$PWD/trex-emu_amd/lib/libemurx.so
    [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
    EMURX_LIB=$lib timeout -k 10 300 python -u tools/tx_scale_probe.py 20 > $out/scale_${v}_$rep.json 2> $out/scale_${v}_$rep.err || exit $?
    echo "$v #$rep $(python -c "
import json; r=json.load(open('$out/scale_${v}_$rep.json')); print({k: v['us_per_call'] for k, v in r.items()})")"
  done
done
