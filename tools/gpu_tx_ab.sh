#!/bin/bash
# The tx framing: parity tests and bench.py --tx-path (B and E) for the in-tree library and the
# variants named (trex-emu_amd/lib/libemurx_<name>.so), then rocprofv3 of B's tx path.
#   tools/gpu_tx_ab.sh [variant...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/txab; mkdir -p $out
for v in default "$@"; do
  case $v in noup*) continue ;; esac  # timing-only builds (wrong results by design): noup*
  lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
  EMURX_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_txzmq.py -m gpu -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread > $out/pytest_$v.log 2>&1
  rc=$?; echo "$v tx parity rc=$rc"; tail -n 2 $out/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in default "$@"; do
    lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
    for c in ${TX_CONFIGS:-B E}; do
      EMURX_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --tx-path --no-exchange-run \
        --no-cpu-baseline --no-check > $out/tx_${c}_${v}_$rep.log 2>&1 || { tail -5 $out/tx_${c}_${v}_$rep.log; exit 1; }
      grep '^{' $out/tx_${c}_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$c' '$v' '$rep'", json.dumps(d["tx_zmq"]))'
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_B -o run --output-format csv -- python bench.py --config B \
  --steps 20 --warmup 5 --tx-path --no-exchange-run --no-cpu-baseline --no-check > $out/prof_B.log 2>&1 || { tail -5 $out/prof_B.log; exit 1; }
f=$(ls $out/prof_B/*/run_kernel_stats.csv 2>/dev/null | head -n 1)
[ -n "$f" ] && grep -E "txz" "$f" | cut -d, -f1-4
echo done
