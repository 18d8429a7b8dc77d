#!/bin/bash
# The tx paths: their GPU parity tests (checksums, ZMQ framing), then bench.py --tx-path on B and E.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/txc; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_txzmq.py -m gpu -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "tx" > $out/pytest_tx.log 2>&1
rc=$?; echo "tx parity rc=$rc"; tail -n 2 $out/pytest_tx.log; [ $rc -eq 0 ] || exit $rc
for c in B E; do
  timeout -k 10 300 python -u bench.py --config $c --steps 50 --warmup 5 --tx-path --no-exchange-run --no-cpu-baseline \
    > $out/tx_$c.log 2>&1 || { tail -5 $out/tx_$c.log; exit 1; }
  grep '^{' $out/tx_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$c'", json.dumps(d["tx_zmq"]), json.dumps(d["tx_checksum"]))'
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_B -o run --output-format csv -- python bench.py --config B \
  --steps 20 --warmup 5 --tx-path --no-exchange-run --no-cpu-baseline > $out/prof_B.log 2>&1 || { tail -5 $out/prof_B.log; exit 1; }
f=$(ls $out/prof_B/*/run_kernel_stats.csv 2>/dev/null | head -n 1)
[ -n "$f" ] && grep -E "txz|tx_csum" "$f" | cut -d, -f1-4
echo done
