set -u
mkdir -p gpurun_out/r05d
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "ingest or stream or walk" --timeout 300 --timeout-method thread > gpurun_out/r05d/pytest_ingest.log 2>&1
rc=$?; echo "ingest tests rc=$rc"; tail -3 gpurun_out/r05d/pytest_ingest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 --host-path --no-exchange-run --no-cpu-baseline > gpurun_out/r05d/bench_B_host.log 2>&1 || { echo host fail; tail -5 gpurun_out/r05d/bench_B_host.log; exit 1; }
grep '^{' gpurun_out/r05d/bench_B_host.log | python -c '
import json,sys; d=json.loads(sys.stdin.read()); h=d["host_inclusive"]
b=h["batch_latency_by_msgs"]; t=h["two_slot_rate_by_msgs"]
for k in b: print(k, json.dumps(b[k]), json.dumps(t.get(k)))
print("with_copy", h.get("mpkts_with_host_copy"), "prefilled", h.get("mpkts_prefilled"))'
