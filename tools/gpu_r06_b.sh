#!/bin/bash
# round 6 (b): the changed GPU tests, the bucket-order probe of k_lookup, the receive-fill
# thread count of the host-inclusive pass
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_comm.py tests/test_abi.py \
  "tests/test_gpu_parity.py::test_ingest_small_degraded" "tests/test_gpu_parity.py::test_tx_checksum_unaligned_first_frame_at_zero" \
  "tests/test_gpu_tables.py::test_owner_flags_heads_without_tuple" "tests/test_gpu_tables.py::test_table_allocation_fallback" \
  "tests/test_bench_launch.py::test_two_rank_exchange_fields" > gpurun_out/tb.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/tb.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/lookup_sorted_probe.py > gpurun_out/sorted_probe.json 2> gpurun_out/sorted_probe.err || exit $?
for t in 8 16; do
  EMURX_BENCH_FILL_THREADS=$t timeout -k 10 200 python -u bench.py --steps 50 --no-exchange-run --no-cpu-baseline \
    > gpurun_out/bench_fill$t.json 2> gpurun_out/bench_fill$t.err || exit $?
done
