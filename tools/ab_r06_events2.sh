#!/bin/bash
# After moving the events out of the timed region (--sync-poll was removed after this A/B): the driver's 20-step command of config B
# (headline only) with and without --sync-poll, interleaved; then the full driver command, the
# bench's GPU tests and the N = 2 gloo command (the exchange's timing pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/ab_events2; mkdir -p $out
for k in 1 2 3 4; do
  for tr in "" "--sync-poll"; do
    tag=x$(echo "$tr" | tr -d ' -')
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exchange-run --no-host-inclusive \
      $tr > $out/run${tag}_$k.log 2>&1 || exit $?
    python - "$out/run${tag}_$k.log" "$tr" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d["roofline"].get("pipelined", {})
print(repr(sys.argv[2]), d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_mean"], p.get("interval_ms"),
      d["host_submit_ms_per_step"], flush=True)
PY
  done
done
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.log 2>&1 || exit $?
tail -c 600 $out/bench_driver.log
timeout -k 10 600 python -u -m pytest tests/test_bench_launch.py -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $out/pytest_bench.log 2>&1 || exit $?
tail -n 2 $out/pytest_bench.log
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29571 bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_N2_gloo.log 2>&1 || exit $?
tail -c 400 $out/bench_N2_gloo.log
