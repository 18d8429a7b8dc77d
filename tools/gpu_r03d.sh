# host mirror (memo + OnRxBatch) on the GPU, a stream-hold diagnostic, the batched-ingest latency sweep, then the split A/B
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r03d gpurun_out/ab
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_host_mirror.py -m gpu > gpurun_out/r03d/host_mirror.log 2>&1 || { tail -30 gpurun_out/r03d/host_mirror.log; exit 1; }
tail -3 gpurun_out/r03d/host_mirror.log
timeout -k 10 120 python -u tools/sleep_diag.py > gpurun_out/r03d/sleep_diag.log 2>&1; echo "sleep_diag rc=$?"; cat gpurun_out/r03d/sleep_diag.log
timeout -k 10 300 python bench.py --host-path --steps 50 --warmup 5 --no-cpu-baseline --no-replay > gpurun_out/r03d/host_path.log 2>&1 || { tail -30 gpurun_out/r03d/host_path.log; exit 1; }
tail -1 gpurun_out/r03d/host_path.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d["host_inclusive"]))'
bash tools/gpu_ab_split.sh
