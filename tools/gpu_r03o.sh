# rocprofv3 kernel trace + stats of the default bench command (python bench.py, no flags) on
# the final tree, and the trace's launch interval / one-launch duration (tools/prof_interval.py)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03o
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r03o/prof_B -o run --output-format csv \
    -- python bench.py > gpurun_out/r03o/bench_B_default.log 2>&1 || { tail -20 gpurun_out/r03o/bench_B_default.log; exit 1; }
steps=$(grep '^{' gpurun_out/r03o/bench_B_default.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["steps"])')
python tools/prof_interval.py gpurun_out/r03o/prof_B/run_kernel_trace.csv "$steps" > gpurun_out/r03o/prof_B_interval.json
cat gpurun_out/r03o/prof_B_interval.json
