#!/bin/bash
# GPU-box check sequence (run via gpurun from the repo root).  Every GPU step has its own
# time limit; a fault / abort / timeout ends the script (no further GPU work).
#   tools/gpu_check.sh [tests|bench|prof|pmc|all] ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_fault() {  # rc 1 = assertion/test failures: keep going; anything else: stop
  local rc=$1
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "FAULT/TIMEOUT rc=$rc -> stop"; exit "$rc"; fi
}
run() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  return $rc
}
for what in "${@:-all}"; do
  case $what in
  tests|all)
    run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread; stop_on_fault $? ;;&
  smoke|all)
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; stop_on_fault $? ;;&
  bench|all)
    run bench_B 600 python -u bench.py --steps 200 --warmup 20; stop_on_fault $?
    run bench_B_driver 600 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline; stop_on_fault $?
    run bench_C 600 python bench.py --config C --steps 100 --warmup 10 --no-cpu-baseline; stop_on_fault $?
    run bench_E 600 python bench.py --config E --steps 50 --warmup 5 --no-cpu-baseline; stop_on_fault $? ;;&
  dclass)
    run bench_DN 600 python bench.py --config D --tables none --no-exchange-run --steps 50 --warmup 5 --no-cpu-baseline; stop_on_fault $?
    run bench_D 600 python bench.py --config D --no-exchange-run --steps 50 --warmup 5 --no-cpu-baseline; stop_on_fault $? ;;&
  prof|all)
    run prof_B 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_B -o run --output-format csv \
        -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline; stop_on_fault $?
    t=$(ls gpurun_out/prof_B/*/run_kernel_trace.csv gpurun_out/prof_B/run_kernel_trace.csv 2>/dev/null | head -n 1)
    [ -n "$t" ] && python tools/prof_interval.py "$t" 50 | tee gpurun_out/prof_B_interval.json ;;&
  exchange)
    run bench_D1 900 python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline; stop_on_fault $?
    run bench_D2_gloo 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 2 --config D --backend gloo --frames 262144 --steps 10 --warmup 2; stop_on_fault $?
    run bench_B2_gloo 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29534 bench.py --gpus 2 --backend gloo --steps 20 --warmup 2; stop_on_fault $? ;;
  rehearse)
    run bench_B2x_gloo 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29535 bench.py --gpus 2 --backend gloo --steps 20 --warmup 2; stop_on_fault $? ;;&
  profD)
    run prof_D 900 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_D -o run --output-format csv \
        -- python bench.py --config D --steps 20 --warmup 3 --no-cpu-baseline; stop_on_fault $? ;;
  pmc)
    for c in FETCH_SIZE WRITE_SIZE; do
      run pmc_$c 600 rocprofv3 --pmc $c -T -d gpurun_out/pmc_$c -o run --output-format csv \
          -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline; stop_on_fault $?
    done ;;
  esac
done
echo "done $(date +%T)"
