# The driver's N = 2 command at full default sizes, both ranks on the one GPU over gloo
# (RCCL needs one GPU per rank): the headline, the Namespace exchange side entry and the
# replicated alternative end to end with the final bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03m
( while sleep 50; do echo "alive $(date +%T)"; done ) &
tick=$!
timeout -k 10 900 python -u bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 > gpurun_out/r03m/bench_N2_gloo.log 2>&1
rc=$?
kill $tick
echo "rc=$rc"
tail -c 3000 gpurun_out/r03m/bench_N2_gloo.log
exit $rc
