# staged-only nt (default build) against the previous build (libemurx_base.so), then a kernel trace of partitioned D
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab gpurun_out/r03g
AB_ARGS="--no-replay" bash tools/ab_variants.sh "B C E" base || exit 1
for rep in 1 2; do
  for v in default base; do
    lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
    EMURX_LIB=$lib timeout -k 10 300 python bench.py --config D --tables none --no-exchange-run --steps 50 --warmup 5 --no-cpu-baseline --no-check --no-replay > gpurun_out/ab/DN_${v}_$rep.log 2>&1 || exit 1
    echo "DN $v #$rep $(grep '^{' gpurun_out/ab/DN_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_mean"], d["roofline"]["frac"], d["roofline"]["pipelined"]["interval_ms"])')"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03g/prof_D -o run --output-format csv -- python bench.py --config D --steps 30 --warmup 5 --no-cpu-baseline --no-check --no-replay > gpurun_out/r03g/prof_D.log 2>&1 || { tail -5 gpurun_out/r03g/prof_D.log; exit 1; }
f=$(ls gpurun_out/r03g/prof_D/*/run_kernel_stats.csv gpurun_out/r03g/prof_D/run_kernel_stats.csv 2>/dev/null | head -n 1)
[ -n "$f" ] && cut -d, -f1-4 "$f" | head -n 14
