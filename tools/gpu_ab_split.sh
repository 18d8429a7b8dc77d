set -u
cd "${GRAFT_REPO_ROOT:-.}"
AB_ARGS="--no-replay" bash tools/ab_variants.sh "B C" nosplit head
for v in default nosplit; do
  lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
  EMURX_LIB=$lib timeout -k 10 300 python bench.py --config D --tables none --no-exchange-run --steps 50 --warmup 5 --no-cpu-baseline --no-check --no-replay > gpurun_out/ab/DN_$v.log 2>&1 || exit 1
  echo "DN $v $(tail -1 gpurun_out/ab/DN_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_mean"], d["roofline"]["pipelined"]["interval_ms"])')"
done
