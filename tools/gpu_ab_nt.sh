# counter calibration (tools/pmc_calib.sh), then nt LDS-DMA frame loads (libemurx_nt.so) against the default
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
bash tools/pmc_calib.sh gpurun_out/calib || exit 1
AB_ARGS="--no-replay" bash tools/ab_variants.sh "B C E" nt || exit 1
for rep in 1 2; do
  for v in default nt; do
    lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
    EMURX_LIB=$lib timeout -k 10 300 python bench.py --config D --tables none --no-exchange-run --steps 50 --warmup 5 --no-cpu-baseline --no-check --no-replay > gpurun_out/ab/DN_${v}_$rep.log 2>&1 || exit 1
    echo "DN $v #$rep $(grep '^{' gpurun_out/ab/DN_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_mean"], d["roofline"]["frac"], d["roofline"]["pipelined"]["interval_ms"])')"
  done
done
