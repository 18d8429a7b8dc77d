export TMPDIR=/tmp
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r['kernel_ms_mean'], r['frac'], r['pipelined']['interval_ms'])"; }
for i in 1 2; do timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bd_$i.log 2>&1 || exit 1; summ gpurun_out/bd_$i.log 20/5; done
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bd_3.log 2>&1 || exit 1; summ gpurun_out/bd_3.log 200/20
