set -u
mkdir -p gpurun_out/r05c
timeout -k 10 120 tools/host_read_probe > gpurun_out/r05c/host_read_probe.txt 2>&1 || { echo probe fail; tail -3 gpurun_out/r05c/host_read_probe.txt; exit 1; }
echo probe ok
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 --host-path --no-exchange-run --no-cpu-baseline > gpurun_out/r05c/bench_B_host.log 2>&1 || { echo host fail; tail -5 gpurun_out/r05c/bench_B_host.log; exit 1; }
echo host ok
bash tools/ab_variants.sh "B C" dwf
