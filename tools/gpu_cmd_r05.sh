set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "zmq_walk or ingest or stream" --timeout 200 --timeout-method thread > gpurun_out/t8.log 2>&1; echo walktests rc=$?; tail -2 gpurun_out/t8.log
timeout -k 10 300 python -u bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline --no-exchange-run > gpurun_out/c8_D.log 2>&1 || exit 1
EMURX_LIB=$PWD/trex-emu_amd/lib/libemurx_dwf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "config or corpus or edge or fuzz or kat" --timeout 300 --timeout-method thread > gpurun_out/t8_dwf.log 2>&1; echo dwf parity rc=$?; tail -2 gpurun_out/t8_dwf.log
bash tools/ab_variants.sh "B C" dwf
