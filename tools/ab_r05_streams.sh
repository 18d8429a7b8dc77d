set -u
mkdir -p gpurun_out/streams
for s in 2 3 4; do
  timeout -k 10 300 python bench.py --config D --steps 100 --warmup 10 --no-cpu-baseline --no-check --streams $s > gpurun_out/streams/D_s$s.log 2>&1 || exit 1
  echo "D streams $s: $(python tools/exsum.py gpurun_out/streams/D_s$s.log | tail -1)"
done
