#!/bin/bash
# Round evidence on the GPU box: benches (B with CPU baseline + host path, C, E, D), the
# rocprofv3 kernel-trace summary of the config-B bench, and the HBM-traffic PMC passes
# (FETCH_SIZE, WRITE_SIZE: one rocprofv3 run each, as the microarch guide prescribes).
#   tools/round_profile.sh <tag>      -> gpurun_out/round_<tag>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-v}
out=gpurun_out/round_$tag
mkdir -p $out
step() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step bench_B 600 python bench.py --host-path
step bench_C 300 python bench.py --config C --steps 100 --warmup 10 --no-cpu-baseline
step bench_E 300 python bench.py --config E --steps 50 --warmup 5 --no-cpu-baseline
step bench_D 300 python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline
step prof_B 300 rocprofv3 --kernel-trace --stats -d $out/prof_B -o run --output-format csv \
  -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 120 rocprofv3 --pmc $c -T --kernel-include-regex k_rx -d $out/pmc_$c -o run --output-format csv \
    -- python bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-check
done
python tools/pmc_summary.py $out > $out/pmc_summary.txt 2>&1; cat $out/pmc_summary.txt
echo done
