#!/bin/bash
# Round evidence on the GPU box, per BASELINE config:
#   bench    bench.py lines (B with the CPU baseline and the host path)
#   prof     rocprofv3 --kernel-trace --stats of the bench command
#   pmc      HBM traffic of k_rx: FETCH_SIZE and WRITE_SIZE, one rocprofv3 run each (the
#            microarch guide's recipe), folded by tools/pmc_summary.py
#   tools/round_profile.sh <tag> "<configs>" "<phases>"   -> gpurun_out/round_<tag>/
#   e.g. tools/round_profile.sh r02a "B C D E" "bench"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-v}
configs=${2:-"B C D E"}
phases=${3:-"bench prof pmc"}
out=gpurun_out/round_$tag
mkdir -p $out
step() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 2 "$out/$name.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
args() {  # bench arguments per config
  case $1 in
    B) echo "--steps 200 --warmup 20" ;;
    C) echo "--config C --steps 100 --warmup 10" ;;
    D) echo "--config D --steps 50 --warmup 5" ;;
    DR) echo "--config D --tables replicated --no-exchange-run --steps 50 --warmup 5" ;;
    DN) echo "--config D --tables none --no-exchange-run --steps 50 --warmup 5" ;;
    E) echo "--config E --steps 50 --warmup 5" ;;
  esac
}
for ph in $phases; do
  for c in $configs; do
    case $ph in
      bench)
        extra="--no-cpu-baseline"
        [ "$c" = B ] && extra="--host-path"
        step bench_$c 600 python bench.py $(args $c) $extra ;;
      prof)
        step prof_$c 300 rocprofv3 --kernel-trace --stats -d $out/prof_$c -o run --output-format csv \
          -- python bench.py $(args $c) --no-cpu-baseline --no-exchange-run
        f=$(ls $out/prof_$c/*/run_kernel_stats.csv $out/prof_$c/run_kernel_stats.csv 2>/dev/null | head -n 1)
        [ -n "$f" ] && cut -d, -f1-4 "$f" | head -n 12
        t=$(ls $out/prof_$c/*/run_kernel_trace.csv $out/prof_$c/run_kernel_trace.csv 2>/dev/null | head -n 1)
        # B's default line ends with the host-inclusive block's isolated ingest launches: trimmed
        trim=""; [ "$c" = B ] && trim="--kernel k_rx<1, --trim-isolated"
        [ -n "$t" ] && python tools/prof_interval.py "$t" $(args $c | sed 's/.*--steps \([0-9]*\).*/\1/') $trim \
          | tee $out/prof_${c}_interval.json ;;
      pmc)
        for k in FETCH_SIZE WRITE_SIZE; do
          step pmc_${c}_$k 180 rocprofv3 --pmc $k -T --kernel-include-regex k_rx -d $out/pmc_${c}/pmc_$k -o run \
            --output-format csv -- python bench.py $(args $c) --steps 40 --warmup 8 --no-cpu-baseline --no-check --no-replay \
            --no-exchange-run
        done
        xs=""  # E's excess is probe lines since the window-skip checksum (round 4); --excess-streamed before
        python tools/pmc_summary.py $out/pmc_${c} $xs > $out/pmc_config$c.json 2>&1; cat $out/pmc_config$c.json ;;
    esac
  done
done
echo done
