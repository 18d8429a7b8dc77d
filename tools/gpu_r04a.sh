#!/bin/bash
# Round 4: GPU tests, smoke, the default bench line with the host path, and a rocprofv3 kernel
# trace of the partitioned config-D step (keyed descriptors).  A fault / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04a
mkdir -p $out
step() {  # name seconds cmd...
  local name=$1 to=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 3 "$out/$name.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_B_host 600 python -u bench.py --host-path
step prof_D 300 rocprofv3 --kernel-trace --stats -d $out/prof_D -o run --output-format csv \
  -- python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline --no-exchange-run
f=$(ls $out/prof_D/*/run_kernel_stats.csv $out/prof_D/run_kernel_stats.csv 2>/dev/null | head -n 1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -n 14
echo done
