#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench command on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof_final; mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python bench.py \
  > $out/bench_default_prof.log 2>&1 || { tail -5 $out/bench_default_prof.log; exit 1; }
f=$(ls $out/prof/*/run_kernel_stats.csv 2>/dev/null | head -n 1)
[ -n "$f" ] && cp "$f" $out/prof_default_kernel_stats.csv && cut -d, -f1-5 "$f" | head -12
echo done
