#!/bin/bash
# k_lookup against config D's partitioned step at N = 1: the Namespace table's spread
# (EMURX_TABLE_SPREAD ns,mac,ip,ci) and the non-temporal head loads / write-through outputs
# (libemurx_lnt.so), interleaved, two rounds; then a kernel trace of the default step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/ab_lookup; mkdir -p $out
for rep in 1 2; do
  for v in default lnt ns4 ns2 lnt_ns2; do
    lib=$PWD/trex-emu_amd/lib/libemurx.so; e=""
    case $v in lnt*) lib=$PWD/trex-emu_amd/lib/libemurx_lnt.so ;; esac
    case $v in *ns4) e="EMURX_TABLE_SPREAD=4,8,16,16" ;; *ns2) e="EMURX_TABLE_SPREAD=2,8,16,16" ;; esac
    log=$out/D_${v}_$rep.log
    env $e EMURX_LIB=$lib timeout -k 10 300 python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline --no-check \
      --no-exchange-run > $log 2>&1 || { echo "fail $v"; tail -3 $log; exit 1; }
    echo "$v #$rep $(python tools/exsum.py $log | tail -1)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $out/prof_D -o run --output-format csv -- python bench.py --config D \
  --steps 20 --warmup 3 --no-cpu-baseline --no-check --no-exchange-run > $out/prof_D.log 2>&1 || { echo prof fail; tail -5 $out/prof_D.log; exit 1; }
echo done
