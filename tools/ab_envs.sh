#!/bin/bash
# A/B of several environment settings with the in-tree library, interleaved per repetition:
#   tools/ab_envs.sh "<configs>" <reps> "<VAR=val ...>" ["<VAR=val ...>" ...]
# ("-" as a setting = the defaults).  Prints value / one launch ms / frac / pipelined ms per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
configs=$1; reps=$2; shift 2
mkdir -p gpurun_out/ab
for cfg in $configs; do
  case $cfg in
    B) args="--steps 200 --warmup 20" ;;
    C) args="--config C --steps 100 --warmup 10" ;;
    DN) args="--config D --tables none --no-exchange-run --steps 50 --warmup 5" ;;
    DR) args="--config D --tables replicated --no-exchange-run --steps 50 --warmup 5" ;;
    D) args="--config D --steps 50 --warmup 5" ;;
    E) args="--config E --steps 50 --warmup 5" ;;
  esac
  for r in $(seq 1 $reps); do
    i=0
    for e in "$@"; do
      i=$((i + 1))
      [ "$e" = - ] && e="EMURX_AB_NONE=1"
      log=gpurun_out/ab/${cfg}_${i}_$r.log
      env $e timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-check > $log 2>&1 \
        || { echo "fail $cfg [$e]"; tail -3 $log; exit 1; }
      echo "$cfg #$r [$e] $(tail -1 $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; x=d.get("exchange") or {}; print(round(d["value"]), "one", r["kernel_ms_mean"], r["frac"], "pipe", r.get("pipelined",{}).get("interval_ms"), "step", d["ms_per_step"], ("xchg " + str(x.get("value"))) if x else "")')"
    done
  done
done
