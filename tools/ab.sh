#!/bin/bash
# A/B of the two k_rx forms on configs B, C, E (EMURX_KRX=once: one tile per workgroup)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in B C E; do
  for form in once pipe; do
    EMURX_KRX=$form timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline \
      > gpurun_out/ab_${cfg}_${form}.log 2>&1 || { echo "fail $cfg $form"; tail -3 gpurun_out/ab_${cfg}_${form}.log; exit 1; }
    python - "$cfg" "$form" <<'PY'
import json,sys
l=[x for x in open(f"gpurun_out/ab_{sys.argv[1]}_{sys.argv[2]}.log") if x.startswith("{")][-1]
d=json.loads(l); print(sys.argv[1], sys.argv[2], d["value"], d["roofline"]["kernel_ms_mean"], d["roofline"]["frac"])
PY
  done
done
