#!/bin/bash
# k_q ablation: 1 skip group-total reads, 2 skip histogram fold, 4 skip done counters,
# 8 skip qlist writes (timings only; outputs are wrong for non-zero masks)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for m in 0 1 2 4 6 8 15 0; do
  EMURX_DBG_KQ=$m timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/exp_kq_$m.log 2>&1 || { echo "fail $m rc=$?"; tail -3 gpurun_out/exp_kq_$m.log; [ $m -eq 0 ] && exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/exp_kq_$m.log').read().strip().splitlines()[-1]); r=d['roofline']; print('mask $m', d['value'], r['kernel_ms_mean'], r['queue_kernel_ms_mean'])"
done
