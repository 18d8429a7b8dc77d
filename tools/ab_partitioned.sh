#!/bin/bash
# The partitioned config-D step (k_owner_count + k_rx<2> + k_lookup) with the in-tree library
# and alternative builds, interleaved:  tools/ab_partitioned.sh <name>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abp
for rep in 1 2; do
  for v in default "$@"; do
    lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
    log=gpurun_out/abp/D_${v}_$rep.log
    EMURX_LIB=$lib timeout -k 10 300 python bench.py --config D --steps 40 --warmup 5 --no-cpu-baseline \
      --no-exchange-run > $log 2>&1 || { echo "fail $v"; tail -3 $log; exit 1; }
    echo "D-partitioned $v #$rep $(grep '^{' $log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["exchange"]["step_device_ms_mean"], d["roofline"]["kernel_ms_mean"])')"
  done
done
