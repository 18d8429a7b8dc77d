#!/bin/bash
# Host-inclusive ingest latencies (bench.py --host-path) of the in-tree library and variants,
# plus the small-ingest phase stamps (tools/lat_probe.py on the EMURX_SMALL_STAMP build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_ingest
EMURX_LIB=$PWD/trex-emu_amd/lib/libemurx_sstamp.so timeout -k 10 200 python tools/lat_probe.py > gpurun_out/ab_ingest/lat_stamp.log 2>&1 || exit 1
for v in default "$@"; do
  lib=$PWD/trex-emu_amd/lib/libemurx.so; [ $v != default ] && lib=$PWD/trex-emu_amd/lib/libemurx_$v.so
  EMURX_LIB=$lib timeout -k 10 300 python bench.py --host-path --steps 20 --warmup 5 --no-cpu-baseline \
    --no-exchange-run > gpurun_out/ab_ingest/host_$v.log 2>&1 || { echo "fail $v"; tail -3 gpurun_out/ab_ingest/host_$v.log; exit 1; }
  python - "$v" gpurun_out/ab_ingest/host_$v.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])["host_inclusive"]
lat = {m: v["us_median"] for m, v in d["batch_latency_by_msgs"].items()}
thr = {m: v["mpkts"] for m, v in d["two_slot_rate_by_msgs"].items()}
print(sys.argv[1], "copy", d["mpkts_with_host_copy"], "prefilled", d["mpkts_prefilled"], "lat_us", lat, "two_slot_mpkts", thr)
PY
done
