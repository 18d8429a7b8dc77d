#!/bin/bash
# Round 4: where the small ingest batch's latency goes (tools/lat_probe.py), small path with and
# without the completion-word spin, the multi-launch path, and the kernel's own duration.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04c
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread -k "ingest or stream or zmq" > $out/pytest_ingest.log 2>&1 || { tail -30 $out/pytest_ingest.log; exit 1; }
tail -1 $out/pytest_ingest.log
timeout -k 10 120 python tools/lat_probe.py > $out/lat_spin.log 2>&1 || { tail -5 $out/lat_spin.log; exit 1; }
tail -1 $out/lat_spin.log
EMURX_INGEST_SPIN=0 timeout -k 10 120 python tools/lat_probe.py > $out/lat_nospin.log 2>&1 || { tail -5 $out/lat_nospin.log; exit 1; }
tail -1 $out/lat_nospin.log
EMURX_INGEST_SMALL=0 timeout -k 10 120 python tools/lat_probe.py > $out/lat_multi.log 2>&1 || { tail -5 $out/lat_multi.log; exit 1; }
tail -1 $out/lat_multi.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python tools/lat_probe.py \
  > $out/prof.log 2>&1 || { tail -5 $out/prof.log; exit 1; }
f=$(ls $out/prof/*/run_kernel_stats.csv $out/prof/run_kernel_stats.csv 2>/dev/null | head -n 1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -n 8

EMURX_LIB=$PWD/trex-emu_amd/lib/libemurx_sstamp.so timeout -k 10 120 python tools/lat_probe.py > $out/lat_stamp.log 2>&1 || { tail -5 $out/lat_stamp.log; exit 1; }
tail -1 $out/lat_stamp.log
echo done
