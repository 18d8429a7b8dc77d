#!/bin/bash
# round 6 (h): the host-inclusive pass over 2, 3 and 4 ingest slots (config B)
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out/slots
for rep in 1 2; do
  for sl in 2 3 4; do
    timeout -k 10 200 python -u bench.py --steps 50 --no-exchange-run --no-cpu-baseline --ingest-slots $sl \
      > gpurun_out/slots/B_s${sl}_$rep.json 2> gpurun_out/slots/B_s${sl}_$rep.err || exit $?
    python -c "
import json; r=json.loads(open('gpurun_out/slots/B_s${sl}_$rep.json').read().strip().splitlines()[-1]); h=r['host_inclusive']
print('slots', h['slots'], 'copy', h['with_host_copy']['mpkts'], 'fill_threads', h['with_host_copy']['fill_threads'], '1thr', h['with_host_copy_1_thread']['mpkts'], 'prefilled', h['prefilled']['mpkts'])"
  done
done
