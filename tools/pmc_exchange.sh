#!/bin/bash
# PMC traffic (FETCH_SIZE, WRITE_SIZE; one rocprofv3 pass each) of config D's partitioned step kernels.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
out=gpurun_out/pmcD; mkdir -p $out
for k in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $k -T --kernel-include-regex "k_lookup|k_rx|k_owner_count" -d $out/$k -o run \
    --output-format csv -- python bench.py --config D --steps 30 --warmup 5 --no-cpu-baseline --no-check --no-replay \
    --no-exchange-run > $out/$k.log 2>&1 || { echo "fail $k"; tail -3 $out/$k.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections, statistics
for k in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/pmcD/{k}/**/run_counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == k:
            per[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    for name, v in per.items():
        print(k, name, "median KB", round(statistics.median(v), 1), "n", len(v))
PY
