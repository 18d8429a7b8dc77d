"""Per-launch HBM traffic of k_rx from the FETCH_SIZE / WRITE_SIZE passes of round_profile.sh.

gfx950: FETCH_SIZE reports half of the bytes of wide streaming reads (MI355X_MICROARCH.md,
HBM section), so HBM read = 2 x FETCH_SIZE (KiB) x 1024; WRITE_SIZE (KiB) x 1024 as is.
Dispatches after the first three (warm tables and caches) are averaged."""
import csv
import glob
import json
import sys


def per_dispatch(d, counter):
    vals = {}
    for f in glob.glob(f"{d}/pmc_{counter}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "k_rx" not in row.get("Kernel_Name", ""):
                continue
            k = int(row.get("Dispatch_Id", len(vals)))
            vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
    v = [vals[k] for k in sorted(vals)]
    return v[3:] if len(v) > 4 else v


d = sys.argv[1]
f, w = per_dispatch(d, "FETCH_SIZE"), per_dispatch(d, "WRITE_SIZE")
if not f or not w:
    print("no PMC rows found")
    sys.exit(0)
rd = 2 * sum(f) / len(f) * 1024
wr = sum(w) / len(w) * 1024
print(json.dumps({"k_rx_hbm_read_bytes": round(rd), "k_rx_hbm_write_bytes": round(wr),
                  "k_rx_hbm_bytes_per_launch": round(rd + wr), "dispatches": [len(f), len(w)],
                  "rule": "read = 2 x FETCH_SIZE(KiB) x 1024 (gfx950), write = WRITE_SIZE(KiB) x 1024"}))
