"""Fold tools/pmc_calib.sh's passes: per mode, counters per launch (the cold first launch
dropped) against the bytes the mode moves; the factor FETCH_SIZE x 1024 / bytes per pattern.

    python tools/pmc_calib_summary.py gpurun_out/calib
"""
import csv
import glob
import json
import sys
from pathlib import Path


def per_launch(d):
    """{counter: mean per dispatch, first dispatch dropped}."""
    rows = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_calib" not in r.get("Kernel_Name", ""):
                continue
            k = (r["Counter_Name"], int(r["Dispatch_Id"]))
            rows[k] = rows.get(k, 0.0) + float(r["Counter_Value"])
    out = {}
    for name in {c for c, _ in rows}:
        v = [rows[(c, i)] for c, i in sorted(rows) if c == name]
        v = v[1:] if len(v) > 1 else v
        out[name] = sum(v) / len(v)
    return out


def main(root):
    res = {}
    for j in sorted(Path(root).glob("calib_*.json")):
        mode = j.stem.split("_", 1)[1]
        m = json.loads(j.read_text())
        c = per_launch(f"{root}/pmc_{mode}_fetch")
        c.update(per_launch(f"{root}/pmc_{mode}_req"))
        known = m["stream_bytes"] + m["probe_bytes"]
        e = dict(m, counters={k: round(v) for k, v in sorted(c.items())})
        if "FETCH_SIZE" in c and known:
            e["fetch_bytes"] = round(c["FETCH_SIZE"] * 1024)
            e["fetch_over_known"] = round(c["FETCH_SIZE"] * 1024 / known, 4)
        if "TCC_EA0_RDREQ_sum" in c and known:
            e["rdreq_x64_over_known"] = round(c["TCC_EA0_RDREQ_sum"] * 64 / known, 4)
        e["gbs"] = round(known / (m["us_per_launch"] * 1e3), 1)
        res[mode] = e
    # the probe part alone in a mixed launch: (mixed - stream-only), against the probe bytes
    if "S" in res and "fetch_bytes" in res.get("S", {}):
        for mix in ("M", "MH"):
            if mix in res and "fetch_bytes" in res[mix]:
                extra = res[mix]["fetch_bytes"] - res["S"]["fetch_bytes"]
                res[mix]["probe_fetch_over_probe_bytes"] = round(extra / res[mix]["probe_bytes"], 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/calib")
