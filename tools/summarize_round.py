"""One line per config from a tools/round_profile.sh output directory: the bench value, the
k_rx time by events and by rocprof, the roofline fractions and the PMC bytes.

    python tools/summarize_round.py gpurun_out/round_<tag>
"""
import csv
import glob
import json
import sys
from pathlib import Path


def main(d):
    d = Path(d)
    for log in sorted(d.glob("bench_*.log")):
        c = log.stem[len("bench_"):]
        lines = [x for x in log.read_text().splitlines() if x.startswith("{")]
        if not lines:
            print(c, "no JSON line")
            continue
        j = json.loads(lines[-1])
        r = j["roofline"]
        print(f"{c}: {j['value']} Mpkt/s, {j['ms_per_step']} ms/step, k_rx {r['kernel_ms_mean']} ms, "
              f"frac {r['frac']}, copy ceiling {r.get('copy_ceiling_gbs')} GB/s ({r.get('frac_of_copy_ceiling')})")
        for k in ("alternative", "exchange", "host_inclusive"):
            if k in j:
                print(f"   {k}: {json.dumps(j[k])[:300]}")
        stats = glob.glob(str(d / f"prof_{c}" / "**" / "run_kernel_stats.csv"), recursive=True)
        for f in stats[:1]:
            for row in csv.DictReader(open(f)):
                if "emurx" in row["Name"]:
                    print(f"     {row['Name'][:40]} calls {row['Calls']} avg {float(row['AverageNs']) / 1e3:.1f} us")
    for p in sorted(d.glob("pmc_config*.json")):
        try:
            print(p.stem, json.loads(p.read_text())["k_rx_hbm_bytes_per_launch"])
        except Exception as e:  # noqa: BLE001
            print(p.stem, "unreadable", e)


if __name__ == "__main__":
    main(sys.argv[1])
