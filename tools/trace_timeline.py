"""Per-launch timeline of k_rx in a rocprofv3 kernel trace of one bench run: the timed region's
`steps` launches and the interval region's `steps` after them (bench.py order: warmup, timed
region, interval region, one-stream launches, replay).  Start / end relative to the timed
region's first start, duration, and the queue each ran on.
    python tools/trace_timeline.py <run_kernel_trace.csv> <steps> [--no-replay] [--kernel TEXT]"""
import csv
import json
import sys


def col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    return None


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    replay = "--no-replay" not in sys.argv
    kern = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "k_rx"
    ks = []
    for row in csv.DictReader(open(path)):
        name = col(row, "Kernel_Name", "Kernel-Name", "KernelName") or ""
        if kern not in name:
            continue
        ks.append((int(col(row, "Start_Timestamp", "BeginNs")), int(col(row, "End_Timestamp", "EndNs")),
                   col(row, "Queue_Id", "Stream_Id", "Queue-Id")))
    ks.sort()
    one = max(steps, 100)
    end = len(ks) - (steps if replay else 0) - one
    interval = ks[end - steps:end]
    timed = ks[end - 2 * steps:end - steps]
    t0 = timed[0][0]
    res = {}
    for label, grp in (("timed", timed), ("interval_region", interval)):
        rows = [[round((s - t0) / 1e3, 2), round((e - t0) / 1e3, 2), round((e - s) / 1e3, 2), q] for s, e, q in grp]
        span = (max(e for _, e, _ in grp) - min(s for s, _, _ in grp)) / 1e3
        res[label] = {"span_us": round(span, 2), "per_step_us": round(span / steps, 3), "launches": rows}
    prev = ks[end - 2 * steps - 1]
    res["gap_before_timed_us"] = round((t0 - prev[1]) / 1e3, 2)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
