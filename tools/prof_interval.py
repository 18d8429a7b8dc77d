"""k_rx launch duration and launch interval from a rocprofv3 kernel trace of one bench run.

    python tools/prof_interval.py <run_kernel_trace.csv> <steps>

bench.py's pipelined steps (--streams 2, --batches 8) enqueue: the warmup launches, then the
`steps` launches of the timed region alternating between the streams over the rotating slots
(roofline.pipelined), then `steps` launches back to back on one stream over the rotating batch
slots (each launch alone: roofline.kernel_ms_mean / frac), then `steps` launches replaying one
batch per stream (roofline.cache_resident_replay).  (Before the end of round 3 the timed region
came last: --old-order.)  For those three groups of
`steps` k_rx dispatches this prints the mean per-dispatch duration (what `--stats` averages)
and the interval (last end - first start) / launches, which is what the bench's one event pair
around a group measures.  With --batches <= --streams there is no replay group: pass
`--no-replay` as the third argument.
"""
import csv
import json
import sys


def col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def main(path, steps, replay=True, old_order=False):
    ks = []
    for row in csv.DictReader(open(path)):
        name = col(row, "Kernel_Name", "Kernel-Name", "KernelName")
        if "k_rx" not in name:
            continue
        ks.append((int(col(row, "Start_Timestamp", "Start-Timestamp", "BeginNs")),
                   int(col(row, "End_Timestamp", "End-Timestamp", "EndNs"))))
    ks.sort()
    out = {"k_rx_dispatches": len(ks), "steps": steps}
    g = [ks[len(ks) - (i + 1) * steps:len(ks) - i * steps] for i in range(3)]  # last, second to last, ...
    if old_order:
        groups = [("timed_region", g[0])]
        groups += [("cache_resident_replay", g[1]), ("one_stream", g[2])] if replay else [("one_stream", g[1])]
    elif replay:
        groups = [("cache_resident_replay", g[0]), ("one_stream", g[1]), ("timed_region", g[2])]
    else:
        groups = [("one_stream", g[0]), ("timed_region", g[1])]
    for label, grp in groups:
        if len(grp) < steps:
            continue
        dur = sum(e - s for s, e in grp) / len(grp)
        span = max(e for _, e in grp) - min(s for s, _ in grp)
        out[label] = {"mean_duration_us": round(dur / 1e3, 3), "interval_us": round(span / len(grp) / 1e3, 3),
                      "overlap": round(dur * len(grp) / span, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), replay="--no-replay" not in sys.argv[3:], old_order="--old-order" in sys.argv[3:])
