"""k_rx launch duration and launch interval from a rocprofv3 kernel trace of one bench run.

    python tools/prof_interval.py <run_kernel_trace.csv> <steps>

bench.py's pipelined steps (--streams 2, --batches 8) enqueue: the warmup launches, then the
`steps` launches of the timed region alternating between the streams over the rotating slots,
then (since round 6) the same `steps` again between the interval events (roofline.pipelined;
the group this tool reports as timed_region: the same pipeline), then max(`steps`, 100) launches back to back on one stream over the
rotating batch slots (each launch alone: roofline.kernel_ms_mean / frac), then `steps` launches
replaying one batch per stream (roofline.cache_resident_replay).  (Before the end of round 3 the timed region
came last: --old-order.)  For those three groups of
`steps` k_rx dispatches this prints the mean per-dispatch duration (what `--stats` averages)
and the interval (last end - first start) / launches, which is what the bench's one event pair
around a group measures.  With --batches <= --streams there is no replay group: pass
`--no-replay` as the third argument.  `--kernel <text>` keeps only the k_rx dispatches whose name
holds <text> (the default command also runs config D's exchange after the headline: pass
`--kernel "k_rx<1, 6144u>"` for config B's narrow-slab launches).  `--trim-isolated` drops the
trailing isolated launches of the default line's host_inclusive block (ingest batches, each on its
own after its copies).
"""
import csv
import json
import sys


def col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def main(path, steps, replay=True, old_order=False, one=None, kernel="k_rx", trim=False):
    one = max(steps, 100) if one is None else one  # bench.py times one launch alone over max(--steps, 100)
    ks = []
    for row in csv.DictReader(open(path)):
        name = col(row, "Kernel_Name", "Kernel-Name", "KernelName")
        if "k_rx" not in name or kernel not in name:
            continue
        ks.append((int(col(row, "Start_Timestamp", "Start-Timestamp", "BeginNs")),
                   int(col(row, "End_Timestamp", "End-Timestamp", "EndNs"))))
    ks.sort()
    out = {"k_rx_dispatches": len(ks), "steps": steps}
    if trim:  # the default command's host_inclusive block runs after the headline: its batches'
        # k_rx launches each start > 30 us after the previous one ended; drop them from the end
        n0 = len(ks)
        while len(ks) > 1 and ks[-1][0] - ks[-2][1] > 30000:
            ks.pop()
        out["trimmed_isolated_dispatches"] = n0 - len(ks)
    if old_order:
        g = [ks[len(ks) - (i + 1) * steps:len(ks) - i * steps] for i in range(3)]  # last, second to last, ...
        groups = [("timed_region", g[0])]
        groups += [("cache_resident_replay", g[1]), ("one_stream", g[2])] if replay else [("one_stream", g[1])]
    else:
        # from the end: the replay (steps), the one-stream launches (max(steps, 100)), the timed region
        sizes = ([("cache_resident_replay", steps)] if replay else []) + [("one_stream", one), ("timed_region", steps)]
        groups, end = [], len(ks)
        for label, size in sizes:
            groups.append((label, ks[max(0, end - size):end]))
            end -= size
    for label, grp in groups:
        if not grp or len(grp) < min(steps, len(grp)) or (label != "one_stream" and len(grp) < steps):
            continue
        dur = sum(e - s for s, e in grp) / len(grp)
        span = max(e for _, e in grp) - min(s for s, _ in grp)
        out[label] = {"mean_duration_us": round(dur / 1e3, 3), "interval_us": round(span / len(grp) / 1e3, 3),
                      "overlap": round(dur * len(grp) / span, 3)}
    print(json.dumps(out))


if __name__ == "__main__":
    rest = sys.argv[3:]
    one = int(rest[rest.index("--one") + 1]) if "--one" in rest else None  # traces before max(steps, 100): --one <steps>
    kernel = rest[rest.index("--kernel") + 1] if "--kernel" in rest else "k_rx"
    main(sys.argv[1], int(sys.argv[2]), replay="--no-replay" not in rest, old_order="--old-order" in rest, one=one,
         kernel=kernel, trim="--trim-isolated" in rest)
