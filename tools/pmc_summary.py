"""Per-launch memory traffic of k_rx from the FETCH_SIZE / WRITE_SIZE passes of round_profile.sh,
with the round-3 calibration of FETCH_SIZE (tools/pmc_calib.hip, profiles/r03/pmc_calib.json):

  * a wide coalesced streaming read (16 B per lane) is counted at 1/2 of its bytes (one
    TCC_EA0_RDREQ per 128-B line, tallied at 64 B);
  * a random 64-B bucket read (ld_bucket: four 16-B loads of one line by one lane) that misses
    L2 is counted at its 64 bytes (one request, tallied at 64 B); L2 hits are not counted;
  * WRITE_SIZE reads the bytes of 16-B streaming stores exactly.

The batch slot (frames, their ZMQ headers, descriptors) is read once as a stream (alg_read
bytes, taken from the pass's own bench line), so FETCH_SIZE - alg_read / 2 is the excess: table-probe lines that left L2
(config B, C, D) or, on the window path (config E), the long spans read a second time (a
stream again).  Reported per launch (the first three dispatches dropped):
  bytes_if_excess_probe_lines   alg_read + excess x 1 + write   (excess as probe lines)
  bytes_if_excess_streamed      alg_read + excess x 2 + write   (excess as streaming re-reads)
  k_rx_hbm_bytes_per_launch     the first, or with --excess-streamed (config E) the second
Both count Infinity-Cache hits as memory traffic (FETCH_SIZE cannot tell them apart).
"""
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


def alg_read_bytes(d):
    """The bytes one launch streams in: the batch slot's frames with their ZMQ frame headers
    (the staging reads the wave's whole range) and the 8-B descriptors, from the bench line of
    the FETCH_SIZE pass (config.input_bytes_per_batch)."""
    for f in glob.glob(f"{d}_FETCH_SIZE.log"):
        for line in open(f):
            if line.startswith("{"):
                c = json.loads(line)["config"]
                return c["input_bytes_per_batch"]
    return None


d = sys.argv[1]
streamed = "--excess-streamed" in sys.argv[2:]  # the window path's re-read spans (config E)
f, w = per_dispatch(d, "FETCH_SIZE"), per_dispatch(d, "WRITE_SIZE")
if not f or not w:
    print("no PMC rows found")
    sys.exit(0)
fetch = sum(f) / len(f) * 1024
wr = sum(w) / len(w) * 1024
out = {"k_rx_fetch_size_bytes": round(fetch), "k_rx_hbm_write_bytes": round(wr), "dispatches": [len(f), len(w)]}
ar = alg_read_bytes(d)
if ar:
    excess = max(fetch - ar / 2, 0.0)
    out.update({"alg_read_bytes": ar, "excess_fetch_bytes": round(excess),
                "bytes_if_excess_probe_lines": round(ar + excess + wr),
                "bytes_if_excess_streamed": round(ar + 2 * excess + wr),
                "excess_read_as": "streamed (window-path re-reads)" if streamed else "probe lines"})
    out["k_rx_hbm_bytes_per_launch"] = out["bytes_if_excess_streamed" if streamed else "bytes_if_excess_probe_lines"]
else:  # no bench line: the round-2 rule (every fetch a streaming read)
    out["k_rx_hbm_bytes_per_launch"] = round(2 * fetch + wr)
out["rule"] = ("calibrated (profiles/r03/pmc_calib.json): stream reads = 2 x FETCH_SIZE share, probe lines = "
               "1 x FETCH_SIZE share, writes = WRITE_SIZE; Infinity-Cache hits included")
print(json.dumps(out))
