"""k_lookup at one Namespace owner of N = 8, on one GPU (no RCCL needed): eight sources' config-D
shards (2M frames each, as bench.py's ranks hold) go through parse_route_dev with 8 parts, the
all-to-all is played on the device (owner 0's receive buffer = region 0 of every source), and
owner 0's lookup_dev runs over them against its 1/8 tables; beside it the N = 1 case (one
handle, all tables, one source).  Prints each case's k_lookup time per launch (HIP events around
back-to-back launches on one stream) and records per launch.  The library is the one EMURX_LIB
names (tools/build_variant.sh builds), so library variants compare on the same script.
    python tools/lookup_owner_probe.py [frames_per_source] [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "trex-emu_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from emurx import abi, synth  # noqa: E402
from emurx import exchange as X  # noqa: E402
from emurx.rx import RxPath  # noqa: E402


def dev(a, pad=64):
    """A host array on the device with `pad` zero bytes after it (the staging loads' overrun)."""
    b = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    t = torch.zeros(b.size + pad, dtype=torch.uint8, device="cuda")
    t[: b.size] = torch.from_numpy(b.copy()).cuda()
    return t


def handle(n, parts, part, w):
    h = RxPath(0, max_ns=32768, max_clients=1 << 20, max_frames=n)
    h.register_all()
    if parts > 1:
        h.set_partition(parts, part)
    synth.load_tables(w, h)
    return h


def sources(h, shards, parts, cap):
    n = len(shards[0]["desc"])
    qcap = abi.queue_cap(n)
    ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda")
    tc = torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device="cuda")
    hist = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
    sends = []
    for s, w in enumerate(shards):
        buf, desc = dev(w["buf"]), dev(w["desc"])
        send = torch.empty(parts * X.region_bytes(cap, abi.tail_capacity(cap)), dtype=torch.uint8, device="cuda")
        sc = torch.zeros(2 * parts, dtype=torch.int32, device="cuda")
        h.parse_route_dev(buf, desc, n, None, ql, qcap, tc, hist, parts, s, cap, send, sc)
        torch.cuda.synchronize()
        sends.append((send, sc.cpu().numpy()))
        del buf, desc
    return sends


def time_lookup(h, recv, rc, parts, cap, reps):
    out = torch.empty(parts * cap * X.REC_BYTES, dtype=torch.uint8, device="cuda")
    for _ in range(5):
        h.lookup_dev(recv, rc, parts, cap, out)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        h.lookup_dev(recv, rc, parts, cap, out)
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    t0 = time.time()
    parts = 8
    shards = [synth.config_d(n, rank=s) for s in range(parts)]
    print(f"[probe] shards ready {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    res = {"lib": os.path.basename(os.environ.get("EMURX_LIB", "libemurx.so")), "frames_per_source": n}
    # N = 1: one handle with every table, one source, one region
    h1 = handle(n, 1, 0, shards[0])
    cap1 = X.capacity(n, 1)
    (send1, sc1), = sources(h1, shards[:1], 1, cap1)
    rc1 = torch.from_numpy(sc1.astype(np.int32)).cuda()
    res["n1"] = {"records": int(sc1[0::2].sum()), "ms": round(time_lookup(h1, send1, rc1, 1, cap1, reps), 5),
                 "table_bytes": h1.table_stats()["table_bytes"]}
    del h1, send1
    torch.cuda.empty_cache()
    print(f"[probe] N=1 done {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    # owner 0 of 8: its 1/8 tables, region 0 of every source
    h8 = handle(n, parts, 0, shards[0])
    cap = X.capacity(n, parts, slack=1.06)
    sends = sources(h8, shards, parts, cap)
    rb = X.region_bytes(cap, abi.tail_capacity(cap))
    recv = torch.cat([s[0][0:rb] for s in sends])
    rc = torch.tensor([int(s[1][k]) for s in sends for k in range(2)], dtype=torch.int32, device="cuda")
    del sends
    res["owner0_of_8"] = {"records": int(rc[0::2].sum()), "ms": round(time_lookup(h8, recv, rc, parts, cap, reps), 5),
                          "table_bytes": h8.table_stats()["table_bytes"]}
    for k in ("n1", "owner0_of_8"):
        r = res[k]
        r["ns_per_record"] = round(r["ms"] * 1e6 / max(r["records"], 1), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
