"""What bucket-ordered probing could buy the owner's k_lookup, measured
before building it: config D, 2M frames, one owner with every table (N = 1), the lookup heads
as parse_route_dev packs them (frame order) against the same heads permuted so that the MAC-keyed
ones come in the order of their client-table bucket (then the IPv4-keyed ones in theirs, then the
rest).  The permutation is made on the host (the tables' hash, emurx_tables.h, restated in
numpy) and is not timed: the sorted figure is the floor a device-side bucketing pass would have
to pay for.  Prints both k_lookup times per launch (HIP events around back-to-back launches),
and checks that the sorted run's records are the frame-order run's, permuted.
    python tools/lookup_sorted_probe.py [frames] [reps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "trex-emu_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from emurx import abi, synth  # noqa: E402
from emurx import exchange as X  # noqa: E402
from emurx.rx import RxPath  # noqa: E402

U = np.uint32


def fmix(h):
    h = h ^ (h >> U(16))
    h = h * U(0x85EBCA6B)
    h = h ^ (h >> U(13))
    h = h * U(0xC2B2AE35)
    return h ^ (h >> U(16))


def ehash(a, b, c, d, e):
    """emurx_hash (emurx_tables.h) over uint32 arrays"""
    a, b, c, d, e = (np.asarray(x, U) for x in (a, b, c, d, e))
    h = a * U(0x9E3779B1)
    h = (h ^ (h >> U(15))) + b * U(0x85EBCA77)
    h = (h ^ (h >> U(13))) + c * U(0xC2B2AE3D)
    h = (h ^ (h >> U(16))) + d * U(0x27D4EB2F)
    h = (h ^ (h >> U(15))) + e * U(0x165667B1)
    return fmix(h)


def dev(a, pad=64):
    b = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    t = torch.zeros(b.size + pad, dtype=torch.uint8, device="cuda")
    t[: b.size] = torch.from_numpy(b.copy()).cuda()
    return t


def time_lookup(h, recv, rc, cap, tcap, reps, out):
    for _ in range(5):
        h.lookup_dev(recv, rc, 1, cap, out, tail_cap=tcap)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        h.lookup_dev(recv, rc, 1, cap, out, tail_cap=tcap)
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    import pyoracle
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    t0 = time.time()
    w = synth.config_d(n, rank=0)
    h = RxPath(0, max_ns=32768, max_clients=1 << 20, max_frames=n)
    h.register_all()
    synth.load_tables(w, h)
    o = pyoracle.Oracle()
    synth.load_tables(w, o)
    orec = o.rx_batch(w["buf"], w["desc"])[0]
    print(f"[probe] tables ready {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    cap, tcap = n, abi.tail_capacity(n)
    rb = abi.lookup_region_bytes(cap, tcap)
    buf, desc = dev(w["buf"]), dev(w["desc"])
    qcap = abi.queue_cap(n)
    ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda")
    tc = torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device="cuda")
    hist = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
    send = torch.empty(rb, dtype=torch.uint8, device="cuda")
    sc = torch.zeros(2, dtype=torch.int32, device="cuda")
    h.parse_route_dev(buf, desc, n, None, ql, qcap, tc, hist, 1, 0, cap, send, sc, tail_cap=tcap)
    torch.cuda.synchronize()
    del buf, desc
    cnt = int(sc[0].item())
    heads = send[: cnt * 32].cpu().numpy().view(abi.LOOKUP_REC_DTYPE)
    fr = heads["frame"].astype(np.int64)
    r = orec[fr]
    tk = ehash(r["vport"].astype(U), r["vlan0"], r["vlan1"], np.full(cnt, 0x6E73, U), np.zeros(cnt, U))
    key = (heads["w4"] >> U(28)) & U(7)
    tup = (heads["w4"] >> U(31)) == 1
    lo = np.where(tup, heads["dlo"], heads["x"]).astype(U)
    hi = np.where(tup, heads["dhi"] & U(0xFFFF), heads["dhi"] >> U(16)).astype(U)
    mac_slot = ehash(tk, lo, hi, np.full(cnt, 0x6D6163, U), np.zeros(cnt, U)) & U((1 << 21) - 1)
    ip4_slot = ehash(tk, heads["x"], np.full(cnt, 0x697034, U), np.zeros(cnt, U), np.zeros(cnt, U)) & U((1 << 23) - 1)
    is_mac, is_ip4 = (key == 3), (key == 5)
    sk = np.where(is_mac, mac_slot.astype(np.int64),
                  np.where(is_ip4, (1 << 22) + ip4_slot.astype(np.int64), 1 << 40))
    perm = np.argsort(sk, kind="stable")
    sorted_send = send.clone()
    sorted_send[: cnt * 32] = torch.from_numpy(np.ascontiguousarray(heads[perm]).view(np.uint8).reshape(-1)).cuda()
    rc = sc.clone()
    out_a = torch.empty(cap * X.REC_BYTES, dtype=torch.uint8, device="cuda")
    out_b = torch.empty_like(out_a)
    res = {"frames": n, "heads": cnt, "mac_keyed": int(is_mac.sum()), "ip4_keyed": int(is_ip4.sum()),
           "table_bytes": h.table_stats()["table_bytes"]}
    for k in range(2):  # alternate, twice
        res[f"frame_order_ms_{k}"] = round(time_lookup(h, send, rc, cap, tcap, reps, out_a), 5)
        res[f"bucket_order_ms_{k}"] = round(time_lookup(h, sorted_send, rc, cap, tcap, reps, out_b), 5)
    a = out_a[: cnt * 40].cpu().numpy().view(abi.ROUTE_REC_DTYPE)
    b = out_b[: cnt * 40].cpu().numpy().view(abi.ROUTE_REC_DTYPE)
    res["same_records_permuted"] = bool(a[perm].tobytes() == b.tobytes())
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
