"""Helpers shared by the GPU tests: run the device path through the C-ABI and fetch the
outputs, build tables for frame sets."""
import numpy as np

from emurx import abi


def to_dev(a: np.ndarray, pad: int = 64):
    import torch
    b = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    t = torch.zeros(b.size + pad, dtype=torch.uint8, device="cuda")
    if b.size:
        t[: b.size] = torch.from_numpy(b.copy()).to("cuda")
    return t


def run_dev(rx, buf, desc, classify=True, qcap=None, flows=False):
    """-> rec, qlist (packed in queue order), qoff(14), hist(2*64) as numpy, via
    emurx_classify_dev / emurx_parse_dev (per-tile queue segments, sharded histogram)."""
    import torch
    from emurx.rx import hist_fold, pack_queues
    n = len(desc)
    qcap = qcap or max(abi.queue_cap(n), abi.QUEUE_TILE)
    nt = max(abi.ntiles(n), 1)
    tb, td = to_dev(buf), to_dev(desc)
    rec = torch.zeros(max(n, 1) * 32, dtype=torch.uint8, device="cuda")
    qlist = torch.full((abi.NUM_QUEUES * qcap,), -1, dtype=torch.int32, device="cuda")
    tile_cnt = torch.full((nt * 16,), -1, dtype=torch.int32, device="cuda")
    hist = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
    flow = torch.full((max(n, 1),), 0x5A5A5A5A, dtype=torch.int32, device="cuda") if flows else None
    rx.classify_dev(tb, td, n, rec, qlist, qcap, tile_cnt, hist, classify=classify, flow=flow)
    torch.cuda.synchronize()
    r = rec.cpu().numpy()[: n * 32].view(abi.REC_DTYPE)
    packed, qoff = pack_queues(qlist.cpu().numpy(), qcap, tile_cnt.cpu().numpy(), n)
    out = (r, packed, qoff, hist_fold(hist.cpu().numpy().view(np.uint64)))
    if flows:
        out += (flow.cpu().numpy().view(np.uint32)[:n],)
    return out


def rec_diff(a, b, limit=5):
    """Human-readable first differences between two record arrays."""
    a = np.asarray(a)
    b = np.asarray(b)
    if len(a) != len(b):
        return f"length {len(a)} != {len(b)}"
    A = np.ascontiguousarray(a).view(np.uint8).reshape(-1, 32)
    B = np.ascontiguousarray(b).view(np.uint8).reshape(-1, 32)
    bad = np.nonzero((A != B).any(1))[0]
    out = [f"{len(bad)} differing records"]
    for i in bad[:limit]:
        fa = {k: int(a[i][k]) for k in abi.REC_DTYPE.names}
        fb = {k: int(b[i][k]) for k in abi.REC_DTYPE.names}
        out.append(f"  [{i}] gpu={fa}\n       orc={fb}")
    return "\n".join(out)


def frames_tables(frames, vport=1):
    """Namespace + Client tables derived from a frame set: a Namespace per distinct
    (vport, tags) and, for unicast destination MACs, a client owning that MAC and the
    frame's destination IPv4 / IPv6 (deduplicated)."""
    from emurx import frames as F
    import struct
    ns = {}
    clients = {}
    used4, used6 = set(), set()
    for f in frames:
        if len(f) < 14:
            continue
        et = struct.unpack(">H", f[12:14])[0]
        off, vl = 14, []
        while et in (0x8100, 0x88A8) and len(f) >= off + 4 and len(vl) < 2:
            vl.append(struct.unpack(">I", f[off - 2:off + 2])[0] & 0xFFFF0FFF)
            et = struct.unpack(">H", f[off + 2:off + 4])[0]
            off += 4
        vl += [0] * (2 - len(vl))
        key = F.tunnel_key(vport, vl[0], vl[1])
        nsid = ns.setdefault(key, len(ns))
        dmac = bytes(f[0:6])
        if dmac[0] & 1 or dmac == bytes(6):
            continue
        ip4 = ip6 = None
        if et == 0x0800 and len(f) >= off + 20:
            ip4 = bytes(f[off + 16:off + 20])
        if et == 0x86DD and len(f) >= off + 40:
            ip6 = bytes(f[off + 24:off + 40])
        k = (nsid, dmac)
        if k not in clients:
            if ip4 is not None and ((nsid, ip4) in used4 or ip4 == bytes(4)):
                ip4 = None
            if ip6 is not None and ((nsid, ip6) in used6 or ip6 == bytes(16)):
                ip6 = None
            if ip4:
                used4.add((nsid, ip4))
            if ip6:
                used6.add((nsid, ip6))
            clients[k] = (len(clients), ip4, ip6)
    return ns, clients


def load_frame_tables(targets, ns, clients, plug_ns=abi.PLUG_ALL, plug_cl=abi.PLUG_ALL):
    for t in targets:
        for key, nsid in ns.items():
            assert t.ns_add(key, nsid, plug_ns) == 0
        for (nsid, mac), (cid, ip4, ip6) in clients.items():
            p = plug_cl if cid % 7 else plug_cl & ~(1 << 7)  # some clients without transport
            assert t.client_add(nsid, cid, mac, ip4, ip6, None, p) == 0


def frame_tuples(buf, desc, rec):
    """The reference's c5tuplekey bytes of every tcp/udp frame reaching a client (client_ctx.go:
    89-112): 13 bytes for IPv4, 37 for IPv6; None elsewhere."""
    out = []
    for d, r in zip(desc, rec):
        if r["status"] != 0 or r["proto"] not in (abi.CB_TCP, abi.CB_UDP) or (r["flags"] >> 4) & 7 != abi.LK["CLIENT"]:
            out.append(None)
            continue
        p = buf[d["off"]:d["off"] + d["len"]].tobytes()
        l3, l4 = int(r["l3"]), int(r["l4"])
        if p[l3] >> 4 == 4:
            out.append(p[l3 + 12:l3 + 20] + p[l4:l4 + 4] + bytes([p[l3 + 9]]))
        else:
            out.append(p[l3 + 8:l3 + 40] + p[l4:l4 + 4] + bytes([int(r["next_hdr"])]))
    return out


def owner_keys(rec):
    """The descriptor owner key (EMURX_DESC_KEYED | digest) of every record's CTunnelKey."""
    from emurx import frames as F
    from emurx.rx import owner_key
    if len(rec) == 0:
        return np.zeros(0, np.uint8)
    k = np.stack([rec["vport"].astype(np.uint64), rec["vlan0"].astype(np.uint64), rec["vlan1"].astype(np.uint64)], 1)
    uk, inv = np.unique(k, axis=0, return_inverse=True)
    ok = np.array([owner_key(F.tunnel_key(int(a), int(b), int(c))) for a, b, c in uk], np.uint8)
    return ok[inv.reshape(-1)]
