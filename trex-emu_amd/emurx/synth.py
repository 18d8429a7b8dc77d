"""Seeded synthetic workloads of BASELINE.json's configs, vectorised numpy.

    config_b  1M x 64 B untagged IPv4/UDP, 1 Namespace / 1 Client (seed 0xE3E3_0001)
    config_c  1M mixed dot1q/QinQ IPv4/IPv6 (10 % of IPv6 with an 8-B HBH/DST header),
              UDP 60 / TCP 30 / ICMP(v6) echo 10 %, 4K Namespaces / 64K Clients,
              1 % bad IPv4/L4 checksum, 1 % unknown Namespace, 1 % unknown MAC (0xE3E3_0002)
    config_d  config_c at 16M frames, 32K Namespaces / 1M Clients (0xE3E3_0003)
    config_e  IMIX 7:4:1 of 64/594/1518 B, TCP 70 % / UDP 30 % with valid checksums over the
              whole segment, tables as config_c (0xE3E3_0004)

A workload is a dict: buf (uint8, frames in ZMQ layout: a 4-byte 0xAA|vport|len header in
front of every frame, 64 zero bytes of tail padding), desc (DESC_DTYPE), n, nbytes (frame
bytes), ns (list of (key12, ns_id)), clients (dict of arrays ns/cid/mac/ipv4/ipv6).
Data is synthetic; frame bytes are valid wire formats (gopacket layouts, frames.py).
"""
from __future__ import annotations

import numpy as np

from .abi import DESC_DTYPE

SEED_B, SEED_C, SEED_D, SEED_E = 0xE3E30001, 0xE3E30002, 0xE3E30003, 0xE3E30004
_SPECIAL_UDP = np.array([67, 68, 546, 547, 5353])


def _be16(F, rows, col, v):
    v = np.asarray(v, dtype=np.uint32)
    F[rows, col] = (v >> 8) & 0xFF
    F[rows, col + 1] = v & 0xFF


def _be32(F, rows, col, v):
    v = np.asarray(v, dtype=np.uint64)
    for k in range(4):
        F[rows, col + k] = (v >> (8 * (3 - k))) & 0xFF


def _pair_sum(F, rows, start, length):
    """sum of big-endian byte pairs of F[rows, start:start+length] (odd tail byte << 8)."""
    maxlen = int(length.max()) if len(length) else 0
    maxlen += maxlen & 1
    W = F[rows, start:start + maxlen].astype(np.uint64)
    M = np.arange(maxlen)[None, :] < length[:, None]
    W = W * M
    return (W[:, 0::2] << 8).sum(1) + W[:, 1::2].sum(1)


def _fold_inv(s):
    s = s.astype(np.uint64)
    for _ in range(4):
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def _udp_ports(rng, m):
    sp = rng.integers(1024, 65536, m)
    bad = np.isin(sp, _SPECIAL_UDP)
    sp[bad] = 40000
    return sp


def build_frames(rng, spec):
    """Vectorised frame builder.  spec: dict of per-frame arrays
    ntag (0..2), tpid0, vid0, vid1, ipver (4|6), ext (0 none, 1 HBH+RouterAlert, 2 DST PadN),
    l4 (17|6|1; 1 means ICMPv4 / ICMPv6 echo by ipver), dmac (n,6), smac (n,6),
    sip4/dip4 (n,4), sip6/dip6 (n,16), sport, dport, plen, bad (0, 1 IPv4 hdr, 2 L4).
    Returns (F uint8 (n, L), length uint32 (n,))."""
    n = len(spec["ntag"])
    hdr = 14 + 4 * spec["ntag"] + np.where(spec["ipver"] == 4, 20, 40 + 8 * (spec["ext"] > 0))
    l4h = np.where(spec["l4"] == 6, 20, 8)
    length = (hdr + l4h + spec["plen"]).astype(np.uint32)
    L = int(length.max()) + 8
    F = np.zeros((n, L), dtype=np.uint8)
    F[:, 0:6] = spec["dmac"]
    F[:, 6:12] = spec["smac"]
    keys = (spec["ntag"] * 100 + spec["ipver"] * 10 + spec["ext"]) * 1000 + spec["l4"]
    for key in np.unique(keys):
        rows = np.nonzero(keys == key)[0]
        ntag = int(spec["ntag"][rows[0]])
        v6 = int(spec["ipver"][rows[0]]) == 6
        ext = int(spec["ext"][rows[0]])
        l4 = int(spec["l4"][rows[0]])
        plen = spec["plen"][rows].astype(np.int64)
        m = len(rows)
        o = 12
        if ntag >= 1:
            _be16(F, rows, o, spec["tpid0"][rows])
            _be16(F, rows, o + 2, spec["vid0"][rows])
            o += 4
        if ntag >= 2:
            _be16(F, rows, o, np.full(m, 0x8100))
            _be16(F, rows, o + 2, spec["vid1"][rows])
            o += 4
        _be16(F, rows, o, np.full(m, 0x86DD if v6 else 0x0800))
        L3 = o + 2
        l4hdr = 20 if l4 == 6 else 8
        if v6:
            extlen = 8 if ext else 0
            L4 = L3 + 40 + extlen
            nh_l4 = 58 if l4 == 1 else l4
            F[rows, L3] = 0x60
            _be16(F, rows, L3 + 4, extlen + l4hdr + plen)
            F[rows, L3 + 6] = (0 if ext == 1 else 60) if ext else nh_l4
            F[rows, L3 + 7] = 64
            F[rows, L3 + 8:L3 + 24] = spec["sip6"][rows]
            F[rows, L3 + 24:L3 + 40] = spec["dip6"][rows]
            if ext == 1:   # HBH: Router Alert (type 5, len 2) + Pad1-free PadN(0)
                F[rows, L3 + 40:L3 + 48] = np.array([nh_l4, 0, 5, 2, 0, 0, 1, 0], np.uint8)
            elif ext == 2:  # DST: PadN(4)
                F[rows, L3 + 40:L3 + 48] = np.array([nh_l4, 0, 1, 4, 0, 0, 0, 0], np.uint8)
            l4len = l4hdr + plen
            pcs = _pair_sum(F, rows, L3 + 8, np.full(m, 32)) + l4len + nh_l4
        else:
            L4 = L3 + 20
            totlen = 20 + l4hdr + plen
            F[rows, L3] = 0x45
            _be16(F, rows, L3 + 2, totlen)
            _be16(F, rows, L3 + 4, rows & 0xFFFF)
            _be16(F, rows, L3 + 6, np.full(m, 0x4000))  # DF
            F[rows, L3 + 8] = 64
            F[rows, L3 + 9] = l4
            F[rows, L3 + 12:L3 + 16] = spec["sip4"][rows]
            F[rows, L3 + 16:L3 + 20] = spec["dip4"][rows]
            ipcs = _fold_inv(_pair_sum(F, rows, L3, np.full(m, 20)))
            bad_ip = spec["bad"][rows] == 1
            ipcs = np.where(bad_ip, ipcs ^ 0x0100, ipcs)
            _be16(F, rows, L3 + 10, ipcs)
            l4len = l4hdr + plen
            pcs = _pair_sum(F, rows, L3 + 12, np.full(m, 8)) + l4 + l4len
        # L4 header
        if l4 == 17:
            _be16(F, rows, L4, spec["sport"][rows])
            _be16(F, rows, L4 + 2, spec["dport"][rows])
            _be16(F, rows, L4 + 4, 8 + plen)
            cso = 6
        elif l4 == 6:
            _be16(F, rows, L4, spec["sport"][rows])
            _be16(F, rows, L4 + 2, spec["dport"][rows])
            _be32(F, rows, L4 + 4, rows.astype(np.uint64) * 1000 + 1)
            F[rows, L4 + 12] = 5 << 4
            F[rows, L4 + 13] = spec["tcpflags"][rows] if "tcpflags" in spec else 0x18
            _be16(F, rows, L4 + 14, np.full(m, 8192))
            cso = 16
        else:
            F[rows, L4] = 128 if v6 else 8
            _be16(F, rows, L4 + 4, rows & 0xFFFF)
            _be16(F, rows, L4 + 6, (rows >> 16) & 0xFFFF)
            cso = 2
            if not v6:
                pcs = np.zeros(m, dtype=np.uint64)  # ICMPv4 checksum has no pseudo header
        # payload
        maxp = int(plen.max()) if m else 0
        if maxp:
            P = rng.integers(0, 256, (m, maxp), dtype=np.uint8)
            P *= (np.arange(maxp)[None, :] < plen[:, None])
            F[rows, L4 + l4hdr:L4 + l4hdr + maxp] = P
        cs = _fold_inv(pcs + _pair_sum(F, rows, L4, l4hdr + plen))
        if l4 == 17:
            cs = np.where(cs == 0, 0xFFFF, cs)  # valid, non-zero (RFC 768)
        bad_l4 = (spec["bad"][rows] == 2) | ((spec["bad"][rows] == 1) & v6)
        flipped = cs ^ 0x0100
        flipped = np.where(flipped == 0, cs ^ 0x0200, flipped)
        cs = np.where(bad_l4, flipped, cs)
        _be16(F, rows, L4 + cso, cs)
    return F, length


def pack_zmq_layout(F, length, vport):
    """frames -> one buffer, each frame preceded by its 4-byte ZMQ frame header."""
    n = len(length)
    length = length.astype(np.int64)
    off = np.zeros(n, dtype=np.int64)
    if n:
        off[1:] = np.cumsum(length[:-1] + 4)
    off += 4
    total = int(off[-1] + length[-1]) if n else 0
    buf = np.zeros(total + 64, dtype=np.uint8)
    hdr = (0xAA << 24) | ((vport.astype(np.int64) & 0xFF) << 16) | length
    hb = np.stack([(hdr >> 24) & 0xFF, (hdr >> 16) & 0xFF, (hdr >> 8) & 0xFF, hdr & 0xFF], 1)
    idx = (off - 4)[:, None] + np.arange(4)[None, :]
    buf[idx] = hb.astype(np.uint8)
    # scatter frames grouped by length (vectorised per length)
    for ln in np.unique(length):
        rows = np.nonzero(length == ln)[0]
        cols = off[rows][:, None] + np.arange(ln)[None, :]
        buf[cols] = F[rows, :ln]
    desc = np.zeros(n, dtype=DESC_DTYPE)
    desc["off"] = off
    desc["len"] = length
    desc["vport"] = vport
    return buf, desc


def _mac_of(ns, c):
    """client MAC 02:<ns 3 bytes>:<c 2 bytes>  (locally administered, unique, non-zero)."""
    ns = np.asarray(ns, dtype=np.int64)
    c = np.asarray(c, dtype=np.int64)
    return np.stack([np.full_like(ns, 2), (ns >> 16) & 0xFF, (ns >> 8) & 0xFF, ns & 0xFF,
                     (c >> 8) & 0xFF, c & 0xFF], -1).astype(np.uint8)


def _ipv4_of(ns, c):
    ns = np.asarray(ns, dtype=np.int64)
    c = np.asarray(c, dtype=np.int64)
    return np.stack([10 + ((ns >> 16) & 0x3F), (ns >> 8) & 0xFF, ns & 0xFF, (c & 0xFF) + 1],
                    -1).astype(np.uint8)


def _ipv6_of(ns, c):
    ns = np.asarray(ns, dtype=np.int64)
    c = np.asarray(c, dtype=np.int64)
    out = np.zeros(ns.shape + (16,), dtype=np.uint8)
    out[..., 0], out[..., 1], out[..., 2], out[..., 3] = 0x20, 0x01, 0x0D, 0xB8
    out[..., 4], out[..., 5], out[..., 6] = (ns >> 16) & 0xFF, (ns >> 8) & 0xFF, ns & 0xFF
    out[..., 14], out[..., 15] = (c >> 8) & 0xFF, (c & 0xFF) + 1
    return out


def _ns_layout(n_ns, pairs_per_vport):
    """Namespace k: vport = k // pairs, pair j = k % pairs.  The first half of the pairs are
    single dot1q (VID j+1), the second half QinQ (outer TPID 0x88a8 / 0x8100 alternating)."""
    k = np.arange(n_ns)
    vport = k // pairs_per_vport
    j = k % pairs_per_vport
    half = pairs_per_vport // 2
    single = j < half
    q = j - half
    ntag = np.where(single, 1, 2)
    tpid0 = np.where(single, 0x8100, np.where(q % 2 == 0, 0x88A8, 0x8100))
    vid0 = np.where(single, j + 1, 1 + (q // 16) % 4000)
    vid1 = np.where(single, 0, 1 + q % 16)
    v0 = (tpid0.astype(np.int64) << 16) | vid0
    v1 = np.where(single, 0, (0x8100 << 16) | vid1)
    return dict(vport=vport, ntag=ntag, tpid0=tpid0, vid0=vid0, vid1=vid1, vlan0=v0, vlan1=v1)


def _keys(lay):
    from .frames import tunnel_key
    return [(tunnel_key(int(lay["vport"][k]), int(lay["vlan0"][k]), int(lay["vlan1"][k])), k)
            for k in range(len(lay["vport"]))]


def config_b(n=1 << 20, seed=SEED_B):
    rng = np.random.default_rng(seed)
    cmac = _mac_of(np.array([0]), np.array([0]))[0]
    cip = np.array([10, 0, 0, 1], np.uint8)
    sip = np.zeros((n, 4), np.uint8)
    sip[:, 0], sip[:, 1] = 16, 0
    sip[:, 2:4] = rng.integers(0, 256, (n, 2), dtype=np.uint8)
    spec = dict(ntag=np.zeros(n, np.int64), tpid0=np.zeros(n, np.int64), vid0=np.zeros(n, np.int64),
                vid1=np.zeros(n, np.int64), ipver=np.full(n, 4), ext=np.zeros(n, np.int64),
                l4=np.full(n, 17), dmac=np.broadcast_to(cmac, (n, 6)),
                smac=np.broadcast_to(np.array([0, 0x11, 0x22, 0x33, 0x44, 0x55], np.uint8), (n, 6)),
                sip4=sip, dip4=np.broadcast_to(cip, (n, 4)), sip6=None, dip6=None,
                sport=_udp_ports(rng, n), dport=np.full(n, 5000), plen=np.full(n, 22),
                bad=np.zeros(n, np.int64))
    F, length = build_frames(rng, spec)
    assert (length == 64).all()
    buf, desc = pack_zmq_layout(F, length, np.zeros(n, np.int64))
    from .frames import tunnel_key
    clients = dict(ns=np.array([0]), cid=np.array([0]), mac=cmac[None], ipv4=cip[None],
                   ipv6=np.zeros((1, 16), np.uint8))
    return dict(name="B", buf=buf, desc=desc, n=n, nbytes=int(length.sum()),
                ns=[(tunnel_key(0, 0, 0), 0)], clients=clients, seed=seed)


def _mixed(n, seed, n_ns, clients_per_ns, vports, imix=False, name="C", rank=0, syn=0.0):
    rng = np.random.default_rng([seed, rank])
    lay = _ns_layout(n_ns, n_ns // vports)
    ns_of = rng.integers(0, n_ns, n)
    u = rng.random(n)
    unknown_ns = u < 0.01
    unknown_mac = (u >= 0.01) & (u < 0.02)
    bad = np.where((u >= 0.02) & (u < 0.03), np.where(rng.random(n) < 0.5, 1, 2), 0)
    ntag = lay["ntag"][ns_of]
    tpid0 = lay["tpid0"][ns_of]
    vid0 = lay["vid0"][ns_of].copy()
    vid1 = lay["vid1"][ns_of]
    vid0[unknown_ns] = 4090 + (vid0[unknown_ns] % 5)  # never allocated by _ns_layout
    vport = lay["vport"][ns_of]
    if imix:
        size = rng.choice(np.array([64, 594, 1518]), n, p=np.array([7, 4, 1]) / 12)
        l4 = np.where(rng.random(n) < 0.7, 6, 17)
        ipver = np.where(rng.random(n) < 0.5, 4, 6)
        ipver[size == 64] = 4
    else:
        ipver = np.where(rng.random(n) < 0.5, 4, 6)
        r = rng.random(n)
        l4 = np.where(r < 0.6, 17, np.where(r < 0.9, 6, 1))
    ext = np.where((ipver == 6) & (rng.random(n) < 0.1), np.where(rng.random(n) < 0.5, 1, 2), 0)
    if imix:
        ext[size == 64] = 0
    c_of = rng.integers(0, clients_per_ns, n)
    dmac = _mac_of(ns_of, c_of)
    dmac[unknown_mac, 0] = 0x06  # locally administered, never allocated
    smac = _mac_of(ns_of + 1_000_000, c_of)
    smac[:, 0] = 0x0A
    sip4 = rng.integers(0, 256, (n, 4), dtype=np.uint8)
    sip4[:, 0] = 16
    dip4 = _ipv4_of(ns_of, c_of)
    sip6 = _ipv6_of(ns_of + 77, c_of)
    dip6 = _ipv6_of(ns_of, c_of)
    hdr = 14 + 4 * ntag + np.where(ipver == 4, 20, 40 + 8 * (ext > 0)) + np.where(l4 == 6, 20, 8)
    if imix:
        plen = np.maximum(size - hdr, 0)
    else:
        lo = np.maximum(64 - hdr, 0)
        plen = lo + (rng.random(n) * (110 - hdr - lo + 1)).astype(np.int64)
    sport = np.where(l4 == 17, _udp_ports(rng, n), rng.integers(1024, 65536, n))
    dport = np.where(l4 == 17, _udp_ports(rng, n), rng.integers(1, 1024, n))
    spec = dict(ntag=ntag, tpid0=tpid0, vid0=vid0, vid1=vid1, ipver=ipver, ext=ext, l4=l4,
                dmac=dmac, smac=smac, sip4=sip4, dip4=dip4, sip6=sip6, dip6=dip6, sport=sport,
                dport=dport, plen=plen, bad=bad)
    if syn:  # a share of bare SYNs (new TCP flows); the default keeps PSH|ACK
        spec["tcpflags"] = np.where(rng.random(n) < syn, 0x02, 0x18)
    F, length = build_frames(rng, spec)
    buf, desc = pack_zmq_layout(F, length, vport)
    del F
    nsk = np.repeat(np.arange(n_ns), clients_per_ns)
    ck = np.tile(np.arange(clients_per_ns), n_ns)
    clients = dict(ns=nsk, cid=nsk * clients_per_ns + ck, mac=_mac_of(nsk, ck), ipv4=_ipv4_of(nsk, ck),
                   ipv6=_ipv6_of(nsk, ck))
    return dict(name=name, buf=buf, desc=desc, n=n, nbytes=int(length.sum()), ns=_keys(lay),
                clients=clients, seed=seed, layout=lay)


def config_c(n=1 << 20, seed=SEED_C, rank=0, syn=0.0):
    return _mixed(n, seed, 4096, 16, 4, name="C", rank=rank, syn=syn)


def config_d(n=1 << 24, seed=SEED_D, rank=0):
    return _mixed(n, seed, 32768, 32, 8, name="D", rank=rank)


def config_e(n=1 << 20, seed=SEED_E, rank=0):
    return _mixed(n, seed, 4096, 16, 4, imix=True, name="E", rank=rank)


def load_tables(w, target):
    """Populate an RxPath (or the test oracle, same method names) with a workload's tables."""
    for key, ns_id in w["ns"]:
        rc = target.ns_add(key, ns_id, 0x7FF)
        assert rc == 0, rc
    rc, k = target.clients_add(client_specs(w))
    assert rc == 0 and k == len(w["clients"]["cid"]), (rc, k)


def client_specs(w, plugins=0x7FF):
    """The workload's clients as one ctx_client_add list (CLIENT_SPEC_DTYPE rows)."""
    from .abi import CLIENT_SPEC_DTYPE
    c = w["clients"]
    s = np.zeros(len(c["cid"]), CLIENT_SPEC_DTYPE)
    s["ns_id"], s["client_id"], s["plugin_mask"] = c["ns"], c["cid"], plugins
    s["mac"], s["ipv4"], s["ipv6"] = c["mac"], c["ipv4"], c["ipv6"]
    return s
