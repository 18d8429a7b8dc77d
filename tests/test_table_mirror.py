"""The host side of the tables, no GPU (host-only handles, emurx_open with device < 0):

* Go map semantics: every table call returns what the oracle (the Go restatement) returns.
* The device image: after every mutation the kernels' bucket walk over the host image
  (emurx_image_lookup) finds exactly the live map entries -- through tombstones, rebuilds and
  growth -- so the blocks the library ships to the device hold the tables Go would probe.
* Partitioned images hold only the owned Namespaces and about 1/n of the bytes.
* The mid-batch rule (include/emu_rx.h emurx_recs_stale): a record of a batch classified at
  batch start that is NOT flagged stale equals Go's classification of that frame against the
  maps as the callbacks of the earlier frames of the batch left them (DHCP's UpdateClientIpv4
  dhcp.go:718, client add / remove, plugin changes, Namespace add / remove mid-batch)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from emurx import abi, synth
from emurx import frames as F
from emurx.rx import RxPath, ns_owner

NS, MAC, IP4, IP6, CI, FT4, FT6, SRV = range(8)


def le32(b):
    return int.from_bytes(bytes(b[:4]), "little")


def mac_key(ns, mac):
    return [ns, le32(mac), mac[4] | (mac[5] << 8)]


def ip6_key(ns, ip):
    return [ns] + [le32(ip[4 * k:4 * k + 4]) for k in range(4)]


class Model:
    """Python truth of the Go maps (only what the image must answer)."""

    def __init__(self):
        self.ns, self.mac, self.ip4, self.ip6, self.cl = {}, {}, {}, {}, {}

    def check(self, rx, owned=None, sample=None):
        items = list(self.ns.items())
        for key, nsid in items:
            w = [le32(key[0:4]), le32(key[4:8]), le32(key[8:12])]
            want = nsid if owned is None or owned(nsid) else None
            assert rx.image_lookup(NS, w) == want, (key.hex(), nsid)
        for (ns, mac), cid in self.mac.items():
            want = cid if owned is None or owned(ns) else None
            assert rx.image_lookup(MAC, mac_key(ns, mac)) == want
        for (ns, ip), cid in self.ip4.items():
            want = cid if owned is None or owned(ns) else None
            assert rx.image_lookup(IP4, [ns, le32(ip)]) == want
        for (ns, ip), cid in self.ip6.items():
            want = cid if owned is None or owned(ns) else None
            assert rx.image_lookup(IP6, ip6_key(ns, ip)) == want
        for cid, c in self.cl.items():
            want = c["plugins"] if owned is None or owned(c["ns"]) else None
            assert rx.image_lookup(CI, [cid]) == want


def host_pair(max_ns=512, max_clients=4096):
    import pyoracle
    return RxPath(-1, max_ns=max_ns, max_clients=max_clients, max_frames=1024), pyoracle.Oracle()


def test_host_only_handle_needs_no_gpu(lib):
    rx = RxPath(-1, max_ns=16, max_clients=16, max_frames=64)
    key = F.tunnel_key(1, 0x81000005, 0)
    assert rx.ns_add(key, 3, abi.PLUG_ALL) == 0
    assert rx.image_lookup(NS, [1, 0x81000005, 0]) == 3
    rx.sync()  # nothing to ship to: a no-op
    with pytest.raises(RuntimeError, match="HIP runtime error"):
        rx.classify_dev(0, 0, 0, hist=1)


def random_ops(rx, o, m, rng, steps, keys, owned=None, check_every=50):
    """Random AddNs / RemoveNs / AddClient / RemoveClient / UpdateClientIpv4 / Ipv6 /
    DIpv6 / plugin changes on both, return codes compared; the image checked against m."""
    next_cid = [max(m.cl) + 1 if m.cl else 0]
    for step in range(steps):
        op = int(rng.integers(0, 9))
        nss = list(m.ns.values())
        cids = list(m.cl)
        if op == 0 or not nss:  # AddNs (sometimes a duplicate key or id)
            key = keys[int(rng.integers(0, len(keys)))]
            nsid = int(rng.integers(0, 512))
            rc = rx.ns_add(key, nsid, abi.PLUG_ALL)
            assert rc == o.ns_add(key, nsid, abi.PLUG_ALL)
            if rc == 0:
                m.ns[key] = nsid
        elif op == 1:  # RemoveNs (refused while it has clients)
            key = list(m.ns)[int(rng.integers(0, len(m.ns)))]
            rc = rx.ns_remove(key)
            assert rc == o.ns_remove(key)
            if rc == 0:
                del m.ns[key]
        elif op in (2, 3):  # AddClient
            ns = nss[int(rng.integers(0, len(nss)))]
            cid = next_cid[0] % 4096
            next_cid[0] += 1
            mac = bytes([2, 0, ns >> 8, ns & 255, (cid >> 8) & 255, cid & 255])
            if rng.random() < 0.05:
                mac = bytes(6)  # refused (EINVAL)
            ip4 = bytes([10, int(rng.integers(0, 4)), int(rng.integers(0, 4)), int(rng.integers(1, 250))])
            ip6 = bytes([0x20, 1, 0xd, 0xb8] + [0] * 10 + [int(rng.integers(0, 8)), int(rng.integers(1, 250))])
            d6 = ip6 if rng.random() < 0.05 else (bytes(16) if rng.random() < 0.5 else bytes([0xfd] + [0] * 14 + [int(rng.integers(1, 99))]))
            rc = rx.client_add(ns, cid, mac, ip4, ip6, d6, abi.PLUG_ALL)
            assert rc == o.client_add(ns, cid, mac, ip4, ip6, d6, abi.PLUG_ALL)
            if rc == 0:
                m.mac[(ns, mac)] = cid
                m.ip4[(ns, ip4)] = cid
                m.ip6[(ns, ip6)] = cid
                if d6 != bytes(16):
                    m.ip6[(ns, d6)] = cid
                m.cl[cid] = dict(ns=ns, mac=mac, ip4=ip4, ip6=ip6, d6=d6, plugins=abi.PLUG_ALL)
        elif op == 4 and cids:  # RemoveClient
            cid = cids[int(rng.integers(0, len(cids)))]
            c = m.cl[cid]
            rc = rx.client_remove(c["ns"], c["mac"])
            assert rc == o.client_remove(c["ns"], c["mac"]) == 0
            del m.mac[(c["ns"], c["mac"])]
            for k, t in (("ip4", m.ip4), ("ip6", m.ip6), ("d6", m.ip6)):
                if c[k] != bytes(len(c[k])):
                    t.pop((c["ns"], c[k]), None)
            del m.cl[cid]
        elif op in (5, 6) and cids:  # UpdateClientIpv4 / Ipv6 (sometimes to a taken or zero address)
            cid = cids[int(rng.integers(0, len(cids)))]
            c = m.cl[cid]
            v6 = op == 6
            if v6:
                nw = bytes([0x20, 1, 0xd, 0xb8] + [0] * 10 + [int(rng.integers(0, 8)), int(rng.integers(0, 250))])
                rc = rx.client_update_ipv6(cid, nw)
                assert rc == o.client_update_ipv6(cid, nw)
            else:
                nw = bytes([10, int(rng.integers(0, 4)), int(rng.integers(0, 4)), int(rng.integers(0, 250))])
                rc = rx.client_update_ipv4(cid, nw)
                assert rc == o.client_update_ipv4(cid, nw)
            t, k = (m.ip6, "ip6") if v6 else (m.ip4, "ip4")
            cur = c[k]
            if cur != nw:  # Go: drop the old entry, add the new one unless it is taken
                if cur != bytes(len(cur)):
                    t.pop((c["ns"], cur), None)
                if rc == 0:
                    if nw != bytes(len(nw)):
                        t[(c["ns"], nw)] = cid
                    c[k] = nw
                else:
                    c[k] = bytes(len(cur))
        elif op == 7 and cids:  # client plugins
            cid = cids[int(rng.integers(0, len(cids)))]
            p = int(rng.integers(0, 1 << 11))
            assert rx.client_set_plugins(cid, p) == o.client_set_plugins(cid, p) == 0
            m.cl[cid]["plugins"] = p
        elif op == 8 and nss:
            nsid = nss[int(rng.integers(0, len(nss)))]
            p = int(rng.integers(0, 1 << 11))
            assert rx.ns_set_plugins(nsid, p) == o.ns_set_plugins(nsid, p) == 0
        if step % check_every == 0:
            m.check(rx, owned)
    m.check(rx, owned)


def _keys(k):
    return [F.tunnel_key(v % 4, 0x81000000 | (v + 1), 0 if v % 2 else 0x81000000 | (v % 7 + 1)) for v in range(k)]


def test_image_follows_random_mutations(oracle_built):
    rx, o = host_pair()
    random_ops(rx, o, Model(), np.random.default_rng(7), 6000, _keys(300))


def test_tombstone_churn_rebuilds(oracle_built):
    """Thousands of add / remove cycles on a small table: tombstones force rebuilds at the
    same size, and the image keeps answering every live key."""
    rx, o = host_pair(max_ns=8, max_clients=64)
    m = Model()
    key = F.tunnel_key(0, 0, 0)
    assert rx.ns_add(key, 0, abi.PLUG_ALL) == o.ns_add(key, 0, abi.PLUG_ALL) == 0
    m.ns[key] = 0
    live = []
    rng = np.random.default_rng(3)
    for i in range(5000):
        if len(live) < 40 and (not live or rng.random() < 0.55):
            cid = int(rng.integers(0, 64))
            mac = bytes([2, 0, 0, 0, i >> 8 & 255, i & 255])
            rc = rx.client_add(0, cid, mac, bytes([10, 0, i >> 8 & 255, i & 255]), None, None, abi.PLUG_ALL)
            assert rc == o.client_add(0, cid, mac, bytes([10, 0, i >> 8 & 255, i & 255]), None, None, abi.PLUG_ALL)
            if rc == 0:
                live.append((cid, mac, bytes([10, 0, i >> 8 & 255, i & 255])))
                m.mac[(0, mac)] = cid
                m.ip4[(0, live[-1][2])] = cid
                m.cl[cid] = dict(ns=0, plugins=abi.PLUG_ALL)
        else:
            cid, mac, ip = live.pop(int(rng.integers(0, len(live))))
            assert rx.client_remove(0, mac) == o.client_remove(0, mac) == 0
            del m.mac[(0, mac)], m.ip4[(0, ip)], m.cl[cid]
        if i % 97 == 0:
            m.check(rx)
    m.check(rx)


def test_transport_tables_grow(oracle_built):
    """Flow and listener tables start at 16 buckets and grow; every live flow stays findable."""
    rx, o = host_pair(max_ns=4, max_clients=16)
    key = F.tunnel_key(0, 0, 0)
    assert rx.ns_add(key, 0, abi.PLUG_ALL) == 0
    assert rx.client_add(0, 5, bytes([2, 0, 0, 0, 0, 5]), bytes([10, 0, 0, 5]), None, None, abi.PLUG_ALL) == 0
    rng = np.random.default_rng(9)
    flows = {}
    for i in range(3000):
        t = bytes(rng.integers(0, 256, 13 if i % 3 else 37, dtype=np.uint8))
        assert rx.flow_add(5, t, i) == 0
        flows[t] = i
        if i % 5 == 0:
            k = list(flows)[int(rng.integers(0, len(flows)))]
            assert rx.flow_remove(5, k) == 0
            del flows[k]
    for t, fid in flows.items():
        if len(t) == 13:
            w = [5, le32(t[0:4]), le32(t[4:8]), le32(t[8:12]), t[12]]
            assert rx.image_lookup(FT4, w) == fid
        else:
            w = [5] + [le32(t[4 * k:4 * k + 4]) for k in range(8)] + [le32(t[32:36]), t[36]]
            assert rx.image_lookup(FT6, w) == fid
    for port in range(200):
        assert rx.server_add(5, 1000 + port, 6) == 0
    assert all(rx.image_lookup(SRV, [5, 1000 + p | 6 << 16]) == 1 for p in range(200))
    assert rx.image_lookup(SRV, [5, 999 | 6 << 16]) is None


@pytest.mark.parametrize("parts", [2, 3, 8])
def test_partitioned_image(oracle_built, parts):
    """With set_partition(n, p) the image holds exactly the Namespaces p owns and their
    clients; the n images of config C together are about the replicated image's bytes."""
    w = synth.config_c(64)
    full = RxPath(-1, max_ns=4096, max_clients=65536, max_frames=64)
    synth.load_tables(w, full)
    total = full.table_stats()["table_bytes"]
    sizes = []
    for p in range(parts):
        rx = RxPath(-1, max_ns=4096, max_clients=65536, max_frames=64)
        rx.set_partition(parts, p)
        synth.load_tables(w, rx)
        sizes.append(rx.table_stats()["table_bytes"])
        owner = {nsid: ns_owner(key, parts) for key, nsid in w["ns"]}
        m = Model()
        m.ns = {key: nsid for key, nsid in w["ns"][::17]}
        c = w["clients"]
        for i in range(0, len(c["cid"]), 97):
            m.mac[(int(c["ns"][i]), c["mac"][i].tobytes())] = int(c["cid"][i])
            m.ip4[(int(c["ns"][i]), c["ipv4"][i].tobytes())] = int(c["cid"][i])
            m.ip6[(int(c["ns"][i]), c["ipv6"][i].tobytes())] = int(c["cid"][i])
            m.cl[int(c["cid"][i])] = dict(ns=int(c["ns"][i]), plugins=0x7FF)
        m.check(rx, owned=lambda nsid: owner[nsid] == p)
    # + the dense ns info and the transport tables' minimum sizes (a few tens of KB a partition);
    # power-of-two tables: 1/parts of the bytes for parts = 2, 8, at most 2/parts for 3
    share = 1 if parts & (parts - 1) == 0 else 2
    assert max(sizes) <= share * total / parts + 4096 * 16 + (1 << 16), (sizes, total)


def test_partition_growth(oracle_built):
    """A partition that receives far more than its share grows its tables."""
    rx, o = host_pair(max_ns=512, max_clients=4096)
    rx.set_partition(8, 3)
    keys = [k for k in _keys(400) if ns_owner(k, 8) == 3]
    m = Model()
    for i, key in enumerate(keys):
        assert rx.ns_add(key, i, abi.PLUG_ALL) == o.ns_add(key, i, abi.PLUG_ALL) == 0
        m.ns[key] = i
    cid = 0
    for i in range(len(keys)):
        for j in range(40):
            mac = bytes([2, 1, i >> 8, i & 255, 0, j + 1])
            ip4 = bytes([10, 9, i & 255, j + 1])
            assert rx.client_add(i, cid, mac, ip4, None, None, abi.PLUG_ALL) == 0
            m.mac[(i, mac)] = cid
            m.ip4[(i, ip4)] = cid
            m.cl[cid] = dict(ns=i, plugins=abi.PLUG_ALL)
            cid += 1
            if cid >= 4096:
                break
    m.check(rx)


# ---- the mid-batch rule ----------------------------------------------------------------
def test_mid_batch_rule(oracle_built):
    """Frames dispatched in order while "callbacks" mutate the maps between them: every record
    of the batch-start snapshot that emurx_recs_stale does not flag equals the live
    classification (oracle single-frame parse against the mutated maps); flagged ones are the
    ones the shim re-probes.  The mutations target Namespaces and clients of later frames."""
    import pyoracle
    n = 6000
    w = synth.config_c(n, seed=0xB0B)
    live, snap = pyoracle.Oracle(), pyoracle.Oracle()
    rx = RxPath(-1, max_ns=4096 + 64, max_clients=65536 + 64, max_frames=n)
    for t in (live, snap, rx):
        synth.load_tables(w, t)
    srec, _, _, _ = snap.rx_batch(w["buf"], w["desc"])
    g0 = rx.table_gen()
    rng = np.random.default_rng(5)
    c = w["clients"]
    cid_of = {(int(c["ns"][i]), c["mac"][i].tobytes()): int(c["cid"][i]) for i in range(len(c["cid"]))}
    key_of = {nsid: key for key, nsid in w["ns"]}
    frames = [w["buf"][d["off"]:d["off"] + d["len"]].tobytes() for d in w["desc"]]
    stale_n = differ = 0
    spare = 65536
    for j in range(n):
        rec_live = live.parse_frame(frames[j], int(w["desc"]["vport"][j]))
        st = rx.recs_stale(srec[j:j + 1], g0)[0]
        if rec_live.tobytes() != srec[j].tobytes():
            differ += 1
            assert st, (j, srec[j], rec_live)
        stale_n += int(st)
        if rng.random() < 0.02:  # a callback mutates the tables
            t = srec[min(n - 1, j + int(rng.integers(1, 40)))]  # a later frame's Namespace / client
            op = int(rng.integers(0, 6))
            nsid, cid = int(t["ns_id"]), int(t["client_id"])
            for target in (live, rx):
                if op == 0 and cid != abi.ID_NONE:  # DHCP ack: UpdateClientIpv4 (dhcp.go:718)
                    rc = target.client_update_ipv4(cid, bytes([172, 31, j >> 8 & 255, j & 255]))
                elif op == 1 and cid != abi.ID_NONE:  # the client goes away
                    mac = bytes(c["mac"][cid])
                    rc = target.client_remove(int(c["ns"][cid]), mac)
                elif op == 2 and nsid != abi.ID_NONE:  # a plugin is removed from the Namespace
                    rc = target.ns_set_plugins(nsid, 0x7FF & ~(1 << abi.PLUG_NAMES.index("transport")))
                elif op == 3 and nsid != abi.ID_NONE:  # a new client in that Namespace
                    rc = target.client_add(nsid, spare, bytes([6, 6, j >> 8 & 255, j & 255, 0, 1]), None, None,
                                           None, 0x7FF)
                elif op == 4 and cid != abi.ID_NONE:  # client plugins change
                    rc = target.client_set_plugins(cid, 0)
                elif op == 5 and nsid == abi.ID_NONE:  # an unknown tunnel key becomes a Namespace
                    k = F.tunnel_key(int(t["vport"]), int(t["vlan0"]), int(t["vlan1"]))
                    rc = target.ns_add(k, 4096 + (j % 64), 0x7FF)
                else:
                    rc = None
            spare += op == 3
    assert differ > 20, differ           # the mutations did change later classifications
    assert stale_n < n // 2, stale_n     # and the rule flags a minority of the batch


def _image_bytes(max_ns, max_clients):
    return RxPath(-1, max_ns=max_ns, max_clients=max_clients, max_frames=64).table_stats()["table_bytes"]


def _sparse_bytes(max_ns, max_clients, sp):
    """Expected image bytes of an empty handle: slots = next power of two >= spread x entries
    (emurx_mirror.cpp set_partition), times the slot size, plus the dense ns info."""
    def p2(v):
        p = 16
        while p < v:
            p <<= 1
        return p
    ns, mac, ip, ci = sp
    return (p2(ns * max_ns) * 16 + p2(mac * max_clients) * 16 + 2 * p2(ip * max_clients) * 32
            + p2(ci * max_clients) * 32 + p2(16 * 8) * 32 + p2(32 * 8) * 64 + p2(8 * 16) * 16 + max_ns * 16)


def test_sparse_table_sizes(oracle_built):
    """Tables start at their target spread (slots per entry: 8 for ns / MAC, 16 for IPv4 /
    IPv6 / client info), so that almost every key of a 64-lane wave sits in its home bucket."""
    assert _image_bytes(1024, 4096) == _sparse_bytes(1024, 4096, (8, 8, 16, 16))


def test_table_spread_override():
    """EMURX_TABLE_SPREAD="ns,mac,ip,ci" (read once per process) sets the spreads; malformed
    values keep the defaults."""
    code = ("import sys; sys.path.insert(0, 'trex-emu_amd'); from emurx.rx import RxPath; "
            "print(RxPath(-1, max_ns=1024, max_clients=4096, max_frames=64).table_stats()['table_bytes'])")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for env, sp in (("2,2,2,2", (2, 2, 2, 2)), ("4,8,32,2", (4, 8, 32, 2)), ("3,8,16,16", (8, 8, 16, 16)),
                    ("junk", (8, 8, 16, 16))):
        out = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=120,
                             env={**os.environ, "EMURX_TABLE_SPREAD": env})
        assert out.returncode == 0, out.stderr
        assert int(out.stdout.split()[-1]) == _sparse_bytes(1024, 4096, sp), env
