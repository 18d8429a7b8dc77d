"""ctypes binding of the CPU oracle (oracle/liborc.so) — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, and only
as the checker.  Layouts are restated here independently of the product binding
(tests assert both agree byte-for-byte).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = Path(os.environ.get("ORC_LIB", HERE / "liborc.so"))  # ORC_LIB: the sanitized build (tests/test_sanitizers.py)

REC_DTYPE = np.dtype([
    ("ns_id", "<u4"), ("client_id", "<u4"), ("vlan0", "<u4"), ("vlan1", "<u4"),
    ("vport", "<u2"), ("l3", "<u2"), ("l4", "<u2"), ("l7", "<u2"), ("l7_len", "<u2"),
    ("next_hdr", "u1"), ("proto", "u1"), ("status", "u1"), ("flags", "u1"), ("rsv", "<u2")])
DESC_DTYPE = np.dtype([("off", "<u4"), ("len", "<u2"), ("vport", "u1"), ("pad", "u1")])
TX_DESC_DTYPE = np.dtype([("off", "<u4"), ("len", "<u2"), ("l3", "<u2"), ("l4", "<u2"), ("osize", "<u2"),
                          ("ops", "u1"), ("nh", "u1"), ("pad", "u1", 2)])
NPC = 50
NQ = 13


class Counters(C.Structure):
    _fields_ = [("parser", C.c_uint64 * NPC), ("rx_pkts", C.c_uint64), ("rx_bytes", C.c_uint64),
                ("rx_batch", C.c_uint64), ("rx_parse_err", C.c_uint64), ("ref_panic", C.c_uint64)]


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        P = C.c_void_p
        for name, res, args in [
            ("orc_new", P, []), ("orc_free", None, [P]),
            ("orc_set_callbacks_mask", None, [P, C.c_uint32]),
            ("orc_ns_add", C.c_int, [P, P, C.c_uint32, C.c_uint32]),
            ("orc_ns_remove", C.c_int, [P, P]),
            ("orc_ns_set_plugins", C.c_int, [P, C.c_uint32, C.c_uint32]),
            ("orc_client_add", C.c_int, [P, C.c_uint32, C.c_uint32, P, P, P, P, C.c_uint32]),
            ("orc_clients_add", C.c_int, [P, P, C.c_uint32, C.POINTER(C.c_uint32)]),
            ("orc_client_remove", C.c_int, [P, C.c_uint32, P]),
            ("orc_client_set_plugins", C.c_int, [P, C.c_uint32, C.c_uint32]),
            ("orc_client_update_ipv4", C.c_int, [P, C.c_uint32, P]),
            ("orc_client_update_ipv6", C.c_int, [P, C.c_uint32, P]),
            ("orc_client_update_dipv6", C.c_int, [P, C.c_uint32, P]),
            ("orc_client_set_ra", C.c_int, [P, C.c_uint32, P, C.c_uint8]),
            ("orc_checksum", C.c_uint16, [P, C.c_size_t, C.c_uint32]),
            ("orc_parse_frame", None, [P, P, C.c_uint32, C.c_uint16, P]),
            ("orc_parse_only", None, [C.c_uint32, P, C.c_uint32, C.c_uint16, P]),
            ("orc_rx_batch", None, [P, P, P, C.c_uint32, P, P, P, C.POINTER(Counters)]),
            ("orc_rx_stream", C.c_int, [P, P, C.c_size_t, P, P, C.c_uint32,
                                        C.POINTER(C.c_uint32), P, C.POINTER(Counters)]),
            ("orc_zmq_descriptors", C.c_int, [P, C.c_size_t, P, C.c_uint32,
                                              C.POINTER(C.c_uint32), C.POINTER(C.c_int)]),
            ("orc_tx_checksum", None, [P, P, C.c_uint32, P]),
            ("orc_tx_zmq", C.c_uint64, [P, P, C.c_uint32, P, C.c_uint64, P, P]),
            ("orc_flow_add", C.c_int, [P, C.c_uint32, P, C.c_uint32, C.c_uint32]),
            ("orc_flow_remove", C.c_int, [P, C.c_uint32, P, C.c_uint32]),
            ("orc_server_add", C.c_int, [P, C.c_uint32, C.c_uint16, C.c_uint8]),
            ("orc_server_remove", C.c_int, [P, C.c_uint32, C.c_uint16, C.c_uint8]),
            ("orc_client_set_transport", C.c_int, [P, C.c_uint32, C.c_int]),
            ("orc_flows", None, [P, P, P, P, C.c_uint32, P]),
        ]:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _b(x, n=None):
    if x is None:
        return None
    a = np.frombuffer(bytes(x), dtype=np.uint8).copy()
    if n is not None:
        assert a.size == n, (a.size, n)
    return a


class Oracle:
    """Thread/Namespace/Client tables + ParsePacket restatement."""

    def __init__(self, cb_mask: int = (1 << 12) - 1):
        self._h = lib().orc_new()
        self._keep = []
        lib().orc_set_callbacks_mask(self._h, cb_mask)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_free(self._h)
            self._h = None

    def set_callbacks_mask(self, m):
        lib().orc_set_callbacks_mask(self._h, m)

    def ns_add(self, key: bytes, ns_id: int, plugins: int) -> int:
        k = _b(key, 12)
        return lib().orc_ns_add(self._h, k.ctypes.data, ns_id, plugins)

    def ns_remove(self, key: bytes) -> int:
        k = _b(key, 12)
        return lib().orc_ns_remove(self._h, k.ctypes.data)

    def ns_set_plugins(self, ns_id, plugins):
        return lib().orc_ns_set_plugins(self._h, ns_id, plugins)

    def client_add(self, ns_id, cid, mac, ipv4=None, ipv6=None, dhcpv6=None, plugins=0x7FF):
        a = [_b(mac, 6), _b(ipv4, 4), _b(ipv6, 16), _b(dhcpv6, 16)]
        p = [x.ctypes.data if x is not None else None for x in a]
        return lib().orc_client_add(self._h, ns_id, cid, p[0], p[1], p[2], p[3], plugins)

    def clients_add(self, spec):
        """orc_clients_add over emurx_client_spec rows (56 B each) -> (rc, added)."""
        a = np.ascontiguousarray(spec)
        assert a.dtype.itemsize == 56
        k = C.c_uint32()
        rc = lib().orc_clients_add(self._h, a.ctypes.data if len(a) else None, len(a), C.byref(k))
        return rc, k.value

    def client_remove(self, ns_id, mac):
        m = _b(mac, 6)
        return lib().orc_client_remove(self._h, ns_id, m.ctypes.data)

    def client_set_plugins(self, cid, plugins):
        return lib().orc_client_set_plugins(self._h, cid, plugins)

    def client_update_ipv4(self, cid, ip):
        a = _b(ip, 4)
        return lib().orc_client_update_ipv4(self._h, cid, a.ctypes.data)

    def client_update_ipv6(self, cid, ip):
        a = _b(ip, 16)
        return lib().orc_client_update_ipv6(self._h, cid, a.ctypes.data)

    def client_update_dipv6(self, cid, ip):
        a = _b(ip, 16)
        return lib().orc_client_update_dipv6(self._h, cid, a.ctypes.data)

    def client_set_ra(self, cid, prefix, plen):
        a = _b(prefix, 16)
        return lib().orc_client_set_ra(self._h, cid, a.ctypes.data, plen)

    # ---- transport flow tables --------------------------------------------------------
    def flow_add(self, cid, tuple_bytes, flow_id):
        t = _b(tuple_bytes)
        return lib().orc_flow_add(self._h, cid, t.ctypes.data, len(t), flow_id)

    def flow_remove(self, cid, tuple_bytes):
        t = _b(tuple_bytes)
        return lib().orc_flow_remove(self._h, cid, t.ctypes.data, len(t))

    def server_add(self, cid, port, proto):
        return lib().orc_server_add(self._h, cid, port, proto)

    def server_remove(self, cid, port, proto):
        return lib().orc_server_remove(self._h, cid, port, proto)

    def client_set_transport(self, cid, has_ctx):
        return lib().orc_client_set_transport(self._h, cid, int(has_ctx))

    def flows(self, buf, desc, rec):
        """TransportCtx.handleRxPacket's decision per classified frame (EMURX_FLOW_* / id)."""
        n = len(desc)
        out = np.zeros(max(n, 1), np.uint32)
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        d = np.ascontiguousarray(desc).view(DESC_DTYPE)
        r = np.ascontiguousarray(rec).view(REC_DTYPE)
        lib().orc_flows(self._h, buf.ctypes.data, d.ctypes.data, r.ctypes.data, n, out.ctypes.data)
        return out[:n]

    # ---- data path ------------------------------------------------------------------
    def parse_frame(self, frame: bytes, vport: int = 0):
        f = _b(frame) if len(frame) else np.zeros(1, np.uint8)
        r = np.zeros(1, dtype=REC_DTYPE)
        lib().orc_parse_frame(self._h, f.ctypes.data, len(frame), vport, r.ctypes.data)
        return r[0]

    def rx_batch(self, buf: np.ndarray, desc: np.ndarray):
        n = len(desc)
        rec = np.zeros(n, dtype=REC_DTYPE)
        qlist = np.zeros(max(n, 1), dtype=np.uint32)
        qoff = np.zeros(NQ + 1, dtype=np.uint32)
        cnt = Counters()
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        desc = np.ascontiguousarray(desc).view(DESC_DTYPE)
        lib().orc_rx_batch(self._h, buf.ctypes.data, desc.ctypes.data, n, rec.ctypes.data,
                           qlist.ctypes.data, qoff.ctypes.data, C.byref(cnt))
        return rec, qlist[:n], qoff, cnt

    def rx_stream(self, msg: bytes, cap: int = 1 << 16):
        m = _b(msg) if len(msg) else np.zeros(1, np.uint8)
        rec = np.zeros(cap, dtype=REC_DTYPE)
        qlist = np.zeros(cap, dtype=np.uint32)
        qoff = np.zeros(NQ + 1, dtype=np.uint32)
        cnt = Counters()
        n = C.c_uint32()
        rc = lib().orc_rx_stream(self._h, m.ctypes.data, len(msg), rec.ctypes.data,
                                 qlist.ctypes.data, cap, C.byref(n), qoff.ctypes.data,
                                 C.byref(cnt))
        assert rc == 0, rc
        return rec[:n.value], qlist[:n.value], qoff, cnt


def checksum(data: bytes, init: int = 0) -> int:
    a = _b(data) if len(data) else np.zeros(1, np.uint8)
    return int(lib().orc_checksum(a.ctypes.data, len(data), init))


def parse_only(frame: bytes, vport=0, cb_mask=(1 << 12) - 1):
    f = _b(frame) if len(frame) else np.zeros(1, np.uint8)
    r = np.zeros(1, dtype=REC_DTYPE)
    lib().orc_parse_only(cb_mask, f.ctypes.data, len(frame), vport, r.ctypes.data)
    return r[0]


def zmq_descriptors(msg: bytes, cap=1 << 16):
    m = _b(msg) if len(msg) else np.zeros(1, np.uint8)
    d = np.zeros(cap, dtype=DESC_DTYPE)
    n = C.c_uint32()
    e = C.c_int()
    rc = lib().orc_zmq_descriptors(m.ctypes.data, len(msg), d.ctypes.data, cap, C.byref(n),
                                   C.byref(e))
    return rc, d[:n.value], e.value


def tx_checksum(buf: np.ndarray, desc: np.ndarray):
    """orc_tx_checksum on a copy of buf -> (new buffer, status[n])."""
    out = np.ascontiguousarray(buf, dtype=np.uint8).copy()
    d = np.ascontiguousarray(desc).view(TX_DESC_DTYPE)
    st = np.zeros(max(len(d), 1), np.uint8)
    lib().orc_tx_checksum(out.ctypes.data, d.ctypes.data, len(d), st.ctypes.data)
    return out, st[: len(d)]


def tx_zmq(buf: np.ndarray, desc: np.ndarray, cap=None):
    """orc_tx_zmq: VethIFZmq.Send per frame + FlushTx -> (bytes, msg_off[n_msgs + 1])."""
    d = np.ascontiguousarray(desc)
    n = len(d)
    need = 8 * n + int(d["len"].astype(np.int64).sum())
    cap = need if cap is None else cap
    out = np.zeros(max(cap, 1), np.uint8)
    off = np.zeros(n + 1, np.uint64)
    nm = C.c_uint64()
    b = np.ascontiguousarray(buf, dtype=np.uint8)
    total = lib().orc_tx_zmq(b.ctypes.data, d.ctypes.data, n, out.ctypes.data, cap, off.ctypes.data,
                             C.byref(nm))
    return out[:min(total, cap)], off[: nm.value + 1], int(total)


def counters_dict(cnt: Counters):
    from_names = [
        "errInternalHandler", "errParser", "errEAPolTooShort", "errArpTooShort",
        "errIcmpv4TooShort", "errIgmpv4TooShort", "errUdpTooShort", "errTcpTooShort",
        "errDot1qTooShort", "errToManyDot1q", "errIPv4TooShort", "errIPv4HeaderTooShort",
        "errIPv4Fragment", "errIPv4cs", "errTCP", "errUDP", "eapolPkts", "eapolBytes", "arpPkts",
        "arpBytes", "icmpPkts", "icmpBytes", "igmpPkts", "igmpBytes", "dhcpPkts", "dhcpBytes",
        "dhcpSrvPkts", "dhcpSrvBytes", "mDnsPkts", "mDnsBytes", "tcpPkts", "tcpBytes", "udpPkts",
        "udpBytes", "udpCsErr", "tcpCsErr", "errIPv6TooShort", "errIPv6HopLimitDrop",
        "errIPv6Empty", "errIPv6OptJumbo", "errIPv6Fragment", "errIcmpv6TooShort",
        "errIcmpv6Cse", "errIcmpv4Cse", "errIcmpv6Unsupported", "Icmpv6Pkt", "Icmpv6Bytes",
        "errL4ProtoUnsupported", "errL3ProtoUnsupported", "errPacketIsTooShort"]
    d = {n: int(cnt.parser[i]) for i, n in enumerate(from_names)}
    for k in ("rx_pkts", "rx_bytes", "rx_batch", "rx_parse_err", "ref_panic"):
        d[k] = int(getattr(cnt, k))
    return d
