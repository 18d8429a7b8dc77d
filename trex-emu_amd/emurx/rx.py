"""RxPath — Python surface of the C-ABI, shaped like the reference's rx entry points.

    RxPath.register(name)         Parser.Register          src/emu/core/parser.go:528-565
    RxPath.ns_add / ns_remove     CThreadCtx.AddNs/RemoveNs src/emu/core/thread_ctx.go:786-812
    RxPath.client_add / remove    CNSCtx.AddClient/RemoveClient src/emu/core/ns_ctx.go:332-440
    RxPath.on_rx_stream(msg)      VethIFZmq.OnRxStream     src/emu/core/veth_zmq.go:277-320
    RxPath.classify_dev(...)      the same, device-resident (frames already in HBM)

Device memory is plain torch CUDA tensors (plumbing only); every call goes through
libemurx.so — there is no Python or CPU implementation of the data path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi


def _u8(x, n):
    if x is None:
        return None
    a = np.frombuffer(bytes(x), dtype=np.uint8).copy()
    if a.size != n:
        raise ValueError(f"expected {n} bytes, got {a.size}")
    return a


def _p(a):
    return None if a is None else a.ctypes.data


class RxPath:
    """device < 0: a host-only handle (table mirror, generations, image queries; no GPU)."""

    def __init__(self, device: int = 0, max_ns: int = 4096, max_clients: int = 65536,
                 max_frames: int = 1 << 20, max_bytes: int = 1 << 20):
        self.lib = abi.load()
        cfg = abi.Cfg(device, max_ns, max_clients, max_frames, max_bytes)
        h = C.c_void_p()
        abi.check(self.lib.emurx_open(C.byref(cfg), C.byref(h)), "emurx_open")
        self.h = h
        self.cfg = cfg

    def close(self):
        if getattr(self, "h", None):
            self.lib.emurx_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    # ---- registration ----------------------------------------------------------------
    def register(self, protocol: str):
        return abi.check(self.lib.emurx_register(self.h, protocol.encode()), "register")

    def register_all(self):
        for p in ("arp", "icmp", "igmp", "dhcp", "dhcpsrv", "icmpv6", "dhcpv6", "dot1x", "mdns",
                  "ppp", "transport"):
            self.register(p)

    def set_callbacks_mask(self, mask: int):
        return abi.check(self.lib.emurx_set_callbacks_mask(self.h, mask), "set_callbacks_mask")

    @property
    def callbacks_mask(self) -> int:
        return int(self.lib.emurx_get_callbacks_mask(self.h))

    # ---- tables (return codes are passed through: they mirror Go's error returns) ------
    def ns_add(self, key: bytes, ns_id: int, plugins: int = abi.PLUG_ALL) -> int:
        k = _u8(key, 12)
        return self.lib.emurx_ns_add(self.h, _p(k), ns_id, plugins)

    def ns_remove(self, key: bytes) -> int:
        k = _u8(key, 12)
        return self.lib.emurx_ns_remove(self.h, _p(k))

    def ns_set_plugins(self, ns_id: int, plugins: int) -> int:
        return self.lib.emurx_ns_set_plugins(self.h, ns_id, plugins)

    def client_add(self, ns_id, cid, mac, ipv4=None, ipv6=None, dhcpv6=None,
                   plugins: int = abi.PLUG_ALL) -> int:
        a = [_u8(mac, 6), _u8(ipv4, 4), _u8(ipv6, 16), _u8(dhcpv6, 16)]
        return self.lib.emurx_client_add(self.h, ns_id, cid, *[_p(x) for x in a], plugins)

    def clients_add(self, spec: np.ndarray) -> tuple[int, int]:
        """ctx_client_add: CLIENT_SPEC_DTYPE rows in order -> (rc of the first failure or 0,
        clients added)."""
        a = np.ascontiguousarray(spec, dtype=abi.CLIENT_SPEC_DTYPE)
        k = C.c_uint32()
        rc = self.lib.emurx_clients_add(self.h, _p(a) if len(a) else None, len(a), C.byref(k))
        return rc, k.value

    def client_remove(self, ns_id, mac) -> int:
        m = _u8(mac, 6)
        return self.lib.emurx_client_remove(self.h, ns_id, _p(m))

    def client_set_plugins(self, cid, plugins) -> int:
        return self.lib.emurx_client_set_plugins(self.h, cid, plugins)

    def client_update_ipv4(self, cid, ip) -> int:
        a = _u8(ip, 4)
        return self.lib.emurx_client_update_ipv4(self.h, cid, _p(a))

    def client_update_ipv6(self, cid, ip) -> int:
        a = _u8(ip, 16)
        return self.lib.emurx_client_update_ipv6(self.h, cid, _p(a))

    def client_update_dipv6(self, cid, ip) -> int:
        a = _u8(ip, 16)
        return self.lib.emurx_client_update_dipv6(self.h, cid, _p(a))

    def client_set_ra(self, cid, prefix, plen) -> int:
        a = _u8(prefix, 16)
        return self.lib.emurx_client_set_ra(self.h, cid, _p(a), plen)

    # transport flow tables (TransportCtx.addFlowv4/6, serverCb; include/emu_rx.h)
    def flow_add(self, cid, tuple_bytes, flow_id) -> int:
        t = np.frombuffer(bytes(tuple_bytes), np.uint8).copy()
        rc = self.lib.emurx_flow_add(self.h, cid, _p(t), len(t), flow_id)
        self._transport = self.any_transport or rc == 0
        return rc

    def flow_remove(self, cid, tuple_bytes) -> int:
        t = np.frombuffer(bytes(tuple_bytes), np.uint8).copy()
        return self.lib.emurx_flow_remove(self.h, cid, _p(t), len(t))

    def server_add(self, cid, port, proto) -> int:
        rc = self.lib.emurx_server_add(self.h, cid, port, proto)
        self._transport = self.any_transport or rc == 0
        return rc

    def server_remove(self, cid, port, proto) -> int:
        return self.lib.emurx_server_remove(self.h, cid, port, proto)

    def client_set_transport(self, cid, has_ctx) -> int:
        rc = self.lib.emurx_client_set_transport(self.h, cid, int(has_ctx))
        self._transport = self.any_transport or (rc == 0 and bool(has_ctx))
        return rc

    def sync(self, stream=None):
        return abi.check(self.lib.emurx_sync(self.h, stream), "sync")

    # ---- host batch (ZMQ message) ------------------------------------------------------
    def on_rx_stream(self, msg: bytes, cap: int | None = None):
        cap = cap or int(self.cfg.max_frames)
        m = np.frombuffer(bytes(msg), dtype=np.uint8).copy() if len(msg) else np.zeros(1, np.uint8)
        rec = np.zeros(cap, dtype=abi.REC_DTYPE)
        qlist = np.zeros(cap, dtype=np.uint32)
        qoff = np.zeros(abi.NUM_QUEUES + 1, dtype=np.uint32)
        cnt = abi.Counters()
        n = C.c_uint32()
        abi.check(self.lib.emurx_rx_stream(self.h, _p(m), len(msg), _p(rec), _p(qlist), cap,
                                           C.byref(n), _p(qoff), C.byref(cnt)), "rx_stream")
        k = n.value
        return rec[:k], qlist[:k], qoff, cnt

    # ---- device-resident batch -----------------------------------------------------------
    def classify_dev(self, frames, desc, n: int, rec=None, qlist=None, qcap: int = 0, tile_cnt=None,
                     hist=None, stream=None, classify: bool = True, flow=None):
        """frames/desc/rec/qlist/tile_cnt/hist: device tensors (or raw device addresses).
        Tile t's frames of queue q land in qlist[q*qcap + t*QUEUE_TILE :][:tile_cnt[t*16+q]]
        (see pack_queues); hist holds HIST_SHARDS accumulating copies (see hist_fold)."""
        out = abi.DevOut(_addr(rec), _addr(qlist), qcap, _addr(tile_cnt), _addr(hist), _addr(flow))
        fn = self.lib.emurx_classify_dev if classify else self.lib.emurx_parse_dev
        return abi.check(fn(self.h, _addr(frames), _addr(desc), n, C.byref(out),
                            _stream(stream)), "classify_dev")

    def classify_call(self, frames, desc, n: int, rec=None, qlist=None, qcap: int = 0, tile_cnt=None,
                      hist=None, stream=None, classify: bool = True, flow=None):
        """classify_dev with every argument resolved once: returns a zero-argument callable
        that enqueues the same batch again (one C call, no Python-side argument work)."""
        out = abi.DevOut(_addr(rec), _addr(qlist), qcap, _addr(tile_cnt), _addr(hist), _addr(flow))
        fn = self.lib.emurx_classify_dev if classify else self.lib.emurx_parse_dev
        args = (self.h, _addr(frames), _addr(desc), n, C.byref(out), _stream(stream))

        def call():
            rc = fn(*args)
            if rc:
                abi.check(rc, "classify_dev")
        call.keep = out
        return call

    def set_timing(self, slots: int = 1024, stride: int = 1):
        """Time every `stride`-th batch with HIP events (0 slots disables)."""
        return abi.check(self.lib.emurx_set_timing(self.h, slots, stride), "set_timing")

    def kernel_times(self, cap: int = 1 << 16):
        """Device ms of every batch launched since the previous call (HIP events recorded on
        the launch stream around the k_rx launch)."""
        a = np.zeros(cap, np.float32)
        n = C.c_uint32()
        abi.check(self.lib.emurx_kernel_times(self.h, _p(a), cap, C.byref(n)), "kernel_times")
        return a[: n.value]

    def last_stage(self) -> int:
        """LDS staging bytes per wave of the most recent k_rx launch (7168 or 6144)."""
        return int(self.lib.emurx_last_stage(self.h))

    def last_txz(self) -> int:
        """LDS image bytes per wave of the last tx framing write (6144, 4608, 0; -1 before)."""
        return int(self.lib.emurx_last_txz(self.h))

    # ---- batched host ingest (many ZMQ messages per GPU round trip) -------------------------
    def ingest_buffer(self, slot: int, nbytes: int) -> np.ndarray:
        """The slot's pinned staging buffer as a writable uint8 view of `nbytes`."""
        p = C.c_void_p()
        abi.check(self.lib.emurx_ingest_buffer(self.h, slot, nbytes, C.byref(p)), "ingest_buffer")
        return np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(max(nbytes, 1),))[:nbytes]

    def ingest_submit(self, slot: int, msgs) -> None:
        """msgs: MSG_DTYPE array (or [(off, len), ...]) of messages in the slot buffer."""
        a = np.asarray(msgs)
        a = np.ascontiguousarray(a).view(np.uint32) if a.dtype.names else np.asarray(msgs, dtype=np.uint32)
        m = np.ascontiguousarray(a).reshape(-1, 2)
        abi.check(self.lib.emurx_ingest_submit(self.h, slot, _p(m) if len(m) else None, len(m)),
                  "ingest_submit")

    def ingest_stream(self, slot: int) -> int:
        """The slot's hipStream_t as an integer (for torch.cuda.ExternalStream)."""
        p = C.c_void_p()
        abi.check(self.lib.emurx_ingest_stream(self.h, slot, C.byref(p)), "ingest_stream")
        return int(p.value)

    def ingest_wait(self, slot: int, copy: bool = True) -> dict:
        """Results of the slot's batch: rec, desc, qlist, qoff, msg_frames, msg_status,
        counters (views into library memory unless copy)."""
        r = abi.IngestResult()
        abi.check(self.lib.emurx_ingest_wait(self.h, slot, C.byref(r)), "ingest_wait")
        n, m = int(r.n_frames), int(r.n_msgs)

        def view(ptr, count, dt):
            if not count:
                return np.zeros(0, dt)
            b = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(count * np.dtype(dt).itemsize,))
            v = b.view(dt)
            return v.copy() if copy else v
        return dict(rec=view(r.rec, n, abi.REC_DTYPE), desc=view(r.desc, n, abi.DESC_DTYPE),
                    qlist=view(r.qlist, n, np.uint32), qoff=np.array(r.qoff, np.uint32),
                    msg_frames=view(r.msg_frames, m, np.uint32), msg_status=view(r.msg_status, m, np.uint8),
                    counters=r.delta.as_dict(), n=n, one_launch=bool(r.one_launch), degraded=bool(r.degraded))

    # ---- tx-side checksum generation ------------------------------------------------------
    def tx_checksum_dev(self, frames, desc, n: int, status=None, stream=None):
        """Rewrite the checksums selected by each TX_DESC_DTYPE descriptor, in place on the
        device buffer `frames` (include/emu_rx.h emurx_tx_checksum_dev)."""
        return abi.check(self.lib.emurx_tx_checksum_dev(self.h, _addr(frames), _addr(desc), n, _addr(status),
                                                        _stream(stream)), "tx_checksum_dev")

    def tx_zmq_dev(self, frames, desc, n: int, out, cap: int, msg_off, info, stream=None):
        """Pack the n frames into ZMQ messages as VethIFZmq.Send x n + FlushTx would
        (include/emu_rx.h emurx_tx_zmq_dev): messages back to back in `out`, msg_off u64
        [n + 1], info u64 {n_msgs, total bytes}."""
        return abi.check(self.lib.emurx_tx_zmq_dev(self.h, _addr(frames), _addr(desc), n, _addr(out), cap,
                                                   _addr(msg_off), _addr(info), _stream(stream)), "tx_zmq_dev")

    # ---- Namespace-partitioned exchange ---------------------------------------------------
    def classify_route_dev(self, frames, desc, n: int, rec, qlist, qcap: int, tile_cnt, hist, n_parts: int,
                           my_rank: int, cap: int, send, send_count, stream=None, flow=None):
        """classify_dev + route_dev in one call, the route's counting pass inside k_rx
        (include/emu_rx.h emurx_classify_route_dev)."""
        out = abi.DevOut(_addr(rec), _addr(qlist), qcap, _addr(tile_cnt), _addr(hist), _addr(flow))
        return abi.check(self.lib.emurx_classify_route_dev(self.h, _addr(frames), _addr(desc), n, C.byref(out),
                                                           n_parts, my_rank, cap, _addr(send), _addr(send_count),
                                                           _stream(stream)), "classify_route_dev")

    def route_dev(self, rec, n: int, n_parts: int, my_rank: int, cap: int, send, send_count, stream=None):
        """Pack the batch's records with a Namespace into their owners' send regions
        (send[d*cap:][:send_count[d]], frame order; include/emu_rx.h emurx_route_dev)."""
        return abi.check(self.lib.emurx_route_dev(self.h, _addr(rec), n, n_parts, my_rank, cap, _addr(send),
                                                  _addr(send_count), _stream(stream)), "route_dev")

    # ---- owner-partitioned classification ----------------------------------------------------
    def set_partition(self, n_parts: int, part: int):
        """Device tables hold only the Namespaces this partition owns (emurx_set_partition)."""
        return abi.check(self.lib.emurx_set_partition(self.h, n_parts, part), "set_partition")

    def parse_route_dev(self, frames, desc, n: int, rec, qlist, qcap: int, tile_cnt, hist, n_parts: int,
                        my_rank: int, cap: int, send, send_count, stream=None, tail_cap=None):
        """Parse + lookup keys, packed into the owners' regions (abi.lookup_region_bytes(cap,
        tail_cap) bytes each: LOOKUP_REC_DTYPE heads + tail shards); send_count [2 * n_parts]
        {heads, tail overflow}.  tail_cap defaults to default_tail_cap(cap)."""
        if tail_cap is None:
            tail_cap = self.default_tail_cap(cap)
        out = abi.DevOut(_addr(rec), _addr(qlist), qcap, _addr(tile_cnt), _addr(hist), None)
        return abi.check(self.lib.emurx_parse_route_dev(self.h, _addr(frames), _addr(desc), n, C.byref(out),
                                                        n_parts, my_rank, cap, tail_cap, _addr(send),
                                                        _addr(send_count), _stream(stream)), "parse_route_dev")

    def default_tail_cap(self, cap: int) -> int:
        """Tail units per shard when the caller gives none: room for a sixteenth of
        the heads to carry one unit (ICMPv6 keys), or, once any client has a TransportCtx (tcp /
        udp heads then carry their c5tuplekey: 1 unit over IPv4, 3 over IPv6), for every head to
        carry three.  A shard that still overflows is reported in send_count[2 d + 1]."""
        return abi.tail_capacity(cap, 3.0 if self.any_transport else 1 / 16)

    @property
    def any_transport(self) -> bool:
        """Some client has a TransportCtx on this handle (flows, listeners or the mark): what
        makes the source attach tuples (emurx_parse_route_dev)."""
        return bool(getattr(self, "_transport", False))

    def desc_keys_dev(self, frames, desc, n: int, stream=None):
        """Write every frame's owner key into its descriptor's pad byte, in place
        (include/emu_rx.h emurx_desc_keys_dev): what the device framing walk does."""
        return abi.check(self.lib.emurx_desc_keys_dev(self.h, _addr(frames), _addr(desc), n, _stream(stream)),
                         "desc_keys_dev")

    def zmq_walk_dev(self, buf, ctl, nmsg: int, desc, msg_stat, keys: bool = True, stream=None):
        """The framing walk alone on device-resident messages (include/emu_rx.h
        emurx_zmq_walk_dev): ctl = emurx_msg[nmsg] then slot_base[nmsg + 1] (uint32)."""
        return abi.check(self.lib.emurx_zmq_walk_dev(self.h, _addr(buf), _addr(ctl), nmsg, _addr(desc),
                                                     _addr(msg_stat), 0 if keys else abi.WALK_NO_KEYS,
                                                     _stream(stream)), "zmq_walk_dev")

    def lookup_dev(self, recv, recv_count, n_parts: int, cap: int, out, flow=None, stream=None, tail_cap=None):
        """The owner's lookups over received lookup regions (parse_route_dev's layout; recv_count
        [2 * n_parts]) -> ROUTE_REC_DTYPE slots."""
        if tail_cap is None:
            tail_cap = self.default_tail_cap(cap)
        return abi.check(self.lib.emurx_lookup_dev(self.h, _addr(recv), _addr(recv_count), n_parts, cap, tail_cap,
                                                   _addr(out), _addr(flow), _stream(stream)), "lookup_dev")

    # ---- the library-owned communicator (include/emu_rx.h emurx_comm_*, emurx_exchange_dev) ----
    def comm_init(self, uid: bytes, nranks: int, rank: int):
        """Join the exchange's communicator (ncclCommInitRank; blocks until every rank joined).
        uid: comm_unique_id() of one rank, handed to every rank out of band."""
        u = _u8(uid, abi.COMM_ID_BYTES)
        _torch_first()
        return abi.check(self.lib.emurx_comm_init(self.h, _p(u), nranks, rank), "comm_init")

    def comm_destroy(self):
        return abi.check(self.lib.emurx_comm_destroy(self.h), "comm_destroy")

    def comm_info(self):
        """(nranks, rank) of the handle's communicator, or None."""
        a, b = C.c_uint32(), C.c_uint32()
        rc = self.lib.emurx_comm_info(self.h, C.byref(a), C.byref(b))
        if rc == abi.EMURX_ENOENT:
            return None
        abi.check(rc, "comm_info")
        return a.value, b.value

    def exchange_dev(self, send, send_count, recv, recv_count, cap: int, tail_cap=None, payload: bool = False,
                     route: bool = False, stream=None) -> int:
        """One exchange of the owners' regions over the handle's communicator (RCCL): region r
        of every rank's send into region s of rank r's recv, counts alongside.  Lookup regions
        (parse_route_dev) unless route (classify_route_dev's route records).  Returns the bytes
        sent to other ranks."""
        tail_cap = (self.default_tail_cap(cap) if tail_cap is None else tail_cap) if not route else 0
        moved = C.c_uint64()
        flags = (abi.XCH_PAYLOAD if payload else abi.XCH_EQUAL) | (abi.XCH_ROUTE if route else 0)
        abi.check(self.lib.emurx_exchange_dev(self.h, _addr(send), _addr(send_count), _addr(recv), _addr(recv_count),
                                              cap, tail_cap, flags, C.byref(moved), _stream(stream)), "exchange_dev")
        return moved.value

    # ---- table generations / image diagnostics -------------------------------------------------
    def table_gen(self) -> int:
        return int(self.lib.emurx_table_gen(self.h))

    def recs_stale(self, rec: np.ndarray, gen: int) -> np.ndarray:
        """emurx_recs_stale: 1 where a record may differ from the live tables' answer."""
        r = np.ascontiguousarray(rec, dtype=abi.REC_DTYPE)
        out = np.zeros(max(len(r), 1), np.uint8)
        abi.check(self.lib.emurx_recs_stale(self.h, _p(r) if len(r) else None, len(r), gen, _p(out)),
                  "recs_stale")
        return out[: len(r)]

    def image_lookup(self, table: int, key) -> int | None:
        k = np.ascontiguousarray(key, dtype=np.uint32)
        v = C.c_uint32()
        rc = self.lib.emurx_image_lookup(self.h, table, _p(k), C.byref(v))
        if rc == abi.EMURX_ENOENT:
            return None
        abi.check(rc, "image_lookup")
        return v.value

    def image_check(self) -> int:
        """32-bit words where the device tables differ from the host image (0 = in sync)."""
        v = C.c_uint64()
        abi.check(self.lib.emurx_image_check(self.h, C.byref(v)), "image_check")
        return v.value

    def table_stats(self) -> dict:
        """Blocks shipped as deltas, whole tables uploaded, bytes of the device tables."""
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        abi.check(self.lib.emurx_table_stats(self.h, C.byref(a), C.byref(b), C.byref(c)), "table_stats")
        return dict(delta_blocks=a.value, whole_tables=b.value, table_bytes=c.value)


def comm_library():
    """Path of the RCCL the library's communicators use (emurx_comm_library: bound at the first
    call), or None when none loads."""
    _torch_first()
    b = C.create_string_buffer(1024)
    rc = abi.load().emurx_comm_library(b, 1024)
    return b.value.decode() if rc == abi.EMURX_OK else None


def _torch_first():
    """Before the library binds RCCL (its first communicator call): torch, when installed, is
    imported first, so that the process has one ROCm runtime and one RCCL (torch's bundled
    ones).  The system's RCCL bound ahead of a later torch import mixes two copies of ROCm's
    libraries, and such a process aborts at exit."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def comm_unique_id() -> bytes:
    """A fresh communicator id (emurx_comm_unique_id, ncclGetUniqueId): one rank makes it, every
    rank passes it to RxPath.comm_init."""
    _torch_first()
    b = np.zeros(abi.COMM_ID_BYTES, np.uint8)
    abi.check(abi.load().emurx_comm_unique_id(_p(b)), "comm_unique_id")
    return b.tobytes()


def comm_init_all(paths) -> None:
    """One communicator over several handles of this process, one GPU each (emurx_comm_init_all):
    handle k is rank k."""
    _torch_first()
    hs = (C.c_void_p * len(paths))(*[p.h.value for p in paths])
    abi.check(abi.load().emurx_comm_init_all(hs, len(paths)), "comm_init_all")


def group_start():
    _torch_first()
    abi.check(abi.load().emurx_group_start(), "group_start")


def group_end():
    abi.check(abi.load().emurx_group_end(), "group_end")


def owner_key(key: bytes) -> int:
    """The descriptor owner key of a 12-byte CTunnelKey (EMURX_DESC_KEYED | 7-bit digest)."""
    return int(abi.load().emurx_owner_key(_p(_u8(key, 12))))


def ns_owner(key: bytes, n_parts: int) -> int:
    """Partition (GPU) owning the Namespace with this 12-byte CTunnelKey."""
    k = np.frombuffer(bytes(key), np.uint8).copy()
    assert k.size == 12
    return int(abi.load().emurx_ns_owner(_p(k), n_parts))


def _addr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    return x.data_ptr()


def _stream(s):
    if s is None:
        return None
    if isinstance(s, int):
        return s
    return s.cuda_stream


def zmq_descriptors(msg: bytes, cap: int = 1 << 16):
    lib = abi.load()
    m = np.frombuffer(bytes(msg), dtype=np.uint8).copy() if len(msg) else np.zeros(1, np.uint8)
    d = np.zeros(cap, dtype=abi.DESC_DTYPE)
    n, e = C.c_uint32(), C.c_int()
    rc = lib.emurx_zmq_descriptors(_p(m), len(msg), _p(d), cap, C.byref(n), C.byref(e))
    return rc, d[:n.value], e.value


def hist_fold(shards: np.ndarray) -> np.ndarray:
    """[HIST_SHARDS * 2 * HIST_BINS] device histogram copies -> [2 * HIST_BINS] (C-ABI)."""
    lib = abi.load()
    s = np.ascontiguousarray(shards, dtype=np.uint64).reshape(-1)
    assert s.size == abi.HIST_SHARDS * 2 * abi.HIST_BINS
    out = np.zeros(2 * abi.HIST_BINS, np.uint64)
    lib.emurx_hist_fold(_p(s), _p(out))
    return out


def pack_queues(qlist: np.ndarray, qcap: int, tile_cnt: np.ndarray, n: int):
    """Per-tile queue segments -> (frame indices in queue order, qoff[NUM_QUEUES + 1]):
    queue q = qlist_packed[qoff[q]:qoff[q+1]], frames in order (the host side of
    emurx_rx_stream's packing)."""
    nt = abi.ntiles(n)
    ql = np.asarray(qlist).view(np.uint32).reshape(abi.NUM_QUEUES, -1)[:, : nt * abi.QUEUE_TILE]
    cnt = np.asarray(tile_cnt).view(np.uint32).reshape(-1, 16)[:nt, : abi.NUM_QUEUES].astype(np.int64)
    assert (cnt <= abi.QUEUE_TILE).all()
    seg = ql.reshape(abi.NUM_QUEUES, nt, abi.QUEUE_TILE)
    keep = np.arange(abi.QUEUE_TILE)[None, None, :] < cnt.T[:, :, None]
    packed = seg[keep].astype(np.uint32)  # C order: queue, tile, slot
    qoff = np.zeros(abi.NUM_QUEUES + 1, np.uint32)
    qoff[1:] = np.cumsum(cnt.sum(0))
    return packed, qoff


def hist_to_counters(hist: np.ndarray) -> dict:
    lib = abi.load()
    h = np.ascontiguousarray(hist, dtype=np.uint64)
    cnt = abi.Counters()
    lib.emurx_hist_to_counters(_p(h), C.byref(cnt))
    return cnt.as_dict()
