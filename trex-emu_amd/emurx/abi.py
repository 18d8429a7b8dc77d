"""ctypes binding of the C-ABI declared in include/emu_rx.h (libemurx.so).

The shared library is built in-tree by `make -C trex-emu_amd` (or __graft_entry__.build()).
Loading fails loudly when it is missing: there is no CPU fallback for the product path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parent.parent          # trex-emu_amd/
REPO_ROOT = PKG_ROOT.parent
LIB_PATH = PKG_ROOT / "lib" / "libemurx.so"

# ---- constants (emu_rx.h) ---------------------------------------------------------------
EMURX_OK = 0
EMURX_EINVAL, EMURX_ENOMEM, EMURX_EEXIST, EMURX_ENOENT = -22, -12, -17, -2
EMURX_EDEVICE, EMURX_ENOSPC = -5, -28
EMURX_ECOMM = -71      # RCCL error of the library-owned communicator
COMM_ID_BYTES = 128    # EMURX_COMM_ID_BYTES (ncclUniqueId)
XCH_EQUAL, XCH_PAYLOAD, XCH_ROUTE = 0, 1, 2  # emurx_exchange_dev flags
ID_NONE = 0xFFFFFFFF
MAX_FRAME = 9216

CB_NAMES = ["arp", "icmp", "igmp", "dhcp", "dhcpsrv", "dhcpv6", "mdns", "tcp", "udp",
            "icmpv6", "eapol", "ppp"]
(CB_ARP, CB_ICMP, CB_IGMP, CB_DHCP, CB_DHCPSRV, CB_DHCPV6, CB_MDNS, CB_TCP, CB_UDP,
 CB_ICMPV6, CB_EAPOL, CB_PPP) = range(12)
NUM_CB = 12
CB_NONE = 0xFF
Q_DROP = 12
NUM_QUEUES = 13

PLUG_NAMES = ["arp", "icmp", "igmp", "dhcp", "dhcpsrv", "dhcpv6", "mdns", "transport", "ipv6",
              "dot1x", "ppp"]
PLUG_ALL = (1 << len(PLUG_NAMES)) - 1

STATUS_NAMES = [
    "OK", "NOT_SUPPORTED", "PACKET_TOO_SHORT", "EAPOL_TOO_SHORT", "ARP_TOO_SHORT",
    "DOT1Q_TOO_SHORT", "TOO_MANY_DOT1Q", "IPV4_TOO_SHORT", "IPV4_HDR_TOO_SHORT", "IPV4_FRAGMENT",
    "IPV4_CS", "IPV6_TOO_SHORT", "IPV6_HOPLIMIT", "IPV6_EMPTY", "IPV6_JUMBO", "IPV6_FRAGMENT",
    "ICMPV4_TOO_SHORT", "ICMPV4_CS", "TCP_TOO_SHORT", "TCP_CS", "UDP_TOO_SHORT", "UDP_CS",
    "ICMPV6_TOO_SHORT", "ICMPV6_CS", "ICMPV6_UNSUPPORTED", "L4_UNSUPPORTED", "L3_UNSUPPORTED",
    "PANIC_L4LEN", "PANIC_IPV6_OPT", "PANIC_NIL_EAPOL", "PANIC_MBUF"]
ST = {n: i for i, n in enumerate(STATUS_NAMES)}
LOOKUP_NAMES = ["NONE", "NO_NS", "NS_NO_PLUGIN", "NS_LEVEL", "NO_CLIENT", "CLIENT_NO_PLUGIN",
                "CLIENT"]
LK = {n: i for i, n in enumerate(LOOKUP_NAMES)}
FLAG_RTALERT = 0x01

PARSER_COUNTER_NAMES = [
    "errInternalHandler", "errParser", "errEAPolTooShort", "errArpTooShort", "errIcmpv4TooShort",
    "errIgmpv4TooShort", "errUdpTooShort", "errTcpTooShort", "errDot1qTooShort", "errToManyDot1q",
    "errIPv4TooShort", "errIPv4HeaderTooShort", "errIPv4Fragment", "errIPv4cs", "errTCP", "errUDP",
    "eapolPkts", "eapolBytes", "arpPkts", "arpBytes", "icmpPkts", "icmpBytes", "igmpPkts",
    "igmpBytes", "dhcpPkts", "dhcpBytes", "dhcpSrvPkts", "dhcpSrvBytes", "mDnsPkts", "mDnsBytes",
    "tcpPkts", "tcpBytes", "udpPkts", "udpBytes", "udpCsErr", "tcpCsErr", "errIPv6TooShort",
    "errIPv6HopLimitDrop", "errIPv6Empty", "errIPv6OptJumbo", "errIPv6Fragment",
    "errIcmpv6TooShort", "errIcmpv6Cse", "errIcmpv4Cse", "errIcmpv6Unsupported", "Icmpv6Pkt",
    "Icmpv6Bytes", "errL4ProtoUnsupported", "errL3ProtoUnsupported", "errPacketIsTooShort"]
NUM_PARSER_COUNTERS = len(PARSER_COUNTER_NAMES)
HIST_BINS = 64
HIST_SHARDS = 64   # EMURX_HIST_SHARDS: accumulating copies of the device histogram
QUEUE_TILE = 256   # EMURX_QUEUE_TILE: frames per tile / queue segment

# ---- record / descriptor layouts --------------------------------------------------------
REC_DTYPE = np.dtype([
    ("ns_id", "<u4"), ("client_id", "<u4"), ("vlan0", "<u4"), ("vlan1", "<u4"),
    ("vport", "<u2"), ("l3", "<u2"), ("l4", "<u2"), ("l7", "<u2"), ("l7_len", "<u2"),
    ("next_hdr", "u1"), ("proto", "u1"), ("status", "u1"), ("flags", "u1"), ("rsv", "<u2")])
assert REC_DTYPE.itemsize == 32
ROUTE_REC_DTYPE = np.dtype([("rec", REC_DTYPE), ("src_index", "<u4"), ("src_rank", "<u4")])
assert ROUTE_REC_DTYPE.itemsize == 40
# emurx_lookup_rec (owner-partitioned classification): the 32-byte head of a frame's lookup
# record: the source frame index, the packed parse (VLAN codes, vport / l3 / next header, l4 /
# l7, l7_len / proto / status / key kind / tuple bit), the destination MAC, and x (MAC / IPv4
# key, or the index of the record's first 16-byte tail unit); csrc/emurx_parse.h
LOOKUP_REC_DTYPE = np.dtype([("frame", "<u4"), ("vlans", "<u4"), ("w2", "<u4"), ("w3", "<u4"), ("w4", "<u4"),
                             ("dlo", "<u4"), ("dhi", "<u4"), ("x", "<u4")])
assert LOOKUP_REC_DTYPE.itemsize == 32
WALK_NO_KEYS = 1          # EMURX_WALK_NO_KEYS
TAIL_SHARDS = 64          # EMURX_TAIL_SHARDS: tail cursors (and shards) per region
TAIL_NONE = 0xFFFFFFFF    # EMURX_TAIL_NONE: a head whose tail did not fit its shard


def lookup_region_bytes(cap: int, tail_cap: int) -> int:
    """EMURX_LOOKUP_REGION_BYTES: one owner's region of 32-byte heads and tail shards."""
    return cap * 32 + TAIL_SHARDS * tail_cap * 16


def tail_capacity(cap: int, frac: float = 1 / 16) -> int:
    """16-byte tail units per shard for regions of `cap` heads: room for `frac` of them to
    carry a one-unit tail (config D: the 5 % ICMPv6 echo frames), plus slack for the spread of
    the shards.  A shard that overflows reports the units it needed (emurx_parse_route_dev)."""
    return int(cap * frac / TAIL_SHARDS) + 32
ST_HOLE = 0xFF     # EMURX_ST_HOLE: status of the record of an empty descriptor slot
MAX_PARTS = 8
DESC_DTYPE = np.dtype([("off", "<u4"), ("len", "<u2"), ("vport", "u1"), ("pad", "u1")])
assert DESC_DTYPE.itemsize == 8
DESC_HOLE = 0xFF   # EMURX_DESC_HOLE: an empty descriptor slot
DESC_KEYED = 0x80  # EMURX_DESC_KEYED | k: the frame's Namespace-owner key
INGEST_SLOTS = 4   # EMURX_INGEST_SLOTS
SMALL_TILES, SMALL_LDS, SMALL_MSGS = 256, 40960, 1024  # the one-launch ingest's limits (csrc/emurx_kernels.h)
MSG_OK, MSG_PARSE_ERR, MSG_PANIC = 0, 1, 2
MSG_DTYPE = np.dtype([("off", "<u4"), ("len", "<u4")])
TX_IPV4_HDR, TX_V6_NH, TX_L4_SHIFT = 0x01, 0x02, 4
TX_L4_NONE, TX_L4_TCP4, TX_L4_UDP4, TX_L4_TCP6, TX_L4_UDP6, TX_L4_ICMP6, TX_L4_ICMP4 = range(7)
TX_OK, TX_RANGE = 0, 1
ZMQ_TX_BURST, ZMQ_TX_MAX_BUFFER, ZMQ_PKT_MAGIC = 64, 32768, 0xAA  # veth_zmq.go:36-37, :167
FLOW_NONE, FLOW_NO_CTX, FLOW_NO_SYN, FLOW_NO_SERVER, FLOW_NEW = (0xFFFFFFFF, 0xFFFFFFF0, 0xFFFFFFF1,
                                                                0xFFFFFFF2, 0xFFFFFFF3)
FLOW_UNKNOWN = 0xFFFFFFF4  # emurx_lookup_dev: the head came without its c5tuplekey
FLOW_ID_MAX = 0xFFFFFFEF
# emurx_client_spec (ctx_client_add list entry)
CLIENT_SPEC_DTYPE = np.dtype([("ns_id", "<u4"), ("client_id", "<u4"), ("plugin_mask", "<u4"), ("mac", "u1", 6),
                              ("ipv4", "u1", 4), ("ipv6", "u1", 16), ("dhcpv6", "u1", 16), ("pad", "u1", 2)])
assert CLIENT_SPEC_DTYPE.itemsize == 56
TX_DESC_DTYPE = np.dtype([("off", "<u4"), ("len", "<u2"), ("l3", "<u2"), ("l4", "<u2"), ("osize", "<u2"),
                          ("ops", "u1"), ("nh", "u1"), ("pad", "u1", 2)])
assert TX_DESC_DTYPE.itemsize == 16


class Cfg(C.Structure):
    _fields_ = [("device", C.c_int), ("max_ns", C.c_uint32), ("max_clients", C.c_uint32),
                ("max_frames", C.c_uint32), ("max_bytes", C.c_uint32)]


class Counters(C.Structure):
    _fields_ = [("parser", C.c_uint64 * NUM_PARSER_COUNTERS), ("rx_pkts", C.c_uint64),
                ("rx_bytes", C.c_uint64), ("rx_batch", C.c_uint64),
                ("rx_parse_err", C.c_uint64), ("ref_panic", C.c_uint64)]

    def as_dict(self):
        d = {n: int(self.parser[i]) for i, n in enumerate(PARSER_COUNTER_NAMES)}
        for k in ("rx_pkts", "rx_bytes", "rx_batch", "rx_parse_err", "ref_panic"):
            d[k] = int(getattr(self, k))
        return d


class IngestResult(C.Structure):
    _fields_ = [("rec", C.c_void_p), ("desc", C.c_void_p), ("qlist", C.c_void_p),
                ("msg_frames", C.c_void_p), ("msg_status", C.c_void_p), ("n_frames", C.c_uint32),
                ("n_msgs", C.c_uint32), ("qoff", C.c_uint32 * (NUM_QUEUES + 1)), ("delta", Counters),
                ("one_launch", C.c_uint32), ("degraded", C.c_uint32)]


class DevOut(C.Structure):
    _fields_ = [("rec", C.c_void_p), ("qlist", C.c_void_p), ("qcap", C.c_uint32),
                ("tile_cnt", C.c_void_p), ("hist", C.c_void_p), ("flow", C.c_void_p)]


def ntiles(n: int) -> int:
    return (n + QUEUE_TILE - 1) // QUEUE_TILE


def queue_cap(n: int) -> int:
    """Smallest per-queue region (DevOut.qcap) a batch of n frames accepts."""
    return ntiles(n) * QUEUE_TILE


# (name, restype, argtypes) — every symbol include/emu_rx.h declares
_P = C.c_void_p
_U8P = C.c_void_p
SIGNATURES = [
    ("emurx_abi_version", C.c_int, []),
    ("emurx_build_id", C.c_char_p, []),
    ("emurx_open", C.c_int, [C.POINTER(Cfg), C.POINTER(C.c_void_p)]),
    ("emurx_close", None, [_P]),
    ("emurx_strerror", C.c_char_p, [C.c_int]),
    ("emurx_register", C.c_int, [_P, C.c_char_p]),
    ("emurx_set_callbacks_mask", C.c_int, [_P, C.c_uint32]),
    ("emurx_get_callbacks_mask", C.c_uint32, [_P]),
    ("emurx_ns_add", C.c_int, [_P, _U8P, C.c_uint32, C.c_uint32]),
    ("emurx_ns_remove", C.c_int, [_P, _U8P]),
    ("emurx_ns_set_plugins", C.c_int, [_P, C.c_uint32, C.c_uint32]),
    ("emurx_client_add", C.c_int, [_P, C.c_uint32, C.c_uint32, _U8P, _U8P, _U8P, _U8P, C.c_uint32]),
    ("emurx_clients_add", C.c_int, [_P, _P, C.c_uint32, C.POINTER(C.c_uint32)]),
    ("emurx_client_remove", C.c_int, [_P, C.c_uint32, _U8P]),
    ("emurx_client_set_plugins", C.c_int, [_P, C.c_uint32, C.c_uint32]),
    ("emurx_client_update_ipv4", C.c_int, [_P, C.c_uint32, _U8P]),
    ("emurx_client_update_ipv6", C.c_int, [_P, C.c_uint32, _U8P]),
    ("emurx_client_update_dipv6", C.c_int, [_P, C.c_uint32, _U8P]),
    ("emurx_client_set_ra", C.c_int, [_P, C.c_uint32, _U8P, C.c_uint8]),
    ("emurx_sync", C.c_int, [_P, _P]),
    ("emurx_rx_stream", C.c_int, [_P, _U8P, C.c_size_t, _P, _P, C.c_uint32,
                                  C.POINTER(C.c_uint32), _P, C.POINTER(Counters)]),
    ("emurx_classify_dev", C.c_int, [_P, _P, _P, C.c_uint32, C.POINTER(DevOut), _P]),
    ("emurx_parse_dev", C.c_int, [_P, _P, _P, C.c_uint32, C.POINTER(DevOut), _P]),
    ("emurx_zmq_descriptors", C.c_int, [_U8P, C.c_size_t, _P, C.c_uint32,
                                        C.POINTER(C.c_uint32), C.POINTER(C.c_int)]),
    ("emurx_hist_to_counters", None, [_P, C.POINTER(Counters)]),
    ("emurx_hist_fold", None, [_P, _P]),
    ("emurx_set_timing", C.c_int, [_P, C.c_uint32, C.c_uint32]),
    ("emurx_kernel_times", C.c_int, [_P, _P, C.c_uint32, C.POINTER(C.c_uint32)]),
    ("emurx_last_stage", C.c_uint32, [_P]),
    ("emurx_last_txz", C.c_int32, [_P]),
    ("emurx_copy_ceiling_dev", C.c_int, [_P, _P, C.c_size_t, _P]),
    ("emurx_ns_owner", C.c_uint32, [_U8P, C.c_uint32]),
    ("emurx_owner_key", C.c_uint8, [_U8P]),
    ("emurx_desc_keys_dev", C.c_int, [_P, _P, _P, C.c_uint32, _P]),
    ("emurx_route_dev", C.c_int, [_P, _P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P]),
    ("emurx_classify_route_dev", C.c_int, [_P, _P, _P, C.c_uint32, C.POINTER(DevOut), C.c_uint32, C.c_uint32,
                                           C.c_uint32, _P, _P, _P]),
    ("emurx_parse_route_dev", C.c_int, [_P, _P, _P, C.c_uint32, C.POINTER(DevOut), C.c_uint32, C.c_uint32,
                                        C.c_uint32, C.c_uint32, _P, _P, _P]),
    ("emurx_lookup_dev", C.c_int, [_P, _P, _P, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P]),
    ("emurx_zmq_walk_dev", C.c_int, [_P, _P, _P, C.c_uint32, _P, _P, C.c_uint32, _P]),
    ("emurx_set_partition", C.c_int, [_P, C.c_uint32, C.c_uint32]),
    ("emurx_table_gen", C.c_uint64, [_P]),
    ("emurx_recs_stale", C.c_int, [_P, _P, C.c_uint32, C.c_uint64, _P]),
    ("emurx_image_lookup", C.c_int, [_P, C.c_uint32, _P, C.POINTER(C.c_uint32)]),
    ("emurx_image_check", C.c_int, [_P, C.POINTER(C.c_uint64)]),
    ("emurx_table_stats", C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    ("emurx_ingest_buffer", C.c_int, [_P, C.c_uint32, C.c_size_t, C.POINTER(C.c_void_p)]),
    ("emurx_ingest_submit", C.c_int, [_P, C.c_uint32, _P, C.c_uint32]),
    ("emurx_ingest_wait", C.c_int, [_P, C.c_uint32, C.POINTER(IngestResult)]),
    ("emurx_ingest_stream", C.c_int, [_P, C.c_uint32, C.POINTER(C.c_void_p)]),
    ("emurx_tx_checksum_dev", C.c_int, [_P, _P, _P, C.c_uint32, _P, _P]),
    ("emurx_tx_zmq_dev", C.c_int, [_P, _P, _P, C.c_uint32, _P, C.c_uint64, _P, _P, _P]),
    ("emurx_flow_add", C.c_int, [_P, C.c_uint32, _U8P, C.c_uint32, C.c_uint32]),
    ("emurx_flow_remove", C.c_int, [_P, C.c_uint32, _U8P, C.c_uint32]),
    ("emurx_server_add", C.c_int, [_P, C.c_uint32, C.c_uint16, C.c_uint8]),
    ("emurx_server_remove", C.c_int, [_P, C.c_uint32, C.c_uint16, C.c_uint8]),
    ("emurx_client_set_transport", C.c_int, [_P, C.c_uint32, C.c_int]),
    ("emurx_comm_unique_id", C.c_int, [_P]),
    ("emurx_comm_init", C.c_int, [_P, _P, C.c_uint32, C.c_uint32]),
    ("emurx_comm_init_all", C.c_int, [_P, C.c_uint32]),
    ("emurx_comm_destroy", C.c_int, [_P]),
    ("emurx_comm_info", C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    ("emurx_comm_library", C.c_int, [C.c_char_p, C.c_size_t]),
    ("emurx_group_start", C.c_int, []),
    ("emurx_group_end", C.c_int, []),
    ("emurx_exchange_dev", C.c_int, [_P, _P, _P, _P, _P, C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.POINTER(C.c_uint64), _P]),
]

_lib = None


def load(path: str | os.PathLike | None = None):
    """Load libemurx.so (raises OSError when it was not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else Path(os.environ.get("EMURX_LIB", LIB_PATH))
    if not p.exists():
        raise OSError(f"libemurx.so not built at {p}: run `make -C {PKG_ROOT}` "
                      "(there is no CPU fallback for the product path)")
    lib = C.CDLL(str(p), mode=C.RTLD_GLOBAL)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
        # provenance: which source tree the loaded library was built from (GPU test logs)
        built, tree = lib.emurx_build_id().decode(), source_id()
        import sys
        print(f"emurx: {p} built from source tree {built}" +
              ("" if tree in (built, None) else f" -- STALE: this tree is {tree}"), file=sys.stderr)
    return lib


def source_id() -> str | None:
    """The id of the source tree (trex-emu_amd/Makefile SRC_ID: sha1 of the concatenated
    sources, headers and Makefile, first 16 hex digits); None when a file is missing."""
    import hashlib
    src = ["emurx_kernels.hip", "emurx_route.hip", "emurx_ingest.hip", "emurx_tx.hip", "emurx_txzmq.hip",
           "emurx_api.cpp", "emurx_mirror.cpp", "emurx_comm.cpp"]
    hdr = ["emurx_kernels.h", "emurx_tables.h", "emurx_parse.h", "emurx_mirror.h"]
    files = [PKG_ROOT / "csrc" / f for f in src + hdr] + [REPO_ROOT / "include" / "emu_rx.h", PKG_ROOT / "Makefile"]
    h = hashlib.sha1()
    try:
        for f in files:
            h.update(f.read_bytes())
    except OSError:
        return None
    return h.hexdigest()[:16]


def check(rc: int, what: str = ""):
    if rc != EMURX_OK:
        msg = load().emurx_strerror(rc).decode()
        raise RuntimeError(f"{what}: emurx error {rc} ({msg})")
    return rc


def ptr(a) -> int | None:
    """Address of a numpy array / bytes / torch tensor (None passes NULL)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    raise TypeError(f"pass numpy arrays or tensors, not {type(a)}")
