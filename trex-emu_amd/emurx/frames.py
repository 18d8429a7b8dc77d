"""Scalar frame builders with gopacket's serialization semantics.

Used to rebuild the reference's own test frames byte-for-byte
(src/emu/core/parser_test.go builds them with gopacket.SerializeLayers) and to build
edge-case frames for the parity tests.  Layouts follow the vendored gopacket:
  Ethernet  layers/ethernet.go:117-154  (dst, src, type; pads the frame to 60 bytes)
  Dot1Q     layers/dot1q.go:56-71       (PCP<<13 | DEI<<12 | VID, type)
  IPv4      layers/ip4.go:212-265       (FixLengths -> IHL, Length; ComputeChecksums)
  UDP       layers/udp.go:79-114
  ICMPv4    layers/icmp4.go:316-331
  ARP       layers/arp.go:107-140
  DHCPv4    layers/dhcpv4.go:175-243
  PPPoE     layers/pppoe.go:102-135
"""
from __future__ import annotations

import ipaddress
import struct

ETH_IPV4 = 0x0800
ETH_ARP = 0x0806
ETH_IPV6 = 0x86DD
ETH_DOT1Q = 0x8100
ETH_QINQ = 0x88A8
ETH_PPPOE_DISC = 0x8863
ETH_PPPOE_SESS = 0x8864
ETH_EAPOL = 0x888E


def mac(s) -> bytes:
    if isinstance(s, (bytes, bytearray)):
        return bytes(s)
    if isinstance(s, (list, tuple)):
        return bytes(s)
    return bytes(int(x, 16) for x in s.split(":"))


def ip4(s) -> bytes:
    if isinstance(s, (bytes, bytearray)):
        return bytes(s)
    if isinstance(s, int):
        return struct.pack(">I", s)
    return ipaddress.IPv4Address(s).packed


def ip6(s) -> bytes:
    if isinstance(s, (bytes, bytearray)):
        return bytes(s)
    return ipaddress.IPv6Address(s).packed


def csum_fold(data: bytes, init: int = 0) -> int:
    """tcpipChecksum (layers/tcpip.go:76-94): byte-pair sum into uint32, fold, invert."""
    c = init
    n = len(data)
    for i in range(0, n - 1, 2):
        c += (data[i] << 8) + data[i + 1]
    if n % 2 == 1:
        c += data[n - 1] << 8
    c &= 0xFFFFFFFF
    while c > 0xFFFF:
        c = (c >> 16) + (c & 0xFFFF)
    return (~c) & 0xFFFF


def _pair_sum(b: bytes) -> int:
    return sum((b[i] << 8) + b[i + 1] for i in range(0, len(b), 2))


def ipv4_pseudo(src: bytes, dst: bytes, proto: int, length: int) -> int:
    """IPv4Header.GetPhCs layout (ip4.go:49-58)."""
    return _pair_sum(src + dst + bytes([0, proto]) + struct.pack(">H", length & 0xFFFF))


def ipv6_pseudo(src: bytes, dst: bytes, length: int, nh: int) -> int:
    """IPv6Header.GetPhCs layout (ip6.go:126-134)."""
    return _pair_sum(src + dst + struct.pack(">I", length & 0xFFFF) + bytes([0, 0, 0, nh]))


# ---------------------------------------------------------------------------------------
# layers
# ---------------------------------------------------------------------------------------
def ethernet(dst, src, etype: int, payload: bytes, pad: bool = True) -> bytes:
    f = mac(dst) + mac(src) + struct.pack(">H", etype) + payload
    if pad and len(f) < 60:
        f += bytes(60 - len(f))
    return f


def dot1q(vid: int, etype: int, pcp: int = 0, dei: bool = False) -> bytes:
    tci = (pcp << 13) | vid | (0x1000 if dei else 0)
    return struct.pack(">HH", tci, etype)


def ipv4(src, dst, proto: int, payload: bytes, *, ttl=64, tos=0, ident=0, flags=0, frag=0,
         options: bytes = b"", length=None, ihl=None, csum="auto", version=4) -> bytes:
    if ihl is None:
        ihl = 5 + len(options) // 4
    if length is None:
        length = 20 + len(options) + len(payload)
    hdr = bytearray(struct.pack(">BBHHHBBH4s4s", (version << 4) | ihl, tos, length & 0xFFFF,
                                ident, (flags << 13) | frag, ttl, proto, 0, ip4(src), ip4(dst)))
    hdr += options
    if csum == "auto":
        c = csum_fold(bytes(hdr))
    else:
        c = int(csum)
    hdr[10:12] = struct.pack(">H", c)
    return bytes(hdr) + payload


def ipv6(src, dst, nh: int, payload: bytes, *, hop=64, plen=None, tc=0, flow=0,
         version=6) -> bytes:
    if plen is None:
        plen = len(payload)
    w0 = (version << 28) | (tc << 20) | flow
    return struct.pack(">IHBB", w0, plen & 0xFFFF, nh, hop) + ip6(src) + ip6(dst) + payload


def ipv6_ext(nh: int, body: bytes) -> bytes:
    """Generic extension header (HBH / DST / ROUTING ...): nh, hdrlen, body padded to 8n-2."""
    total = 2 + len(body)
    if total % 8:
        body = body + bytes(8 - total % 8)
        total = 2 + len(body)
    return bytes([nh, total // 8 - 1]) + body


def udp(sport: int, dport: int, payload: bytes, *, csum=0, pseudo: int | None = None,
        length=None) -> bytes:
    """csum: int value, or "auto" with `pseudo` = pseudo-header partial sum (GetPhCs)."""
    if length is None:
        length = 8 + len(payload)
    h = bytearray(struct.pack(">HHHH", sport, dport, length & 0xFFFF, 0)) + payload
    if csum == "auto":
        c = csum_fold(bytes(h), pseudo or 0)
    else:
        c = int(csum)
    h[6:8] = struct.pack(">H", c)
    return bytes(h)


def tcp(sport: int, dport: int, payload: bytes, *, seq=1, ack=0, flags=0x18, win=8192,
        doff=5, options: bytes = b"", csum="auto", pseudo: int | None = None) -> bytes:
    h = bytearray(struct.pack(">HHIIBBHHH", sport, dport, seq, ack, doff << 4, flags, win, 0, 0))
    h += options
    h += payload
    if csum == "auto":
        c = csum_fold(bytes(h), pseudo or 0)
    else:
        c = int(csum)
    h[16:18] = struct.pack(">H", c)
    return bytes(h)


def icmp4(typ: int, code: int, ident: int, seq: int, payload: bytes, csum="auto") -> bytes:
    h = bytearray(struct.pack(">BBHHH", typ, code, 0, ident, seq)) + payload
    c = csum_fold(bytes(h)) if csum == "auto" else int(csum)
    h[2:4] = struct.pack(">H", c)
    return bytes(h)


def icmp6(typ: int, code: int, body: bytes, *, pseudo: int, csum="auto") -> bytes:
    h = bytearray(struct.pack(">BBH", typ, code, 0)) + body
    c = csum_fold(bytes(h), pseudo) if csum == "auto" else int(csum)
    h[2:4] = struct.pack(">H", c)
    return bytes(h)


def arp(op: int, sha, spa, tha, tpa, htype=1, ptype=0x0800) -> bytes:
    return (struct.pack(">HHBBH", htype, ptype, 6, 4, op) + mac(sha) + ip4(spa) + mac(tha)
            + ip4(tpa))


def dhcp_option(t: int, data: bytes | None = None) -> bytes:
    if t in (0, 255):
        return bytes([t])
    return bytes([t, len(data)]) + data


def dhcpv4(op: int, xid: int, chaddr, options: list[bytes], *, htype=1, hlen=None, flags=0,
           ciaddr="0.0.0.0", yiaddr="0.0.0.0", siaddr="0.0.0.0", giaddr="0.0.0.0",
           magic=0x63825363) -> bytes:
    ch = mac(chaddr)
    if hlen is None:
        hlen = len(ch)
    d = bytearray(240)
    d[0], d[1], d[2], d[3] = op, htype, hlen, 0
    d[4:8] = struct.pack(">I", xid)
    d[10:12] = struct.pack(">H", flags)
    d[12:16] = ip4(ciaddr)
    d[16:20] = ip4(yiaddr)
    d[20:24] = ip4(siaddr)
    d[24:28] = ip4(giaddr)
    d[28:28 + len(ch)] = ch
    d[236:240] = struct.pack(">I", magic)
    if options:
        for o in options:
            d += o
        d += b"\xff"
    return bytes(d)


def pppoe_padi() -> bytes:
    """PPPoE PADI with one empty Service-Name tag (as parser_test.go:50-60)."""
    return bytes([0x11, 0x09]) + struct.pack(">HH", 0, 4) + struct.pack(">HH", 0x0101, 0)


# ---------------------------------------------------------------------------------------
# ZMQ batch wire format (src/emu/core/veth_zmq.go:8-22)
# ---------------------------------------------------------------------------------------
def zmq_pack(frames, vports=None) -> bytes:
    out = bytearray(struct.pack(">I", (0xBEEF << 16) | (len(frames) & 0xFFFF)))
    for i, f in enumerate(frames):
        vp = 0 if vports is None else vports[i]
        out += struct.pack(">I", (0xAA << 24) | ((vp & 0xFF) << 16) | (len(f) & 0xFFFF))
        out += f
    return bytes(out)


def zmq_messages(buf, desc, per_msg: int = 64):
    """A batch in the ZMQ layout (synth.pack_zmq_layout: each frame preceded by its 4-byte
    frame header) -> (stream, msgs): consecutive groups of `per_msg` frames as ZMQ messages
    (a 4-byte batch header each) laid back to back in `stream`, and msgs[i] = (off, len) of
    message i in it (emurx.abi.MSG_DTYPE).  Frames must be in buffer order, contiguous."""
    import numpy as np
    from .abi import MSG_DTYPE
    n = len(desc)
    off = desc["off"].astype(np.int64)
    end = off + desc["len"].astype(np.int64)
    first = np.arange(0, n, per_msg)
    last = np.minimum(first + per_msg, n) - 1
    src_lo, src_hi = off[first] - 4, end[last]
    cnt = last - first + 1
    mlen = 4 + (src_hi - src_lo)
    moff = np.zeros(len(first), np.int64)
    moff[1:] = np.cumsum(mlen[:-1])
    total = int(mlen.sum())
    stream = np.empty(total, np.uint8)
    hdr = ((0xBEEF << 16) | (cnt & 0xFFFF)).astype(">u4").view(np.uint8).reshape(-1, 4)
    idx = moff[:, None] + np.arange(4)[None, :]
    stream[idx] = hdr
    # frame bytes (with their frame headers) are contiguous per message in the source
    lens = src_hi - src_lo
    body = int(lens.sum())
    if body:
        k = np.arange(body) - np.repeat(np.cumsum(lens) - lens, lens)  # byte index inside its message body
        stream[np.repeat(moff + 4, lens) + k] = np.asarray(buf)[np.repeat(src_lo, lens) + k]
    msgs = np.zeros(len(first), MSG_DTYPE)
    msgs["off"], msgs["len"] = moff, mlen
    return stream, msgs


def pack_frames(frames, vports=None, header: int = 4):
    """Concatenate frames with a `header`-byte gap before each (ZMQ layout when 4) and
    return (buffer, desc) with desc a numpy structured array (see emurx.abi.DESC_DTYPE)."""
    import numpy as np
    from .abi import DESC_DTYPE
    n = len(frames)
    desc = np.zeros(n, dtype=DESC_DTYPE)
    buf = bytearray()
    for i, f in enumerate(frames):
        buf += bytes(header)
        desc[i]["off"] = len(buf)
        desc[i]["len"] = len(f)
        desc[i]["vport"] = 0 if vports is None else vports[i]
        buf += f
    buf += bytes(16)
    return np.frombuffer(bytes(buf), dtype=np.uint8).copy(), desc


def tunnel_key(vport: int, vlan0: int = 0, vlan1: int = 0) -> bytes:
    """CTunnelKey bytes (thread_ctx.go:92-97)."""
    return struct.pack("<HHII", vport, 0, vlan0, vlan1)
