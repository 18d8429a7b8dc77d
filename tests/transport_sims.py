"""Transport flow decisions pinned by the reference's transport simulations.

src/emu/plugins/transport/trans_sim.go builds one Namespace (vport 1, tags 0x8100/1 and
0x8100/2) with two clients (newTransportSim :644-680): a client (MAC 00:00:01:00:00:01,
16.0.0.1, 2001:db8::1000:1) that Dials 48.0.0.1:80 or [2001:db8::3000:1]:80 over TCP or UDP
(newSimCtx :50-57), and a server (MAC 00:00:01:00:00:02, 48.0.0.1, 2001:db8::3000:1)
listening on :80 (:41-45).  Every frame either sends is recorded as "tx" in
unit-test/exp/<test>.json and, after a 500 ms timer, handed to the peer's
TransportCtx.handleRxPacket (ProcessTxToRx :731-747: dst MAC byte 5 == 2 -> the server;
pktEventTxRx.OnEvent :693-728), the function emurx's flow decision restates
(client_ctx.go:912-969).  Some tests drop each delivery with a probability (param.drop,
trans_test.go); a dropped frame is recorded but never delivered.

What the capture vouches for, per frame (TCP or UDP, IPv4 or IPv6):
  * the flow table holds the client's connection from Dial on, keyed "in respect to the
    return packet" (client_ctx.go:44-45): the swap of its first frame's tuple;
  * the server accepted the last client SYN before its first frame (a SYN-ACK only follows an
    accept, handleRxTcpNewFlow :829-864 -> OnAccept), or, for UDP, the client's first
    datagram (handleRxUdpNewFlow :866-898): that frame was a NEW flow at the server, and so
    would any client SYN before it have been, had it been delivered;
  * a frame to the server after the accept, followed in the capture by a frame from the
    server, found the server's flow (a socket that answers later was alive: no flow is removed
    and recreated in these tests), and likewise a frame to the client followed by a frame from
    the client found the client's flow; in the tests without drops the closing frames did too
    (the last ACK of a FIN reaches a socket in LAST_ACK or TIME_WAIT).

NEW and the found flows are pinned this way.  NO_SYN (a non-SYN frame without a flow) and
NO_SERVER (a SYN without a listener) have no frame in the captures; the tests derive them
from the same frames with the flow or the listener taken away (a restatement of
handleRxTcpNewFlow :838-850, not a capture outcome).
"""
import struct

import numpy as np

NS_KEY = struct.pack("<HHII", 1, 0, 0x81000001, 0x81000002)
CLIENT = dict(cid=0, mac=bytes([0, 0, 1, 0, 0, 1]), ipv4=bytes([16, 0, 0, 1]),
              ipv6=bytes([0x20, 0x01, 0x0D, 0xB8] + [0] * 8 + [16, 0, 0, 1]))
SERVER = dict(cid=1, mac=bytes([0, 0, 1, 0, 0, 2]), ipv4=bytes([48, 0, 0, 1]),
              ipv6=bytes([0x20, 0x01, 0x0D, 0xB8] + [0] * 8 + [48, 0, 0, 1]))
PORT = 80
CLIENT_FLOW, SERVER_FLOW = 100, 200
# trans_test.go: the tests with param.drop > 0 (TestPluginTrans11 / 12: 0.1, TestPluginTransSc4: 0.02)
DROPS = {"tcp1-11.json", "tcp1-12.json", "tcpsc-4.json"}
CAPTURES = ["tcp1.json", "tcp1-6.json", "tcp1-7.json", "tcp1-8.json", "tcp1-9.json", "tcp1-10.json",
            "tcp1-11.json", "tcp1-12.json", "tcp1-v6.json", "tcp1-v6-02.json", "tcp-udp1.json", "tcp-udp2.json",
            "tcprr-1.json", "tcpsc-1.json", "tcpsc-2.json", "tcpsc-3.json", "tcpsc-4.json"]


def frames(z, capture):
    """The capture's frames in recording order (tests/golden/corpus_frames.npz)."""
    fi = [str(f) for f in z["files"]].index(capture)
    idx = np.nonzero(z["src"] == fi)[0]
    return [z["data"][z["off"][i]:z["off"][i] + z["len"][i]].tobytes() for i in idx]


def l3l4(f):
    """(ipv6, L3, L4, protocol) of a simulation frame: two tags, IPv4 (IHL from the header) or
    IPv6 without extension headers, as trans_sim.go:699-710 lays them out."""
    l3 = 22
    v6 = f[20:22] == b"\x86\xdd"
    return (v6, l3, l3 + 40, f[l3 + 6]) if v6 else (v6, l3, l3 + (f[l3] & 15) * 4, f[l3 + 9])


def tuple_of(f):
    """The frame's c5tuplekey as the receiver builds it (fillv4tuple / fillv6tuple, client_ctx.go:720-765)."""
    v6, l3, l4, proto = l3l4(f)
    if v6:
        return f[l3 + 8:l3 + 40] + f[l4:l4 + 4] + bytes([proto])
    return f[l3 + 12:l3 + 20] + f[l4:l4 + 4] + bytes([proto])


def swapped(t):
    """The key of the return direction (the client's flow, registered at Dial)."""
    n = 16 if len(t) == 37 else 4
    return t[n:2 * n] + t[:n] + t[2 * n + 2:2 * n + 4] + t[2 * n:2 * n + 2] + t[-1:]


def to_server(f):
    return f[5] == 2  # ProcessTxToRx, trans_sim.go:740


def is_syn(f):
    _, _, l4, proto = l3l4(f)
    return proto == 6 and (f[l4 + 13] & 0x3F) == 0x02


def plan(capture, fr):
    """-> (proto, client flow key, server flow key, accept index, expectations) where
    expectations = [(frame index, receiver cid, "NEW" | "SERVER_FLOW" | "CLIENT_FLOW", state)] and
    state "before" (listener + client flow) or "after" (+ the server's accepted flow)."""
    proto = l3l4(fr[0])[3]
    first_reply = next(i for i, f in enumerate(fr) if not to_server(f))
    if proto == 6:
        accept = max(i for i in range(first_reply) if to_server(fr[i]) and is_syn(fr[i]))
    else:
        accept = next(i for i in range(first_reply) if to_server(fr[i]))
    client_key = swapped(tuple_of(fr[0]))
    server_key = tuple_of(fr[accept])
    drops = capture in DROPS
    exp = []
    for i, f in enumerate(fr):
        later_from_receiver = any(to_server(g) != to_server(f) for g in fr[i + 1:])
        if to_server(f):
            if i <= accept:
                if proto == 17 or is_syn(f):
                    exp.append((i, SERVER["cid"], "NEW", "before"))
            elif later_from_receiver or not drops:
                exp.append((i, SERVER["cid"], "SERVER_FLOW", "after"))
        elif later_from_receiver or not drops:
            exp.append((i, CLIENT["cid"], "CLIENT_FLOW", "after"))
    return proto, client_key, server_key, accept, exp


def load(t, proto, client_key, plugins_all):
    """The simulation's tables on `t` (RxPath or oracle): the Namespace, both clients with a
    TransportCtx, the server's listener on :80 and the client's connection."""
    assert t.ns_add(NS_KEY, 0, plugins_all) == 0
    for c in (CLIENT, SERVER):
        assert t.client_add(0, c["cid"], c["mac"], c["ipv4"], c["ipv6"], None, plugins_all) == 0
        assert t.client_set_transport(c["cid"], 1) == 0
    assert t.server_add(SERVER["cid"], PORT, proto) == 0
    assert t.flow_add(CLIENT["cid"], client_key, CLIENT_FLOW) == 0
