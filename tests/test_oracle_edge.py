"""Pin the oracle on every return path of ParsePacket / parsePacketL4 (expected outcomes
read off src/emu/core/parser.go by hand, see tests/edge_frames.py), plus the table
semantics of AddNs / AddClient / RemoveClient / UpdateClient* and the ZMQ framing quirks."""
import pytest

import edge_frames as E
from emurx import abi
from emurx import frames as F

CASES = E.cases()


@pytest.mark.parametrize("name,frame,vport,exp,cb", CASES, ids=[c[0] for c in CASES])
def test_edge_outcome(oracle_built, name, frame, vport, exp, cb):
    import pyoracle
    r = pyoracle.parse_only(frame, vport)
    assert abi.STATUS_NAMES[r["status"]] == exp
    if cb is not None:
        assert abi.CB_NAMES[r["proto"]] == cb
    else:
        assert r["proto"] == abi.CB_NONE


def test_eapol_unregistered_is_panic(oracle_built):
    import pyoracle
    f = E.eth(F.ETH_EAPOL, b"\x01\x00\x00\x05")
    assert pyoracle.parse_only(f, 0, 0)["status"] == abi.ST["PANIC_NIL_EAPOL"]
    assert pyoracle.parse_only(f, 0, 1 << abi.CB_EAPOL)["status"] == abi.ST["OK"]


def test_wrapped_l7len(oracle_built):
    import pyoracle
    f = E.v4(17, F.udp(1, 2, b"abcd", csum=0), length=10)
    r = pyoracle.parse_only(f, 0)
    assert r["l7_len"] == (10 - 20 - 8) & 0xFFFF


def test_table_semantics(oracle_built):
    import pyoracle
    o = pyoracle.Oracle()
    k = F.tunnel_key(1, 0x81000001, 0)
    assert o.ns_add(k, 0, 0x7FF) == 0
    assert o.ns_add(k, 1, 0x7FF) == abi.EMURX_EEXIST
    mac = bytes([2, 0, 0, 0, 0, 1])
    assert o.client_add(0, 0, bytes(6)) == abi.EMURX_EINVAL           # zero MAC
    assert o.client_add(0, 0, mac, bytes([10, 0, 0, 1])) == 0
    assert o.client_add(0, 1, mac) == abi.EMURX_EEXIST                # same MAC
    assert o.client_add(0, 1, bytes([2, 0, 0, 0, 0, 2]), bytes([10, 0, 0, 1])) == abi.EMURX_EEXIST
    assert o.ns_remove(k) == abi.EMURX_EEXIST                        # active clients
    assert o.client_update_ipv4(0, bytes([10, 0, 0, 9])) == 0
    assert o.client_remove(0, mac) == 0
    assert o.ns_remove(k) == 0


def test_zmq_walk(oracle_built):
    import pyoracle
    fr = [bytes(60), bytes(100), bytes(14)]
    msg = F.zmq_pack(fr, [1, 2, 3])
    rc, d, err = pyoracle.zmq_descriptors(msg)
    assert rc == 0 and err == 0 and len(d) == 3
    assert list(d["len"]) == [60, 100, 14] and list(d["vport"]) == [1, 2, 3]
    assert list(d["off"]) == [8, 72, 176]
    # truncated message: RxParseErr, frames before the error survive
    rc, d, err = pyoracle.zmq_descriptors(msg[:-1])
    assert err == 1 and len(d) == 2
    # bad magic
    assert pyoracle.zmq_descriptors(b"\x12\x34\x00\x01")[2] == 1
    # bad per-frame magic
    bad = bytearray(msg)
    bad[4] = 0xAB
    assert pyoracle.zmq_descriptors(bytes(bad))[1].size == 0
    # frame larger than MAX_PACKET_SIZE: MbufPoll.Alloc panics
    big = F.zmq_pack([bytes(9217)])
    assert pyoracle.zmq_descriptors(big)[2] == 2
