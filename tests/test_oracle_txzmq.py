"""The oracle's tx ZMQ framing (orc_tx_zmq, a statement-by-statement restatement of
VethIFZmq.Send / FlushTx, veth_zmq.go:149-200).  The reference holds no captured tx
messages, so the restatement is checked by its rules and by a round trip through the rx
framing restatement (OnRxStream, veth_zmq.go:277-320, pinned by the reference's fixtures):
every message decodes to the frames that went in, in order."""
import numpy as np
import pytest

from emurx import abi
import txzmq_util as U


def _decode(msg):
    """message -> [(vport, bytes)] by the format of FlushTx :157-171"""
    cnt = int.from_bytes(msg[2:4].tobytes(), "big")
    at, res = 4, []
    for _ in range(cnt):
        h = int.from_bytes(msg[at:at + 4].tobytes(), "big")
        assert h >> 24 == abi.ZMQ_PKT_MAGIC
        ln = h & 0xFFFF
        res.append(((h >> 16) & 0xFF, msg[at + 4:at + 4 + ln].tobytes()))
        at += 4 + ln
    assert at == len(msg)
    return res


def _roundtrip(buf, d, out, off):
    import pyoracle
    k = 0
    for m in range(len(off) - 1):
        msg = out[int(off[m]):int(off[m + 1])]
        assert int.from_bytes(msg[:2].tobytes(), "big") == 0xBEEF
        frames = _decode(msg)
        assert 1 <= len(frames) <= abi.ZMQ_TX_BURST
        # OnRxStream walks a message with u16 offsets and allocates mbufs of at most
        # EMURX_MAX_FRAME bytes: check the messages it can take
        if len(msg) <= 0xFFFF and all(len(b) <= abi.MAX_FRAME for _, b in frames):
            rc, got, err = pyoracle.zmq_descriptors(msg.tobytes(), cap=128)
            assert rc == 0 and err == 0, (m, rc, err)
            assert [(int(g["vport"]), msg[int(g["off"]):int(g["off"]) + int(g["len"])].tobytes())
                    for g in got] == frames
        for vp, b in frames:
            e = d[k]
            assert vp == int(e["vport"]) and b == buf[int(e["off"]):int(e["off"]) + int(e["len"])].tobytes()
            k += 1
    assert k == len(d)


@pytest.mark.parametrize("n,kind", [(0, 0), (1, 0), (63, 3), (64, 3), (65, 3), (1000, 0), (300, 1),
                                    (700, 2), (5000, 3)])
def test_tx_zmq_roundtrip(oracle_built, n, kind):
    import pyoracle
    buf, d = U.batch(n, kind)
    out, off, total = pyoracle.tx_zmq(buf, d)
    assert total == len(out) == int(off[-1]) == 4 * (len(off) - 1) + 4 * n + int(d["len"].astype(np.int64).sum())
    _roundtrip(buf, d, out, off)


def test_tx_zmq_rules(oracle_built):
    """Send :186 closes before a frame reaching 32 KiB; :198 after 64 frames; a lone frame of
    32 KiB or more is its own message."""
    import pyoracle
    buf, d = U.threshold_batch()
    out, off, _ = pyoracle.tx_zmq(buf, d)
    counts = [int.from_bytes(out[int(o) + 2:int(o) + 4].tobytes(), "big") for o in off[:-1]]
    # 32767 | 1 32766 | 1 1 16384 | 16383 1 | 16384 | 16384 0 0 10 x61 | 10 x64 | 10 x5 | 32768
    # | 5 | 65535 | 0 7   (a frame reaching 32768 with the open message's bytes closes it
    # first; the zero-length frame after 65535 still sees 65535 open bytes)
    assert counts == [1, 2, 3, 2, 1, 64, 64, 5, 1, 1, 1, 2], counts
    _roundtrip(buf, d, out, off)


def test_tx_zmq_capacity(oracle_built):
    import pyoracle
    buf, d = U.batch(200, 2)
    full, off, total = pyoracle.tx_zmq(buf, d)
    part, off2, total2 = pyoracle.tx_zmq(buf, d, cap=total // 3)
    assert total2 == total and np.array_equal(off2, off)
    assert part.tobytes() == full[: total // 3].tobytes()
