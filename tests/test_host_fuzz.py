"""Host-side fuzz, no GPU: the oracle's parse + classify over mutated capture frames, and the
C-ABI's host framing walk (emurx_zmq_descriptors, the OnRxStream restatement veth_zmq.go:277-320)
over random, truncated, corrupted and over-announcing ZMQ messages against the oracle's walk.
These are the inputs tests/test_sanitizers.py drives through the ASan + UBSan builds of the
oracle and of the library's host code; here they also run plain."""
import numpy as np

import edge_frames as E
from emurx import frames as F
from gpu_util import frames_tables, load_frame_tables
from test_gpu_parity import corpus_frames, mutate


def test_oracle_fuzz_frames(oracle_built):
    """20K mutated frames (bytes overwritten, truncated, bits flipped, tails appended) through
    the oracle's rx_batch and its per-frame parse; the two agree and every record's offsets
    stay inside what a uint16 can hold."""
    rng = np.random.default_rng(0xA5A1)
    base = corpus_frames() + [c[1] for c in E.cases()]
    frames = mutate(base, rng, 20000)
    o = oracle_built.Oracle()
    ns, cl = frames_tables(base)
    load_frame_tables([o], ns, cl)
    buf, desc = F.pack_frames(frames, list(rng.integers(0, 4, len(frames))))
    rec, qlist, qoff, cnt = o.rx_batch(buf, desc)
    assert len(rec) == len(frames) and int(qoff[-1]) == len(frames)
    assert len(set(rec["status"].tolist())) >= 20
    for i in rng.integers(0, len(frames), 500):
        r = o.parse_frame(frames[i], int(desc["vport"][i]))
        assert r["status"] == rec["status"][i] and r["l4"] == rec["l4"][i] and r["l7_len"] == rec["l7_len"][i]


def _hostile_msgs(rng, count=400):
    """ZMQ rx messages (0xBEEF | count, then 0xAA | vport | len + bytes per frame) of every
    kind the walk must survive: announced counts larger than present, frame lengths past the
    message end, truncated headers, bad magics, empty and > 64 KiB messages."""
    out = []
    for _ in range(count):
        nf = int(rng.integers(0, 10))
        fr = [rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes() for _ in range(nf)]
        m = bytearray(F.zmq_pack(fr, list(rng.integers(0, 256, nf))))
        k = int(rng.integers(0, 7))
        if k == 0 and len(m) > 4:
            m = m[: int(rng.integers(0, len(m)))]                       # truncated anywhere
        elif k == 1:
            m[2:4] = int(rng.integers(nf + 1, 65536)).to_bytes(2, "big")  # over-announcing count
        elif k == 2 and nf:
            at = 4
            j = int(rng.integers(0, nf))
            for f in fr[:j]:
                at += 4 + len(f)
            m[at + 2:at + 4] = int(rng.integers(len(fr[j]) + 1, 65536)).to_bytes(2, "big")  # frame past the end
        elif k == 3 and nf:
            m[4] = int(rng.integers(0, 256))                            # frame magic
        elif k == 4:
            m[0:2] = (0xFEEB).to_bytes(2, "big")                        # compressed batch (never handled)
        elif k == 5:
            m += rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8).tobytes()  # trailing garbage
        out.append(bytes(m))
    out += [b"", b"\xbe", b"\xbe\xef\x00\x01", F.zmq_pack([bytes(9000)] * 9), F.zmq_pack([bytes(65000)]),
            F.zmq_pack([bytes(9217)]), F.zmq_pack([b""] * 70)]
    return out


def test_zmq_walk_hostile_messages(lib, oracle_built):
    from emurx.rx import zmq_descriptors
    rng = np.random.default_rng(0xBEEF)
    for m in _hostile_msgs(rng):
        for cap in (1 << 16, 3):
            a = zmq_descriptors(m, cap)
            b = oracle_built.zmq_descriptors(m, cap)
            assert a[0] == b[0] and a[2] == b[2], (m[:16].hex(), cap)
            assert a[1].tobytes() == b[1].tobytes()
