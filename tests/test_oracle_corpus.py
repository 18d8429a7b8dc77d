"""The oracle over the reference's golden capture corpus (tests/golden/corpus_frames.npz,
extracted from unit-test/exp by tests/golden/make_corpus.py).

Pins: every rx frame the reference's plugin simulations answered reaches a callback
(SURVEY.md §4), and the per-callback distribution of the whole corpus.
"""
import collections
from pathlib import Path

import numpy as np

from emurx import abi

GOLD = Path(__file__).resolve().parent / "golden" / "corpus_frames.npz"

# SURVEY.md §4 (scratch restatement, recomputed here)
RX_EXPECT = {"udp": 268, "mdns": 249, "arp": 69, "icmpv6": 62, "dhcpsrv": 34, "igmp": 25,
             "dhcp": 24, "icmp": 11, "eapol": 9, "dhcpv6": 8}
TX_EXPECT = {"udp": 4398, "tcp": 1214, "igmp": 703, "arp": 620, "icmpv6": 377, "mdns": 251,
             "ICMPV6_UNSUPPORTED": 209, "dhcpsrv": 107, "dhcp": 21, "L3_UNSUPPORTED": 20,
             "eapol": 13, "icmp": 11}


def load_corpus():
    z = np.load(GOLD, allow_pickle=False)
    return z["data"], z["off"], z["len"], z["meta"]


def corpus_batch():
    """Corpus as one batch in the ZMQ layout (4-byte gap before each frame), vport 1."""
    data, off, ln, meta = load_corpus()
    from emurx import frames as F
    fr = [data[o:o + l].tobytes() for o, l in zip(off, ln)]
    buf, desc = F.pack_frames(fr, vports=[1] * len(fr))
    return buf, desc, meta


def test_corpus_distribution(oracle_built):
    import pyoracle
    buf, desc, meta = corpus_batch()
    o = pyoracle.Oracle()
    rec, qlist, qoff, cnt = o.rx_batch(buf, desc)
    for m, expect in ((1, RX_EXPECT), (0, TX_EXPECT)):
        sel = rec[meta == m]
        c = collections.Counter(abi.CB_NAMES[p] if s == 0 else abi.STATUS_NAMES[s]
                                for s, p in zip(sel["status"], sel["proto"]))
        assert dict(c) == expect
    # all rx frames reached a callback
    assert (rec[meta == 1]["status"] == 0).all()
    # queues partition the batch, each stable
    assert qoff[-1] == len(rec)
    for q in range(abi.NUM_QUEUES):
        idx = qlist[qoff[q]:qoff[q + 1]]
        assert (np.diff(idx.astype(np.int64)) > 0).all()
        want = (rec["status"] == 0) & (rec["proto"] == q) if q < 12 else rec["status"] != 0
        assert set(idx.tolist()) == set(np.nonzero(want)[0].tolist())
    d = pyoracle.counters_dict(cnt)
    assert d["udpPkts"] == sum(((rec["status"] == 0) & np.isin(rec["proto"], [3, 4, 5, 6, 8])))
    assert d["errParser"] == int((rec["status"] != 0).sum())
