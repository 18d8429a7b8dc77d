"""The oracle over the reference's golden capture corpus (tests/golden/corpus_frames.npz,
extracted from unit-test/exp by tests/golden/make_corpus.py).

Pins: every rx frame the reference's plugin simulations answered reaches a callback
(SURVEY.md §4), and the callback it reaches is the one of the plugin whose simulation the
capture records (its file name: arp*.json -> arp, dns*.json -> udp, the DNS plugin's sockets
ride the transport plugin's UDP, ipv6nd / mld / ipv6ping -> icmpv6, dot1x -> eapol, ...); the
per-callback distribution of the whole corpus is recomputed here (scratch counts).
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


# capture name prefix -> the callback of the plugin under simulation (src/emu/plugins/<name>,
# registered as in src/cmd/trex-emu.go:47-67; dns rides transport UDP sockets)
CAPTURE_CB = [("dhcpsrv", "dhcpsrv"), ("dhcpv6", "dhcpv6"), ("dhcp", "dhcp"), ("arp", "arp"),
              ("dns", "udp"), ("dot1x", "eapol"), ("icmpv6", "icmpv6"), ("icmp", "icmp"),
              ("igmp", "igmp"), ("ipv6nd", "icmpv6"), ("ipv6ping", "icmpv6"), ("mdns", "mdns"),
              ("mld", "icmpv6")]


def capture_callback(name):
    for pre, cb in CAPTURE_CB:
        if name.startswith(pre):
            return cb
    return None


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


def test_rx_frames_reach_their_plugin(oracle_built):
    """Each answered rx frame reaches the callback of the plugin its capture simulates."""
    import pyoracle
    z = np.load(GOLD, allow_pickle=False)
    files, src = z["files"], z["src"]
    buf, desc, meta = corpus_batch()
    rec, _, _, _ = pyoracle.Oracle().rx_batch(buf, desc)
    rx = np.nonzero(meta == 1)[0]
    assert len(rx) == sum(RX_EXPECT.values())
    checked = 0
    for i in rx:
        want = capture_callback(str(files[src[i]]))
        assert want is not None, files[src[i]]
        assert rec["status"][i] == 0 and abi.CB_NAMES[rec["proto"][i]] == want, (files[src[i]], i)
        checked += 1
    assert checked == len(rx)


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
