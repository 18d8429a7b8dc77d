"""The oracle's transport flow decision (TransportCtx.handleRxPacket, client_ctx.go:912-969)
against the outcomes the reference's transport simulations vouch for (tests/transport_sims.py):
every frame of the 17 tcp / udp captures, delivered to its peer, classifies to the peer
(tcp / udp callback, client found) and takes the flow decision its successors in the capture
imply (NEW, the server's flow, the client's flow).  The GPU twin is
tests/test_gpu_parity.py::test_transport_reference_sims."""
import numpy as np
import pytest

import transport_sims as T
from emurx import abi
from emurx import frames as F

OUT = {"NEW": abi.FLOW_NEW, "SERVER_FLOW": T.SERVER_FLOW, "CLIENT_FLOW": T.CLIENT_FLOW}


def corpus():
    toc = __import__("test_oracle_corpus")
    return np.load(toc.GOLD, allow_pickle=False)


def run_oracle(o, buf, desc):
    rec, _, _, _ = o.rx_batch(buf, desc)
    return rec, o.flows(buf, desc, rec)


@pytest.mark.parametrize("capture", T.CAPTURES)
def test_oracle_transport_sim(capture, oracle_built):
    fr = T.frames(corpus(), capture)
    proto, ckey, skey, accept, exp = T.plan(capture, fr)
    buf, desc = F.pack_frames(fr, [1] * len(fr))
    o = oracle_built.Oracle()
    T.load(o, proto, ckey, abi.PLUG_ALL)
    rec, flow = run_oracle(o, buf, desc)
    cb = abi.CB_TCP if proto == 6 else abi.CB_UDP
    assert (rec["status"] == 0).all() and (rec["proto"] == cb).all()
    assert (((rec["flags"] >> 4) & 7) == abi.LK["CLIENT"]).all()
    want_cid = np.array([T.SERVER["cid"] if T.to_server(f) else T.CLIENT["cid"] for f in fr])
    assert np.array_equal(rec["client_id"], want_cid)
    before = [(i, k) for i, _, k, s in exp if s == "before"]
    assert before and all(int(flow[i]) == OUT[k] for i, k in before), [(i, hex(flow[i])) for i, _ in before]
    # NO_SYN / NO_SERVER (restatement, no capture frame): non-SYN frames to the server before it
    # holds the flow, and the SYN without the listener
    for i, f in enumerate(fr):
        if T.to_server(f) and proto == 6 and not T.is_syn(f):
            assert flow[i] == abi.FLOW_NO_SYN
    assert o.flow_add(T.SERVER["cid"], skey, T.SERVER_FLOW) == 0
    rec, flow = run_oracle(o, buf, desc)
    after = [(i, k) for i, _, k, s in exp if s == "after"]
    assert len(after) >= len(fr) // 2
    bad = [(i, k, hex(int(flow[i]))) for i, k in after if int(flow[i]) != OUT[k]]
    assert not bad, bad[:5]
    assert o.server_remove(T.SERVER["cid"], T.PORT, proto) == 0
    assert o.flow_remove(T.SERVER["cid"], skey) == 0
    _, flow = run_oracle(o, buf, desc)
    assert flow[accept] == abi.FLOW_NO_SERVER
