"""GPU: the Namespace-owner exchange behind the C-ABI (include/emu_rx.h emurx_comm_*,
emurx_exchange_dev): a library-owned RCCL communicator, driven through ctypes exactly as the
cgo shim drives it, no torch.distributed anywhere.

The box has one GPU, so the communicator has one rank (RCCL refuses two ranks on one device).
A 1-rank exchange still runs the library's whole protocol: the count and region phases of
both transfer modes (whole regions; counts first, then the spans that carry data), and with
EMURX_COMM_SELF=rccl the own region goes through RCCL's send / receive path instead of a
device copy.  Every owner output is bit-exact against the oracle on config D shards
(32,768 Namespaces / 1,048,576 clients: SURVEY.md §8d), the reference's classification
(thread_ctx.go:772-784, ns_ctx.go:262-329) of every frame.  The N > 1 protocol (which rank
receives which region) is the one the gloo tests of tests/test_exchange_cpu.py and
tests/test_bench_launch.py check with world size 2.
"""
import os

import numpy as np
import pytest

from emurx import abi, synth
from gpu_util import rec_diff, to_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dtabs(gpu_ok, oracle_built):
    """One handle with config D's full tables (1 partition: every Namespace is rank 0's), the
    oracle with the same tables, and two config D shards."""
    import pyoracle
    from emurx.rx import RxPath
    n = 1 << 18
    shards = [synth.config_d(n, rank=s) for s in range(2)]
    rx = RxPath(0, max_ns=32768, max_clients=1 << 20, max_frames=n)
    rx.register_all()
    synth.load_tables(shards[0], rx)
    o = pyoracle.Oracle()
    synth.load_tables(shards[0], o)
    yield rx, o, shards
    rx.close()


def owner_step(rx, w, cap, tcap, payload, stream=None, group=False):
    """parse_route_dev -> exchange_dev -> lookup_dev on one rank: (route records, counts,
    bytes moved, the send and receive buffers).  group: the exchange between
    emurx_group_start / emurx_group_end (the one-process, N-GPU form), its consumer after."""
    from emurx.rx import group_end, group_start
    import torch
    from emurx import exchange as X
    n = len(w["desc"])
    buf, desc = to_dev(w["buf"]), to_dev(w["desc"])
    qcap = abi.queue_cap(n)
    ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda")
    tc = torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device="cuda")
    hi = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
    rb = abi.lookup_region_bytes(cap, tcap)
    send = torch.full((rb,), 0xEE, dtype=torch.uint8, device="cuda")
    sc = torch.full((2,), -1, dtype=torch.int32, device="cuda")
    recv = torch.full((rb,), 0x5A, dtype=torch.uint8, device="cuda")
    rc = torch.full((2,), -1, dtype=torch.int32, device="cuda")
    out = torch.full((cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda")
    rx.parse_route_dev(buf, desc, n, None, ql, qcap, tc, hi, 1, 0, cap, send, sc, tail_cap=tcap, stream=stream)
    if group:
        group_start()
    try:
        moved = rx.exchange_dev(send, sc, recv, rc, cap, tcap, payload=payload, stream=stream)
    finally:
        if group:
            group_end()
    rx.lookup_dev(recv, rc, 1, cap, out, tail_cap=tcap, stream=stream)
    torch.cuda.synchronize()
    return (out.cpu().numpy().view(abi.ROUTE_REC_DTYPE), rc.cpu().numpy(), moved, send.cpu().numpy(),
            recv.cpu().numpy(), sc.cpu().numpy())


def check_owner(o, w, got, rc, cap):
    orec = o.rx_batch(w["buf"], w["desc"])[0]
    n = len(orec)
    assert int(rc[0]) == n and int(rc[1]) == 0
    want = np.zeros(n, abi.ROUTE_REC_DTYPE)
    want["rec"], want["src_index"], want["src_rank"] = orec, np.arange(n), 0
    g = got[:n]
    assert g.tobytes() == want.tobytes(), rec_diff(g["rec"], want["rec"])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("self_path", ["copy", "rccl"])
def test_one_rank_comm_config_d(dtabs, self_path):
    """a 1-rank library communicator (emurx_comm_unique_id +
    emurx_comm_init through ctypes), both transfer modes, config D shards on full tables: the
    owner's records are bit-exact against the oracle, the heads and the tail units arrive as
    sent, and a 1-rank exchange moves no byte to another rank."""
    from emurx import exchange as X
    from emurx.rx import comm_unique_id
    rx, o, shards = dtabs
    old = os.environ.get("EMURX_COMM_SELF")
    os.environ["EMURX_COMM_SELF"] = self_path  # read when the communicator is made
    try:
        rx.comm_init(comm_unique_id(), 1, 0)
    finally:
        if old is None:
            os.environ.pop("EMURX_COMM_SELF")
        else:
            os.environ["EMURX_COMM_SELF"] = old
    try:
        assert rx.comm_info() == (1, 0)
        for w in shards:
            n = len(w["desc"])
            cap = n
            tcap = abi.tail_capacity(cap)
            for payload in (False, True):
                got, rc, moved, send, recv, sc = owner_step(rx, w, cap, tcap, payload)
                check_owner(o, w, got, rc, cap)
                assert moved == 0 and np.array_equal(rc, sc)
                # what arrived: the valid heads byte for byte, and every head's tail
                assert recv[: n * 32].tobytes() == send[: n * 32].tobytes()
                a = X.lookup_records(send, n, cap, tcap)
                b = X.lookup_records(recv, n, cap, tcap)
                assert a.tobytes() == b.tobytes()
                if not payload:  # whole regions: every byte
                    assert recv.tobytes() == send.tobytes()
    finally:
        rx.comm_destroy()
    assert rx.comm_info() is None


def test_comm_init_all_group(dtabs):
    """The one-process model (emurx_comm_init_all over the process's handles, one GPU each; here
    one): the exchange issued between emurx_group_start / emurx_group_end, on a stream of the
    caller's, bit-exact against the oracle; the payload mode is refused inside a group (it
    waits on the host between its phases); a second communicator on the handle is refused."""
    import torch
    from emurx.rx import comm_init_all, comm_unique_id, group_end, group_start
    rx, o, shards = dtabs
    comm_init_all([rx])
    try:
        assert rx.comm_info() == (1, 0)
        with pytest.raises(RuntimeError, match="already exists"):
            rx.comm_init(comm_unique_id(), 1, 0)
        w = shards[1]
        n = len(w["desc"])
        cap, tcap = n, abi.tail_capacity(n)
        st = torch.cuda.Stream()
        group_start()
        try:
            with pytest.raises(RuntimeError, match="invalid argument"):
                dummy = torch.zeros(abi.lookup_region_bytes(cap, tcap), dtype=torch.uint8, device="cuda")
                cnt = torch.zeros(2, dtype=torch.int32, device="cuda")
                rx.exchange_dev(dummy, cnt, dummy.clone(), cnt.clone(), cap, tcap, payload=True)
        finally:
            group_end()
        # a whole-region exchange inside a group: the group's end issues it
        got, rc, moved, send, recv, sc = owner_step(rx, w, cap, tcap, False, stream=st, group=True)
        check_owner(o, w, got, rc, cap)
        assert recv.tobytes() == send.tobytes()
    finally:
        rx.comm_destroy()


def _comm(rx):
    from emurx.rx import comm_unique_id
    rx.comm_init(comm_unique_id(), 1, 0)


def test_route_records_exchange(dtabs):
    """EMURX_XCH_ROUTE: the replicated alternative's 40-byte route records (emurx_classify_route_dev's
    regions, one count per region) through the library communicator, both transfer modes: the
    counts and every routed record arrive as sent, and they are the host restatement's routing of
    the oracle's records."""
    import torch
    import route_ref
    from emurx import exchange as X
    rx, o, shards = dtabs
    w = shards[0]
    n = len(w["desc"])
    orec = o.rx_batch(w["buf"], w["desc"])[0]
    want = route_ref.route(orec, 1, 0)[0]
    buf, desc = to_dev(w["buf"]), to_dev(w["desc"])
    qcap = abi.queue_cap(n)
    ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda")
    tc = torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device="cuda")
    hi = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
    rec = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    cap = X.capacity(n, 1)
    send = torch.full((cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda")
    sc = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    rx.classify_route_dev(buf, desc, n, rec, ql, qcap, tc, hi, 1, 0, cap, send, sc)
    _comm(rx)
    try:
        for payload in (False, True):
            recv = torch.full_like(send, 0x5A)
            rc = torch.full_like(sc, -1)
            moved = rx.exchange_dev(send, sc, recv, rc, cap, payload=payload, route=True)
            torch.cuda.synchronize()
            c = int(sc.cpu()[0])
            assert moved == 0 and int(rc.cpu()[0]) == c == len(want)
            got = recv.cpu().numpy()[: c * X.REC_BYTES].view(abi.ROUTE_REC_DTYPE)
            assert got.tobytes() == send.cpu().numpy()[: c * X.REC_BYTES].tobytes()
            assert got.tobytes() == np.asarray(want, dtype=abi.ROUTE_REC_DTYPE).tobytes()
    finally:
        rx.comm_destroy()


def test_exchange_overflow_reports_the_full_count(dtabs):
    """A region sized below the batch (cap = n / 2): the source packs cap heads and reports the
    full count, the exchange moves the cap heads that exist (whole regions, or the spans
    min(count, cap) in payload mode) and delivers the full count, which is how the caller sees
    the overflow and regrows (bench.py exchange_overflow)."""
    import torch
    rx, o, shards = dtabs
    w = shards[1]
    n = len(w["desc"])
    cap = n // 2
    tcap = abi.tail_capacity(cap)
    buf, desc = to_dev(w["buf"]), to_dev(w["desc"])
    qcap = abi.queue_cap(n)
    ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda")
    tc = torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device="cuda")
    hi = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
    send = torch.full((abi.lookup_region_bytes(cap, tcap),), 0xEE, dtype=torch.uint8, device="cuda")
    sc = torch.full((2,), -1, dtype=torch.int32, device="cuda")
    rx.parse_route_dev(buf, desc, n, None, ql, qcap, tc, hi, 1, 0, cap, send, sc, tail_cap=tcap)
    _comm(rx)
    try:
        for payload in (False, True):
            recv = torch.full_like(send, 0x5A)
            rc = torch.full_like(sc, -1)
            rx.exchange_dev(send, sc, recv, rc, cap, tcap, payload=payload)
            torch.cuda.synchronize()
            s, r = send.cpu().numpy(), recv.cpu().numpy()
            assert int(sc.cpu()[0]) == n > cap
            assert np.array_equal(rc.cpu().numpy(), sc.cpu().numpy())
            assert r[: cap * 32].tobytes() == s[: cap * 32].tobytes()
            assert r[cap * 32:].tobytes() == s[cap * 32:].tobytes()  # the tail shards (whole in both modes)
    finally:
        rx.comm_destroy()


def test_empty_batch_exchange(dtabs):
    """An empty batch through the whole owner step (emurx_parse_route_dev with n = 0 writes zero
    counts, the exchange moves the counts and nothing to look up, k_lookup writes nothing), both
    transfer modes; then a one-frame batch on the same buffers, bit-exact."""
    import torch
    rx, o, shards = dtabs
    cap = 1024
    tcap = abi.tail_capacity(cap)
    send = torch.full((abi.lookup_region_bytes(cap, tcap),), 0xEE, dtype=torch.uint8, device="cuda")
    sc = torch.full((2,), -1, dtype=torch.int32, device="cuda")
    qcap = abi.queue_cap(256)
    ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda")
    tc = torch.empty(16, dtype=torch.int32, device="cuda")
    hi = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
    buf = torch.zeros(64, dtype=torch.uint8, device="cuda")
    desc = torch.zeros(8, dtype=torch.uint8, device="cuda")
    rx.parse_route_dev(buf, desc, 0, None, ql, qcap, tc, hi, 1, 0, cap, send, sc, tail_cap=tcap)
    _comm(rx)
    try:
        for payload in (False, True):
            recv = torch.full_like(send, 0x5A)
            rc = torch.full_like(sc, -1)
            out = torch.full((cap * 40,), 0xEE, dtype=torch.uint8, device="cuda")
            assert rx.exchange_dev(send, sc, recv, rc, cap, tcap, payload=payload) == 0
            rx.lookup_dev(recv, rc, 1, cap, out, tail_cap=tcap)
            torch.cuda.synchronize()
            assert rc.cpu().tolist() == [0, 0]
            assert (out.cpu().numpy() == 0xEE).all()  # nothing written
        w = shards[0]
        one = {"buf": w["buf"], "desc": w["desc"][:1]}
        got, rc, moved, s, r, c = owner_step(rx, one, cap, tcap, False)
        check_owner(o, one, got, rc, cap)
    finally:
        rx.comm_destroy()
