"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle, bit-exact.

Records (all 32 bytes), per-callback queues, queue offsets and ParserStats counter deltas
must be identical on: the reference's KAT frames, every edge-case frame, the golden
capture corpus (with tables derived from it), seeded fuzz mutations of those, and the
BASELINE configs B / C / E (full 1M-frame sizes for B and C).
"""
import numpy as np
import pytest

import edge_frames as E
import kat_frames as K
from emurx import abi
from emurx import frames as F
from emurx import synth
from gpu_util import frames_tables, load_frame_tables, owner_keys, rec_diff, run_dev

pytestmark = pytest.mark.gpu
ALL = (1 << 12) - 1


@pytest.fixture(scope="module")
def rxmod(gpu_ok, oracle_built):
    from emurx.rx import RxPath
    return RxPath


def new_pair(RxPath, mask=ALL, **kw):
    import pyoracle
    rx = RxPath(0, max_ns=kw.get("max_ns", 4096), max_clients=kw.get("max_clients", 65536),
                max_frames=kw.get("max_frames", 1 << 20))
    rx.set_callbacks_mask(mask)
    return rx, pyoracle.Oracle(mask)


def check_batch(rx, o, buf, desc, classify=True):
    import pyoracle
    rec, qlist, qoff, hist = run_dev(rx, buf, desc, classify)
    if classify:
        orec, oq, oqoff, ocnt = o.rx_batch(buf, desc)
    else:
        orec = np.zeros(len(desc), dtype=abi.REC_DTYPE)
        for i, d in enumerate(desc):
            orec[i] = pyoracle.parse_only(buf[d["off"]:d["off"] + d["len"]].tobytes(), int(d["vport"]),
                                          rx.callbacks_mask)
        oq = oqoff = ocnt = None
    assert rec.tobytes() == orec.tobytes(), rec_diff(rec, orec)
    if classify:
        assert np.array_equal(qoff, oqoff), (qoff, oqoff)
        assert np.array_equal(qlist, oq)
        from emurx.rx import hist_to_counters
        got = hist_to_counters(hist)
        want = pyoracle.counters_dict(ocnt)
        for k in abi.PARSER_COUNTER_NAMES + ["ref_panic"]:
            assert got[k] == want[k], k
        assert int(hist[0::2].sum()) == len(desc)
    return rec


# ---- reference KATs (parser_test.go) through the host ZMQ entry point ------------------
@pytest.mark.parametrize("case,cb", [("test_parser_arp", "arp"), ("test_parser_arp1", "arp"),
                                     ("test_parser_icmp", "icmp"), ("test_parser_dhcp1", "dhcp"),
                                     ("test_parser_dot1q_ppp", "ppp"), ("test_parser_ppp", "ppp"),
                                     ("test_parser_ipv6_option", "icmpv6")])
def test_kat_on_rx_stream(rxmod, case, cb):
    f, vp = getattr(K, case)()
    rx, o = new_pair(rxmod, 0)
    rx.register(cb if cb not in ("icmpv6",) else "icmpv6")
    o.set_callbacks_mask(rx.callbacks_mask)
    msg = F.zmq_pack([f], [vp])
    rec, qlist, qoff, cnt = rx.on_rx_stream(msg)
    orec, oq, oqoff, ocnt = o.rx_stream(msg)
    assert rec.tobytes() == orec.tobytes(), rec_diff(rec, orec)
    assert np.array_equal(qoff, oqoff) and np.array_equal(qlist, oq)
    import pyoracle
    assert cnt.as_dict() == pyoracle.counters_dict(ocnt)
    if case == "test_parser_icmp":
        assert (rec[0]["l3"], rec[0]["l4"], rec[0]["l7"]) == (22, 42, 50)
    if case == "test_parser_arp":
        assert cnt.as_dict()["errToManyDot1q"] == 1


def test_dhcp_invalid_cs(rxmod):
    f, vp = K.test_parser_dhcp1(valid_ipcs=False)
    rx, o = new_pair(rxmod, 1 << abi.CB_DHCP)
    rec, _, _, cnt = rx.on_rx_stream(F.zmq_pack([f], [vp]))
    assert cnt.as_dict()["errIPv4cs"] == 1 and rec[0]["status"] == abi.ST["IPV4_CS"]


def test_checksum_kats(rxmod):
    rx, o = new_pair(rxmod)
    good4, _, _ = K.tcpip_ipv4_udp()
    good6, _, _ = K.tcpip_ipv6_udp_dstopts()
    bad4, _, _ = K.tcpip_ipv4_udp(K.IPV4_UDP_CSUM ^ 0x10)
    buf, desc = F.pack_frames([good4, good6, bad4])
    rec = check_batch(rx, o, buf, desc)
    assert list(rec["status"]) == [0, 0, abi.ST["UDP_CS"]]


# ---- every return path -------------------------------------------------------------------
@pytest.mark.parametrize("mask", [ALL, 0, ALL & ~(1 << abi.CB_PPP) & ~(1 << abi.CB_UDP)])
@pytest.mark.parametrize("classify", [True, False])
def test_edge_cases(rxmod, mask, classify):
    frames = [c[1] for c in E.cases()]
    rx, o = new_pair(rxmod, mask)
    ns, cl = frames_tables(frames, vport=0)
    load_frame_tables([rx, o], ns, cl)
    buf, desc = F.pack_frames(frames, [c[2] for c in E.cases()])
    check_batch(rx, o, buf, desc, classify)


def test_edge_cases_host_path(rxmod):
    frames = [c[1] for c in E.cases() if len(c[1]) <= 1600]
    rx, o = new_pair(rxmod)
    msg = F.zmq_pack(frames, [3] * len(frames))
    rec, qlist, qoff, cnt = rx.on_rx_stream(msg)
    orec, oq, oqoff, ocnt = o.rx_stream(msg)
    import pyoracle
    assert rec.tobytes() == orec.tobytes(), rec_diff(rec, orec)
    assert np.array_equal(qoff, oqoff) and np.array_equal(qlist, oq)
    assert cnt.as_dict() == pyoracle.counters_dict(ocnt)


# ---- golden corpus -----------------------------------------------------------------------
def corpus_frames():
    z = np.load(__import__("test_oracle_corpus").GOLD, allow_pickle=False)
    return [z["data"][o:o + l].tobytes() for o, l in zip(z["off"], z["len"])]


def test_corpus(rxmod):
    frames = corpus_frames()
    rx, o = new_pair(rxmod)
    ns, cl = frames_tables(frames)
    load_frame_tables([rx, o], ns, cl)
    # RA prefixes for a few clients (CLookupByIPv6LocalGlobal prefix rule)
    for cid in range(0, len(cl), 5):
        p = bytes([0x20, 0x01, 0x0D, 0xB8, 0, 0, 0, 0]) + bytes(8)
        assert rx.client_set_ra(cid, p, 64) == 0 and o.client_set_ra(cid, p, 64) == 0
    buf, desc = F.pack_frames(frames, [1] * len(frames))
    rec = check_batch(rx, o, buf, desc)
    lk = (rec["flags"] >> 4) & 7
    assert (lk == abi.LK["CLIENT"]).sum() > 1000     # the lookups are exercised
    # every answered rx frame reaches the callback of the plugin its capture simulates
    toc = __import__("test_oracle_corpus")
    z = np.load(toc.GOLD, allow_pickle=False)
    for i in np.nonzero(z["meta"] == 1)[0]:
        assert rec["status"][i] == 0 and abi.CB_NAMES[rec["proto"][i]] == toc.capture_callback(str(z["files"][z["src"][i]]))
    # reorder the descriptors: records follow descriptor order, not buffer order
    perm = np.random.default_rng(3).permutation(len(desc))
    check_batch(rx, o, buf, desc[perm])


def mutate(frames, rng, count):
    out = []
    for _ in range(count):
        f = bytearray(frames[int(rng.integers(0, len(frames)))])
        k = int(rng.integers(0, 5))
        if k == 0 and len(f):
            for _ in range(int(rng.integers(1, 4))):
                f[int(rng.integers(0, min(len(f), 80)))] = int(rng.integers(0, 256))
        elif k == 1 and len(f):
            f = f[: int(rng.integers(0, len(f) + 1))]
        elif k == 2 and len(f) > 20:
            i = int(rng.integers(12, min(len(f) - 1, 70)))
            f[i] ^= 1 << int(rng.integers(0, 8))
        elif k == 3:
            f += rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
        out.append(bytes(f))
    return out


def test_fuzz(rxmod):
    rng = np.random.default_rng(0xF022)
    base = corpus_frames() + [c[1] for c in E.cases()]
    frames = mutate(base, rng, 40000)
    rx, o = new_pair(rxmod)
    ns, cl = frames_tables(base)
    load_frame_tables([rx, o], ns, cl)
    buf, desc = F.pack_frames(frames, list(rng.integers(0, 4, len(frames))))
    rec = check_batch(rx, o, buf, desc)
    assert len(set(rec["status"].tolist())) >= 20     # most return paths hit


# ---- ragged / large / empty batches --------------------------------------------------------
def test_big_frames_global_path(rxmod):
    """Waves whose byte range exceeds the LDS stage take the global-memory path."""
    rng = np.random.default_rng(5)
    big = [E.udp4(1, 2, rng.integers(0, 256, int(s), dtype=np.uint8).tobytes())
           for s in rng.integers(1000, 9216 - 42, 150)]
    small = [c[1] for c in E.cases()]
    frames = big + small + big[:20]
    rx, o = new_pair(rxmod)
    buf, desc = F.pack_frames(frames)
    check_batch(rx, o, buf, desc)


def test_long_spans_across_the_window(rxmod):
    """Window-path waves (frames too wide for the stage) whose L4 spans start inside the
    lane's header window and end past it: TCP / UDP / ICMPv4 / ICMPv6 over IPv4 and IPv6,
    valid and corrupted checksums, all-zero ICMPv4 spans (Go's all-zero case), spans ending
    just past the window edge and frames at every 4-byte alignment within a 16-byte vector."""
    from emurx import frames as Fr
    rng = np.random.default_rng(17)
    frames = []
    for size in (130, 200, 600, 1500):
        body = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        frames.append(E.tcp4(body))
        frames.append(E.udp4(5000, 5001, body))
        frames.append(E.udp6(5000, 5001, body))
        frames.append(E.icmp6(128, body=body))
        frames.append(E.v4(1, Fr.icmp4(8, 0, 7, 9, body)))
        frames.append(E.v4(1, bytes(8 + size)))  # all-zero ICMPv4 span: errIcmpv4Cse
        for good in (E.tcp4(body), E.udp6(5000, 5001, body), E.icmp6(128, body=body)):
            bad = bytearray(good)
            bad[-1 - (size % 7)] ^= 0x40  # a payload byte past the window
            frames.append(bytes(bad))
            bad = bytearray(good)
            bad[70] ^= 0x01  # a byte inside the window
            frames.append(bytes(bad))
    frames.append(E.udp4(1, 2, bytes(9000)))  # keeps the waves on the window path
    rx, o = new_pair(rxmod)
    for rot in range(4):  # frame starts at 4, 8, 12, 0 mod 16 (4-byte ZMQ gap per frame)
        fr = frames[rot:] + frames[:rot]
        buf, desc = F.pack_frames(fr)
        check_batch(rx, o, buf, desc)


def test_empty_and_single(rxmod):
    rx, o = new_pair(rxmod)
    rec, qlist, qoff, hist = run_dev(rx, np.zeros(64, np.uint8), np.zeros(0, abi.DESC_DTYPE))
    assert len(rec) == 0 and (qoff == 0).all() and hist.sum() == 0
    buf, desc = F.pack_frames([E.udp4(1, 2)])
    check_batch(rx, o, buf, desc)


def test_ragged_sizes(rxmod):
    """Batch sizes that are not multiples of the wave / workgroup."""
    rx, o = new_pair(rxmod)
    frames = [c[1] for c in E.cases()]
    for n in (1, 63, 64, 65, 255, 256, 257, 1000):
        sel = [frames[i % len(frames)] for i in range(n)]
        buf, desc = F.pack_frames(sel)
        check_batch(rx, o, buf, desc)


def test_queue_region_capacity(rxmod):
    """A per-queue region larger than the minimum leaves the segments in place; one smaller
    than ceil(n / TILE) * TILE is refused before any launch."""
    rx, o = new_pair(rxmod)
    frames = [c[1] for c in E.cases()]
    sel = [frames[i % len(frames)] for i in range(700)]
    buf, desc = F.pack_frames(sel)
    orec, oq, oqoff, _ = o.rx_batch(buf, desc)
    rec, qlist, qoff, _ = run_dev(rx, buf, desc, qcap=abi.queue_cap(700) + 3 * abi.QUEUE_TILE + 5)
    assert rec.tobytes() == orec.tobytes()
    assert np.array_equal(qoff, oqoff) and np.array_equal(qlist, oq)
    with pytest.raises(RuntimeError, match="invalid argument"):
        run_dev(rx, buf, desc, qcap=700)


# ---- table mutations between batches -------------------------------------------------------
def test_table_updates(rxmod):
    w = synth.config_c(8192)
    rx, o = new_pair(rxmod)
    synth.load_tables(w, rx)
    synth.load_tables(w, o)
    check_batch(rx, o, w["buf"], w["desc"])
    c = w["clients"]
    rng = np.random.default_rng(11)
    for i in rng.choice(len(c["cid"]), 300, replace=False):
        ns_id, cid, mac = int(c["ns"][i]), int(c["cid"][i]), c["mac"][i].tobytes()
        op = int(rng.integers(0, 4))
        if op == 0:
            assert rx.client_remove(ns_id, mac) == o.client_remove(ns_id, mac)
        elif op == 1:
            ip = bytes([172, 16, int(rng.integers(0, 256)), int(rng.integers(1, 255))])
            assert rx.client_update_ipv4(cid, ip) == o.client_update_ipv4(cid, ip)
        elif op == 2:
            assert rx.client_set_plugins(cid, 0) == o.client_set_plugins(cid, 0)
        else:
            assert rx.ns_set_plugins(ns_id, 1 << abi.CB_ARP) == o.ns_set_plugins(ns_id, 1 << abi.CB_ARP)
    check_batch(rx, o, w["buf"], w["desc"])


# ---- BASELINE configs -------------------------------------------------------------------
@pytest.mark.parametrize("cfg,n", [("config_b", 1 << 20), ("config_c", 1 << 20), ("config_e", 1 << 20)])
def test_configs(rxmod, cfg, n):
    w = getattr(synth, cfg)(n)
    rx, o = new_pair(rxmod)
    synth.load_tables(w, rx)
    synth.load_tables(w, o)
    rec = check_batch(rx, o, w["buf"], w["desc"])
    if cfg == "config_b":
        assert (rec["status"] == 0).all() and (rec["proto"] == abi.CB_UDP).all()
        assert (rec["ns_id"] == 0).all() and (rec["client_id"] == 0).all()


def test_config_d_full_tables(rxmod):
    """Config D at its full table sizes: 32,768 Namespaces and 1,048,576 Clients (max_clients
    1M, the 2M-bucket IPv6 table), one GPU's 2M-frame shard.  Records, queues and every
    counter bit-exact against the oracle (CThreadCtx.GetNs thread_ctx.go:777-784,
    CNSCtx.CLookupBy* ns_ctx.go:262-329); then the device Namespace-owner packing of those
    records for 8 partitions against the host restatement."""
    import torch
    import route_ref
    from emurx import exchange as X
    n = 1 << 21
    w = synth.config_d(n)
    assert len(w["ns"]) == 32768 and len(w["clients"]["cid"]) == 1 << 20
    rx, o = new_pair(rxmod, max_ns=32768, max_clients=1 << 20, max_frames=n)
    synth.load_tables(w, rx)
    synth.load_tables(w, o)
    rec = check_batch(rx, o, w["buf"], w["desc"])
    lk = (rec["flags"] >> 4) & 7
    assert (lk == abi.LK["CLIENT"]).sum() > 0.9 * n and (lk == abi.LK["NO_NS"]).sum() > 0.005 * n
    assert (lk == abi.LK["NO_CLIENT"]).sum() > 0.005 * n
    d_rec = torch.from_numpy(rec.view(np.uint8).copy()).cuda()
    for parts, me in ((8, 3), (2, 0)):
        cap = X.capacity(n, parts)
        send = torch.full((parts * cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda")
        cnt = torch.full((parts,), -1, dtype=torch.int32, device="cuda")
        rx.route_dev(d_rec, n, parts, me, cap, send, cnt)
        torch.cuda.synchronize()
        got = cnt.cpu().numpy()
        want = route_ref.route(rec, parts, me)
        assert list(got) == [len(x) for x in want] and (got <= cap).all()
        sreg = send.cpu().numpy().view(abi.ROUTE_REC_DTYPE).reshape(parts, cap)
        for d in range(parts):
            assert sreg[d, : got[d]].tobytes() == want[d].tobytes(), d


# ---- the two LDS staging slabs (emurx_launch_batch) ----------------------------------------
@pytest.mark.parametrize("mode", ["wide", "narrow"])
def test_stage_sizes(rxmod, monkeypatch, mode):
    monkeypatch.setenv("EMURX_STAGE", mode)
    for cfg, n in (("config_c", 1 << 17), ("config_e", 1 << 15), ("config_b", 1 << 16)):
        w = getattr(synth, cfg)(n)
        rx, o = new_pair(rxmod)
        synth.load_tables(w, rx)
        synth.load_tables(w, o)
        check_batch(rx, o, w["buf"], w["desc"])
        assert rx.last_stage() == (7168 if mode == "wide" else 6144)


def _spaced(w, stride):
    """The same frames, `stride` bytes apart: every wave spans 64 * stride bytes."""
    d = w["desc"]
    buf = np.zeros(len(d) * stride + 64, np.uint8)
    nd = d.copy()
    for i in range(len(d)):
        o, n = int(d["off"][i]), int(d["len"][i])
        buf[i * stride:i * stride + n] = w["buf"][o:o + n]
    nd["off"] = np.arange(len(d), dtype=np.uint32) * stride
    return buf, nd


def test_stage_auto_choice(rxmod, monkeypatch):
    """Waves spanning 6-7 KiB keep the wide slab; 64-byte frames switch to the narrow one
    after one launch of feedback.  Parity holds either way."""
    monkeypatch.delenv("EMURX_STAGE", raising=False)
    w = synth.config_b(1 << 16)
    rx, o = new_pair(rxmod)
    synth.load_tables(w, rx)
    synth.load_tables(w, o)
    sbuf, sdesc = _spaced(w, 100)  # 6,400 B per wave
    seq = []
    # launches 1, 9, 17, 25 copy their samples back; each batch here is synchronised, so
    # launches 2, 10, 18, 26 decide from them (launch 10 from launch 9's dense frames)
    for buf, desc in [(sbuf, sdesc)] * 8 + [(w["buf"], w["desc"])] * 8 + [(sbuf, sdesc)] * 16:
        check_batch(rx, o, buf, desc)
        seq.append(rx.last_stage())
    assert seq == [7168] * 9 + [6144] * 8 + [7168] * 15, seq


def test_kernel_timing_stride(rxmod):
    """emurx_set_timing(slots, stride): every stride-th batch carries an event pair."""
    rx, _ = new_pair(rxmod)
    frames = [c[1] for c in E.cases()]
    buf, desc = F.pack_frames(frames)
    rx.set_timing(16, 2)
    for _ in range(6):
        run_dev(rx, buf, desc)
    t = rx.kernel_times()
    assert len(t) == 3 and (t > 0).all()
    assert len(rx.kernel_times()) == 0
    rx.set_timing(0)


# ---- Namespace-partitioned exchange: device packing (emurx_route_dev) ---------------------
@pytest.mark.parametrize("n_parts,my_rank", [(1, 0), (2, 1), (3, 2), (8, 5)])
def test_route_dev(rxmod, n_parts, my_rank):
    """Send regions packed on the device == the host restatement, over config C records
    (unknown Namespaces stay local); includes a batch size that is not a tile multiple."""
    import torch
    import route_ref
    from emurx import exchange as X
    n = 20000 + 77
    w = synth.config_c(n, rank=my_rank)
    rx, o = new_pair(rxmod)
    synth.load_tables(w, rx)
    synth.load_tables(w, o)
    orec, _, _, _ = o.rx_batch(w["buf"], w["desc"])
    rec = torch.from_numpy(orec.view(np.uint8).copy()).cuda()
    cap = X.capacity(n, n_parts)
    send = torch.full((n_parts * cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda")
    cnt = torch.full((n_parts,), -1, dtype=torch.int32, device="cuda")
    rx.route_dev(rec, n, n_parts, my_rank, cap, send, cnt)
    torch.cuda.synchronize()
    got_cnt = cnt.cpu().numpy()
    s = send.cpu().numpy().view(abi.ROUTE_REC_DTYPE).reshape(n_parts, cap)
    want = route_ref.route(orec, n_parts, my_rank)
    assert list(got_cnt) == [len(x) for x in want]
    for d in range(n_parts):
        assert s[d, : got_cnt[d]].tobytes() == want[d].tobytes(), d
    assert sum(got_cnt) == int((orec["ns_id"] != abi.ID_NONE).sum())


def _classify_to(rx, w, rec, n):
    import torch
    from emurx import abi as A
    buf = torch.from_numpy(w["buf"]).cuda()
    desc = torch.from_numpy(w["desc"].view(np.uint8).copy()).cuda()
    qcap = A.queue_cap(n)
    qlist = torch.empty(A.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda")
    tile_cnt = torch.empty(A.ntiles(n) * 16, dtype=torch.int32, device="cuda")
    hist = torch.zeros(A.HIST_SHARDS * 2 * A.HIST_BINS, dtype=torch.int64, device="cuda")
    rx.classify_dev(buf, desc, n, rec, qlist, qcap, tile_cnt, hist)
    torch.cuda.synchronize()


def _dev_out(n):
    import torch
    from emurx import abi as A
    qcap = A.queue_cap(n)
    return dict(rec=torch.zeros(max(n, 1) * 32, dtype=torch.uint8, device="cuda"),
                qlist=torch.empty(A.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda"), qcap=qcap,
                tile_cnt=torch.empty(max(A.ntiles(n), 1) * 16, dtype=torch.int32, device="cuda"),
                hist=torch.zeros(A.HIST_SHARDS * 2 * A.HIST_BINS, dtype=torch.int64, device="cuda"))


@pytest.mark.parametrize("n_parts,my_rank", [(1, 0), (2, 1), (8, 3)])
def test_classify_route_dev(rxmod, n_parts, my_rank):
    """emurx_classify_route_dev (the owner counts taken inside k_rx) gives the oracle's
    records and the send regions of the host restatement, the same as classify_dev followed
    by route_dev; back-to-back batches of different sizes reuse the route scratch."""
    import torch
    import route_ref
    from emurx import exchange as X
    rx, o = new_pair(rxmod)
    for n, seed in ((30000 + 5, 0), (777, 1), (30000 + 5, 2)):
        w = synth.config_c(n, rank=my_rank + 10 * seed)
        if seed == 0:
            synth.load_tables(w, rx)
            synth.load_tables(w, o)
        orec, _, _, _ = o.rx_batch(w["buf"], w["desc"])
        buf = torch.from_numpy(w["buf"]).cuda()
        desc = torch.from_numpy(w["desc"].view(np.uint8).copy()).cuda()
        cap = X.capacity(n, n_parts)
        d = _dev_out(n)
        send = torch.full((n_parts * cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda")
        cnt = torch.full((n_parts,), -1, dtype=torch.int32, device="cuda")
        rx.classify_route_dev(buf, desc, n, d["rec"], d["qlist"], d["qcap"], d["tile_cnt"], d["hist"], n_parts,
                              my_rank, cap, send, cnt)
        torch.cuda.synchronize()
        assert d["rec"].cpu().numpy()[: n * 32].view(abi.REC_DTYPE).tobytes() == orec.tobytes()
        want = route_ref.route(orec, n_parts, my_rank)
        c = cnt.cpu().numpy()
        assert list(c) == [len(x) for x in want]
        sreg = send.cpu().numpy().view(abi.ROUTE_REC_DTYPE).reshape(n_parts, cap)
        for k in range(n_parts):
            assert sreg[k, : c[k]].tobytes() == want[k].tobytes(), k


def test_routes_on_many_streams(rxmod):
    """Batches classified and routed on six streams at once (more streams than route scratch
    sets, so sets change hands behind events): every batch's records and send regions equal
    the oracle's and the host restatement's."""
    import torch
    import route_ref
    from emurx import exchange as X
    rx, o = new_pair(rxmod)
    n_parts, my_rank = 4, 2
    jobs = []
    for j in range(12):
        n = 20000 + 3 * j
        w = synth.config_c(n, rank=40 + j)
        if j == 0:
            synth.load_tables(w, rx)
            synth.load_tables(w, o)
        cap = X.capacity(n, n_parts)
        d = _dev_out(n)
        jobs.append(dict(w=w, n=n, cap=cap, d=d, buf=torch.from_numpy(w["buf"]).cuda(),
                         desc=torch.from_numpy(w["desc"].view(np.uint8).copy()).cuda(),
                         send=torch.full((n_parts * cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda"),
                         cnt=torch.full((n_parts,), -1, dtype=torch.int32, device="cuda")))
    streams = [torch.cuda.Stream() for _ in range(6)]
    torch.cuda.synchronize()
    for j, b in enumerate(jobs):
        d = b["d"]
        rx.classify_route_dev(b["buf"], b["desc"], b["n"], d["rec"], d["qlist"], d["qcap"], d["tile_cnt"], d["hist"],
                              n_parts, my_rank, b["cap"], b["send"], b["cnt"], stream=streams[j % len(streams)])
    torch.cuda.synchronize()
    for j, b in enumerate(jobs):
        orec, _, _, _ = o.rx_batch(b["w"]["buf"], b["w"]["desc"])
        assert b["d"]["rec"].cpu().numpy()[: b["n"] * 32].view(abi.REC_DTYPE).tobytes() == orec.tobytes(), j
        want = route_ref.route(orec, n_parts, my_rank)
        c = b["cnt"].cpu().numpy()
        assert list(c) == [len(x) for x in want], j
        sreg = b["send"].cpu().numpy().view(abi.ROUTE_REC_DTYPE).reshape(n_parts, b["cap"])
        for k in range(n_parts):
            assert sreg[k, : c[k]].tobytes() == want[k].tobytes(), (j, k)


def test_max_batch(rxmod):
    """The largest batch one call takes: 16,777,216 descriptors (65,536 tiles: config D's whole
    batch on one GPU, and the route scan's limit of 1,024 groups of 64 tiles), 1M config-C
    frames each referenced 16 times.  Records, queues and counters against the oracle over the
    same descriptors; then classify + route to 8 owners against the host restatement."""
    import torch
    import route_ref
    from emurx import exchange as X
    n1, rep = 1 << 20, 16
    w = synth.config_c(n1, rank=3)
    desc = np.tile(w["desc"], rep)
    n = len(desc)
    rx, o = new_pair(rxmod, max_frames=n)
    synth.load_tables(w, rx)
    synth.load_tables(w, o)
    rec = check_batch(rx, o, w["buf"], desc)
    n_parts, my_rank = 8, 5
    own = np.tile(route_ref.owners(rec[:n1], n_parts), rep)
    want = np.bincount(own[own != 0xFF], minlength=n_parts)
    tb, td = torch.from_numpy(w["buf"]).cuda(), torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    d = _dev_out(n)
    cap = X.capacity(n, n_parts, slack=1.06)
    for attempt in range(2):  # the fair share + 6 % overflows here: true counts, then grow and redo
        send = torch.empty(n_parts * cap * X.REC_BYTES, dtype=torch.uint8, device="cuda")
        cnt = torch.full((n_parts,), -1, dtype=torch.int32, device="cuda")
        rx.classify_route_dev(tb, td, n, d["rec"], d["qlist"], d["qcap"], d["tile_cnt"], d["hist"], n_parts, my_rank,
                              cap, send, cnt)
        torch.cuda.synchronize()
        c = cnt.cpu().numpy()
        assert list(c) == list(want)
        if (c <= cap).all():
            break
        cap = X.grow(cap, c)
    assert (c <= cap).all()
    sreg = send.cpu().numpy().view(abi.ROUTE_REC_DTYPE).reshape(n_parts, cap)
    for k in range(n_parts):
        idx = np.nonzero(own == k)[0]
        assert c[k] == len(idx), k
        got = sreg[k, : c[k]]
        assert np.array_equal(got["src_index"], idx.astype(got["src_index"].dtype)), k
        assert got["rec"].tobytes() == rec[idx].tobytes(), k
        assert (got["src_rank"] == my_rank).all()


def _hole_rec():
    h = np.zeros(1, abi.REC_DTYPE)
    h["ns_id"] = h["client_id"] = abi.ID_NONE
    h["proto"], h["status"] = abi.CB_NONE, abi.ST_HOLE
    return h[0]


def test_holes_records_and_route(rxmod):
    """Empty descriptor slots (EMURX_DESC_HOLE) get a hole record (no Namespace, status
    EMURX_ST_HOLE), no queue entry and no count; the route, standalone and fused, skips them."""
    import torch
    import route_ref
    from emurx import exchange as X
    n = 20000
    w = synth.config_c(n)
    rx, o = new_pair(rxmod)
    synth.load_tables(w, rx)
    synth.load_tables(w, o)
    rng = np.random.default_rng(44)
    holes = np.sort(rng.choice(n, n // 20, replace=False))
    keep = np.setdiff1d(np.arange(n), holes)
    desc = w["desc"].copy()
    desc["pad"][holes] = abi.DESC_HOLE
    orec, oq, oqoff, ocnt = o.rx_batch(w["buf"], w["desc"][keep])
    want = np.zeros(n, abi.REC_DTYPE)
    want[keep] = orec
    want[holes] = _hole_rec()
    rec, qlist, qoff, hist = run_dev(rx, w["buf"], desc)
    assert rec.tobytes() == want.tobytes(), rec_diff(rec, want)
    assert np.array_equal(qlist, keep[oq].astype(np.uint32)) and np.array_equal(qoff, oqoff)
    assert int(hist[0::2].sum()) == len(keep)
    buf = torch.from_numpy(w["buf"]).cuda()
    ddesc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    drec = torch.from_numpy(want.view(np.uint8).copy()).cuda()
    wroute = route_ref.route(want, 4, 1)
    for fused in (False, True):
        cap = X.capacity(n, 4)
        send = torch.full((4 * cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda")
        cnt = torch.full((4,), -1, dtype=torch.int32, device="cuda")
        if fused:
            d = _dev_out(n)
            rx.classify_route_dev(buf, ddesc, n, d["rec"], d["qlist"], d["qcap"], d["tile_cnt"], d["hist"], 4, 1, cap,
                                  send, cnt)
        else:
            rx.route_dev(drec, n, 4, 1, cap, send, cnt)
        torch.cuda.synchronize()
        c = cnt.cpu().numpy()
        assert list(c) == [len(x) for x in wroute], fused
        sreg = send.cpu().numpy().view(abi.ROUTE_REC_DTYPE).reshape(4, cap)
        for k in range(4):
            assert sreg[k, : c[k]].tobytes() == wroute[k].tobytes(), (fused, k)


def test_route_dev_overflow(rxmod):
    """A region smaller than its records: the count reports the true total, nothing is
    written past the region."""
    import torch
    import route_ref
    n = 5000
    w = synth.config_c(n)
    rx, o = new_pair(rxmod)
    synth.load_tables(w, o)
    orec, _, _, _ = o.rx_batch(w["buf"], w["desc"])
    rec = torch.from_numpy(orec.view(np.uint8).copy()).cuda()
    cap = 1000
    send = torch.full((2 * cap * 40 + 4096,), 0xEE, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(2, dtype=torch.int32, device="cuda")
    rx.route_dev(rec, n, 2, 0, cap, send, cnt)
    torch.cuda.synchronize()
    want = route_ref.route(orec, 2, 0)
    assert list(cnt.cpu().numpy()) == [len(x) for x in want] and min(len(x) for x in want) > cap
    s = send.cpu().numpy()
    assert (s[2 * cap * 40:] == 0xEE).all()
    r = s[: 2 * cap * 40].view(abi.ROUTE_REC_DTYPE).reshape(2, cap)
    for d in range(2):
        assert r[d].tobytes() == want[d][:cap].tobytes()


# ---- batched host ingest: device framing walk + k_rx + device queue packing ---------------
def oracle_messages(o, msgs):
    """What the ingest of `msgs` must return: OnRxStream per message (the oracle's), frames
    numbered across the messages, queues as a stable partition of the whole batch."""
    import collections
    import pyoracle
    recs, nfr, status, tot = [], [], [], collections.Counter()
    for m in msgs:
        rec, _, _, cnt = o.rx_stream(m)
        recs.append(rec)
        nfr.append(len(rec))
        status.append(pyoracle.zmq_descriptors(m)[2])
        tot.update(pyoracle.counters_dict(cnt))
    rec = np.concatenate(recs) if recs else np.zeros(0, abi.REC_DTYPE)
    q = np.where(rec["status"] == 0, rec["proto"], abi.Q_DROP).astype(np.int64)
    qoff = np.zeros(abi.NUM_QUEUES + 1, np.uint32)
    qoff[1:] = np.cumsum(np.bincount(q, minlength=abi.NUM_QUEUES))
    return rec, np.argsort(q, kind="stable").astype(np.uint32), qoff, nfr, status, dict(tot)


def place_messages(rx, slot, msgs, rng):
    """Write messages into the slot's pinned buffer at unaligned offsets -> MSG_DTYPE table."""
    gaps = rng.integers(0, 8, len(msgs))
    buf = rx.ingest_buffer(slot, sum(len(m) for m in msgs) + int(gaps.sum()))
    tab = np.zeros(len(msgs), abi.MSG_DTYPE)
    at = 0
    for i, (m, g) in enumerate(zip(msgs, gaps)):
        at += int(g)
        buf[at:at + len(m)] = np.frombuffer(m, np.uint8)
        tab[i] = (at, len(m))
        at += len(m)
    return tab


def check_ingest(res, o, msgs, tab):
    import pyoracle
    rec, qlist, qoff, nfr, status, cnt = oracle_messages(o, msgs)
    assert res["rec"].tobytes() == rec.tobytes(), rec_diff(res["rec"], rec)
    assert np.array_equal(res["qoff"], qoff) and np.array_equal(res["qlist"], qlist)
    assert list(res["msg_frames"]) == nfr and list(res["msg_status"]) == status
    want_desc = [pyoracle.zmq_descriptors(m)[1].copy() for m in msgs]
    for d, t in zip(want_desc, tab):
        d["off"] += t["off"]
    want_desc = np.concatenate(want_desc) if want_desc else np.zeros(0, abi.DESC_DTYPE)
    # the device walk keys every descriptor (EMURX_DESC_KEYED): the owner key of the
    # CTunnelKey the frame's parse leaves; the host walk's descriptors carry none
    got = res["desc"].copy()
    keys = got["pad"].copy()
    got["pad"] = 0
    assert got.tobytes() == want_desc.tobytes()
    assert np.array_equal(keys, owner_keys(rec)), "descriptor owner keys"
    assert res["counters"] == cnt


def test_zmq_walk_dev(rxmod):
    """The framing walk alone on device-resident messages (emurx_zmq_walk_dev): valid, truncated,
    corrupted, over-announcing, oversized and > 64 KiB messages at unaligned offsets give, slot
    for slot, the host walk's descriptors (holes where a message announced more than it
    carried), its per-message frame counts and status, and the owner key of the CTunnelKey
    each frame's parse leaves; EMURX_WALK_NO_KEYS leaves the pad byte 0 and changes nothing
    else (OnRxStream veth_zmq.go:277-320)."""
    import pyoracle
    import test_abi
    import torch
    from gpu_util import to_dev
    rng = np.random.default_rng(0x3A1C)
    frames = [c[1] for c in E.cases()] + corpus_frames()[:2000]
    msgs = test_abi._rand_msgs(rng, 150)
    for i in range(0, len(frames), 64):
        msgs.append(F.zmq_pack(frames[i:i + 64], list(rng.integers(0, 4, len(frames[i:i + 64])))))
    msgs = [msgs[i] for i in rng.permutation(len(msgs))]
    gaps = rng.integers(0, 8, len(msgs))
    buf = np.zeros(sum(len(m) for m in msgs) + int(gaps.sum()) + 64, np.uint8)
    tab = np.zeros(len(msgs), abi.MSG_DTYPE)
    base = [0]
    at = 0
    for i, (m, g) in enumerate(zip(msgs, gaps)):
        at += int(g)
        buf[at:at + len(m)] = np.frombuffer(m, np.uint8)
        tab[i] = (at, len(m))
        at += len(m)
        ann = (int.from_bytes(m[2:4], "big") if len(m) >= 4 and m[:2] == b"\xbe\xef" else 0)
        base.append(base[-1] + min(ann, (min(len(m), 65536) - 4) // 4 if len(m) >= 4 else 0))
    nmsg, ns = len(msgs), base[-1]
    ctl = np.concatenate([tab.view(np.uint32).reshape(-1), np.array(base, np.uint32)])
    d_buf, d_ctl = to_dev(buf), to_dev(ctl)
    out = {}
    for keys in (True, False):
        d_desc = torch.full((ns * 8,), 0x5A, dtype=torch.uint8, device="cuda")
        d_stat = torch.full((nmsg,), -1, dtype=torch.int32, device="cuda")
        rx = rxmod(0, max_ns=16, max_clients=16, max_frames=max(ns, 1))
        rx.zmq_walk_dev(d_buf, d_ctl, nmsg, d_desc, d_stat, keys=keys)
        torch.cuda.synchronize()
        out[keys] = (d_desc.cpu().numpy().view(abi.DESC_DTYPE), d_stat.cpu().numpy().view(np.uint32))
        rx.close()
    o = pyoracle.Oracle()
    for m in range(nmsg):
        _, want, err = pyoracle.zmq_descriptors(msgs[m])
        want = want.copy()
        want["off"] += tab[m]["off"]
        for keys in (True, False):
            d, st = out[keys]
            seg = d[base[m]:base[m + 1]]
            nf = int(st[m] & 0xFFFFFF)
            assert nf == len(want) and int(st[m] >> 24) == err, (m, nf, len(want), st[m] >> 24, err)
            got = seg[:nf].copy()
            k = got["pad"].copy()
            got["pad"] = 0
            assert got.tobytes() == want.tobytes(), m
            if keys:
                recs = o.rx_stream(msgs[m])[0]
                assert np.array_equal(k, owner_keys(recs)), m
            else:
                assert (k == 0).all(), m
            assert (seg["pad"][nf:] == abi.DESC_HOLE).all(), m


@pytest.mark.parametrize("small", ["1", "0"])
def test_ingest_small_limits(rxmod, small, monkeypatch):
    """The one-launch ingest at its limits (256 tiles since round 5): 256 tiles of
    slots exactly (1,024 messages of 64 frames: also the message limit), 257 tiles (1,009
    messages of 65 frames: the pipeline), 1,024 messages of 16 frames, and a tile whose staged
    messages take exactly EMURX_SMALL_LDS / 16 vectors (one launch) or one vector more (the
    pipeline): which path ran (emurx_ingest_result.one_launch), and results equal to the
    oracle's either way (the sizing of s_mk / s_base / s_off and the host's small_fits agree
    exactly)."""
    monkeypatch.setenv("EMURX_INGEST_SMALL", small)
    w = synth.config_b(1 << 14, seed=0xB17)
    frames = [w["buf"][d["off"]:d["off"] + d["len"]].tobytes() for d in w["desc"]]
    rx, o = new_pair(rxmod, max_frames=1 << 17)
    for t in (rx, o):
        synth.load_tables(w, t)
    rng = np.random.default_rng(5)

    def run(msgs, offs=None):
        if offs is None:
            tab = place_messages(rx, 0, msgs, rng)
        else:  # exact offsets (the LDS budget depends on each message's offset mod 16)
            buf = rx.ingest_buffer(0, offs[-1] + len(msgs[-1]) + 64)
            tab = np.zeros(len(msgs), abi.MSG_DTYPE)
            for i, (m, at) in enumerate(zip(msgs, offs)):
                buf[at:at + len(m)] = np.frombuffer(m, np.uint8)
                tab[i] = (at, len(m))
        rx.ingest_submit(0, tab)
        res = rx.ingest_wait(0)
        check_ingest(res, o, msgs, tab)
        return res["one_launch"]

    assert abi.SMALL_TILES == 256 and abi.SMALL_MSGS == 1024
    nf = len(frames)
    big = [F.zmq_pack([frames[(64 * i + j) % nf] for j in range(64)]) for i in range(1024)]  # 65,536 slots = 256 tiles
    assert run(big) == (small == "1")
    over = [F.zmq_pack([frames[(65 * i + j) % nf] for j in range(65)]) for i in range(1009)]  # 65,585 slots: 257 tiles
    assert not run(over)
    many = [F.zmq_pack(frames[16 * i:16 * i + 16]) for i in range(1024)]  # 1,024 messages
    assert run(many) == (small == "1")
    # tile 1 = one message of 255 frames (40,804 bytes at a 16-aligned offset: 2,553 vectors with
    # the 2 of slack) + one of 1 frame at offset mod 16 = 4: 7 vectors (66 bytes) = 2,560 =
    # EMURX_SMALL_LDS / 16, or 8 (80 bytes): one over
    pad = lambda f, n: f + bytes(n - len(f))  # noqa: E731  (bytes past IPv4 totlen: Go ignores them)
    m1 = F.zmq_pack([pad(frames[300 + i], 156) for i in range(255)])
    assert len(m1) == 40804
    head = [F.zmq_pack(frames[64 * i:64 * i + 64]) for i in range(4)]  # tile 0
    for flen, fits in ((64, True), (72, False)):
        m2 = F.zmq_pack([pad(frames[900], flen)])
        msgs = head + [m1, m2]
        offs, at = [], 0
        for m in head:
            offs.append(at)
            at += len(m)
        at = (at + 15) & ~15
        offs += [at, at + len(m1)]
        assert (offs[-1] & 15) == 4
        v = (((offs[-1] & 15) + len(m2) + 15) >> 4) + 2 + (len(m1) + 15) // 16 + 2
        assert v == abi.SMALL_LDS // 16 + (0 if fits else 1), v
        assert run(msgs, offs) == (small == "1" and fits), (flen, fits)


def test_ingest_messages(rxmod):
    """Valid, truncated, corrupted, over-announcing, oversized and > 64 KiB messages in one
    batch at unaligned offsets: records, descriptors, queues, per-message frame counts and
    status, and every counter equal the oracle's OnRxStream per message."""
    import test_abi
    rng = np.random.default_rng(0x16E5)
    frames = [c[1] for c in E.cases()] + corpus_frames()[:3000]
    msgs = test_abi._rand_msgs(rng, 200)
    for i in range(0, len(frames), 57):
        msgs.append(F.zmq_pack(frames[i:i + 57], [1] * len(frames[i:i + 57])))
    msgs = [msgs[i] for i in rng.permutation(len(msgs))]
    rx, o = new_pair(rxmod)
    ns, cl = frames_tables(frames, vport=1)
    load_frame_tables([rx, o], ns, cl)
    tab = place_messages(rx, 0, msgs, rng)
    rx.ingest_submit(0, tab)
    res = rx.ingest_wait(0)
    assert res["n"] > 3000 and (res["msg_status"] != 0).sum() > 50   # holes and aborts exercised
    check_ingest(res, o, msgs, tab)


@pytest.mark.parametrize("small", ["1", "0"])
def test_ingest_small_batches(rxmod, small, monkeypatch):
    """Batches that fit the one-launch path (k_ingest_small: <= 64 tiles, <= 1024 messages, each
    tile's messages within its LDS budget) and, with EMURX_INGEST_SMALL=0, the same batches
    through the multi-launch pipeline: records, descriptors (owner keys included), queues,
    per-message frame counts and status, and every counter equal the oracle's OnRxStream per
    message.  1 to 300 messages of config C frames and hostile messages (truncated, corrupted,
    over-announcing, empty), so that messages span tiles, some carry no slot and the last
    tile's status words include the trailing empty messages; then the limits themselves
    (test_ingest_small_limits)."""
    import test_abi
    monkeypatch.setenv("EMURX_INGEST_SMALL", small)
    rng = np.random.default_rng(0x5A11 + int(small))
    w = synth.config_c(8192, seed=0xC0DE)
    frames = [w["buf"][d["off"]:d["off"] + d["len"]].tobytes() for d in w["desc"]]
    rx, o = new_pair(rxmod)
    for t in (rx, o):
        synth.load_tables(w, t)
    k = 0
    for nm in (1, 2, 3, 5, 16, 17, 40, 64, 300):
        msgs = []
        for j in range(nm):
            per = int(rng.integers(1, 65 if nm < 300 else 24))
            msgs.append(F.zmq_pack(frames[k:k + per], [int(v) for v in w["desc"]["vport"][k:k + per]]))
            k = (k + per) % (len(frames) - 64)
        msgs += test_abi._rand_msgs(rng, 4)[:4] + [b""]
        msgs = [msgs[i] for i in rng.permutation(len(msgs))]
        tab = place_messages(rx, 0, msgs, rng)
        rx.ingest_submit(0, tab)
        res = rx.ingest_wait(0)
        check_ingest(res, o, msgs, tab)
    # runs of equal-sized frames (the walk speculates one stride per round): whole runs, a run
    # broken by one other size, a corrupted header mid-run, a length past the message, an
    # over-announcing header, a run longer than a wave's 64 guesses
    by_len = {}
    for f in frames:
        by_len.setdefault(len(f), []).append(f)
    runs = sorted(by_len.values(), key=len, reverse=True)
    vp = lambda c: [int(rng.integers(0, 4)) for _ in range(c)]
    for nm in (1, 2, 4, 8):
        msgs = []
        for j in range(nm):
            run = runs[j % 3]
            per = int(rng.integers(1, 65)) if j % 2 else 64
            fr = [run[i % len(run)] for i in range(per)]
            kind = (j + nm) % 6
            if kind == 1 and per > 3:
                fr[per // 2] = runs[(j + 1) % 3][0]
            m = bytearray(F.zmq_pack(fr, vp(len(fr))))
            at = 4 + sum(4 + len(x) for x in fr[: len(fr) // 2])
            if kind == 2:
                m[at] = 0x00                                  # magic of the middle frame
            elif kind == 3:
                m[at + 2:at + 4] = (0xFFF0).to_bytes(2, "big")  # a length past the message
            elif kind == 4:
                m[2:4] = (len(fr) + 7).to_bytes(2, "big")      # announces more than it carries
            msgs.append(bytes(m))
        if nm == 8:
            run = runs[0]
            msgs.append(F.zmq_pack([run[i % len(run)] for i in range(150)], vp(150)))
        tab = place_messages(rx, 0, msgs, rng)
        rx.ingest_submit(0, tab)
        check_ingest(rx.ingest_wait(0), o, msgs, tab)


@pytest.mark.parametrize("spin_us", ["0", "200"])
def test_ingest_small_degraded(rxmod, spin_us, monkeypatch):
    """the one-launch ingest's degraded pack (a workgroup that stops
    waiting for the other tiles marks the batch, and the last workgroup packs the queues from
    device scratch).  EMURX_INGEST_SPIN_US=0 takes it on every multi-tile batch; the default
    bound (200 us + 0.1 ns per message byte) on an idle GPU takes the direct pack.  Records, descriptors, queues,
    per-message status and every counter equal the oracle either way, from 2 tiles to the
    256-tile limit, with hostile messages mixed in (OnRxStream veth_zmq.go:277-320)."""
    import test_abi
    monkeypatch.setenv("EMURX_INGEST_SMALL", "1")
    monkeypatch.setenv("EMURX_INGEST_SPIN_US", spin_us)
    rng = np.random.default_rng(0xDE6 + int(spin_us))
    w = synth.config_c(16384, seed=0xC0DF)
    frames = [w["buf"][d["off"]:d["off"] + d["len"]].tobytes() for d in w["desc"]]
    vp = [int(v) for v in w["desc"]["vport"]]
    rx, o = new_pair(rxmod, max_frames=1 << 17)
    for t in (rx, o):
        synth.load_tables(w, t)
    nf = len(frames) - 64
    direct = 0  # multi-tile batches packed directly under the default bound
    for nm in (1, 9, 40, 300, 1024):
        msgs = []
        k = int(rng.integers(0, nf))
        for _ in range(nm - (4 if nm > 8 else 0)):
            per = 64 if nm == 1024 else int(rng.integers(1, 65))
            msgs.append(F.zmq_pack([frames[(k + j) % nf] for j in range(per)], [vp[(k + j) % nf] for j in range(per)]))
            k = (k + per) % nf
        if nm > 8:
            msgs += test_abi._rand_msgs(rng, 4)[:4]
        msgs = [msgs[i] for i in rng.permutation(len(msgs))]
        tab = place_messages(rx, 0, msgs, rng)
        rx.ingest_submit(0, tab)
        res = rx.ingest_wait(0)
        check_ingest(res, o, msgs, tab)
        assert res["one_launch"], nm
        if nm != 9:  # one tile (nm = 1: at most 64 frames), or many (> 1,000 frames)
            multi = nm > 1
            assert res["n"] > abi.QUEUE_TILE or not multi
            if spin_us == "0" or not multi:
                assert res["degraded"] == (multi and spin_us == "0"), (nm, res["n"], res["degraded"])
            else:  # a time bound: one batch slowed by the box may degrade (same results)
                direct += not res["degraded"]
    if spin_us != "0":
        assert direct >= 2, direct  # of the three multi-tile batches


def test_ingest_two_slots_pipelined(rxmod):
    """Config C frames as 64-frame messages, three batches over the two slots with one batch
    always in flight while the next is staged; each equals the oracle."""
    rng = np.random.default_rng(9)
    w = synth.config_c(30000)
    rx, o = new_pair(rxmod)
    synth.load_tables(w, rx)
    synth.load_tables(w, o)
    fr = [w["buf"][d["off"]:d["off"] + d["len"]].tobytes() for d in w["desc"]]
    vp = [int(v) for v in w["desc"]["vport"]]
    msgs = [F.zmq_pack(fr[i:i + 64], vp[i:i + 64]) for i in range(0, len(fr), 64)]
    parts = [msgs[:150], msgs[150:300], msgs[300:]]
    tabs = [None, None]
    tabs[0] = place_messages(rx, 0, parts[0], rng)
    rx.ingest_submit(0, tabs[0])
    tabs[1] = place_messages(rx, 1, parts[1], rng)
    rx.ingest_submit(1, tabs[1])
    check_ingest(rx.ingest_wait(0), o, parts[0], tabs[0])
    t2 = place_messages(rx, 0, parts[2], rng)
    rx.ingest_submit(0, t2)
    check_ingest(rx.ingest_wait(1), o, parts[1], tabs[1])
    check_ingest(rx.ingest_wait(0), o, parts[2], t2)


def test_ingest_limits(rxmod):
    """No messages; a batch that could announce more frames than max_frames (ENOSPC, nothing
    enqueued); wait without a submit (EINVAL); a message outside the buffer (EINVAL)."""
    from emurx.rx import RxPath
    rx = RxPath(0, max_ns=16, max_clients=16, max_frames=100)
    rx.ingest_buffer(0, 64)
    rx.ingest_submit(0, np.zeros(0, abi.MSG_DTYPE))
    res = rx.ingest_wait(0)
    assert res["n"] == 0 and res["counters"]["rx_batch"] == 0 and (res["qoff"] == 0).all()
    m = F.zmq_pack([bytes(60)] * 101)
    buf = rx.ingest_buffer(0, len(m))
    buf[:] = np.frombuffer(m, np.uint8)
    with pytest.raises(RuntimeError, match="output buffer too small"):
        rx.ingest_submit(0, [(0, len(m))])
    with pytest.raises(RuntimeError, match="invalid argument"):
        rx.ingest_wait(0)
    with pytest.raises(RuntimeError, match="invalid argument"):
        rx.ingest_submit(0, [(8, len(m))])
    m = F.zmq_pack([bytes(60)] * 100)
    buf[: len(m)] = np.frombuffer(m, np.uint8)
    rx.ingest_submit(0, [(0, len(m))])
    res = rx.ingest_wait(0)
    assert res["n"] == 100 and res["counters"]["errL3ProtoUnsupported"] == 100


# ---- tx-side checksum generation (emurx_tx_checksum_dev) ---------------------------------
def run_tx(rx, buf, d, skew=0):
    """tx checksums of frames `buf` on the device; skew: d_frames `skew` bytes past a 16-byte
    boundary (the C-ABI takes any frames pointer)."""
    import torch
    from gpu_util import to_dev
    tb, td = to_dev(np.concatenate([np.full(skew, 0x77, np.uint8), buf])), to_dev(d)
    st = torch.full((max(len(d), 1),), 0xEE, dtype=torch.uint8, device="cuda")
    rx.tx_checksum_dev(tb[skew:], td, len(d), st)
    torch.cuda.synchronize()
    out = tb.cpu().numpy()
    assert (out[:skew] == 0x77).all()
    return out[skew: skew + len(buf)], st.cpu().numpy()[: len(d)]


def test_tx_checksum_reference_captures(rxmod):
    """Every checksum the reference's send paths wrote into the golden captures (TCP/UDP over
    IPv4 and IPv6, ICMP, ICMPv6 incl. MLD behind hop-by-hop, IGMP's 24-byte IPv4 header),
    recomputed on the GPU from the cleared fields: byte-identical."""
    import tx_util
    buf, d, want, zeroed = tx_util.corpus_tx_cases()
    rx, _ = new_pair(rxmod)
    got, st = run_tx(rx, zeroed, d)
    assert (st == abi.TX_OK).all()
    assert got.tobytes() == want.tobytes()


def test_tx_checksum_unaligned_frames(rxmod):
    """d_frames at every offset past a 16-byte boundary (the staged path aligned
    its LDS rows relative to d_frames, not to the absolute address): the checksums of the
    reference captures are byte-identical for each, and nothing before d_frames is written."""
    import tx_util
    buf, d, want, zeroed = tx_util.corpus_tx_cases()
    rx, _ = new_pair(rxmod)
    for skew in (1, 2, 3, 5, 8, 13, 15):
        got, st = run_tx(rx, zeroed, d, skew)
        assert (st == abi.TX_OK).all(), skew
        assert got.tobytes() == want.tobytes(), skew


def test_tx_checksum_unaligned_first_frame_at_zero(rxmod):
    """a staged wave whose first frame starts at d_frames + 0..15 with
    d_frames itself unaligned.  The slab's aligned start must come from the absolute address
    (frame offset lo - skew wrapped below zero and pointed ~4 GiB past the buffer).  Small
    frames packed with no header, so wave 0's first frame is at offset 0; every skew 1..15,
    against the oracle, nothing before d_frames written."""
    import pyoracle
    from emurx import frames as F
    rng = np.random.default_rng(0xA1)
    n = 300  # several waves, each one staged (about 64 x 60 B < the 6 KiB slab)
    frames = [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in rng.integers(40, 80, n)]
    buf, desc = F.pack_frames(frames, header=0)
    assert int(desc["off"][0]) == 0
    d = np.zeros(n, abi.TX_DESC_DTYPE)
    d["off"], d["len"] = desc["off"], desc["len"]
    d["l3"] = 14
    d["l4"] = 34
    d["ops"] = abi.TX_IPV4_HDR | (rng.choice([abi.TX_L4_TCP4, abi.TX_L4_UDP4, abi.TX_L4_ICMP4], n) << abi.TX_L4_SHIFT)
    want, wst = pyoracle.tx_checksum(buf, d)
    rx, _ = new_pair(rxmod)
    for skew in range(1, 16):
        got, st = run_tx(rx, buf, d, skew)
        assert np.array_equal(st, wst), skew
        assert got.tobytes() == np.asarray(want).tobytes(), skew


def test_tx_checksum_fuzz_vs_oracle(rxmod):
    """Random frames, ops, offsets (overlapping spans, odd alignments, out of range, IPv6
    next-header override) against the oracle's sequential Go restatement."""
    import pyoracle
    rng = np.random.default_rng(0x7C5)
    n = 20000
    lens = rng.integers(0, 1600, n)
    frames = [rng.integers(0, 256, int(l), dtype=np.uint8).tobytes() for l in lens]
    for k in range(0, n, 7):  # some all-zero frames: the 0xffff / 0 ends of tcpipChecksum
        frames[k] = bytes(len(frames[k]))
    from emurx import frames as F
    buf, desc = F.pack_frames(frames, header=int(rng.integers(0, 4)))
    d = np.zeros(n, abi.TX_DESC_DTYPE)
    d["off"], d["len"] = desc["off"], desc["len"]
    d["l3"] = rng.integers(0, 60, n)
    d["l4"] = np.where(rng.random(n) < 0.8, d["l3"] + rng.choice([20, 24, 40, 48], n), rng.integers(0, 80, n))
    d["osize"] = rng.integers(0, 16, n)
    d["ops"] = rng.integers(0, 4, n) | (rng.integers(0, 8, n) << abi.TX_L4_SHIFT)
    d["nh"] = rng.integers(0, 256, n)
    rx, _ = new_pair(rxmod)
    got, st = run_tx(rx, buf, d)
    want, wst = pyoracle.tx_checksum(buf, d)
    assert np.array_equal(st, wst)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (len(bad), bad[:10])
    assert (wst == abi.TX_OK).sum() > n // 3 and (wst == abi.TX_RANGE).sum() > n // 10


# ---- transport flow decision (TransportCtx.handleRxPacket) -------------------------------
def test_transport_flows(rxmod):
    """Per-frame flow outcome (flow id / no TransportCtx / no SYN / no listener / new) equals the
    oracle's restatement over IPv4 and IPv6 TCP/UDP traffic with flows, listeners and
    TransportCtx marks on a random subset; then after flow, listener and client removals."""
    from gpu_util import frame_tuples
    rng = np.random.default_rng(0xF10)
    w = synth.config_c(30000, syn=0.3)
    rx, o = new_pair(rxmod)
    synth.load_tables(w, rx)
    synth.load_tables(w, o)
    buf, desc = w["buf"], w["desc"]
    orec, _, _, _ = o.rx_batch(buf, desc)
    tup = frame_tuples(buf, desc, orec)
    # no TransportCtx anywhere yet: every tcp/udp frame reaching a client is NO_CTX
    rec0, _, _, _, flow0 = run_dev(rx, buf, desc, flows=True)
    assert np.array_equal(flow0, o.flows(buf, desc, orec)) and (flow0 == abi.FLOW_NO_CTX).sum() > 10000
    idx = np.array([i for i, t in enumerate(tup) if t is not None])
    assert len(idx) > 15000
    for i in rng.choice(idx, len(idx) * 2 // 5, replace=False):
        cid = int(orec[i]["client_id"])
        assert rx.flow_add(cid, tup[i], int(i)) == o.flow_add(cid, tup[i], int(i))
    for i in rng.choice(idx, len(idx) // 4, replace=False):
        cid, t = int(orec[i]["client_id"]), tup[i]
        dport = (t[10] << 8 | t[11]) if len(t) == 13 else (t[34] << 8 | t[35])
        proto = 6 if orec[i]["proto"] == abi.CB_TCP else 17
        assert rx.server_add(cid, dport, proto) == o.server_add(cid, dport, proto)
    cids = np.unique(orec["client_id"][idx])
    for c in rng.choice(cids, len(cids) // 5, replace=False):
        v = int(rng.integers(0, 2))
        assert rx.client_set_transport(int(c), v) == o.client_set_transport(int(c), v) == 0

    def check():
        rec, _, _, _, flow = run_dev(rx, buf, desc, flows=True)
        orec2, _, _, _ = o.rx_batch(buf, desc)
        assert rec.tobytes() == orec2.tobytes(), rec_diff(rec, orec2)
        want = o.flows(buf, desc, orec2)
        bad = np.nonzero(flow != want)[0]
        assert len(bad) == 0, (len(bad), [(int(flow[b]), int(want[b])) for b in bad[:5]])
        return want

    want = check()
    for code in (abi.FLOW_NONE, abi.FLOW_NO_CTX, abi.FLOW_NO_SYN, abi.FLOW_NO_SERVER, abi.FLOW_NEW):
        assert (want == code).sum() > 50, hex(code)
    assert (want <= abi.FLOW_ID_MAX).sum() > 5000
    for i in rng.choice(idx, 2000, replace=False):
        cid = int(orec[i]["client_id"])
        assert rx.flow_remove(cid, tup[i]) == o.flow_remove(cid, tup[i])
    c = w["clients"]
    for k in rng.choice(len(c["cid"]), 200, replace=False):
        assert rx.client_remove(int(c["ns"][k]), c["mac"][k].tobytes()) == \
            o.client_remove(int(c["ns"][k]), c["mac"][k].tobytes())
    check()


# ---- lookup outcomes the reference's plugin simulations vouch for (tests/sim_envs.py) --------
def test_reference_simulations(rxmod):
    import sim_envs as S
    toc = __import__("test_oracle_corpus")
    z = np.load(toc.GOLD, allow_pickle=False)
    for capture, env, lk, cid, _ in S.CASES:
        fr = S.rx_frames(z, capture)
        rx, o = new_pair(rxmod, max_ns=16, max_clients=64, max_frames=1024)
        S.load_env(rx, env)
        S.load_env(o, env)
        buf, desc = F.pack_frames(fr, [1] * len(fr))
        rec = check_batch(rx, o, buf, desc)
        assert (rec["status"] == 0).all() and (rec["ns_id"] == 0).all(), capture
        assert (((rec["flags"] >> 4) & 7) == abi.LK[lk]).all(), capture
        assert (rec["client_id"] == S.expected_clients(fr, cid)).all(), capture
        rx.close()


# ---- flow decisions the reference's transport simulations vouch for (tests/transport_sims.py) ----
def test_transport_reference_sims(rxmod):
    """Every frame of the 17 tcp / udp captures (IPv4 and IPv6) through the GPU path as its peer's
    rx frame: records and flow decisions bit-exact with the oracle, and the flow decision equal to
    the outcome the capture implies -- NEW for the accepted SYN / first datagram, the server's or
    the client's flow for the frames that a later frame of the receiver shows found it -- before
    and after the server's flow exists; then NO_SYN / NO_SERVER with the flow / listener removed."""
    import pyoracle
    import transport_sims as T
    from test_reference_transport_sims import OUT, corpus
    z = corpus()
    for capture in T.CAPTURES:
        fr = T.frames(z, capture)
        proto, ckey, skey, accept, exp = T.plan(capture, fr)
        buf, desc = F.pack_frames(fr, [1] * len(fr))
        rx = rxmod(0, max_ns=16, max_clients=16, max_frames=1024)
        rx.register_all()
        o = pyoracle.Oracle()
        for t in (rx, o):
            T.load(t, proto, ckey, abi.PLUG_ALL)

        def both():
            rec, _, _, _, flow = run_dev(rx, buf, desc, flows=True)
            orec, _, _, _ = o.rx_batch(buf, desc)
            assert rec.tobytes() == orec.tobytes(), (capture, rec_diff(rec, orec))
            assert np.array_equal(flow, o.flows(buf, desc, orec)), capture
            return flow
        flow = both()
        for i, _, k, s in exp:
            if s == "before":
                assert flow[i] == OUT[k], (capture, i, k, hex(int(flow[i])))
        for t in (rx, o):
            assert t.flow_add(T.SERVER["cid"], skey, T.SERVER_FLOW) == 0
        flow = both()
        for i, _, k, s in exp:
            if s == "after":
                assert flow[i] == OUT[k], (capture, i, k, hex(int(flow[i])))
        for t in (rx, o):
            assert t.server_remove(T.SERVER["cid"], T.PORT, proto) == 0 and t.flow_remove(T.SERVER["cid"], skey) == 0
        flow = both()
        assert flow[accept] == abi.FLOW_NO_SERVER
        if proto == 6:
            assert any(flow[i] == abi.FLOW_NO_SYN for i, f in enumerate(fr) if T.to_server(f) and not T.is_syn(f))
        rx.close()
