"""GPU: incremental table shipment, cross-stream ordering, and the owner-partitioned
classification, all bit-exact against the oracle.

* Mutations between batches reach the device as edited 64-byte blocks (no whole-table
  upload): every batch equals the oracle with the same mutations applied, and the device
  tables equal the host image (emurx_image_check).
* A batch in flight on one stream keeps the tables it was launched against while the next
  mutations ship on another stream (no half-old, half-new tables).
* Partitioned: G handles, each holding one Namespace partition; every shard is parsed and
  its lookup records packed per owner (emurx_parse_route_dev), the all-to-all is played on
  the device, and each owner resolves its records (emurx_lookup_dev).  The owners' output
  equals the oracle's records of every frame, grouped by owner, and
  the records with a Namespace equal the replicated path's routed records byte for byte;
  the transport flow decisions equal the oracle's.
"""
import numpy as np
import pytest

from emurx import abi, synth
from emurx import frames as F
from gpu_util import frame_tuples, rec_diff, run_dev

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rxmod(gpu_ok, oracle_built):
    from emurx.rx import RxPath
    return RxPath


def _check(rx, o, w):
    import pyoracle
    rec, qlist, qoff, hist = run_dev(rx, w["buf"], w["desc"])
    orec, oq, oqoff, ocnt = o.rx_batch(w["buf"], w["desc"])
    assert rec.tobytes() == orec.tobytes(), rec_diff(rec, orec)
    assert np.array_equal(qlist, oq) and np.array_equal(qoff, oqoff)
    from emurx.rx import hist_to_counters
    got, want = hist_to_counters(hist), pyoracle.counters_dict(ocnt)
    assert all(got[k] == want[k] for k in abi.PARSER_COUNTER_NAMES)
    return rec


def test_incremental_deltas(rxmod):
    """Rounds of 1 / 64 / 4096 mixed mutations (UpdateClientIpv4 / Ipv6 / DIpv6, AddClient,
    RemoveClient, plugin masks, RA prefixes, AddNs / RemoveNs) between batches; each batch
    bit-exact, the device tables equal to the image, and only deltas shipped."""
    import pyoracle
    n = 1 << 16
    w = synth.config_c(n, seed=0xDE17A)
    rx = rxmod(0, max_ns=4096 + 256, max_clients=65536 + 8192, max_frames=n)
    o = pyoracle.Oracle()
    rx.register_all()
    for t in (rx, o):
        synth.load_tables(w, t)
    _check(rx, o, w)
    base = rx.table_stats()
    c = w["clients"]
    rng = np.random.default_rng(17)
    spare = list(range(65536, 65536 + 8192))
    added = []
    for k in (1, 64, 4096, 64, 1):
        for j in range(k):
            op = int(rng.integers(0, 8))
            i = int(rng.integers(0, len(c["cid"])))
            cid, ns = int(c["cid"][i]), int(c["ns"][i])
            if op == 0:
                ip = bytes([172, 16, int(rng.integers(0, 256)), int(rng.integers(1, 255))])
                assert rx.client_update_ipv4(cid, ip) == o.client_update_ipv4(cid, ip)
            elif op == 1:
                ip = bytes([0x20, 1, 0xd, 0xb8, 9, 9] + [0] * 8 + [int(rng.integers(0, 256)), 1])
                assert rx.client_update_ipv6(cid, ip) == o.client_update_ipv6(cid, ip)
            elif op == 2:
                ip = bytes([0xfe, 0x80] + [0] * 8 + list(rng.integers(0, 256, 6, dtype=np.uint8)))
                assert rx.client_update_dipv6(cid, ip) == o.client_update_dipv6(cid, ip)
            elif op == 3 and spare:
                nc = spare.pop()
                mac = bytes([6, 1, nc >> 16 & 255, nc >> 8 & 255, nc & 255, 7])
                ip4 = bytes([11, nc >> 16 & 255, nc >> 8 & 255, nc & 255])
                assert rx.client_add(ns, nc, mac, ip4, None, None, 0x7FF) == o.client_add(ns, nc, mac, ip4, None, None, 0x7FF)
                added.append((ns, mac, nc))
            elif op == 4 and added:
                ns2, mac, nc = added.pop(int(rng.integers(0, len(added))))
                assert rx.client_remove(ns2, mac) == o.client_remove(ns2, mac) == 0
                spare.append(nc)
            elif op == 5:
                p = int(rng.integers(0, 1 << 11))
                assert rx.client_set_plugins(cid, p) == o.client_set_plugins(cid, p)
            elif op == 6:
                pre = bytes([0x20, 1, 0xd, 0xb8, 0, 0, 0, 0]) + bytes(8)
                assert rx.client_set_ra(cid, pre, 64) == o.client_set_ra(cid, pre, 64)
            else:
                key = F.tunnel_key(int(rng.integers(0, 4)), 0x81000000 | int(rng.integers(4090, 4095)), 0)
                nsid = 4096 + int(rng.integers(0, 256))
                r1, r2 = rx.ns_add(key, nsid, 0x7FF), o.ns_add(key, nsid, 0x7FF)
                assert r1 == r2
                if r1 != 0:
                    assert rx.ns_remove(key) == o.ns_remove(key)
        _check(rx, o, w)
        assert rx.image_check() == 0
    st = rx.table_stats()
    assert st["delta_blocks"] > base["delta_blocks"] + 1000
    assert st["whole_tables"] == base["whole_tables"]  # nothing outgrew its table


def test_mutation_while_batch_in_flight(rxmod):
    """An ingest batch runs on its slot stream while the tables change and the next batch is
    classified on another stream: the in-flight batch sees the old tables, the new one the
    new tables (the shipment waits for the in-flight reader by an event).  The batch is held
    in flight by a spin kernel queued on the slot stream ahead of it, long enough to outlast
    the mutations (checked: the slot stream has not drained when they end)."""
    import time

    import pyoracle
    import torch
    n = 1 << 17
    w = synth.config_c(n)
    rx = rxmod(0, max_ns=4096, max_clients=65536, max_frames=n)
    rx.register_all()
    o_old, o_new = pyoracle.Oracle(), pyoracle.Oracle()
    for t in (rx, o_old, o_new):
        synth.load_tables(w, t)
    fr = [w["buf"][d["off"]:d["off"] + d["len"]].tobytes() for d in w["desc"]]
    vp = [int(v) for v in w["desc"]["vport"]]
    msgs = [F.zmq_pack(fr[i:i + 64], vp[i:i + 64]) for i in range(0, n, 64)]
    total = sum(len(m) for m in msgs)
    buf = rx.ingest_buffer(0, total)
    tab = np.zeros(len(msgs), abi.MSG_DTYPE)
    at = 0
    for i, m in enumerate(msgs):
        buf[at:at + len(m)] = np.frombuffer(m, np.uint8)
        tab[i] = (at, len(m))
        at += len(m)
    # spin rate of torch.cuda._sleep (clock64 cycles per second), then a hold of ~2 s
    s_cal = torch.cuda.Stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s_cal):
        torch.cuda._sleep(1_000_000)  # the first launch loads the module: not part of the rate
        e0.record()
        torch.cuda._sleep(50_000_000)
        e1.record()
    e1.synchronize()
    per_s = 50_000_000 / (e0.elapsed_time(e1) / 1e3)
    rx.sync()  # the first shipment of whole tables waits for the device: done before the hold
    slot_st = torch.cuda.ExternalStream(rx.ingest_stream(0))
    with torch.cuda.stream(slot_st):
        torch.cuda._sleep(int(per_s * 2.0))
    rx.ingest_submit(0, tab)
    t0 = time.perf_counter()
    # mutate every client's IPv4 and half the MACs' plugins while the batch is in flight
    c = w["clients"]
    for i in range(0, len(c["cid"]), 2):
        cid = int(c["cid"][i])
        ip = bytes([172, 20, cid >> 8 & 255, cid & 255])
        assert rx.client_update_ipv4(cid, ip) == o_new.client_update_ipv4(cid, ip) == 0
        assert rx.client_set_plugins(cid, 0x0FF) == o_new.client_set_plugins(cid, 0x0FF) == 0
    assert not slot_st.query(), f"the batch finished during the mutations ({time.perf_counter() - t0:.2f} s)"
    rec_new = _check(rx, o_new, w)  # its own stream: the shipment orders after the ingest
    res = rx.ingest_wait(0)
    orec_old, _, _, _ = o_old.rx_batch(w["buf"], w["desc"])
    assert res["rec"].tobytes() == orec_old.tobytes(), rec_diff(res["rec"], orec_old)
    assert rec_new.tobytes() != orec_old.tobytes()


def _owners_by_key(rec, parts):
    """Owner of every record (the CTunnelKey its parse left)."""
    from emurx.rx import ns_owner
    out = np.full(len(rec), 0xFF, np.uint32)
    ok = np.arange(len(rec))
    k = np.stack([rec["vport"][ok].astype(np.uint64), rec["vlan0"][ok].astype(np.uint64),
                  rec["vlan1"][ok].astype(np.uint64)], 1)
    if len(ok):
        uk, inv = np.unique(k, axis=0, return_inverse=True)
        own = np.array([ns_owner(F.tunnel_key(int(a), int(b), int(c)), parts) for a, b, c in uk], np.uint32)
        out[ok] = own[inv.reshape(-1)]
    return out


def partitioned_vs_oracle(rxmod, shards, load, parts, flows=None, max_ns=4096, max_clients=65536):
    """Shards through the partitioned path (one handle per partition) and through the
    replicated classify + route, against the oracle.  load(target) fills a table target;
    flows(targets, orecs) may add transport state to every target."""
    import pyoracle
    import torch
    import route_ref
    from emurx import exchange as X
    from gpu_util import to_dev
    n = max(len(w["desc"]) for w in shards)
    o = pyoracle.Oracle()
    load(o)
    full = rxmod(0, max_ns=max_ns, max_clients=max_clients, max_frames=n)
    full.register_all()
    load(full)
    owners = []
    for p in range(parts):
        h = rxmod(0, max_ns=max_ns, max_clients=max_clients, max_frames=n)
        h.register_all()
        h.set_partition(parts, p)
        load(h)
        owners.append(h)
    if flows:
        flows([o, full] + owners, [o.rx_batch(w["buf"], w["desc"])[0] for w in shards])
    orecs = [o.rx_batch(w["buf"], w["desc"])[0] for w in shards]
    ts_full = full.table_stats()["table_bytes"]
    # power-of-two tables: 1/parts of the bytes for parts = 2, 4, 8; at most 2/parts otherwise
    assert max(h.table_stats()["table_bytes"] for h in owners) <= 2 * ts_full / parts + (1 << 16)

    cap = n  # no region can overflow (the edge / corpus frames share few tunnel keys)
    tcap = tail_cap_max(n)  # nor any tail shard (with flows, most tcp / udp heads carry a tuple)
    rb = abi.lookup_region_bytes(cap, tcap)
    send, cnt, rep_send, rep_cnt = [], [], [], []
    for s, w in enumerate(shards):
        m = len(w["desc"])
        buf, desc = to_dev(w["buf"]), to_dev(w["desc"])
        qcap = abi.queue_cap(m)
        mk = lambda: (torch.zeros(m * 32, dtype=torch.uint8, device="cuda"),  # noqa: E731
                      torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda"),
                      torch.empty(abi.ntiles(m) * 16, dtype=torch.int32, device="cuda"),
                      torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda"))
        rec, ql, tc, hi = mk()
        sd = torch.full((parts * rb,), 0xEE, dtype=torch.uint8, device="cuda")
        sc = torch.full((2 * parts,), -1, dtype=torch.int32, device="cuda")
        owners[s % parts].parse_route_dev(buf, desc, m, rec, ql, qcap, tc, hi, parts, s, cap, sd, sc, tail_cap=tcap)
        rrec, rql, rtc, rhi = mk()
        rsd = torch.full((parts * cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda")
        rsc = torch.full((parts,), -1, dtype=torch.int32, device="cuda")
        full.classify_route_dev(buf, desc, m, rrec, rql, qcap, rtc, rhi, parts, s, cap, rsd, rsc)
        torch.cuda.synchronize()
        # the source's parse-only records equal the oracle's parse (no lookups)
        pr = rec.cpu().numpy().view(abi.REC_DTYPE)
        assert (pr["ns_id"] == abi.ID_NONE).all()
        assert np.array_equal(pr["status"], orecs[s]["status"]) and np.array_equal(pr["l4"], orecs[s]["l4"])
        send.append(sd)
        cnt.append(sc.cpu().numpy())
        assert (cnt[-1][1::2] == 0).all(), cnt[-1]  # no tail shard overflowed
        rep_send.append(rsd)
        rep_cnt.append(rsc.cpu().numpy())
    for p in range(parts):
        # the all-to-all, played on the device: region s of owner p's receive buffer = region p of s
        recv = torch.empty(parts * rb, dtype=torch.uint8, device="cuda")
        rc = torch.tensor([int(cnt[s][2 * p + k]) for s in range(parts) for k in range(2)], dtype=torch.int32,
                          device="cuda")
        for s in range(parts):
            recv[s * rb:(s + 1) * rb] = send[s][p * rb:(p + 1) * rb]
        out = torch.full((parts * cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda")
        flow = torch.full((parts * cap,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
        owners[p].lookup_dev(recv, rc, parts, cap, out, flow, tail_cap=tcap)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(abi.ROUTE_REC_DTYPE).reshape(parts, cap)
        fl = flow.cpu().numpy().view(np.uint32).reshape(parts, cap)
        rep = [rep_send[s].cpu().numpy().view(abi.ROUTE_REC_DTYPE).reshape(parts, cap)[p, : rep_cnt[s][p]]
               for s in range(parts)]
        for s in range(parts):
            own = _owners_by_key(orecs[s], parts)
            sel = np.nonzero(own == p)[0]
            assert cnt[s][2 * p] == len(sel)
            want = np.zeros(len(sel), abi.ROUTE_REC_DTYPE)
            want["rec"], want["src_index"], want["src_rank"] = orecs[s][sel], sel, s
            g = got[s, : len(sel)]
            assert g.tobytes() == want.tobytes(), rec_diff(g["rec"], want["rec"])
            # the records with a Namespace = the replicated path's routed records
            hasns = g[g["rec"]["ns_id"] != abi.ID_NONE]
            assert hasns.tobytes() == rep[s].tobytes()
            assert hasns.tobytes() == route_ref.route(orecs[s], parts, s)[p].tobytes()
            wf = o.flows(shards[s]["buf"], shards[s]["desc"][sel], orecs[s][sel])
            assert np.array_equal(fl[s, : len(sel)], wf), (s, p)
    return o, orecs


def tail_cap_max(n):
    """Tail units per shard that no batch of n frames can overflow: every frame of every tile
    of the fullest shard with a 3-unit tail (an IPv6 c5tuplekey)."""
    return 768 * -(-abi.ntiles(n) // abi.TAIL_SHARDS)


def transport_state(shards):
    """flows(targets, orecs) for partitioned_vs_oracle: flows for a third of shard 0's TCP / UDP
    frames and listeners on a fifth of their destination ports, on every target."""
    def flows(targets, orecs):
        tup = frame_tuples(shards[0]["buf"], shards[0]["desc"], orecs[0])
        rng = np.random.default_rng(0xAB)
        idx = [i for i, t in enumerate(tup) if t is not None]
        for i in rng.choice(idx, len(idx) // 3, replace=False):
            cid = int(orecs[0][i]["client_id"])
            assert len({t.flow_add(cid, tup[i], int(i)) for t in targets}) == 1
        for i in rng.choice(idx, len(idx) // 5, replace=False):
            cid, t = int(orecs[0][i]["client_id"]), tup[i]
            dport = (t[10] << 8 | t[11]) if len(t) == 13 else (t[34] << 8 | t[35])
            proto = 6 if orecs[0][i]["proto"] == abi.CB_TCP else 17
            assert len({x.server_add(cid, dport, proto) for x in targets}) == 1
    return flows


@pytest.mark.parametrize("parts", [2, 3, 4])
def test_partitioned_lookups_equal_replicated(rxmod, parts):
    """Config C shards with bare SYNs, flows and listeners: records and flow decisions."""
    n = 40000
    shards = [synth.config_c(n, rank=s, syn=0.3) for s in range(parts)]
    o, orecs = partitioned_vs_oracle(rxmod, shards, lambda t: synth.load_tables(shards[0], t), parts,
                                     transport_state(shards))
    allf = o.flows(shards[0]["buf"], shards[0]["desc"], orecs[0])
    assert (allf <= abi.FLOW_ID_MAX).sum() > 1000 and (allf == abi.FLOW_NEW).sum() > 100


def test_partitioned_edge_and_fuzz_frames(rxmod):
    """Every return path of the parser (edge frames, the golden corpus, fuzzed frames: short
    frames, tag errors, PPPoE after a tag, three tags ...) through the partitioned path: the
    owner-count pass routes each frame by the CTunnelKey its full parse leaves."""
    import edge_frames as E
    from gpu_util import frames_tables, load_frame_tables
    from test_gpu_parity import corpus_frames, mutate
    base = corpus_frames() + [c[1] for c in E.cases()]
    rng = np.random.default_rng(0x9A27)
    shards = []
    for s in range(3):
        fr = mutate(base, rng, 12000) + base[s::3]
        buf, desc = F.pack_frames(fr, list(rng.integers(0, 4, len(fr))))
        shards.append(dict(buf=buf, desc=desc))
    ns, cl = frames_tables(base, vport=1)
    for v in (0, 2, 3):  # Namespaces on every vport the shards use
        n2, _ = frames_tables(base, vport=v)
        for k in n2:
            ns.setdefault(k, len(ns))
    partitioned_vs_oracle(rxmod, shards, lambda t: load_frame_tables([t], ns, cl), 3)


def test_capture_refused_before_enqueue(rxmod):
    """Every device entry point that ships tables or takes route scratch refuses a capturing
    stream with EMURX_EINVAL BEFORE it enqueues anything: the capture ends cleanly
    (no foreign event waited on, no scratch allocated inside it), replaying the graph changes
    nothing, and the same calls on the same stream work once it no longer captures."""
    import torch
    from emurx import exchange as X
    from gpu_util import to_dev
    n = 4096
    w = synth.config_c(n)
    rx = rxmod(0, max_ns=4096, max_clients=65536, max_frames=n)
    rx.register_all()
    synth.load_tables(w, rx)
    # table edits pending at capture time: a call that shipped them would enqueue k_apply
    c0 = int(w["clients"]["cid"][0])
    rx.client_update_ipv4(c0, bytes([10, 9, 8, 7]))
    buf, desc = to_dev(w["buf"]), to_dev(w["desc"])
    qcap = abi.queue_cap(n)
    rec = torch.full((n * 32,), 0xEE, dtype=torch.uint8, device="cuda")
    ql = torch.full((abi.NUM_QUEUES * qcap,), -1, dtype=torch.int32, device="cuda")
    tc = torch.full((abi.ntiles(n) * 16,), -1, dtype=torch.int32, device="cuda")
    hist = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
    cap = X.capacity(n, 2)
    send = torch.full((2 * abi.lookup_region_bytes(cap, abi.tail_capacity(cap)),), 0xEE, dtype=torch.uint8,
                      device="cuda")
    sc = torch.full((4,), -1, dtype=torch.int32, device="cuda")
    rsc = torch.full((2,), -1, dtype=torch.int32, device="cuda")
    out = torch.full((2 * cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda")
    rsend = torch.full((2 * cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda")
    calls = {
        "classify_dev": lambda s: rx.classify_dev(buf, desc, n, rec, ql, qcap, tc, hist, stream=s),
        "classify_route_dev": lambda s: rx.classify_route_dev(buf, desc, n, rec, ql, qcap, tc, hist, 2, 0, cap,
                                                              rsend, rsc, stream=s),
        "parse_route_dev": lambda s: rx.parse_route_dev(buf, desc, n, None, ql, qcap, tc, hist, 2, 0, cap, send, sc,
                                                        stream=s),
        "lookup_dev": lambda s: rx.lookup_dev(send, sc, 2, cap, out, stream=s),
        "route_dev": lambda s: rx.route_dev(rec, n, 2, 0, cap, rsend, rsc, stream=s),
    }
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    refused = {}
    with torch.cuda.graph(g, stream=s):
        for name, call in calls.items():
            try:
                call(s)
                refused[name] = False
            except RuntimeError as e:
                refused[name] = "invalid argument" in str(e)
    assert all(refused.values()), refused
    g.replay()
    torch.cuda.synchronize()
    assert (rec == 0xEE).all() and (ql == -1).all() and (tc == -1).all() and (sc == -1).all() and (rsc == -1).all()
    assert (send == 0xEE).all() and (out == 0xEE).all() and (rsend == 0xEE).all() and (hist == 0).all()
    # the edit is still pending and ships with the first real call; the outputs equal the oracle's
    import pyoracle
    from gpu_util import run_dev
    o = pyoracle.Oracle()
    synth.load_tables(w, o)
    o.client_update_ipv4(c0, bytes([10, 9, 8, 7]))
    want = o.rx_batch(w["buf"], w["desc"])[0]
    got = run_dev(rx, w["buf"], w["desc"])[0]
    assert got.tobytes() == want.tobytes(), rec_diff(got, want)
    with torch.cuda.stream(s):
        calls["parse_route_dev"](s)
    torch.cuda.synchronize()
    assert int(sc[0::2].sum()) == n and int(sc[1::2].sum()) == 0


@pytest.mark.timeout(900)
def test_partitioned_config_d_full_tables(rxmod):
    """Config D's full tables (32,768 Namespaces, 1,048,576 clients) split over 8
    partition handles on one GPU, as 8 ranks hold them: each of 8 shards (256K frames each, 2M
    in all) goes through parse_route_dev, the all-to-all is played on the device, and every
    owner's lookup_dev output -- records and flow decisions, with flows and listeners present
    -- is bit-exact against the oracle's classification (ns_ctx.go:262-329,
    thread_ctx.go:772-784), and its records with a Namespace equal the replicated route's."""
    parts = 8
    shards = [synth.config_d(1 << 18, rank=s) for s in range(parts)]
    partitioned_vs_oracle(rxmod, shards, lambda t: synth.load_tables(shards[0], t), parts,
                          transport_state(shards), max_ns=32768, max_clients=1 << 20)


def test_keyed_descriptors_route_the_same(rxmod):
    """Owner counts from descriptor owner keys (EMURX_DESC_KEYED, written by emurx_desc_keys_dev
    as the device framing walk writes them) instead of every frame's L2 header: config D frames
    routed to 8 owners give byte-equal send regions and counts with unkeyed, keyed and
    half-keyed descriptors (holes included), and the keys equal emurx_owner_key of the
    CTunnelKey the oracle's parse leaves."""
    import pyoracle
    import torch
    from emurx import exchange as X
    from gpu_util import owner_keys, to_dev
    n = 1 << 17
    w = synth.config_d(n, rank=3)
    desc = w["desc"].copy()
    holes = np.random.default_rng(4).random(n) < 0.01
    desc["pad"][holes] = abi.DESC_HOLE
    rx = rxmod(0, max_ns=4096, max_clients=65536, max_frames=n)
    buf = to_dev(w["buf"])
    dk = to_dev(desc)
    rx.desc_keys_dev(buf, dk, n)
    torch.cuda.synchronize()
    keyed = dk.cpu().numpy()[: n * 8].view(abi.DESC_DTYPE).copy()
    orec = pyoracle.Oracle().rx_batch(w["buf"], w["desc"])[0]
    assert np.array_equal(keyed["pad"][holes], np.full(holes.sum(), abi.DESC_HOLE, np.uint8))
    assert np.array_equal(keyed["pad"][~holes], owner_keys(orec[~holes]))
    plain = keyed.copy()
    plain["pad"][~holes] = 0
    half = keyed.copy()
    half["pad"][::2] = plain["pad"][::2]
    cap = X.capacity(n, 8)
    tcap = abi.tail_capacity(cap)
    rb = abi.lookup_region_bytes(cap, tcap)
    outs = []
    for d in (plain, keyed, half):
        qcap = abi.queue_cap(n)
        ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda")
        tc = torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device="cuda")
        hi = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
        sd = torch.full((8 * rb,), 0xEE, dtype=torch.uint8, device="cuda")
        sc = torch.full((16,), -1, dtype=torch.int32, device="cuda")
        rx.parse_route_dev(buf, to_dev(d), n, None, ql, qcap, tc, hi, 8, 0, cap, sd, sc, tail_cap=tcap)
        torch.cuda.synchronize()
        c, b = sc.cpu().numpy(), sd.cpu().numpy().reshape(8, rb)
        # the regions' records with their tails (the tail units' order within a shard is not
        # deterministic, what each head's tail holds is)
        outs.append((c, [X.lookup_records(b[k], int(c[2 * k]), cap, tcap).tobytes() for k in range(8)]))
    assert int(outs[0][0][0::2].sum()) == int((~holes).sum()) and (outs[0][0][1::2] == 0).all()
    # config D's ICMPv6 echo frames (5 %) carry a one-unit tail
    assert sum(len(r) for r in outs[0][1]) > 0
    for c, s in outs[1:]:
        assert np.array_equal(c, outs[0][0]) and s == outs[0][1]


def test_tail_shard_overflow(rxmod):
    """A tail shard too small for its units (emurx_parse_route_dev): the send counts report,
    per region, the units the fullest shard needed (> tail_cap), the heads whose tails did not
    fit carry EMURX_TAIL_NONE, and the owner's lookups over such a region stay in bounds.  With
    tail_cap grown to the reported need (exchange.grow_tail) the regions hold every record with
    its tail, equal to a run with room to spare."""
    import torch
    from emurx import exchange as X
    from gpu_util import to_dev
    n = 1 << 16
    w = synth.config_d(n, rank=1)
    rx = rxmod(0, max_ns=32768, max_clients=1 << 20, max_frames=n)
    rx.register_all()
    rx.set_partition(4, 0)
    synth.load_tables(w, rx)
    buf, desc = to_dev(w["buf"]), to_dev(w["desc"])
    rx.desc_keys_dev(buf, desc, n)
    cap = X.capacity(n, 4)
    qcap = abi.queue_cap(n)

    def route(tcap):
        rb = abi.lookup_region_bytes(cap, tcap)
        ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda")
        tc = torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device="cuda")
        hi = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
        sd = torch.full((4 * rb,), 0xEE, dtype=torch.uint8, device="cuda")
        sc = torch.full((8,), -1, dtype=torch.int32, device="cuda")
        rx.parse_route_dev(buf, desc, n, None, ql, qcap, tc, hi, 4, 1, cap, sd, sc, tail_cap=tcap)
        torch.cuda.synchronize()
        return sd, sc.cpu().numpy(), rb

    sd, c, rb = route(1)
    need = c[1::2]
    assert (need > 1).any(), c
    b = sd.cpu().numpy().reshape(4, rb)
    lost = 0
    for k in range(4):
        hd = b[k, : int(c[2 * k]) * 32].view(abi.LOOKUP_REC_DTYPE)
        u = X.tail_units(hd["w4"])
        assert u.sum() > 0
        lost += int((hd["x"][u > 0] == abi.TAIL_NONE).sum())
    assert lost > 0
    # the owner side over the overflowed regions: reads stay inside the buffer
    out = torch.empty(4 * cap * X.REC_BYTES, dtype=torch.uint8, device="cuda")
    rx.lookup_dev(sd, torch.from_numpy(c).cuda(), 4, cap, out, tail_cap=1)
    torch.cuda.synchronize()
    tcap = X.grow_tail(1, need)
    sd2, c2, rb2 = route(tcap)
    assert (c2[1::2] == 0).all() and np.array_equal(c2[0::2], c[0::2])
    sd3, c3, rb3 = route(tail_cap_max(n))
    b2, b3 = sd2.cpu().numpy().reshape(4, rb2), sd3.cpu().numpy().reshape(4, rb3)
    for k in range(4):
        r2 = X.lookup_records(b2[k], int(c2[2 * k]), cap, tcap)
        r3 = X.lookup_records(b3[k], int(c3[2 * k]), cap, tail_cap_max(n))
        assert r2.tobytes() == r3.tobytes()


def test_table_allocation_fallback():
    """A device table whose allocation fails is rebuilt at half its spread and allocated again
    (emurx_cfg) instead of failing emurx_open: with every allocation above 64 MiB
    refused (EMURX_DEBUG_TABLE_LIMIT), config D's tables (1M clients; the IPv4 / IPv6 / client
    info tables are 512 MiB at their default spread) still open, and a config-D batch classified
    on them equals the oracle."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    code = (
        "import sys; sys.path[:0] = ['tests', 'trex-emu_amd', 'oracle']\n"
        "import numpy as np, pyoracle\n"
        "from emurx import synth\n"
        "from emurx.rx import RxPath\n"
        "from gpu_util import run_dev, rec_diff\n"
        "w = synth.config_d(1 << 16)\n"
        "rx = RxPath(0, max_ns=32768, max_clients=1 << 20, max_frames=1 << 16); rx.register_all()\n"
        "synth.load_tables(w, rx)\n"
        "o = pyoracle.Oracle(); synth.load_tables(w, o)\n"
        "want = o.rx_batch(w['buf'], w['desc'])[0]\n"
        "got = run_dev(rx, w['buf'], w['desc'])[0]\n"
        "assert got.tobytes() == want.tobytes(), rec_diff(got, want)\n"
        "print('ok', rx.table_stats()['table_bytes'])\n")
    out = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=600,
                         env={**os.environ, "EMURX_DEBUG_TABLE_LIMIT": str(64 << 20)})
    assert out.returncode == 0 and "ok" in out.stdout, out.stderr[-3000:]
    assert int(out.stdout.split()[-1]) < (400 << 20)  # every table at most 64 MiB


def test_owner_flags_heads_without_tuple(rxmod):
    """a source whose handle has no TransportCtx routes tcp / udp heads without
    their c5tuplekey; an owner whose tables hold flows must not probe them with a zero tuple.
    Those frames' flow is EMURX_FLOW_UNKNOWN (the caller decides); every other flow decision
    and every record equal the oracle's."""
    import pyoracle
    import torch
    from emurx import exchange as X
    from gpu_util import to_dev
    n = 30000
    w = synth.config_c(n, rank=0, syn=0.3)
    o = pyoracle.Oracle()
    src = rxmod(0, max_ns=4096, max_clients=65536, max_frames=n)
    own = rxmod(0, max_ns=4096, max_clients=65536, max_frames=n)
    for t in (o, src, own):
        synth.load_tables(w, t)
        if t is not o:
            t.register_all()
    orec0 = o.rx_batch(w["buf"], w["desc"])[0]
    transport_state([w])([o, own], [orec0])  # flows and listeners on the owner only
    orec = o.rx_batch(w["buf"], w["desc"])[0]
    want_flow = o.flows(w["buf"], w["desc"], orec)
    cap, tcap = n, tail_cap_max(n)
    rb = abi.lookup_region_bytes(cap, tcap)
    buf, desc = to_dev(w["buf"]), to_dev(w["desc"])
    qcap = abi.queue_cap(n)
    ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda")
    tc = torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device="cuda")
    hi = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
    sd = torch.full((rb,), 0xEE, dtype=torch.uint8, device="cuda")
    sc = torch.full((2,), -1, dtype=torch.int32, device="cuda")
    src.parse_route_dev(buf, desc, n, None, ql, qcap, tc, hi, 1, 0, cap, sd, sc, tail_cap=tcap)
    out = torch.full((cap * X.REC_BYTES,), 0xEE, dtype=torch.uint8, device="cuda")
    flow = torch.full((cap,), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    own.lookup_dev(sd, sc, 1, cap, out, flow, tail_cap=tcap)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(abi.ROUTE_REC_DTYPE)[:n]
    assert got["rec"].tobytes() == orec.tobytes(), rec_diff(got["rec"], orec)
    fl = flow.cpu().numpy().view(np.uint32)[:n]
    decided = (want_flow != abi.FLOW_NONE) & (want_flow != abi.FLOW_NO_CTX)
    assert decided.sum() > 1000
    assert (fl[decided] == abi.FLOW_UNKNOWN).all()
    assert np.array_equal(fl[~decided], want_flow[~decided])
