"""Namespace-partitioned exchange protocol on CPU (gloo, world size 2).

Each rank classifies its own shard with the oracle, packs the records into the owners' send
regions with the host restatement of emurx_route_dev (tests/route_ref.py), and runs the same
emurx.exchange.exchange() the GPU bench uses (RCCL there, gloo here).  Every rank must end up
with exactly the records of the Namespaces it owns, from both shards, in (source rank, frame)
order.  The device packing kernel is checked against the same restatement in
tests/test_gpu_parity.py.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

from emurx import abi, synth

ROOT = Path(__file__).resolve().parent.parent
N_FRAMES = 3000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def shard_records(rank):
    import pyoracle
    w = synth.config_c(N_FRAMES, rank=rank)
    o = pyoracle.Oracle()
    synth.load_tables(w, o)
    rec, _, _, _ = o.rx_batch(w["buf"], w["desc"])
    return rec


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "trex-emu_amd"), str(ROOT / "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import route_ref
    from emurx import exchange as X
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        recs = [shard_records(r) for r in range(world)]
        cap = X.capacity(N_FRAMES, world)
        regions = route_ref.route(recs[rank], world, rank)
        send = np.zeros((world, cap), abi.ROUTE_REC_DTYPE)
        for d, rr in enumerate(regions):
            send[d, : len(rr)] = rr
        cnt = np.array([len(rr) for rr in regions], np.int32)
        recv, recv_count = X.exchange(torch.from_numpy(send.view(np.uint8).reshape(-1).copy()),
                                      torch.from_numpy(cnt), cap * X.REC_BYTES)
        got = X.received(recv.numpy(), recv_count.numpy(), cap)
        want = np.concatenate([route_ref.route(recs[s], world, s)[rank] for s in range(world)])
        ok = got.tobytes() == want.tobytes() and len(got) > 0
        owners = route_ref.owners(got["rec"], world)
        ok = ok and bool((owners == rank).all())
        # two exchanges in flight at once (the bench's overlapped steps): started A then B,
        # finished B then A; A equals the blocking exchange, B (no records) delivers none
        send_t = torch.from_numpy(send.view(np.uint8).reshape(-1).copy())
        junk = torch.from_numpy(np.random.default_rng(rank).integers(0, 256, send_t.numel(), dtype=np.uint8))
        pa = X.exchange_start(send_t, torch.from_numpy(cnt), cap * X.REC_BYTES)
        pb = X.exchange_start(junk, torch.zeros(world, dtype=torch.int32), cap * X.REC_BYTES)
        rb, cb = X.exchange_finish(pb)
        ra, ca = X.exchange_finish(pa)
        ok = ok and bool((cb == 0).all()) and torch.equal(ca, recv_count)
        ok = ok and X.received(ra.numpy(), ca.numpy(), cap).tobytes() == got.tobytes()
        # the payload-sized exchange (counts, then only the valid records): junk past every
        # region's count stays home; the records are the same; the bytes sent are the payload
        jsend = junk.numpy().reshape(world, cap * X.REC_BYTES).copy()
        sv = send.view(np.uint8).reshape(world, -1)
        for d in range(world):
            jsend[d, : cnt[d] * X.REC_BYTES] = sv[d, : cnt[d] * X.REC_BYTES]
        rv, cv, moved = X.exchange_v(torch.from_numpy(jsend.reshape(-1)), torch.from_numpy(cnt), cap * X.REC_BYTES,
                                     cap, X.REC_BYTES)
        ok = ok and torch.equal(cv, recv_count) and X.received(rv.numpy(), cv.numpy(), cap).tobytes() == got.tobytes()
        ok = ok and moved == sum(int(cnt[d]) * X.REC_BYTES for d in range(world) if d != rank)
        # two in flight (started A then B, finished B then A)
        pa = X.exchange_v_start(torch.from_numpy(jsend.reshape(-1)), torch.from_numpy(cnt), cap * X.REC_BYTES,
                                cap, X.REC_BYTES)
        pb = X.exchange_v_start(junk, torch.zeros(world, dtype=torch.int32), cap * X.REC_BYTES, cap, X.REC_BYTES)
        rb2, cb2 = X.exchange_finish(pb)
        ra2, ca2 = X.exchange_finish(pa)
        ok = ok and bool((cb2 == 0).all()) and pb[3] == 0
        ok = ok and X.received(ra2.numpy(), ca2.numpy(), cap).tobytes() == got.tobytes()
        Path(out_dir, f"r{rank}").write_text(f"{int(ok)} {len(got)}")
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_exchange_gloo_world2(oracle_built, tmp_path):
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [Path(tmp_path, f"r{r}").read_text().split() for r in range(world)]
    assert all(r[0] == "1" for r in res), res
    # every routed record went to exactly one owner
    total = sum(int(r[1]) for r in res)
    import route_ref
    routed = sum(int((shard_records(r)["ns_id"] != abi.ID_NONE).sum()) for r in range(world))
    assert total == routed


def lookup_regions(rec, world, rank, cap, tcap):
    """Host stand-in for emurx_parse_route_dev's send regions: every frame's 32-byte lookup head
    (the frame index; the other words a function of frame and rank) in the region of the owner
    of its CTunnelKey, frame order; every 5th head an ICMPv6-key head (kIp6) with a one-unit
    tail, every 7th a tcp head with an IPv6 tuple (three units), the tails spread over the
    shards in reverse order (the device's order within a shard is not deterministic).  Returns
    (regions [world] bytes, counts [2 * world], the canonical records per region)."""
    from emurx import exchange as X
    from test_gpu_tables import _owners_by_key
    own = _owners_by_key(rec, world)
    rb = abi.lookup_region_bytes(cap, tcap)
    out, cnt, canon = np.zeros((world, rb), np.uint8), np.zeros(2 * world, np.int32), []
    for d in range(world):
        idx = np.nonzero(own == d)[0]
        hd = np.zeros(len(idx), abi.LOOKUP_REC_DTYPE)
        hd["frame"] = idx
        hd["vlans"], hd["w2"] = rec["vlan0"][idx] & 0xfff, rec["vport"][idx].astype(np.uint32) | (rank << 24)
        hd["x"] = idx * 3 + rank
        ip6 = (idx % 5) == 0
        tup = ((idx % 7) == 0) & ~ip6
        hd["w4"] = np.where(ip6, 6 << 28, np.where(tup, (3 << 28) | (1 << 31) | (1 << 26), 0)).astype(np.uint32)
        tails = out[d, cap * 32:].view("<u4").reshape(-1, 4)
        nxt = [0] * abi.TAIL_SHARDS
        for j in np.nonzero(ip6 | tup)[0][::-1]:
            u = 1 if ip6[j] else 3
            sh = int(idx[j]) % abi.TAIL_SHARDS
            x = sh * tcap + nxt[sh]
            nxt[sh] += u
            assert nxt[sh] <= tcap
            tails[x: x + u] = (int(idx[j]) * 16 + np.arange(4 * u, dtype=np.uint32)).reshape(u, 4)
            hd["x"][j] = x
        out[d, : len(idx) * 32] = hd.view(np.uint8)
        cnt[2 * d] = len(idx)
        canon.append(X.lookup_records(out[d], len(idx), cap, tcap))
    return out, cnt, canon


def _worker_partitioned(rank, world, port, out_dir):
    """The partitioned protocol over gloo: lookup regions (32-byte heads + tail shards) to the
    Namespace owners, two counts per region, the records with their tails intact at the owner;
    and this rank's device-table bytes (host-only handle, emurx_set_partition) ~ 1/world."""
    sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "trex-emu_amd"), str(ROOT / "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from emurx import exchange as X
    from emurx.rx import RxPath
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        recs = [shard_records(r) for r in range(world)]
        cap = X.capacity(N_FRAMES, world)
        tcap = 3 * (N_FRAMES // abi.TAIL_SHARDS + 1)
        rb = abi.lookup_region_bytes(cap, tcap)
        send, cnt, _ = lookup_regions(recs[rank], world, rank, cap, tcap)
        recv, recv_count = X.exchange(torch.from_numpy(send.reshape(-1).copy()), torch.from_numpy(cnt), rb)
        r = recv.numpy().reshape(world, rb)
        c = recv_count.numpy()
        got = np.concatenate([X.lookup_records(r[s], int(c[2 * s]), cap, tcap) for s in range(world)])
        want = np.concatenate([lookup_regions(recs[s], world, s, cap, tcap)[2][rank] for s in range(world)])
        ok = got.tobytes() == want.tobytes() and len(got) > 0 and (c[1::2] == 0).all()
        ok = ok and int((X.tail_units(got["head"]["w4"]) > 0).sum()) > 0
        # payload-sized: the valid heads and the tail shards of every region, nothing else
        noise = np.random.default_rng(7 + rank).integers(0, 256, send.shape, dtype=np.uint8)
        for d in range(world):
            noise[d, : int(cnt[2 * d]) * 32] = send[d, : int(cnt[2 * d]) * 32]
            noise[d, cap * 32:] = send[d, cap * 32:]
        rv, cv, moved = X.exchange_v(torch.from_numpy(noise.reshape(-1).copy()), torch.from_numpy(cnt), rb, cap, 32)
        r2 = rv.numpy().reshape(world, rb)
        got2 = np.concatenate([X.lookup_records(r2[s], int(cv[2 * s]), cap, tcap) for s in range(world)])
        ok = ok and got2.tobytes() == want.tobytes() and torch.equal(cv, recv_count)
        ok = ok and moved == sum(int(cnt[2 * d]) * 32 + (rb - cap * 32) for d in range(world) if d != rank)
        w = synth.config_c(N_FRAMES)
        full = RxPath(-1, max_ns=4096, max_clients=65536, max_frames=64)
        part = RxPath(-1, max_ns=4096, max_clients=65536, max_frames=64)
        part.set_partition(world, rank)
        for t in (full, part):
            synth.load_tables(w, t)
        fb, pb = full.table_stats()["table_bytes"], part.table_stats()["table_bytes"]
        Path(out_dir, f"p{rank}").write_text(f"{int(ok)} {len(got)} {fb} {pb}")
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_exchange_gloo_world2(oracle_built, tmp_path, world):
    """world 2, and 3 (a partition count that is not a power of two)"""
    import torch.multiprocessing as mp
    mp.spawn(_worker_partitioned, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [Path(tmp_path, f"p{r}").read_text().split() for r in range(world)]
    assert all(r[0] == "1" for r in res), res
    assert sum(int(r[1]) for r in res) == world * N_FRAMES  # every frame reached one owner
    share = 1 if world & (world - 1) == 0 else 2  # power-of-two tables: at most 2 / world for 3
    for r in res:  # per-rank device tables: 1 / world of the replicated bytes (+ the dense ns info)
        assert int(r[3]) <= share * int(r[2]) / world + 4096 * 16, r


def test_owner_partition_balance(lib):
    """emurx_ns_owner spreads config D's 32K Namespaces evenly over 8 partitions."""
    from emurx.rx import ns_owner
    keys = synth.config_d(256)["ns"]
    own = np.array([ns_owner(k, 8) for k, _ in keys])
    counts = np.bincount(own, minlength=8)
    assert counts.min() > 0.9 * len(keys) / 8 and counts.max() < 1.1 * len(keys) / 8
    assert all(ns_owner(k, 1) == 0 for k, _ in keys[:100])
