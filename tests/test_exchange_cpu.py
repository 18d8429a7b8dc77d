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
                                      torch.from_numpy(cnt), cap)
        got = X.received(recv.numpy(), recv_count.numpy(), cap)
        want = np.concatenate([route_ref.route(recs[s], world, s)[rank] for s in range(world)])
        ok = got.tobytes() == want.tobytes() and len(got) > 0
        owners = route_ref.owners(got["rec"], world)
        ok = ok and bool((owners == rank).all())
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


def test_owner_partition_balance(lib):
    """emurx_ns_owner spreads config D's 32K Namespaces evenly over 8 partitions."""
    from emurx.rx import ns_owner
    keys = synth.config_d(256)["ns"]
    own = np.array([ns_owner(k, 8) for k, _ in keys])
    counts = np.bincount(own, minlength=8)
    assert counts.min() > 0.9 * len(keys) / 8 and counts.max() < 1.1 * len(keys) / 8
    assert all(ns_owner(k, 1) == 0 for k, _ in keys[:100])
