"""Namespace-partitioned exchange between GPUs.

Frames shard by input offset across the ranks of a node.  Each rank classifies its shard
(emurx_classify_dev), packs the records whose Namespace was found into the send regions of
the Namespaces' owners (emurx_route_dev), and one equal-split all-to-all delivers them:
rank r receives, from every source s, `recv_count[s]` valid records at
`recv[s * cap : s * cap + recv_count[s]]` (frame order of the source).

The collectives are plain torch.distributed calls: RCCL over xGMI with the "nccl" backend
(device tensors, no host synchronisation, the counts travel in their own all-to-all), or
gloo on host copies for CPU tests of the same protocol.
"""
from __future__ import annotations

import numpy as np

from . import abi

REC_BYTES = abi.ROUTE_REC_DTYPE.itemsize


def capacity(n_frames: int, n_parts: int, slack: float = 1.25) -> int:
    """Records per destination region: the fair share plus slack for the owner hash's
    imbalance.  The default (1.25) covers skewed Namespace populations; bench.py passes 1.06
    for config D's uniform synthetic keys (the fullest of 8 partitions holds 1.030x the fair
    share).  A region that overflows anyway is reported by its count (> cap), on every rank
    after the count exchange: the caller must check the counts of every batch, grow the
    capacity (grow()) and route that batch again."""
    if n_parts == 1:
        return max(n_frames, 1)
    return int(n_frames / n_parts * slack) + 1024


def grow(cap: int, counts) -> int:
    """Capacity after an overflow: the largest region count seen plus 1/16 more."""
    m = int(max(int(c) for c in counts))
    return max(cap, m + m // 16 + 1024)


LOOKUP_BYTES = abi.LOOKUP_REC_DTYPE.itemsize


def exchange(send, send_count, cap: int, group=None, rec_bytes: int = REC_BYTES):
    """Equal-split all-to-all of `send` ([world * cap * rec_bytes] uint8 tensor: emurx_route_rec
    regions, or emurx_lookup_rec regions with rec_bytes = LOOKUP_BYTES) and `send_count`
    ([world] int32 tensor).  Returns (recv, recv_count) on the device of the inputs."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    assert send.numel() == world * cap * rec_bytes and send_count.numel() == world
    if dist.get_backend(group) == "gloo" and send.is_cuda:
        r, c = exchange(send.cpu(), send_count.cpu(), cap, group, rec_bytes)
        return r.to(send.device), c.to(send.device)
    recv = torch.empty_like(send)
    recv_count = torch.empty_like(send_count)
    dist.all_to_all_single(recv_count, send_count, group=group)
    dist.all_to_all_single(recv, send, group=group)
    return recv, recv_count


def exchange_start(send, send_count, cap: int, group=None, rec_bytes: int = REC_BYTES):
    """exchange() without waiting: the all-to-alls are enqueued on the collective's stream
    behind the work already on the caller's stream, and the caller's stream goes on (the next
    batch's parse overlaps this batch's transfer).  exchange_finish() makes the caller's
    stream wait for them and returns (recv, recv_count).  gloo on device tensors (CPU
    rehearsals) completes here."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    assert send.numel() == world * cap * rec_bytes and send_count.numel() == world
    if dist.get_backend(group) == "gloo" and send.is_cuda:
        return (None,) + exchange(send, send_count, cap, group, rec_bytes)
    recv = torch.empty_like(send)
    recv_count = torch.empty_like(send_count)
    works = (dist.all_to_all_single(recv_count, send_count, group=group, async_op=True),
             dist.all_to_all_single(recv, send, group=group, async_op=True))
    return works, recv, recv_count


def exchange_finish(pending):
    """(recv, recv_count) of an exchange_start(), the caller's stream ordered after it."""
    works, recv, recv_count = pending
    for w in works or ():
        w.wait()
    return recv, recv_count


def received(recv: np.ndarray, recv_count: np.ndarray, cap: int) -> np.ndarray:
    """Valid records of a receive buffer (host copy), source-rank order."""
    r = np.ascontiguousarray(recv).view(np.uint8).reshape(-1)[: len(recv_count) * cap * REC_BYTES]
    r = r.view(abi.ROUTE_REC_DTYPE).reshape(len(recv_count), cap)
    cnt = np.asarray(recv_count).astype(np.int64)
    if (cnt > cap).any():
        raise RuntimeError(f"exchange region overflow: counts {cnt.tolist()} > cap {cap}")
    return np.concatenate([r[s, : cnt[s]] for s in range(len(cnt))]) if len(cnt) else r[:0, 0]
