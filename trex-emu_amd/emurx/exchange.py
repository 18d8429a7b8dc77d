"""Namespace-partitioned exchange between GPUs.

Frames shard by input offset across the ranks of a node.  Each rank fills one send region per
Namespace owner; the counts travel first (an all-to-all of 1-2 words per region), then only the
bytes that carry data (exchange_v_start: one grouped send / receive per peer and span, the
all-to-all-v of SURVEY §8e); rank r receives, from every source s, region s of its receive
buffer and the counts of that region.  exchange() / exchange_start() move whole regions (one
equal-split all-to-all; the round-4 protocol, kept for comparison).  Two region kinds:

- replicated tables: emurx_classify_route_dev packs the classified records whose Namespace
  was found, `cap` emurx_route_rec (40 B) per region, one count per region;
- partitioned tables: emurx_parse_route_dev packs every frame's lookup record as a 32-byte
  head plus, for ICMPv6 keys and transport tuples, 16-byte tail units
  (abi.lookup_region_bytes(cap, tail_cap) per region), two counts per region (heads, tail
  overflow).

The collectives are plain torch.distributed calls: RCCL over xGMI with the "nccl" backend
(device tensors, no host synchronisation, the counts travel in their own all-to-all), or
gloo on host copies for CPU tests of the same protocol.
"""
from __future__ import annotations

import numpy as np

from . import abi

REC_BYTES = abi.ROUTE_REC_DTYPE.itemsize
LOOKUP_BYTES = abi.LOOKUP_REC_DTYPE.itemsize


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


def grow_tail(tail_cap: int, need) -> int:
    """Tail units per shard after a shard overflowed: the largest need seen plus 1/4 more."""
    m = int(max(int(c) for c in need))
    return max(tail_cap, m + m // 4 + 32)


def region_bytes(cap: int, tail_cap: int | None = None) -> int:
    """Bytes of one region: lookup regions when tail_cap is given, else route records."""
    return cap * REC_BYTES if tail_cap is None else abi.lookup_region_bytes(cap, tail_cap)


def _check(send, send_count, rbytes, world):
    assert send.numel() == world * rbytes, (send.numel(), world, rbytes)
    assert send_count.numel() % world == 0


def exchange(send, send_count, rbytes: int, group=None):
    """Equal-split all-to-all of `send` ([world * rbytes] uint8 tensor: one region per rank)
    and `send_count` ([world * k] int32 tensor: k counts per region).  Returns (recv,
    recv_count) on the device of the inputs."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    _check(send, send_count, rbytes, world)
    if dist.get_backend(group) == "gloo" and send.is_cuda:
        r, c = exchange(send.cpu(), send_count.cpu(), rbytes, group)
        return r.to(send.device), c.to(send.device)
    recv = torch.empty_like(send)
    recv_count = torch.empty_like(send_count)
    dist.all_to_all_single(recv_count, send_count, group=group)
    dist.all_to_all_single(recv, send, group=group)
    return recv, recv_count


def exchange_start(send, send_count, rbytes: int, group=None):
    """exchange() without waiting: the all-to-alls are enqueued on the collective's stream
    behind the work already on the caller's stream, and the caller's stream goes on (the next
    batch's parse overlaps this batch's transfer).  exchange_finish() makes the caller's
    stream wait for them and returns (recv, recv_count).  gloo on device tensors (CPU
    rehearsals) completes here."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    _check(send, send_count, rbytes, world)
    if dist.get_backend(group) == "gloo" and send.is_cuda:
        return (None,) + exchange(send, send_count, rbytes, group)
    recv = torch.empty_like(send)
    recv_count = torch.empty_like(send_count)
    works = (dist.all_to_all_single(recv_count, send_count, group=group, async_op=True),
             dist.all_to_all_single(recv, send, group=group, async_op=True))
    return works, recv, recv_count


def exchange_finish(pending):
    """(recv, recv_count) of an exchange_start() or exchange_v_start(), the caller's stream
    ordered after it."""
    works, recv, recv_count = pending[:3]
    for w in works or ():
        w.wait()
    return recv, recv_count


# ---- payload-sized exchange (round 5): counts first, then only the bytes that carry data ----
def payload_spans(count: int, cap: int, rec_bytes: int, rbytes: int):
    """The byte spans of one region that carry data: its first min(count, cap) records and,
    for lookup regions, the tail shards [cap * rec_bytes, rbytes) (their units are taken by
    atomics, so which of them are used is known on the device only)."""
    heads = min(int(count), cap) * rec_bytes
    spans = [(0, heads)] if heads else []
    if rbytes > cap * rec_bytes:
        spans.append((cap * rec_bytes, rbytes))
    return spans


def _v_ops(send, recv, sc, rc, cs: int, rbytes: int, cap: int, rec_bytes: int, group):
    """The P2P operations of one payload-sized exchange, the own region copied in place; the
    bytes sent to other ranks."""
    import torch.distributed as dist
    world, me = dist.get_world_size(group), dist.get_rank(group)
    ops, moved = [], 0
    for p in range(world):
        peer = dist.get_global_rank(group, p) if group is not None else p
        out_spans = payload_spans(sc[p * cs], cap, rec_bytes, rbytes)
        if p == me:
            for a, b in out_spans:
                recv[p * rbytes + a: p * rbytes + b].copy_(send[p * rbytes + a: p * rbytes + b])
            continue
        for a, b in out_spans:
            ops.append(dist.P2POp(dist.isend, send[p * rbytes + a: p * rbytes + b], peer, group))
            moved += b - a
        for a, b in payload_spans(rc[p * cs], cap, rec_bytes, rbytes):
            ops.append(dist.P2POp(dist.irecv, recv[p * rbytes + a: p * rbytes + b], peer, group))
    return ops, moved


def exchange_v_start(send, send_count, rbytes: int, cap: int, rec_bytes: int, group=None):
    """The payload-sized exchange (all-to-all-v, counts then records): the
    counts' all-to-all, the counts to the host (this waits for the caller's stream: the batch's
    packing), then one grouped send / receive per peer and span that carries data (RCCL
    groups them as its own all-to-all does), enqueued behind the caller's stream; the receive
    buffer keeps the equal-split layout (region s at s * rbytes), its bytes outside the spans
    undefined.  Returns the pending (works, recv, recv_count, moved) for exchange_finish();
    `moved` = the bytes sent to other ranks.  gloo on device tensors (CPU rehearsals) runs on
    host copies and completes here."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    _check(send, send_count, rbytes, world)
    cs = send_count.numel() // world
    if dist.get_backend(group) == "gloo" and send.is_cuda:
        r, c, moved = exchange_v(send.cpu(), send_count.cpu(), rbytes, cap, rec_bytes, group)
        return None, r.to(send.device), c.to(send.device), moved
    recv = torch.empty_like(send)
    recv_count = torch.empty_like(send_count)
    dist.all_to_all_single(recv_count, send_count, group=group)
    sc, rc = send_count.cpu().numpy(), recv_count.cpu().numpy()
    ops, moved = _v_ops(send, recv, sc, rc, cs, rbytes, cap, rec_bytes, group)
    works = dist.batch_isend_irecv(ops) if ops else []
    return works, recv, recv_count, moved


def exchange_v(send, send_count, rbytes: int, cap: int, rec_bytes: int, group=None):
    """exchange_v_start() + exchange_finish(): (recv, recv_count, moved)."""
    pending = exchange_v_start(send, send_count, rbytes, cap, rec_bytes, group)
    recv, recv_count = exchange_finish(pending)
    return recv, recv_count, pending[3]


def received(recv: np.ndarray, recv_count: np.ndarray, cap: int) -> np.ndarray:
    """Valid records of a route receive buffer (host copy), source-rank order."""
    r = np.ascontiguousarray(recv).view(np.uint8).reshape(-1)[: len(recv_count) * cap * REC_BYTES]
    r = r.view(abi.ROUTE_REC_DTYPE).reshape(len(recv_count), cap)
    cnt = np.asarray(recv_count).astype(np.int64)
    if (cnt > cap).any():
        raise RuntimeError(f"exchange region overflow: counts {cnt.tolist()} > cap {cap}")
    return np.concatenate([r[s, : cnt[s]] for s in range(len(cnt))]) if len(cnt) else r[:0, 0]


# the canonical form of a lookup record: the head with x replaced by 0 when it names a tail,
# then the tail's units (zero-padded to 3); what a head's tail holds is deterministic, where
# the units sit in the shards is not (emu_rx.h)
LOOKUP_CANON_DTYPE = np.dtype([("head", abi.LOOKUP_REC_DTYPE), ("tail", "<u4", 12)])


def tail_units(w4: np.ndarray) -> np.ndarray:
    """Tail units of heads from their w4 word (emurx_parse.h lk_tail_units)."""
    w4 = np.asarray(w4, np.uint32)
    key = (w4 >> 28) & 7
    ok = ((w4 >> 20) & 31) == abi.ST["OK"]
    ip6k = (key == 4) | (key == 6)  # kEui, kIp6
    tup = (w4 >> 31) == 1
    units = np.where(ip6k, 1, np.where(tup, np.where((w4 >> 26) & 1, 3, 1), 0))
    return np.where(ok, units, 0).astype(np.int64)


def lookup_records(region: np.ndarray, count: int, cap: int, tail_cap: int) -> np.ndarray:
    """The `count` valid lookup records of one region (host bytes) in canonical form
    (LOOKUP_CANON_DTYPE): each head with its tail's units attached."""
    b = np.ascontiguousarray(region).view(np.uint8).reshape(-1)
    assert b.size == abi.lookup_region_bytes(cap, tail_cap), (b.size, cap, tail_cap)
    if count > cap:
        raise RuntimeError(f"lookup region overflow: {count} heads > cap {cap}")
    heads = b[: cap * 32].view(abi.LOOKUP_REC_DTYPE)[:count].copy()
    tails = b[cap * 32:].view("<u4").reshape(-1, 4)
    out = np.zeros(count, LOOKUP_CANON_DTYPE)
    u = tail_units(heads["w4"])
    for i in np.nonzero(u)[0]:
        x = int(heads["x"][i])
        if x == abi.TAIL_NONE or x + u[i] > len(tails):
            raise RuntimeError(f"lookup record {i}: tail index {x:#x} outside the shards")
        out["tail"][i, : 4 * u[i]] = tails[x: x + u[i]].reshape(-1)
        heads["x"][i] = 0
    out["head"] = heads
    return out
