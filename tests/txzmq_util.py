"""Seeded batches for the tx ZMQ framing (VethIFZmq.Send / FlushTx, veth_zmq.go:149-200)."""
import numpy as np

from emurx import abi


def batch(n, kind, seed=0, gap=3):
    """n frames of a length profile, packed with `gap` bytes between them (unaligned)."""
    rng = np.random.default_rng([seed, n, kind])
    if kind == 0:
        lens = rng.integers(0, 200, n)
    elif kind == 1:  # IMIX + jumbo + frames past the 32 KiB message limit
        lens = rng.choice([64, 594, 1518, 9000, 20000, 32767, 32768, 40000, 65535], n)
    elif kind == 2:
        lens = rng.integers(500, 1200, n)
    else:
        lens = np.full(n, 64)
    lens = lens.astype(np.int64)
    off = np.zeros(n, np.int64)
    if n:
        off[1:] = np.cumsum(lens + gap)[:-1]
    size = int(off[-1] + lens[-1]) + 64 if n else 64
    buf = rng.integers(0, 256, size, dtype=np.uint8)
    d = np.zeros(n, abi.DESC_DTYPE)
    d["off"], d["len"], d["vport"] = off, lens, rng.integers(0, 256, n)
    return buf, d


def threshold_batch():
    """Frames that land exactly on the 32 KiB rule and the 64-frame burst."""
    lens = [32767, 1, 32766, 1, 1, 16384, 16383, 1, 16384, 16384, 0, 0] + [10] * 130 + [32768, 5, 65535, 0, 7]
    lens = np.array(lens, np.int64)
    off = np.zeros(len(lens), np.int64)
    off[1:] = np.cumsum(lens)[:-1]
    buf = np.random.default_rng(5).integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    d = np.zeros(len(lens), abi.DESC_DTYPE)
    d["off"], d["len"], d["vport"] = off, lens, np.arange(len(lens)) % 7
    return buf, d
