"""bench.py's rotating batch slots (permuted_batch): each slot is the workload's frames in a
seeded permutation at new addresses.  Checked on the CPU with torch CPU tensors and the
oracle: the slot's records are the original records in the permuted order (the parse depends
on a frame's bytes alone), every frame's bytes and ZMQ header moved intact, and the slots
occupy distinct bytes (no two slots share an address range)."""
import importlib.util
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("cfg", ["B", "C", "E"])
def test_permuted_batch_is_the_same_workload(cfg, oracle_built):
    import torch
    from emurx import synth
    b = _bench()
    n = 3000
    w = {"B": lambda: synth.config_b(n), "C": lambda: synth.config_c(n), "E": lambda: synth.config_e(n)}[cfg]()
    buf = torch.from_numpy(w["buf"])
    o = oracle_built.Oracle()
    synth.load_tables(w, o)
    ref, _, _, _ = o.rx_batch(w["buf"], w["desc"])
    seed = 77
    pb, pd = b.permuted_batch(torch, buf, w["desc"], seed, "cpu")
    pbuf = pb.numpy()
    pdesc = pd.numpy().view(w["desc"].dtype)
    perm = np.random.default_rng(seed).permutation(n)
    # descriptors: same lengths / vports in permuted order, packed offsets (4-byte header gaps)
    assert np.array_equal(pdesc["len"], w["desc"]["len"][perm])
    assert np.array_equal(pdesc["vport"], w["desc"]["vport"][perm])
    seg = pdesc["len"].astype(np.int64) + 4
    assert pdesc["off"][0] == 4 and np.array_equal(np.diff(pdesc["off"].astype(np.int64)), seg[:-1])
    assert len(pbuf) == int(seg.sum()) + 64 and not pbuf[-64:].any()
    for k in (0, 1, n // 2, n - 1):  # frame bytes and their ZMQ headers moved intact
        so, po, ln = int(w["desc"]["off"][perm[k]]), int(pdesc["off"][k]), int(pdesc["len"][k])
        assert pbuf[po - 4:po + ln].tobytes() == w["buf"][so - 4:so + ln].tobytes()
    rec, _, _, _ = o.rx_batch(pbuf, pdesc)
    assert rec.tobytes() == ref[perm].tobytes()
    # another seed: another order
    pb2, _ = b.permuted_batch(torch, buf, w["desc"], seed + 1, "cpu")
    assert not torch.equal(pb2, pb)
