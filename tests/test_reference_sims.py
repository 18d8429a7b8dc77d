"""The lookup rules against the reference's plugin simulations (tests/sim_envs.py): each
capture's environment rebuilt from its Go test, the capture's rx frames classified by the
oracle, every frame's outcome the one the capture's answers vouch for."""
import numpy as np
import pytest

import sim_envs as S
from emurx import abi, frames as F
from test_oracle_corpus import GOLD



@pytest.mark.parametrize("case", S.CASES, ids=[c[0] for c in S.CASES])
def test_simulation_outcome(oracle_built, case):
    import pyoracle
    capture, env, lk, cid, _ = case
    z = np.load(GOLD, allow_pickle=False)
    fr = S.rx_frames(z, capture)
    assert fr
    o = pyoracle.Oracle()
    S.load_env(o, env)
    buf, desc = F.pack_frames(fr, [1] * len(fr))
    rec, _, _, _ = o.rx_batch(buf, desc)
    assert (rec["status"] == 0).all()
    assert (rec["ns_id"] == 0).all()
    assert (((rec["flags"] >> 4) & 7) == abi.LK[lk]).all()
    assert (rec["client_id"] == S.expected_clients(fr, cid)).all()
