"""CPU: the bench's choice of the N > 1 transfer: --a2a auto times the
sync-free whole-region exchange and the payload-sized one after the warmup and runs the faster;
the line records both rates, their host submit time per step and the choice."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def _res(eq_ms, pl_ms):
    return {"equal": {"value": 1.0 / eq_ms, "ms_per_step": eq_ms, "host_submit_ms_per_step": 0.01},
            "payload": {"value": 1.0 / pl_ms, "ms_per_step": pl_ms, "host_submit_ms_per_step": 0.2}}


def test_faster_transfer_is_chosen():
    b = bench.a2a_choice_block(_res(0.20, 0.25), 20)
    assert b["chosen"] == "equal" and b["steps_each"] == 20
    b = bench.a2a_choice_block(_res(0.30, 0.25), 20)
    assert b["chosen"] == "payload"
    for k in ("equal", "payload"):
        assert set(b[k]) == {"value", "ms_per_step", "host_submit_ms_per_step"}
    assert "max over ranks" in b["source"]


def test_tie_keeps_the_sync_free_transfer():
    assert bench.a2a_choice_block(_res(0.25, 0.25), 10)["chosen"] == "equal"


def test_default_is_auto_over_the_library_communicator(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse_args()
    assert a.a2a == "auto" and a.comm == "library"
