"""bench.py's multi-rank launch path without torchrun (the way the driver runs
`python bench.py --gpus N`): N fresh worker processes rendezvous on 127.0.0.1 and rank 0
prints the JSON line; a failing rank ends the whole run with its exit code instead of
leaving the others waiting in a collective.  --launch-check runs the skeleton without a GPU."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def run(args, env=None, timeout=120):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=e, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.timeout(180)
@pytest.mark.parametrize("n", [2, 3])
def test_spawned_ranks_gloo(n):
    p = run(["--gpus", str(n), "--backend", "gloo", "--launch-check"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    j = json.loads(lines[0])
    assert j["n_gpus"] == n and j["max_over_ranks"] == float(n) and j["master"] == "127.0.0.1"


@pytest.mark.timeout(180)
def test_failed_rank_ends_the_run():
    p = run(["--gpus", "2", "--backend", "gloo", "--launch-check"], env={"EMURX_BENCH_FAIL_RANK": "1"})
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_two_rank_exchange_fields(gpu_ok):
    """The bench's N = 2 line over gloo (both ranks on the one GPU): the config-B headline plus the
    Namespace-partitioned exchange timed with the headline's steps and warmup, its per-phase
    device times and the bytes that crossed to the other rank."""
    p = run(["--gpus", "2", "--backend", "gloo", "--frames", "65536", "--exchange-frames", "65536",
             "--steps", "6", "--warmup", "2", "--batches", "2", "--warmup-seconds", "0.05"], timeout=580)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["value"] > 0
    x = j["namespace_exchange"]
    assert "error" not in x, x
    assert x["steps"] == 6  # the headline's steps, not a side sample
    ph = x["exchange"]["phases"]
    for k in ("source_side_ms", "k_rx_ms", "owner_count_scan_ms", "all_to_all_ms", "owner_lookup_ms"):
        assert ph[k] > 0, (k, ph)
    assert ph["record_bytes"] == 64
    assert ph["bytes_to_other_ranks"] > ph["payload_bytes_to_other_ranks"] > 0
    assert ph["xgmi_gbs"] > 0
