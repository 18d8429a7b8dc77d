"""The reference's parser tests (parser_test.go) over the C++ host mirror
(trex-emu_amd/host/emu_core.*) and the HIP path behind the C-ABI."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "trex-emu_amd" / "build" / "test_parser"
KAT = ROOT / "tests" / "golden" / "kat_frames.bin"


def _build():
    subprocess.run(["make", "-s", "-C", str(ROOT / "trex-emu_amd")], check=True)


def test_mirror_shrink_from_live_entries():
    """The allocation fallback's table shrink (Mirror::shrink): an IPv6 table filled
    to twice its target load (a DHCPv6 address for most clients, ns_ctx.go:442-533) shrinks
    from its live entries, keeps one more insert under the 3/4 bound and every address
    findable, and stops when no denser table is smaller (host-only C++ check)."""
    _build()
    r = subprocess.run([str(ROOT / "trex-emu_amd" / "build" / "test_mirror")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "PASS TestShrinkFromLive" in r.stdout, r.stdout + r.stderr


def test_host_mirror_builds():
    _build()
    assert BIN.exists() and KAT.exists()


@pytest.mark.gpu
def test_parser_go_tests_on_gpu(gpu_ok):
    _build()
    r = subprocess.run([str(BIN), str(KAT)], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("TestParserArp1", "TestParserIcmp", "TestParserDhcp1", "TestParserDhcpInvalidCs",
                 "TestNsClientLookup", "TestOnRxStream"):
        assert f"PASS {name}" in r.stdout


def test_kat_fixture_is_current():
    """tests/golden/kat_frames.bin == what tests/golden/make_kat_frames.py writes now."""
    import struct
    import sys
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    import make_kat_frames as M
    b = bytearray(struct.pack("<I", len(M.frames())))
    for name, f, vp in M.frames():
        n = name.encode()
        b += struct.pack("<H", len(n)) + n + struct.pack("<HI", vp, len(f)) + bytes(f)
    assert KAT.read_bytes() == bytes(b)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_exchange_from_cpp_on_gpu(gpu_ok, oracle_built, tmp_path):
    """The Namespace-owner exchange driven from C++ through the C-ABI alone (host/test_exchange.cpp:
    no Python or torch in that process): a 1-rank communicator made both ways (emurx_comm_init_all,
    the one-process model, with its exchange in a group; emurx_comm_unique_id + emurx_comm_init with
    the payload-sized transfer), config D frames on config D's full tables, the owner's records
    byte-equal to the oracle's."""
    import struct
    import numpy as np
    import pyoracle
    from emurx import abi, synth
    _build()
    n = 1 << 16
    w = synth.config_d(n, rank=5)
    o = pyoracle.Oracle()
    synth.load_tables(w, o)
    orec = o.rx_batch(w["buf"], w["desc"])[0]
    want = np.zeros(n, abi.ROUTE_REC_DTYPE)
    want["rec"], want["src_index"], want["src_rank"] = orec, np.arange(n), 0
    specs = synth.client_specs(w)
    f = tmp_path / "exchange_fixture.bin"
    with open(f, "wb") as fh:
        buf = np.ascontiguousarray(w["buf"], np.uint8)
        fh.write(struct.pack("<6I", n, buf.size, len(w["ns"]), len(specs), 32768, 1 << 20))
        fh.write(buf.tobytes())
        fh.write(np.ascontiguousarray(w["desc"]).tobytes())
        for key, ns_id in w["ns"]:
            fh.write(bytes(key) + struct.pack("<I", ns_id))
        fh.write(np.ascontiguousarray(specs).tobytes())
        fh.write(want.tobytes())
    r = subprocess.run([str(ROOT / "trex-emu_amd" / "build" / "test_exchange"), str(f)], capture_output=True,
                       text=True, timeout=500)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("TestExchangeOneProcess", "TestExchangeCommInit"):
        assert f"PASS {name}" in r.stdout
    assert "rccl: " in r.stdout and "librccl" in r.stdout
