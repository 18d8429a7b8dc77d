"""The host C++ and the C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md
§5), on the CPU: `make asan` builds the library's host side (emurx_api.cpp: ZMQ framing walk,
table shipment bookkeeping, batch checks; emurx_mirror.cpp: the Go-map mirror with its
tombstones, rebuilds, growth and partition images) with -fsanitize=address,undefined
(trex-emu_amd/lib/libemurx_asan.so, linked with the unsanitized gfx950 kernels) and the oracle
(oracle/liborc_asan.so).  A child pytest with gcc's libasan preloaded then drives through them:
the table mirror's random mutation sequences, partitions and mid-batch rule
(test_table_mirror.py), the C-ABI's host functions and hostile ZMQ messages (test_abi.py,
test_host_fuzz.py), and the oracle's known-answer, edge, corpus, flow, tx and fuzz tests.  Any
sanitizer report fails the run (halt_on_error); a positive control proves the instrumentation
is live."""
import fcntl
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
LIB = ROOT / "trex-emu_amd" / "lib" / "libemurx_asan.so"
ORC = ROOT / "oracle" / "liborc_asan.so"
SUITES = ["tests/test_table_mirror.py", "tests/test_abi.py", "tests/test_host_fuzz.py", "tests/test_oracle_kat.py",
          "tests/test_oracle_edge.py", "tests/test_oracle_corpus.py", "tests/test_oracle_flows.py",
          "tests/test_oracle_tx.py", "tests/test_oracle_txzmq.py", "tests/test_reference_sims.py"]


@pytest.fixture(scope="module")
def asan_env():
    # one build at a time: with pytest-xdist both tests of this module may start in two workers,
    # and a library being relinked by one must not be loaded by the other
    (ROOT / "trex-emu_amd" / "build").mkdir(exist_ok=True)
    with open(ROOT / "trex-emu_amd" / "build" / ".asan.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", str(ROOT / "trex-emu_amd"), "asan"], check=True)
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "asan"], check=True)
        fcntl.flock(lk, fcntl.LOCK_UN)
    libasan = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True, text=True,
                             check=True).stdout.strip()
    env = dict(os.environ)
    env.update(LD_PRELOAD=libasan, EMURX_LIB=str(LIB), ORC_LIB=str(ORC),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    return env


def test_host_code_is_clean_under_asan_ubsan(asan_env):
    p = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu",
                        *SUITES], cwd=ROOT, env=asan_env, capture_output=True, text=True, timeout=1500)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]


def test_sanitized_libraries_were_loaded(asan_env):
    """The child really loads the sanitized builds: both show up in its memory map."""
    code = ("import sys; sys.path[:0] = ['trex-emu_amd', 'oracle']\n"
            "from emurx import abi; abi.load()\n"
            "import pyoracle; pyoracle.lib()\n"
            "m = open('/proc/self/maps').read()\n"
            "print('libemurx_asan.so' in m, 'liborc_asan.so' in m)\n")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=asan_env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert p.stdout.split() == ["True", "True"], p.stdout


def test_positive_control_out_of_bounds_read_is_caught(asan_env):
    """A caller that claims a longer ZMQ message than its malloc'd buffer holds (the header
    announces 8 frames, 4 are there): the sanitized framing walk reads the 5th header past the
    allocation and ASan stops the process."""
    code = ("import sys, ctypes as C, numpy as np; sys.path[:0] = ['trex-emu_amd']\n"
            "from emurx import abi, frames as F\n"
            "lib = abi.load()\n"
            "m = bytearray(F.zmq_pack([bytes(60)] * 4)); m[2:4] = (8).to_bytes(2, 'big')\n"
            "libc = C.CDLL(None); libc.malloc.restype = C.c_void_p; libc.malloc.argtypes = [C.c_size_t]\n"
            "p = libc.malloc(len(m)); C.memmove(p, bytes(m), len(m))\n"
            "lib.emurx_zmq_descriptors.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]\n"
            "d = np.zeros(16, dtype=abi.DESC_DTYPE); n = C.c_uint32(); e = C.c_int()\n"
            "lib.emurx_zmq_descriptors(p, len(m) + 64, d.ctypes.data, 16, C.byref(n), C.byref(e))\n")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=asan_env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode != 0 and "heap-buffer-overflow" in p.stderr, (p.returncode, p.stderr[-2000:])
