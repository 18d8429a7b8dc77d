"""Does torch.cuda._sleep hold a library stream (ExternalStream) on this box?"""
import sys
import time

import torch

sys.path.insert(0, "trex-emu_amd")
from emurx.rx import RxPath  # noqa: E402

s_cal = torch.cuda.Stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.cuda.stream(s_cal):
    torch.cuda._sleep(1_000_000)
    e0.record()
    torch.cuda._sleep(50_000_000)
    e1.record()
e1.synchronize()
ms = e0.elapsed_time(e1)
per_s = 50_000_000 / (ms / 1e3)
print(f"_sleep(50M) = {ms:.3f} ms -> {per_s:.3e} cycles/s", flush=True)
rx = RxPath(0, max_ns=16, max_clients=64, max_frames=4096)
p = rx.ingest_stream(0)
print("slot stream", hex(p), flush=True)
st = torch.cuda.ExternalStream(p)
t0 = time.perf_counter()
with torch.cuda.stream(st):
    torch.cuda._sleep(int(per_s * 1.0))
print("queued; query", st.query(), flush=True)
while not st.query():
    time.sleep(0.01)
print(f"external stream drained after {time.perf_counter() - t0:.3f} s", flush=True)
st2 = torch.cuda.Stream()
t0 = time.perf_counter()
with torch.cuda.stream(st2):
    torch.cuda._sleep(int(per_s * 1.0))
while not st2.query():
    time.sleep(0.01)
print(f"torch stream drained after {time.perf_counter() - t0:.3f} s", flush=True)
# Does a not-ready query leave hipErrorNotReady (600) as the thread's last error?
import ctypes  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipGetLastError.restype = ctypes.c_int
hip.hipGetLastError()
st3 = torch.cuda.Stream()
with torch.cuda.stream(st3):
    torch.cuda._sleep(int(per_s * 0.2))
print("query while running:", st3.query(), "-> hipGetLastError() =", hip.hipGetLastError(), flush=True)
st3.synchronize()
