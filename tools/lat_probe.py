"""Latency probe of the batched ingest's small batches (round 4): host time in submit and in
wait, per batch size, beside a torch one-element kernel + synchronize (the launch and
completion floor of this box).  Env EMURX_INGEST_SMALL / EMURX_INGEST_SPIN select the path."""
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "trex-emu_amd"))
import numpy as np
import torch
from emurx import abi, synth
from emurx import frames as F
from emurx.rx import RxPath


def med(v):
    return round(float(np.median(np.array(v[10:]) * 1e6)), 1)


def main():
    dev = torch.device("cuda", 0)
    x = torch.zeros(1, device=dev)
    for _ in range(20):
        x.add_(1)
        torch.cuda.synchronize()
    fl = []
    for _ in range(300):
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        fl.append(time.perf_counter() - t0)
    out = {"env": {k: os.environ.get(k) for k in ("EMURX_INGEST_SMALL", "EMURX_INGEST_SPIN")},
           "torch_one_kernel_sync_us": med(fl)}
    w = synth.config_b(1 << 14, seed=synth.SEED_B)
    rx = RxPath(0, max_ns=4096, max_clients=65536, max_frames=1 << 14)
    rx.register_all()
    synth.load_tables(w, rx)
    stream, msgs = F.zmq_messages(w["buf"], w["desc"], 64)
    np.copyto(rx.ingest_buffer(0, len(stream)), stream)
    lib, h = rx.lib, rx.h
    res = abi.IngestResult()
    mt = np.ascontiguousarray(np.asarray(msgs)).view(np.uint32).reshape(-1, 2)
    for nm in (1, 16, 64, 256):
        tab = np.ascontiguousarray(mt[:nm])
        ptr = tab.ctypes.data
        sub, wt = [], []
        for _ in range(300):
            t0 = time.perf_counter()
            abi.check(lib.emurx_ingest_submit(h, 0, ptr, nm), "submit")
            t1 = time.perf_counter()
            abi.check(lib.emurx_ingest_wait(h, 0, C.byref(res)), "wait")
            t2 = time.perf_counter()
            sub.append(t1 - t0)
            wt.append(t2 - t1)
        out[f"msgs_{nm}"] = {"submit_us": med(sub), "wait_us": med(wt),
                             "total_us": med([a + b for a, b in zip(sub, wt)])}
        if hasattr(lib, "emurx_debug_small_stamps"):  # the EMURX_SMALL_STAMP build: the last batch's phases
            raw = np.zeros(64 * 10 + 16, dtype=np.uint64)
            lib.emurx_debug_small_stamps(raw.ctypes.data_as(C.c_void_p))
            st = raw[:640].reshape(64, 10).astype(np.int64)
            t0 = st[st[:, 0] > 0, 0].min()
            pk = raw[640:646].astype(np.int64)  # the last workgroup's pack phases
            out[f"msgs_{nm}"]["pack_stamps_us"] = [round((v - t0) / 100.0, 2) if v > 0 else None for v in pk]
            out[f"msgs_{nm}"]["stamps_us_from_first_entry"] = [
                [round((v - t0) / 100.0, 2) if v > 0 else None for v in row] for row in st if row[0] > 0]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
