"""Tx framing (emurx_tx_zmq_dev) of config E's IMIX frames at several batch sizes: microseconds per
call and per 1M frames.  With one 64-frame tile per wave and ~2 generations of waves at 1M frames,
a per-frame cost that falls with the batch size says the launch's tail (the last generation's
uneven tiles) is part of the time.  HIP events around `reps` calls back to back.
    python tools/tx_scale_probe.py [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "trex-emu_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from emurx import synth  # noqa: E402
from emurx.rx import RxPath  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    res = {}
    rx = RxPath(0, max_ns=4096, max_clients=65536, max_frames=1 << 22)
    st = torch.cuda.current_stream()
    for cfg in ("E", "B"):
        for n in (1 << 18, 1 << 19, 1 << 20, 1 << 21, 1 << 22):
            w = synth.config_e(n) if cfg == "E" else synth.config_b(n)
            b = np.ascontiguousarray(w["buf"]).view(np.uint8)
            tb = torch.zeros(b.size + 64, dtype=torch.uint8, device="cuda")
            tb[: b.size] = torch.from_numpy(b.copy()).cuda()
            d = np.ascontiguousarray(w["desc"]).view(np.uint8)
            td = torch.from_numpy(d.copy()).cuda()
            need = 8 * n + int(w["desc"]["len"].astype(np.int64).sum())
            out = torch.empty(need + 64, dtype=torch.uint8, device="cuda")
            off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
            info = torch.empty(2, dtype=torch.int64, device="cuda")
            for _ in range(4):
                rx.tx_zmq_dev(tb, td, n, out, need, off, info, stream=st.cuda_stream)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(reps):
                rx.tx_zmq_dev(tb, td, n, out, need, off, info, stream=st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            res[f"{cfg}_{n}"] = {"us_per_call": round(us, 1), "us_per_1M_frames": round(us * (1 << 20) / n, 1),
                                 "gbs_moved": round((int(w["desc"]["len"].astype(np.int64).sum()) + need + 8 * n) / us / 1e3, 1)}
            del tb, td, out, off, info
            torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
