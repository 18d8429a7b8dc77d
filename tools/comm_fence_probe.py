"""The exchange step on a 1-rank library communicator (config D, 2M frames, 32K Namespaces / 1M
clients): parse_route_dev -> exchange_dev (whole regions) -> lookup_dev per batch on one stream,
`steps` batches over two rotating inputs, wall clock.  Run once per EMURX_COMM_FENCE setting
(device: the ordering events' release at device scope, the default; system: the HIP default,
a cache write-back and invalidate at each of the exchange's two event records) and with
EMURX_COMM_SELF=rccl for the own region through RCCL.  Prints one JSON line.
    python tools/comm_fence_probe.py [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "trex-emu_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from emurx import abi, synth  # noqa: E402
from emurx.rx import RxPath, comm_init_all  # noqa: E402


def main():
    import bench
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    n = 1 << 21
    w = synth.config_d(n, rank=0)
    rx = RxPath(0, max_ns=32768, max_clients=1 << 20, max_frames=n)
    rx.register_all()
    synth.load_tables(w, rx)
    comm_init_all([rx])
    dev = torch.device("cuda", 0)
    buf = torch.from_numpy(w["buf"]).to(dev)
    desc = torch.from_numpy(w["desc"].view(np.uint8).copy()).to(dev)
    slots = [(buf, desc), bench.permuted_batch(torch, buf, w["desc"], 77, dev)]
    st = torch.cuda.current_stream(dev)
    for fb, fd in slots:
        rx.desc_keys_dev(fb, fd, n, stream=st.cuda_stream)
    qcap = abi.queue_cap(n)
    ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device=dev)
    tc = torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device=dev)
    hist = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device=dev)
    cap = int(n * 1.06) + 1024
    tcap = abi.tail_capacity(cap)
    rb = abi.lookup_region_bytes(cap, tcap)
    send = torch.empty(rb, dtype=torch.uint8, device=dev)
    sc = torch.zeros(2, dtype=torch.int32, device=dev)
    recv = torch.empty(rb, dtype=torch.uint8, device=dev)
    rc = torch.zeros(2, dtype=torch.int32, device=dev)
    out = torch.empty(cap * 40, dtype=torch.uint8, device=dev)

    def step(k, xch=True):
        fb, fd = slots[k % 2]
        rx.parse_route_dev(fb, fd, n, None, ql, qcap, tc, hist, 1, 0, cap, send, sc, stream=st, tail_cap=tcap)
        if xch:
            rx.exchange_dev(send, sc, recv, rc, cap, tcap, stream=st)
            rx.lookup_dev(recv, rc, 1, cap, out, stream=st, tail_cap=tcap)
        else:
            rx.lookup_dev(send, sc, 1, cap, out, stream=st, tail_cap=tcap)

    res = {"fence": os.environ.get("EMURX_COMM_FENCE", "device"), "self": os.environ.get("EMURX_COMM_SELF", "copy"),
           "frames": n, "steps": steps, "region_bytes": rb}
    for rnd in range(2):
        for name, xch in (("with_exchange", True), ("no_exchange", False)):
            for k in range(8):
                step(k, xch)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(steps):
                step(k, xch)
            torch.cuda.synchronize()
            res[f"{name}_us_{rnd}"] = round((time.perf_counter() - t0) / steps * 1e6, 2)
    print(json.dumps(res), flush=True)
    rx.close()


if __name__ == "__main__":
    main()
