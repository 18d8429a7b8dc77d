"""k_rx's three kinds on the same batch (config D, 2M frames, 32K Namespaces / 1M clients, one
partition): parse only (emurx_parse_dev, k_rx<0>), parse + classify (emurx_classify_dev,
k_rx<1>) and parse + lookup keys packed per owner (emurx_parse_route_dev's k_rx<2>, its owner
counts and scan included and also timed alone), each as `reps` launches back to back on one
stream between one HIP event pair, over two batch slots.  What the partitioned source's packing
costs over the parse it shares with the other kinds.
    python tools/krx_kinds.py [frames] [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "trex-emu_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from emurx import abi, synth  # noqa: E402
from emurx.rx import RxPath  # noqa: E402


def main():
    import bench
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 21
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    w = synth.config_d(n, rank=0)
    rx = RxPath(0, max_ns=32768, max_clients=1 << 20, max_frames=n)
    rx.register_all()
    synth.load_tables(w, rx)
    dev = torch.device("cuda", 0)
    buf = torch.from_numpy(w["buf"]).to(dev)
    desc = torch.from_numpy(w["desc"].view(np.uint8).copy()).to(dev)
    slots = [(buf, desc), bench.permuted_batch(torch, buf, w["desc"], 77, dev)]
    st = torch.cuda.current_stream(dev)
    for fb, fd in slots:
        rx.desc_keys_dev(fb, fd, n, stream=st.cuda_stream)
    qcap = abi.queue_cap(n)
    rec = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device=dev)
    tc = torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device=dev)
    hist = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device=dev)
    cap, tcap = n, abi.tail_capacity(n)
    send = torch.empty(abi.lookup_region_bytes(cap, tcap), dtype=torch.uint8, device=dev)
    sc = torch.zeros(2, dtype=torch.int32, device=dev)
    calls = {
        "parse_k_rx0": lambda k: rx.classify_dev(slots[k % 2][0], slots[k % 2][1], n, rec, ql, qcap, tc, hist,
                                                 classify=False, stream=st),
        "classify_k_rx1": lambda k: rx.classify_dev(slots[k % 2][0], slots[k % 2][1], n, rec, ql, qcap, tc, hist,
                                                    stream=st),
        "parse_route_k_rx2_with_counts": lambda k: rx.parse_route_dev(slots[k % 2][0], slots[k % 2][1], n, None, ql,
                                                                      qcap, tc, hist, 1, 0, cap, send, sc,
                                                                      stream=st, tail_cap=tcap),
    }
    res = {"frames": n, "reps": reps, "lib": os.path.basename(os.environ.get("EMURX_LIB", "libemurx.so"))}
    for rnd in range(2):
        for name, f in calls.items():
            for k in range(6):
                f(k)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for k in range(reps):
                f(k)
            e1.record(st)
            torch.cuda.synchronize()
            res[f"{name}_us_{rnd}"] = round(e0.elapsed_time(e1) / reps * 1e3, 2)
    # k_rx<2> alone: the library's events around its launch
    rx.set_timing(reps + 8, 1)
    for k in range(reps):
        calls["parse_route_k_rx2_with_counts"](k)
    torch.cuda.synchronize()
    t = rx.kernel_times()
    rx.set_timing(0)
    res["k_rx2_alone_us"] = round(float(np.mean(t[2:])) * 1e3, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
