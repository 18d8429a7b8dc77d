"""Where the host-inclusive pass's receive fill goes (bench.py ReceiveFill): the GPU box's NUMA
layout, the GPU's node, and the two-slot ingest rate of config B (1M x 64 B as 16,384 messages)
with the receive threads unpinned, pinned to the GPU's node, and pinned to another node; plus the
fill alone (no GPU work) at each placement.  Prints one JSON line.
    python tools/fill_probe.py [threads] [seconds]"""
import glob
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "trex-emu_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def cpulist(s):
    out = []
    for part in s.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def numa():
    nodes = {}
    for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        try:
            nodes[int(d.rsplit("node", 1)[1])] = cpulist(open(d + "/cpulist").read())
        except OSError:
            pass
    return nodes


def gpu_node():
    import torch
    try:
        p = torch.cuda.get_device_properties(0)
        want = f"{int(p.pci_domain_id):04x}:{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}."
        for f in glob.glob("/sys/bus/pci/devices/*/numa_node"):
            dev = f.split("/")[-2]
            if dev.lower().startswith(want):
                return int(open(f).read()), dev
        return None, want
    except Exception as e:  # noqa: BLE001
        return None, repr(e)


class PinnedFill:
    """ReceiveFill with each worker pinned to a CPU of `cpus` (None: unpinned)."""

    def __init__(self, threads, cpus):
        from concurrent.futures import ThreadPoolExecutor
        self.threads = threads
        self.cpus = cpus
        self.pool = ThreadPoolExecutor(threads)
        if cpus:
            k = [0]
            lock = threading.Lock()

            def pin():
                with lock:
                    c = cpus[k[0] % len(cpus)]
                    k[0] += 1
                os.sched_setaffinity(0, {c})
                time.sleep(0.05)
            for f in [self.pool.submit(pin) for _ in range(threads)]:
                f.result()

    def fill(self, dst, src):
        import ctypes
        n = src.nbytes
        chunk = ((n + self.threads - 1) // self.threads + 4095) & ~4095
        d, s = dst.ctypes.data, src.ctypes.data
        for f in [self.pool.submit(ctypes.memmove, d + o, s + o, min(chunk, n - o)) for o in range(0, n, chunk)]:
            f.result()


def main():
    import numpy as np
    import torch
    from emurx import frames as F
    from emurx import synth
    from emurx.rx import RxPath
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    torch.cuda.init()
    allowed = sorted(os.sched_getaffinity(0))
    nodes = numa()
    gn, gdev = gpu_node()
    res = {"allowed_cpus": len(allowed), "nodes": {k: len(v) for k, v in nodes.items()}, "gpu_node": gn, "gpu_pci": gdev,
           "threads": threads}
    w = synth.config_b(1 << 20)
    zs, msgs = F.zmq_messages(w["buf"], w["desc"], 64)
    rx = RxPath(0, max_ns=4096, max_clients=65536, max_frames=1 << 20)
    rx.register_all()
    synth.load_tables(w, rx)
    bufs = [rx.ingest_buffer(s, len(zs)) for s in range(2)]
    for s in range(2):
        np.copyto(bufs[s], zs)
        rx.ingest_submit(s, msgs)
        rx.ingest_wait(s, copy=False)
    places = {"unpinned": None}
    for k, v in nodes.items():
        c = [x for x in v if x in allowed]
        if c:
            places[f"node{k}"] = c
    for name, cpus in places.items():
        fl = PinnedFill(threads, cpus)
        t0, k = time.perf_counter(), 0
        while time.perf_counter() - t0 < secs / 2:
            fl.fill(bufs[k & 1], zs)
            k += 1
        fill_gbs = k * zs.nbytes / (time.perf_counter() - t0) / 1e9
        pending, k, t0 = [False, False], 0, time.perf_counter()
        while time.perf_counter() - t0 < secs or k < 4:
            s = k & 1
            if pending[s]:
                rx.ingest_wait(s, copy=False)
            fl.fill(bufs[s], zs)
            rx.ingest_submit(s, msgs)
            pending[s] = True
            k += 1
        for s in range(2):
            if pending[s]:
                rx.ingest_wait(s, copy=False)
        el = time.perf_counter() - t0
        res[name] = {"cpus": len(cpus) if cpus else None, "fill_alone_gbs": round(fill_gbs, 1),
                     "ingest_mpkts": round(k * len(w["desc"]) / el / 1e6, 1)}
        fl.pool.shutdown()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
