"""Timeline of one k_rx launch from the stamp build variant (experiment-only).

    tools/build_variant.sh stamp "-DEMURX_STAMP=1"
    EMURX_LIB=trex-emu_amd/lib/libemurx_stamp.so python tools/stamps.py [--replay] [B C E ...]

By default the launches rotate over 8 distinct batches (bench.py's batch slots: the input comes
from HBM); --replay stamps launches that re-read one batch (Infinity-Cache resident).

Every wave stores shader-clock stamps {entry, descriptors read, staging landed, parsed, lookup
key made, tables resolved, histogram, tile barrier entered / left, exit} plus HW_ID / XCC_ID (emurx_kernels.hip,
EMURX_STAMP); a phase a wave skipped (no lane took it) is folded into the next one. Printed per config:
the phase durations per wave, how many waves each CU held on average over the launch, and the
resident-wave profile over the launch (the shader clock is per XCD: spans are taken per CU).
"""
import ctypes
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "trex-emu_amd"))
sys.path.insert(0, str(ROOT))


def run(cfg, n, replay=False):
    import torch
    import bench
    from emurx import abi
    from emurx.rx import RxPath
    from emurx import synth
    w = bench.workload(cfg, n, 0)
    rx = RxPath(0, max_ns=max(4096, len(w["ns"])), max_clients=max(65536, len(w["clients"]["cid"])), max_frames=n)
    rx.register_all()
    synth.load_tables(w, rx)
    dev = torch.device("cuda", 0)
    buf = torch.from_numpy(w["buf"]).to(dev)
    desc = torch.from_numpy(w["desc"].view(np.uint8).copy()).to(dev)
    rec = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    qcap = abi.queue_cap(n)
    qlist = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device=dev)
    nt = abi.ntiles(n)
    tile_cnt = torch.empty(nt * 16, dtype=torch.int32, device=dev)
    hist = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    rx.sync(stream.cuda_stream)
    slots = [(buf, desc)] + ([] if replay else
                             [bench.permuted_batch(torch, buf, w["desc"], 1000 + j, dev) for j in range(1, 8)])
    calls = [rx.classify_call(b, d, n, rec, qlist, qcap, tile_cnt, hist, stream=stream) for b, d in slots]
    k = [0]

    def classify():
        calls[k[0] % len(calls)]()
        k[0] += 1
    lib = abi.load()
    lib.emurx_debug_set_stamps.argtypes = [ctypes.c_void_p]
    st = torch.zeros(nt * 4 * 16, dtype=torch.int64, device=dev)
    for _ in range(30):
        classify()
    torch.cuda.synchronize()
    out = []
    for rep in range(3):
        st.zero_()
        assert lib.emurx_debug_set_stamps(ctypes.c_void_p(st.data_ptr())) == 0
        for _ in range(5):
            classify()
        torch.cuda.synchronize()
        assert lib.emurx_debug_set_stamps(ctypes.c_void_p(0)) == 0
        out.append(st.cpu().numpy().reshape(-1, 16).astype(np.uint64))
    return out


def report(cfg, s):
    t = s[:, :10].astype(np.int64)
    ok = t[:, 0] > 0
    t, hw, xcc = t[ok], s[ok, 10], s[ok, 11]
    for k in range(1, 10):  # a skipped stamp takes the previous one (the phase cost nothing)
        t[:, k] = np.where(t[:, k] == 0, t[:, k - 1], t[:, k])
    END = 9
    cu = (xcc.astype(np.int64) << 16) | ((hw >> 8) & 0xff).astype(np.int64)
    d = np.diff(t, axis=1)
    life = t[:, END] - t[:, 0]
    print(f"== config {cfg}: {len(t)} waves, {len(np.unique(cu))} CUs, {len(np.unique(xcc))} XCDs")
    for k, name in enumerate(["descriptors", "staging", "parse (+coop csum)", "lookups (classify)",
                              "hist + queue ranks", "-", "records + owners", "tile barrier",
                              "queues/counts out"]):
        print(f"  {name:22s} cycles/wave mean {d[:, k].mean():8.0f}  p50 {np.median(d[:, k]):8.0f}  p90 {np.percentile(d[:, k], 90):8.0f}")
    print(f"  {'lifetime':22s} cycles/wave mean {life.mean():8.0f}  p50 {np.median(life):8.0f}  p90 {np.percentile(life, 90):8.0f}")
    spans, occ, nw = [], [], []
    for c in np.unique(cu):
        m = cu == c
        a, b = t[m, 0].min(), t[m, END].max()
        spans.append(b - a)
        occ.append(life[m].sum() / max(b - a, 1))
        nw.append(m.sum())
    spans, occ = np.array(spans), np.array(occ)
    print(f"  per CU: waves {np.mean(nw):.1f} (min {np.min(nw)} max {np.max(nw)}), span cycles mean {spans.mean():.0f} "
          f"min {spans.min()} max {spans.max()}, mean resident waves {occ.mean():.1f} (min {occ.min():.1f})")
    # resident-wave profile over the launch, CU-averaged, in 10 slices of each CU's span
    prof = np.zeros(10)
    for c in np.unique(cu):
        m = cu == c
        a, b = t[m, 0].min(), t[m, END].max()
        edges = np.linspace(a, b, 11)
        for j in range(10):
            lo, hi = edges[j], edges[j + 1]
            ov = np.clip(np.minimum(t[m, END], hi) - np.maximum(t[m, 0], lo), 0, None)
            prof[j] += ov.sum() / (hi - lo)
    prof /= len(np.unique(cu))
    print("  resident waves per CU over the span (10 slices): " + " ".join(f"{v:.1f}" for v in prof))


def main():
    replay = "--replay" in sys.argv
    cfgs = [a for a in sys.argv[1:] if not a.startswith("--")] or ["B"]
    sizes = {"B": 1 << 20, "C": 1 << 20, "E": 1 << 20, "D": 1 << 21}
    for c in cfgs:
        outs = run(c, sizes[c], replay)
        print("input:", "one batch replayed (Infinity Cache)" if replay else "8 rotating batches (HBM)")
        report(c, outs[-1])


if __name__ == "__main__":
    os.makedirs(ROOT / "gpurun_out", exist_ok=True)
    main()
