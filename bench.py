#!/usr/bin/env python3
"""Benchmark: Mpkt/s of device-resident rx parse+classify (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config B|C|D|E] [--frames F]
                    [--exchange] [--backend nccl|gloo] [--batches R] [--streams S]

A step = one batch through the hot path: emurx_classify_dev = one k_rx launch (decode +
checksums + Namespace/Client lookups + 32-B records + stable per-callback queue segments +
outcome histogram) over F frames already resident in HBM.  Default workload = config B
(1M x 64 B untagged IPv4/UDP, 1 Namespace / 1 Client), the configuration the metric is
quoted on.  The steps rotate through R distinct device-resident batches (--batches, default
8: seeded permutations of the workload's frames at distinct addresses, each slot with its own
outputs), so every byte's reuse distance is above the 256 MiB Infinity Cache and the input
comes from HBM, as fresh ZMQ batches do (veth_zmq.go:277-320).  Consecutive batches alternate
between two streams (--streams, default 2; slot j on stream j mod S, so the streams never share
an input), as the ingest path's two slots do: a batch's launch runs beside the previous one
instead of waiting for its last workgroups.  Warmup runs --warmup steps and then keeps going
until --warmup-seconds of wall time have passed (settled clocks for short runs).  For N > 1
(torchrun, one rank per GPU) every rank processes its own F-frame shard against replicated
tables: frames are independent, so there is no data-path collective (weak scaling); value =
frames over all ranks / max-over-ranks time.  At every N (N = 1 included) the Namespace-owner
exchange (config D, 2M frames per GPU, partitioned tables) is timed beside it with the same steps
and warmup (`namespace_exchange`); at N > 1 rank 0 also times its N = 1 twin in the same job
(`namespace_exchange.exchange_scaling_target`: the >= 6x-at-8-GPUs target of the north star).

--exchange (default for config D: 2M frames per GPU, 32K Namespaces / 1M Clients) adds the
Namespace-partitioned exchange to every step: emurx_parse_route_dev packs every frame's
lookup record into its Namespace owner's region, an all-to-all (RCCL over xGMI) delivers the
regions, with the per-region counts in a second all-to-all, and the owner resolves them.

The JSON line carries `roofline` (algorithmic bytes per frame = frame_len + 8 B descriptor
+ 32 B record + 4 B queue entry, over k_rx's duration with each launch alone: the same --steps
launches back to back on one stream over the rotating slots, one HIP event pair around them;
`roofline.pipelined` is the launch interval on the S streams of a second region of the same
steps right after the timed one (the wall-timed region itself carries no events), and
`roofline.cache_resident_replay` the round-2 replay of one batch per stream, labelled as such)
and `cpu_baseline` (the oracle, a single-threaded C restatement of the Go path, timed on this
host's cores over a bounded sample of the same workload; rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "trex-emu_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "Mpkt/s device-resident rx parse+classify, 1M×64B batch, 1/2/4/8 MI355X"


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="B", choices=["B", "C", "D", "E"])
    ap.add_argument("--frames", type=int, default=None,
                    help="frames per GPU per step (default 1M; config D: 2M = 16M over 8 GPUs)")
    ap.add_argument("--exchange", action="store_true",
                    help="route to the Namespace owners each step (= --tables partitioned)")
    ap.add_argument("--tables", choices=["none", "replicated", "partitioned"], default=None,
                    help="none: classify only; replicated / partitioned: Namespace-owner exchange each step "
                         "(default for D: partitioned, with the replicated alternative measured too)")
    ap.add_argument("--table-updates", action="store_true",
                    help="also time batches with 1 / 64 / 4096 table mutations between them")
    ap.add_argument("--a2a", choices=("auto", "v", "equal"), default="auto",
                    help="the exchange's transfer at N > 1: equal = whole regions, no host synchronisation; v = "
                         "counts, then only the spans that carry data (SURVEY §8e's all-to-all-v; the host waits "
                         "for the counts); auto (default) = both timed after the warmup, the faster one runs the "
                         "timed steps (namespace_exchange.exchange.a2a_choice)")
    ap.add_argument("--comm", choices=("library", "torch"), default="library",
                    help="N > 1 over nccl: library = the exchange through the C-ABI's own RCCL communicator "
                         "(emurx_comm_init + emurx_exchange_dev, what a Go caller drives; default); torch = "
                         "torch.distributed collectives.  gloo (CPU rehearsals) always uses torch.distributed")
    ap.add_argument("--exchange-frames", type=int, default=1 << 21,
                    help="frames per GPU of the config-D Namespace-exchange measurement beside the headline")
    ap.add_argument("--no-exchange-run", action="store_true",
                    help="skip the config-D Namespace-exchange measurement beside the config-B headline")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the multi-rank path with ranks sharing a GPU")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--time-stride", type=int, default=4,
                    help="record HIP events around every N-th launch of the timing pass (the timed region's steps once "
                         "more, after it)")
    ap.add_argument("--kernel-timing", default="region", choices=["region", "launch", "off"],
                    help="steps that are one k_rx launch (no exchange): region = an event pair per stream around "
                         "a second region of the same steps (the launch interval) and one around launches "
                         "back to back on one stream (each launch alone); launch = events around every "
                         "--time-stride-th launch of a timing pass; off = wall clock only")
    ap.add_argument("--streams", type=int, default=2,
                    help="steps without an exchange: consecutive batches go round-robin to this many "
                         "streams, each with its own output buffers, so a batch's k_rx runs beside the "
                         "previous one (as the ingest path's two slots do); 1 = back to back on one stream")
    ap.add_argument("--batches", type=int, default=8,
                    help="distinct device-resident batches the steps rotate through (batch k uses batch slot "
                         "k mod this, each slot its own frames, descriptors and outputs; the default 8 keeps "
                         "every byte's reuse distance above the 256 MiB Infinity Cache: the frames come from "
                         "HBM, as fresh batches do in production); 1 = the round-2 replay of one batch")
    ap.add_argument("--no-replay", action="store_true",
                    help="skip the cache-resident replay figure (profiling runs: every launch then reads HBM)")
    ap.add_argument("--warmup-seconds", type=float, default=0.3,
                    help="keep launching warmup steps until this much wall time has passed (clocks settle)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N > 1 with an exchange: run each timed batch's all-to-all to completion "
                         "before the next batch's parse (default: overlap them, two buffer sets)")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the output sanity check (stage-ablation builds, tools/abl_counts.sh)")
    ap.add_argument("--tx-path", action="store_true",
                    help="also time the device tx ZMQ framing (emurx_tx_zmq_dev) over the same frames")
    ap.add_argument("--launch-check", action="store_true",
                    help="rendezvous + max-over-ranks reduction only, no GPU (CPU test of the launch path)")
    ap.add_argument("--no-host-inclusive", action="store_true",
                    help="skip the default line's bounded host-inclusive block (every N)")
    ap.add_argument("--ingest-slots", type=int, default=2,
                    help="ingest slots the host-inclusive passes rotate through (one filled while the others "
                         "are in flight; at most EMURX_INGEST_SLOTS; 3 and 4 measured slower, DESIGN.md §6)")
    ap.add_argument("--host-path", action="store_true",
                    help="also time the host-inclusive path (pinned H2D + kernels + D2H)")
    ap.add_argument("--unkeyed", action="store_true",
                    help="leave the descriptors without owner keys (EMURX_DESC_KEYED): the partitioned source's "
                         "owner-count pass then reads every frame's L2 header instead of the descriptors alone")
    ap.add_argument("--dump-exchange", default=None, metavar="DIR",
                    help="N > 1 with an exchange: after the timed steps, run 4 more overlapped steps and write "
                         "every rank's received and resolved records per step, and its input batches, to DIR "
                         "(tests/test_bench_launch.py checks them against the oracle)")
    return ap.parse_args()


def workload(cfg, n, rank):
    from emurx import synth
    if cfg == "B":
        return synth.config_b(n, seed=synth.SEED_B + rank)
    if cfg == "C":
        return synth.config_c(n, rank=rank)
    if cfg == "D":
        return synth.config_d(n, rank=rank)
    return synth.config_e(n, rank=rank)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores():
    """CPU threads this process may use: the affinity mask, capped by OMP_NUM_THREADS (the GPU
    box exports the share of the machine a job gets; os.cpu_count() there is the whole host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else n


def cpu_baseline(w, budget_s):
    """Oracle (C restatement of the Go path: per-frame parse, byte-pair checksum, hash-map
    lookups) over repeated passes of a bounded sample of the same frames, on 1 host core and
    then on every core this job may use (frames split by offset, one thread per core; ctypes
    drops the GIL, the tables are shared read-only).  Test infrastructure: imported only here."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import threading
    import numpy as np
    import pyoracle
    from emurx import synth
    pyoracle.build()
    o = pyoracle.Oracle()
    synth.load_tables(w, o)
    sample = min(len(w["desc"]), 1 << 18)
    desc = np.ascontiguousarray(w["desc"][:sample])
    o.rx_batch(w["buf"], desc[:1024])  # warm

    def run(d, stop, out, k):
        frames = 0
        while time.perf_counter() < stop:
            o.rx_batch(w["buf"], d)
            frames += len(d)
        out[k] = frames

    one = [0]
    t0 = time.perf_counter()
    run(desc, t0 + budget_s, one, 0)
    el1 = time.perf_counter() - t0
    cores = host_cores()
    parts = np.array_split(desc, cores)
    outs = [0] * cores
    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(parts[k], t0 + budget_s * 0.75, outs, k)) for k in range(cores)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    eln = time.perf_counter() - t0
    return {"value": round(one[0] / el1 / 1e6, 3), "unit": "Mpkt/s", "cores": 1, "kind": "port",
            "sample": f"{sample} frames of config {w['name']} x {one[0] // sample} passes ({el1:.1f} s), "
                      "oracle/emurx_oracle.c rx_batch (parse + classify + queues + counters)",
            "cpu_model": cpu_model(),
            "all_cores": {"value": round(sum(outs) / eln / 1e6, 3), "cores": cores,
                          "seconds": round(eln, 1), "split": "frames by offset, one thread per core"}}


def spawn_ranks(a):
    """`bench.py --gpus N` without torchrun: start N fresh worker processes (one per GPU,
    before any GPU call in this one), rendezvous on 127.0.0.1, forward rank 0's JSON line."""
    import signal
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env,
                                      start_new_session=True))
    rc = 0
    live = list(procs)

    def stop_all(sig=signal.SIGTERM):
        for q in live:  # each rank leads its own session: signal its whole process group
            try:
                os.killpg(q.pid, sig)
            except OSError:
                pass

    # SIGINT / SIGTERM to this launcher reach the ranks too (they are in sessions of their own
    # and would otherwise keep their GPUs, waiting in a collective)
    class Stopped(Exception):
        pass

    def on_signal(signum, frame):
        raise Stopped(signum)
    old = {sg: signal.signal(sg, on_signal) for sg in (signal.SIGINT, signal.SIGTERM)}
    try:
        while live:
            time.sleep(0.2)
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    stop_all()  # a failed rank leaves the others waiting in a collective
    except Stopped as e:
        rc = 128 + int(e.args[0])
    finally:
        if live:  # interrupted (or an error here): end every rank still running, then reap them
            stop_all()
            deadline = time.time() + 10
            for q in live:
                try:
                    q.wait(max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    stop_all(signal.SIGKILL)
                    q.wait()
        for sg, h in old.items():
            signal.signal(sg, h)
    return rc


JSON_OUT = sys.stdout  # main() points it at the process's original stdout


def main():
    a = parse_args()
    if a.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_ranks(a))
    # stdout carries the one JSON line and nothing else: the rest of what this process writes
    # there (RCCL prints a version banner on stdout when a communicator is created) goes to stderr
    global JSON_OUT
    sys.stdout.flush()
    JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(a.gpus)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"warning: WORLD_SIZE={world} != --gpus {a.gpus}", file=sys.stderr)
    import torch
    import torch.distributed as dist
    if a.launch_check:
        sys.exit(launch_check(a, rank, world, dist, torch))
    if a.frames is None:
        a.frames = (1 << 21) if a.config == "D" else (1 << 20)
    mode = a.tables or ("partitioned" if a.config == "D" or a.exchange else "none")
    local = local % max(torch.cuda.device_count(), 1)  # gloo rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    out, rx, w = measure(a, a.config, a.frames, mode, a.steps, a.warmup, rank, world, local, dist, torch)
    if a.config == "B" and not a.no_host_inclusive and not a.host_path:
        # the north star's host-in / host-out rate, at every N (each rank through its own two
        # ingest slots, the node's aggregate): bounded to ~2 s, on the headline's handle
        try:
            out["host_inclusive"] = host_inclusive_block(rx, w, rank, world, dist, torch, a.backend,
                                                         slots=a.ingest_slots)
        except Exception as e:  # noqa: BLE001 - report, keep the headline line
            out["host_inclusive"] = {"error": repr(e)[:300]}
    if a.host_path:
        out["host_inclusive"] = host_path_rate(rx, w, slots=a.ingest_slots)
    if a.config == "D" and not a.no_exchange_run:
        # SURVEY.md §8e asks for both: the Namespace-partitioned lookups (the headline of D)
        # and the "replicas only" alternative (every GPU holds every table)
        other = "replicated" if mode == "partitioned" else "partitioned"
        try:
            rx.close()
            xo, rx, _ = measure(a, "D", a.frames, other, max(10, a.steps // 2), max(2, a.warmup // 2),
                                rank, world, local, dist, torch)
            out["alternative"] = {k: xo[k] for k in ("value", "unit", "ms_per_step", "steps", "exchange")}
            out["alternative"]["k_rx_ms_mean"] = xo["roofline"]["kernel_ms_mean"]
        except Exception as e:  # noqa: BLE001 - report, keep the headline line
            out["alternative"] = {"error": repr(e)[:300]}
    if a.config == "B" and not a.no_exchange_run:
        # The Namespace-owner exchange (MapNsT / GetNs thread_ctx.go:139,772-784
        # split over the GPUs), measured at EVERY N with the headline's steps and warmup: config
        # D, 2M frames per GPU, partitioned tables, lookup records all-to-all'd to the owners.
        # B's headline carries no collective at N > 1 (frames are independent), so the north
        # star's ">= 6x at 8 GPUs after the xGMI Namespace all-to-all" is judged on this block.
        try:
            rx.close()
            xo, rx, _ = measure(a, "D", a.exchange_frames, "partitioned", a.steps, a.warmup, rank, world, local, dist,
                                torch)
            out["namespace_exchange"] = exchange_block(xo)
            if world > 1:
                out["namespace_exchange"]["exchange_scaling_target"] = n1_twin(a, rank, world, local, dist, torch,
                                                                              out["namespace_exchange"])
        except Exception as e:  # noqa: BLE001 - report, keep the headline line
            out["namespace_exchange"] = {"error": repr(e)[:300]}
        out["config"]["scaling_note"] = (
            "B's value carries no collective at any N (frames are independent: weak scaling over offset shards); "
            "the north star's >= 6x-at-8-GPUs target after the xGMI Namespace all-to-all is judged on "
            "namespace_exchange (config D, 2M frames per GPU, partitioned tables), measured at every N with the "
            "same steps and warmup")
    if a.tx_path:
        out["tx_zmq"] = tx_zmq_rate(rx, w, torch)
        out["tx_checksum"] = tx_csum_rate(rx, w, torch)
    if a.table_updates and rank == 0:
        out["table_updates"] = table_update_cost(a, rx, w, torch)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(w, a.cpu_seconds)
        if "host_inclusive" in out and a.config == "B" and "batch_latency_by_msgs" in out["host_inclusive"]:
            out["host_inclusive"]["crossover"] = crossover(out["host_inclusive"], out["cpu_baseline"]["value"])
    if rank == 0:
        print(json.dumps(out), file=JSON_OUT, flush=True)
    rx.close()
    if world > 1:
        dist.destroy_process_group()


def progress(rank, msg):
    """A progress line on stderr (rank 0): a long run shows it is alive, and a log shows where
    a run that was stopped had got to (the JSON line comes only at the end)."""
    if rank == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def exchange_block(xo):
    """The namespace_exchange entry of the line: the exchange step's own measurement (value =
    frames over all ranks / max-over-ranks time; at N = 1 the two-stream pipelined rate, with
    the one-stream steps beside it in exchange.one_stream_steps) and its per-phase times."""
    b = {k: xo[k] for k in ("value", "unit", "n_gpus", "ms_per_step", "steps", "warmup", "config", "exchange",
                            "host_submit_ms_per_step")}
    b["k_rx_ms_mean"] = xo["roofline"]["kernel_ms_mean"]
    b["roofline"] = {k: xo["roofline"][k] for k in ("kernel", "achieved", "frac", "alg_bytes_per_launch")}
    return b


def n1_twin(a, rank, world, local, dist, torch, blk):
    """The N = 1 counterpart of an N > 1 namespace_exchange run, measured in the same job: rank 0
    runs the same exchange step (config D, its own 2M-frame shard, every table on its GPU, one
    partition, the same steps and warmup) while the other ranks wait; ratio = the N-GPU value /
    the faster of the two N = 1 figures (two-stream pipelined or one-stream steps)."""
    res = None
    if rank == 0:
        xo, rx1, _ = measure(a, "D", a.exchange_frames, "partitioned", a.steps, a.warmup, 0, 1, local, dist, torch)
        rx1.close()
        one = xo["exchange"].get("one_stream_steps", {}).get("value", xo["value"])
        best = max(xo["value"], one)
        res = {"n1_value": round(best, 2), "n1_pipelined_value": xo["value"], "n1_one_stream_value": one,
               "n_value": blk["value"], "n_gpus": world, "ratio": round(blk["value"] / best, 3),
               "target": 6.0, "target_n_gpus": 8, "target_ratio_at_this_n": round(6.0 * world / 8, 3),
               "source": "n1 measured in this job on rank 0's GPU after the N-rank run: the same exchange step "
                         "(config D, 2M frames, 32K ns / 1M clients, partitioned with 1 part), same steps and warmup; "
                         "ratio against the faster N = 1 figure"}
    if world > 1:
        dist.barrier()
    return res


def launch_check(a, rank, world, dist, torch):
    """The multi-rank skeleton of a bench run without the GPU: rendezvous on MASTER_ADDR,
    barrier, the max-over-ranks time reduction, rank 0's JSON line."""
    if os.environ.get("EMURX_BENCH_FAIL_RANK") == str(rank):
        return 3  # test hook: a rank that dies before the rendezvous completes
    if os.environ.get("EMURX_BENCH_HANG"):
        time.sleep(600)  # test hook: every rank stuck (as in a collective whose peer is gone)
    if os.environ.get("EMURX_BENCH_STDOUT_NOISE"):
        os.write(1, b"RCCL version : banner\n")  # test hook: a library writing to the stdout fd
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"launch_check": "ok", "n_gpus": world, "max_over_ranks": float(t.item()),
                          "master": os.environ.get("MASTER_ADDR")}), file=JSON_OUT, flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def permuted_batch(torch, buf_dev, desc_np, seed, dev):
    """Another device-resident batch of the same workload: the frames (each with its 4-byte ZMQ
    header) in a seeded permutation, laid out contiguously at new addresses, and its
    descriptors.  Same tables, same mix of shapes, distinct bytes at every address; gathered on
    the device (one index per byte)."""
    import numpy as np
    n = len(desc_np)
    perm = np.random.default_rng(seed).permutation(n)
    d = desc_np[perm].copy()
    seg = d["len"].astype(np.int64) + 4
    start = np.zeros(n, np.int64)
    if n > 1:
        start[1:] = np.cumsum(seg[:-1])
    total = int(seg.sum())
    shift = torch.from_numpy(desc_np["off"][perm].astype(np.int64) - 4 - start).to(dev)
    idx = torch.arange(total, device=dev, dtype=torch.int64)
    idx += torch.repeat_interleave(shift, torch.from_numpy(seg).to(dev), output_size=total)
    out = torch.zeros(total + 64, dtype=torch.uint8, device=dev)
    out[:total] = buf_dev[idx]
    del idx, shift
    d["off"] = (start + 4).astype(d["off"].dtype)
    return out, torch.from_numpy(d.view(np.uint8).copy()).to(dev)


def measure(a, cfg, n, mode, steps, warmup, rank, world, local, dist, torch):
    """Run `steps` timed batches of workload `cfg` (n frames per rank) -> (JSON dict, rx, w).
    mode: "none" (classify, no collective), "replicated" (every GPU holds every table:
    classify + route the found records to their Namespace owners + all-to-all), or
    "partitioned" (each GPU holds its Namespace partition: parse + lookup keys, all-to-all of
    the lookup records to the owners, lookups at the owner).  Step k reads batch slot k mod
    --batches (distinct frames and descriptors each, permuted_batch), so the input comes from
    HBM and not from the Infinity Cache a replayed batch would stay in."""
    import numpy as np
    from emurx import abi
    from emurx.rx import RxPath
    t_start = time.perf_counter()
    progress(rank, f"measure config {cfg}, {n} frames per GPU, tables {mode}, {world} rank(s)")
    w = workload(cfg, n, rank)
    max_ns = max(4096, len(w["ns"]))
    max_cl = max(65536, len(w["clients"]["cid"]) + (8192 if a.table_updates else 0))  # spare ids
    rx = RxPath(local, max_ns=max_ns, max_clients=max_cl, max_frames=n)
    rx.register_all()
    if mode == "partitioned":
        rx.set_partition(world, rank)  # device tables: this rank's Namespaces only
    from emurx import synth
    synth.load_tables(w, rx)

    dev = torch.device("cuda", local)
    S = max(1, a.streams) if mode == "none" else 1
    R = max(1, a.batches, S)
    R -= R % S  # every stream reads its own batch slots (slot j on stream j mod S)
    buf = torch.from_numpy(w["buf"]).to(dev)
    desc = torch.from_numpy(w["desc"].view(np.uint8).copy()).to(dev)
    inputs = [(buf, desc)] + [permuted_batch(torch, buf, w["desc"], (int(w["seed"]) << 8) + j + 1000 * rank, dev)
                              for j in range(1, R)]
    if not a.unkeyed:
        # the descriptors as the device framing walk hands them over (veth_zmq.go:277-320): each
        # with its frame's Namespace-owner key (EMURX_DESC_KEYED), which the walk derives from
        # the frame header it reads anyway; untimed, as the rest of the descriptors' making
        for fb, fd in inputs:
            rx.desc_keys_dev(fb, fd, n, stream=torch.cuda.current_stream(dev).cuda_stream)
    qcap = abi.queue_cap(n)

    def outputs():
        return (torch.empty(n * 32, dtype=torch.uint8, device=dev),
                torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device=dev),
                torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device=dev))
    rec, qlist, tile_cnt = outputs()
    hist = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device=dev)  # accumulates
    stream = torch.cuda.current_stream(dev)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    rx.sync(stream.cuda_stream)
    calls = one_calls = None
    if mode == "none":
        # batch slot j: its own frames, descriptors, records, queues and tile counts (the
        # histogram accumulates atomically: shared); launched on stream j mod S in the timed
        # steps, and all on one stream for the one-launch-at-a-time figure
        outs = [(rec, qlist, tile_cnt)] + [outputs() for _ in range(R - 1)]
        calls = [rx.classify_call(inputs[j][0], inputs[j][1], n, *outs[j][:2], qcap, outs[j][2], hist,
                                  stream=streams[j % S]) for j in range(R)]
        one_calls = [rx.classify_call(inputs[j][0], inputs[j][1], n, *outs[j][:2], qcap, outs[j][2], hist,
                                      stream=stream) for j in range(R)]

    xch = None
    if mode != "none":
        from emurx import exchange as X
        rb = X.LOOKUP_BYTES if mode == "partitioned" else X.REC_BYTES
        cap0 = X.capacity(n, world, slack=1.06)
        # partitioned: 32-byte lookup heads + tail shards per region, two counts per region
        # (heads, tail overflow); replicated: 40-byte classified records, one count
        xch = dict(cap=cap0, tcap=abi.tail_capacity(cap0) if mode == "partitioned" else None, ev=[], timing=False,
                   k=0, rb=rb, cs=2 if mode == "partitioned" else 1)
        xch["region"] = X.region_bytes(xch["cap"], xch["tcap"])

        # two buffer sets when the timed steps overlap batch k's exchange with batch k+1's parse,
        # each on its own compute stream (as the N = 1 pipelined steps): batch k+1's parse runs
        # beside batch k's all-to-all AND beside batch k-1's owner lookups
        nsets = 2 if world > 1 and not a.no_overlap else 1
        side = torch.cuda.Stream(dev) if nsets > 1 else None
        # the transfer: the library's own communicator (RCCL through the C-ABI) at N > 1 over
        # nccl, else torch.distributed (gloo rehearsals); whole regions or payload spans
        xch["lib"] = world > 1 and a.backend == "nccl" and a.comm == "library"
        xch["payload"] = a.a2a == "v"
        if xch["lib"]:
            # every rank binds RCCL before any joins the communicator (ncclCommInitRank waits for
            # all ranks): should one fail to, every rank takes torch.distributed instead, together
            from emurx.rx import comm_library
            xch["comm_library"] = comm_library()
            lib_ok = torch.tensor([1 if xch["comm_library"] else 0], dtype=torch.int64, device=dev)
            dist.all_reduce(lib_ok, op=dist.ReduceOp.MIN)
            if not int(lib_ok.item()):
                xch["lib"] = False
                xch["comm_fallback"] = "a rank could not bind RCCL (emurx_comm_library): torch.distributed"
                progress(rank, xch["comm_fallback"])
        if xch["lib"]:
            from emurx.rx import comm_unique_id
            uid = torch.zeros(128, dtype=torch.uint8, device=dev)
            if rank == 0:
                uid.copy_(torch.frombuffer(bytearray(comm_unique_id()), dtype=torch.uint8))
            dist.broadcast(uid, 0)  # the id out of band (a Go caller sends it its own way)
            rx.comm_init(bytes(uid.cpu().numpy()), world, rank)

        def alloc_regions():
            xch["sets"] = []
            for j in range(nsets):
                b = dict(send=torch.empty(world * xch["region"], dtype=torch.uint8, device=dev),
                         send_count=torch.zeros(world * xch["cs"], dtype=torch.int32, device=dev), pending=None,
                         st=stream if j == 0 else side, ev=None)
                # set 0 writes the handle's record / queue buffers (the sanity checks read them)
                b["rec"], b["qlist"], b["tile_cnt"] = (rec, qlist, tile_cnt) if j == 0 else outputs()
                if xch["lib"]:  # the library exchange's receive buffers (stream-ordered reuse)
                    b["recv"], b["recv_count"] = torch.empty_like(b["send"]), torch.empty_like(b["send_count"])
                if mode == "partitioned":
                    b["out"] = torch.empty(world * xch["cap"] * X.REC_BYTES, dtype=torch.uint8, device=dev)
                xch["sets"].append(b)
            xch.update(send=xch["sets"][0]["send"], send_count=xch["sets"][0]["send_count"],
                       out=xch["sets"][0].get("out"))
        alloc_regions()

        def lib_exchange(b, st):
            """batch b's transfer through the library's communicator, enqueued on st"""
            return rx.exchange_dev(b["send"], b["send_count"], b["recv"], b["recv_count"], xch["cap"],
                                   xch["tcap"] or 0, payload=xch["payload"], route=mode == "replicated", stream=st)

        def x_start(b):
            """batch b's transfer enqueued behind its stream (the payload form waits on the host
            for the batch's counts first)"""
            if xch["lib"]:
                b["pending"] = (None, b["recv"], b["recv_count"], lib_exchange(b, b["st"]))
                return
            with torch.cuda.stream(b["st"]):  # the collective waits for this set's stream
                if xch["payload"]:
                    b["pending"] = X.exchange_v_start(b["send"], b["send_count"], xch["region"], xch["cap"], rb)
                else:
                    b["pending"] = X.exchange_start(b["send"], b["send_count"], xch["region"])

        def x_sync(b):
            """(recv, recv_count, bytes sent to other ranks) of set b's transfer, on the launch
            stream, waited for.  A failure fails the run on every rank (no per-rank fallback:
            ranks that changed protocol alone would hang in mismatched collectives)"""
            if xch["lib"]:
                moved = lib_exchange(b, stream)
                return b["recv"], b["recv_count"], moved
            if xch["payload"]:
                return X.exchange_v(b["send"], b["send_count"], xch["region"], xch["cap"], rb)
            r, c = X.exchange(b["send"], b["send_count"], xch["region"])
            return r, c, (world - 1) * xch["region"]

        def produce(b, k):
            b["k"] = k
            fb, fd = inputs[k % R]
            if mode == "replicated":
                # classify + route in one call: the route's owner counts are taken inside k_rx
                rx.classify_route_dev(fb, fd, n, b["rec"], b["qlist"], qcap, b["tile_cnt"], hist, world, rank,
                                      xch["cap"], b["send"], b["send_count"], stream=b["st"])
            else:
                # no source records: every frame's lookup record carries its parse to the owner
                rx.parse_route_dev(fb, fd, n, None, b["qlist"], qcap, b["tile_cnt"], hist, world, rank, xch["cap"],
                                   b["send"], b["send_count"], stream=b["st"], tail_cap=xch["tcap"])

        def consume(b):
            with torch.cuda.stream(b["st"]):  # the set's stream waits for its all-to-all
                xch["recv"], xch["recv_count"] = X.exchange_finish(b["pending"])
            b["pending"] = None
            if mode == "partitioned":
                rx.lookup_dev(xch["recv"], xch["recv_count"], world, xch["cap"], b["out"], stream=b["st"],
                              tail_cap=xch["tcap"])
            if xch.get("dump") is not None:  # --dump-exchange: this step's owner records, as they are now
                torch.cuda.synchronize()
                cnt = xch["recv_count"].cpu().numpy().astype(np.int64)[0::xch["cs"]]
                res = (b["out"] if mode == "partitioned" else xch["recv"]).cpu().numpy()
                res = res.reshape(world, -1)[:, : xch["cap"] * X.REC_BYTES]  # owner outputs: cap route records
                xch["dump"].append(dict(k=b["k"], cnt=cnt, recs=np.concatenate(
                    [res[sr, : min(int(cnt[sr]), xch["cap"]) * X.REC_BYTES] for sr in range(world)])))

        def finish(b):
            consume(b)
            if b["ev"] is not None:
                b["ev"][1].record(b["st"])
                xch["ev"].append(b["ev"])
                b["ev"] = None

        def step_overlapped():
            """Batch k on set k mod 2's stream.  equal: parse + pack, then its all-to-all starts
            on the collective stream (behind that parse), then the previous batch's owner lookups
            are queued on ITS stream behind its own all-to-all.  v: the lookups of batch k-2 (the
            set's last batch, whose transfer started a step ago) are queued first, then batch k's
            parse + pack, and only then batch k-1's transfer, whose counts the host waits for:
            by then batch k's parse is queued behind it, so the GPU does not idle while the host
            waits.  Either way batch k's parse, batch k-1's transfer and batch k-2's lookups
            overlap.  Events time a batch from its parse to its lookups' end, on its stream."""
            k = xch["k"]
            xch["k"] += 1
            b, prev = xch["sets"][k % 2], xch["sets"][(k + 1) % 2]
            if xch["payload"] and b["pending"] is not None:
                finish(b)  # batch k - 2
            if xch["timing"] and k % a.time_stride == 0 and xch["pool"]:
                b["ev"] = xch["pool"].pop()
                b["ev"][0].record(b["st"])
            produce(b, k)
            if not xch["payload"]:
                x_start(b)
                if prev["pending"] is not None:
                    finish(prev)
                return
            b["await_x"] = True
            if prev.get("await_x"):  # batch k - 1
                prev["await_x"] = False
                x_start(prev)

        def drain():
            order = sorted(xch["sets"], key=lambda x: x.get("k", 0))
            for b in order:
                if b.get("await_x"):
                    b["await_x"] = False
                    x_start(b)
            for b in order:
                if b["pending"] is not None:
                    finish(b)

    kk = [0]

    def pipelined_rate():
        """N = 1 with the exchange's packing (no collective): consecutive batches alternate
        between two streams, each with its own records, queues, regions and owner outputs, as
        the timed steps of B / C / E do; wall clock over `steps` batches."""
        sets = []
        for j in range(max(2, a.streams)):
            b = dict(st=stream if j == 0 else torch.cuda.Stream(dev), send=torch.empty_like(xch["send"]),
                     send_count=torch.zeros_like(xch["send_count"]), r=torch.empty_like(rec),
                     q=torch.empty_like(qlist), t=torch.empty_like(tile_cnt))
            if mode == "partitioned":
                b["out"] = torch.empty_like(xch["out"])
            sets.append(b)

        def one(b, k):
            fb, fd = inputs[k % R]
            if mode == "replicated":
                rx.classify_route_dev(fb, fd, n, b["r"], b["q"], qcap, b["t"], hist, 1, 0, xch["cap"],
                                      b["send"], b["send_count"], stream=b["st"])
            else:
                rx.parse_route_dev(fb, fd, n, None, b["q"], qcap, b["t"], hist, 1, 0, xch["cap"],
                                   b["send"], b["send_count"], stream=b["st"], tail_cap=xch["tcap"])
                rx.lookup_dev(b["send"], b["send_count"], 1, xch["cap"], b["out"], stream=b["st"], tail_cap=xch["tcap"])
        for k in range(2 * len(sets)):
            one(sets[k % len(sets)], k)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for k in range(steps):
            one(sets[k % len(sets)], k)
        torch.cuda.synchronize()
        el1 = time.perf_counter() - t1
        return {"value": round(n * steps / el1 / 1e6, 2), "unit": "Mpkt/s", "ms_per_step": round(el1 / steps * 1e3, 4),
                "steps": steps, "streams": len(sets), "batches": R,
                "source": "wall clock; batch k on stream k mod streams with its own buffers"}

    def step():
        if xch is None:
            calls[kk[0] % R]()
            kk[0] += 1
            return
        ev = None
        if xch["timing"] and xch["k"] % a.time_stride == 0 and xch["pool"]:
            ev = xch["pool"].pop()  # created before the timed region: creating one costs ~50 us
            ev[0].record(stream)
        k = xch["k"]
        xch["k"] += 1
        produce(xch["sets"][0], k)
        if world > 1:
            xch["recv"], xch["recv_count"], _ = x_sync(xch["sets"][0])
        else:
            xch["recv"], xch["recv_count"] = xch["send"], xch["send_count"]
        if mode == "partitioned":
            rx.lookup_dev(xch["recv"], xch["recv_count"], world, xch["cap"], xch["out"], stream=stream,
                          tail_cap=xch["tcap"])
        if ev is not None:
            ev[1].record(stream)
            xch["ev"].append(ev)

    def phase_breakdown(reps=None):
        """Device time per phase of the exchange step, each phase as `reps` calls back to back
        on the launch stream between one HIP event pair (an event between two phases adds a
        barrier and a cache write-back of its own: round 6 measured the old per-phase events
        inflating the owner-count + scan phase from 12 to 69 us): the source side (owner counts +
        group scan + k_rx packing the lookup records, or k_rx + scan + route packing), k_rx alone
        (the library's events around its launch, a second pass), the all-to-all (counts +
        regions; RCCL's stream joined back into the launch stream), the owner's k_lookup; and
        the bytes that crossed to other ranks (whole regions: the all-to-all is equal-split) and
        the payload among them (heads + tail units, or routed records)."""
        reps = reps or max(4, min(steps, 30))
        b = xch["sets"][0]
        pairs = {}

        def group(name, fn):
            """fn(k) for k < reps between one event pair on the launch stream (one warm call
            first); the host enqueues them behind a spin so the pair times the device work"""
            fn(0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            with torch.cuda.stream(stream):
                torch.cuda._sleep(20_000_000)
            e0.record(stream)
            for k in range(reps):
                fn(k)
            e1.record(stream)
            torch.cuda.synchronize()
            pairs[name] = e0.elapsed_time(e1) / reps

        res = {}

        def a2a(k):
            res["x"] = x_sync(b) if world > 1 else (b["send"], b["send_count"], 0)

        group("src", lambda k: produce(b, k))
        a2a(0)
        recv, rc, sent = res["x"]
        if world > 1:
            group("a2a", a2a)
        if mode == "partitioned":
            group("look", lambda k: rx.lookup_dev(recv, rc, world, xch["cap"], b["out"], stream=stream,
                                                  tail_cap=xch["tcap"]))
        # k_rx alone: the library's events around each launch of a second source-side group
        rx.set_timing(reps + 8, 1)
        group("src_timed", lambda k: produce(b, k))
        krx = rx.kernel_times()
        rx.set_timing(0)
        src, a2a_ms = pairs["src"], pairs.get("a2a", 0.0)
        look = pairs.get("look")
        look_b2b = look
        k_rx_ms = float(np.mean(krx[1:])) if len(krx) > 1 else float("nan")
        sc = b["send_count"].cpu().numpy().astype(np.int64)[0::xch["cs"]]
        others = [d for d in range(world) if d != rank]
        # what crossed to other ranks: the counts and, per --a2a, the spans that carry data (v)
        # or whole regions (equal); the last step's, as every step of one batch sends the same
        moved = (sent if world > 1 else 0) + len(others) * 4 * xch["cs"]
        # payload per region: the heads (or routed records) and, partitioned, their tail units
        units = [0] * world
        if mode == "partitioned":
            sb = b["send"].cpu().numpy().reshape(world, -1)
            for d in range(world):
                hd = sb[d, : int(min(sc[d], xch["cap"])) * rb].view(abi.LOOKUP_REC_DTYPE)
                units[d] = int(X.tail_units(hd["w4"]).sum())
        payload = int(sum(int(sc[d]) * rb + 16 * units[d] for d in others))
        to_others = int(sum(int(sc[d]) for d in others))
        out = {"steps": reps, "source_side_ms": round(src, 5), "k_rx_ms": round(k_rx_ms, 5),
               ("owner_count_scan_ms" if mode == "partitioned" else "scan_pack_ms"): round(src - k_rx_ms, 5),
               "all_to_all_ms": round(a2a_ms, 5), "owner_lookup_ms": round(look, 5) if mode == "partitioned" else 0.0,
               "owner_lookup_kernel_ms": round(look_b2b, 5) if look_b2b is not None else None,
               "record_bytes": rb, "tail_units_per_shard": xch["tcap"], "region_bytes": xch["region"],
               "tail_bytes_per_frame": round(16 * sum(units) / max(int(sc.sum()), 1), 3),
               "transfer": ("counts, then the spans that carry data (grouped sends / receives)" if xch["payload"]
                            else "whole regions and counts in one grouped exchange"),
               "bytes_to_other_ranks": moved, "payload_bytes_to_other_ranks": payload,
               "frames_to_other_ranks": to_others,
               "bytes_per_frame_to_other_ranks": round(moved / to_others, 2) if to_others else None,
               "payload_bytes_per_frame_to_other_ranks": round(payload / to_others, 2) if to_others else None,
               "source": f"each phase as {reps} calls back to back on the launch stream between one HIP event pair "
                         "(no events between phases); k_rx by the library's events around each launch of a "
                         "second source-side group"}
        if world > 1 and a2a_ms > 0:
            out["xgmi_gbs"] = round(moved / (a2a_ms * 1e-3) / 1e9, 2)
            out["xgmi_payload_gbs"] = round(payload / (a2a_ms * 1e-3) / 1e9, 2)
        return out

    def warm_for_time():
        """Warmup floor in wall time (--warmup-seconds): a short --warmup would otherwise time
        the first launches at unsettled clocks.  Every rank runs the same number of rounds."""
        t_w = time.perf_counter()
        more = warmup > 0
        while more:
            for _ in range(max(R, 16)):
                step()
            torch.cuda.synchronize()
            go = torch.tensor([int(time.perf_counter() - t_w < a.warmup_seconds)], dtype=torch.int64)
            if world > 1:
                go = go.to(dev) if dist.get_backend() == "nccl" else go
                dist.all_reduce(go, op=dist.ReduceOp.MAX)
            more = bool(go.cpu().item())
        return time.perf_counter() - t_w

    for attempt in range(4):
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        if xch is None or not exchange_overflow(xch, world, dist, torch, dev):
            break
        # a region overflowed (send_count > cap, or a tail shard > tcap): grow every rank's
        # regions and redo
        xch["cap"], xch["tcap"] = grow_cap(xch, world, dist, torch, dev)
        xch["region"] = X.region_bytes(xch["cap"], xch["tcap"])
        alloc_regions()
        hist.zero_()
    def sanity():
        """The outcome on this rank (counts only; parity lives in tests/), after some steps."""
        from emurx.rx import hist_fold, pack_queues
        h = hist_fold(hist.cpu().numpy().view(np.uint64))
        assert int(h[0::2].sum()) % n == 0, "histogram does not cover the batches"
        _, qoff = pack_queues(qlist.cpu().numpy(), qcap, tile_cnt.cpu().numpy(), n)
        assert int(qoff[-1]) == n, "queues do not cover the batch"
        if xch is not None:
            xcheck(xch, rec, n, world, rank, dist, torch, dev, mode)
    if not a.no_check and warmup > 0:
        sanity()
    def choose_a2a(k_steps):
        """--a2a auto at N > 1: the two transfers timed one after the other over the same
        pipeline as the timed steps (k_steps each after 4 untimed, max over ranks), the faster
        kept.  Every rank decides on the same reduced times."""
        over = len(xch["sets"]) > 1
        res = {}
        for name, pl in (("equal", False), ("payload", True)):
            xch["payload"] = pl
            for reps in (4, k_steps):
                torch.cuda.synchronize()
                dist.barrier()
                xch["k"] = 0
                t0 = time.perf_counter()
                for _ in range(reps):
                    step_overlapped() if over else step()
                if over:
                    drain()
                t_sub = time.perf_counter() - t0
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
            t = torch.tensor([el, t_sub], dtype=torch.float64)
            t = t.to(dev) if dist.get_backend() == "nccl" else t
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el, t_sub = (float(x) for x in t.cpu())
            res[name] = {"value": round(n * world * k_steps / el / 1e6, 2), "ms_per_step": round(el / k_steps * 1e3, 4),
                         "host_submit_ms_per_step": round(t_sub / k_steps * 1e3, 4)}
        return a2a_choice_block(res, k_steps)

    # the time-based warmup last, right before the measurements: the host-side check above
    # leaves the GPU idle long enough for its clocks to drop, which a 20-step region would time
    warm_s = warm_for_time()
    if xch is not None and world > 1 and a.a2a == "auto":
        xch["a2a_choice"] = choose_a2a(max(10, min(steps, 40)))
        xch["payload"] = xch["a2a_choice"]["chosen"] == "payload"
        progress(rank, f"transfer: {xch['a2a_choice']['chosen']} ({xch['a2a_choice']})")
        warm_s += warm_for_time()

    progress(rank, f"config {cfg} {mode}: tables and batches ready, warmed up ({time.perf_counter() - t_start:.1f} s)")
    region = xch is None and a.kernel_timing == "region"
    # per-launch / per-batch HIP events (the exchange's phases, --kernel-timing launch) are
    # recorded in a second pass of the same steps after the timed region, never inside it
    timed_pass = xch is not None or a.kernel_timing == "launch"
    if xch is not None:
        xch["timing"] = False
        xch["ev"] = []
        xch["pool"] = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(steps // a.time_stride + 1)]
    reg_ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    for e in reg_ev:  # instantiate the events outside the timed region
        e.record(stream)
    # the region: a start and an end event on every stream (all recorded after the device-wide
    # synchronize), timed from the earliest start to the latest end.  No cross-stream wait: a
    # second stream held behind the first stream's start event began its first launch ~20 us
    # after the first one's (rocprofv3 trace, profiles/r03/prof_B_r03d_kernel_trace.csv.gz), a
    # stagger the short driver region paid once per run
    s_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in streams]
    for e0, e1 in s_ev:  # instantiate the events outside the timed region
        e0.record(stream)
        e1.record(stream)

    def region_open():
        for (e0, _), s2 in zip(s_ev, streams):
            e0.record(s2)

    def region_close():
        for (_, e1), s2 in zip(s_ev, streams):
            e1.record(s2)

    def region_ms():
        """Earliest start to latest end over the streams' event pairs (after a synchronize)."""
        base = s_ev[0][0]
        first = min([0.0] + [base.elapsed_time(e0) for e0, _ in s_ev[1:]])
        return max(base.elapsed_time(e1) for _, e1 in s_ev) - first

    one = replay = None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    overlapped = xch is not None and len(xch["sets"]) > 1
    if overlapped:
        xch["k"] = 0
    # the timed region holds the steps alone: its launch-interval events come from a second
    # region of the same steps right after it (an event pair per stream inside the wall-timed
    # region cost the 20-step command ~3 %, profiles/r06/ab_events/)
    t0 = time.perf_counter()
    for _ in range(steps):
        step_overlapped() if overlapped else step()
    if overlapped:
        drain()
    t_submit = time.perf_counter() - t0
    torch.cuda.synchronize()
    # this rank's time: its K steps up to the synchronize that drains them.  The closing barrier
    # aligns the ranks after it and stays out of the interval (its own latency, tens of us on
    # nccl, is not step work); the max over ranks below is the slowest rank's time
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    if not a.no_check and warmup == 0 and steps > 0:  # no warmup: check the timed steps' outputs
        sanity()
    interval = None
    if region:
        # the launch interval: the same steps again (the batch rotation continuing), an event
        # pair on every stream, earliest start to latest end
        region_open()
        for _ in range(steps):
            step()
        region_close()
        torch.cuda.synchronize()
        interval = region_ms() / steps
        # each launch alone (after the timed region, which runs straight after the time-based
        # warmup): the same rotation of batch slots, back to back on one stream
        # at least 100 launches, so that a short --steps still times the launch, not the
        # clocks' first reaction to the work
        n_one = max(steps, 100)
        reg_ev[0].record(stream)
        for k in range(n_one):
            one_calls[k % R]()
        reg_ev[1].record(stream)
        torch.cuda.synchronize()
        one = reg_ev[0].elapsed_time(reg_ev[1]) / n_one
        if R > S and not a.no_replay:
            # the round-2 replay: each stream re-reads one batch, which stays in the Infinity Cache
            region_open()
            for k in range(steps):
                calls[k % S]()
            region_close()
            torch.cuda.synchronize()
            replay = region_ms() / steps
        pk = [one]
    else:
        pk = []
        if timed_pass:
            # the timing pass: the timed region's steps once more with the library's launch
            # events (every --time-stride-th launch) and the batches' event pairs on
            rx.set_timing(steps + 8, a.time_stride)
            if xch is not None:
                xch["timing"] = True
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            for _ in range(steps):
                step_overlapped() if overlapped else step()
            if overlapped:
                drain()
            torch.cuda.synchronize()
            pk = rx.kernel_times()
            rx.set_timing(0)
            if xch is not None:
                xch["timing"] = False
    if xch is not None and any(exchange_overflow(dict(xch, send_count=b["send_count"]), world, dist, torch, dev)
                               for b in xch["sets"]):
        raise RuntimeError("exchange region overflow in the timed region")

    if a.dump_exchange and xch is not None and overlapped:
        dump_exchange(a, xch, inputs, R, rank, world, dist, torch, step_overlapped, drain)
    phases = None
    if xch is not None:
        phases = phase_breakdown()
    pipelined = None
    if xch is not None and world == 1 and a.streams > 1:
        pipelined = pipelined_rate()
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev if a.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total_frames = n * steps * world
    value = total_frames / el / 1e6
    ms_per_step = el / steps * 1e3

    # roofline of the dominant kernel (k_rx): algorithmic bytes / its mean launch duration.
    # Per frame: the frame, its 8-B descriptor and the 32-B record (104 B for a
    # 64-B frame), plus the 4-B queue entry k_rx also writes (the 32-B lookup head and the
    # batch's tail units instead of the record in the partitioned mode's k_rx)
    per_frame = 8 + 4 + 32
    tail_bytes = int(round((phases or {}).get("tail_bytes_per_frame", 0.0) * n)) if mode == "partitioned" else 0
    alg_bytes = w["nbytes"] + per_frame * n + tail_bytes
    parse_s = float(np.mean(pk)) * 1e-3 if len(pk) else float("nan")
    achieved = alg_bytes / parse_s / 1e9
    traffic, pmc_src = None, None
    # the PMC passes of the same config and table mode (tools/round_profile.sh: D = partitioned,
    # DN = --tables none, DR = replicated)
    tag = cfg + ({"none": "N", "replicated": "R"}.get(mode, "") if cfg == "D" else "")
    pmc = ROOT / "profiles" / f"pmc_config{tag}.json"
    if pmc.exists():
        try:
            traffic = json.loads(pmc.read_text()).get("k_rx_hbm_bytes_per_launch")
            pmc_src = str(pmc.relative_to(ROOT))
        except Exception:  # noqa: BLE001
            traffic = None
    copy_gbs = copy_ceiling(torch, dev, stream)
    # the Namespace + Client bucket reads of every frame that reaches a callback (two 64-B
    # buckets, issued together): outside the algorithmic bytes, served by L2 / MALL / HBM
    r = rec.cpu().numpy().view(abi.REC_DTYPE)
    probed = int((r["status"] == 0).sum()) if mode != "partitioned" else 0
    ts = rx.table_stats()
    par = {"none": f"frame shards x{world}, replicated tables, no collective",
           "replicated": f"frame shards x{world}, replicated tables, classified records to the Namespace "
                         f"owners (all-to-all, {a.backend})",
           "partitioned": f"frame shards x{world}, Namespace-partitioned tables, lookup records to the "
                          f"Namespace owners (all-to-all, {a.backend}), lookups at the owner"}[mode]
    in_bytes = w["nbytes"] + 4 * n + 64 + 8 * n  # a batch slot's frames (ZMQ layout) + descriptors
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Mpkt/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic (seeded, valid wire-format frames); {R} distinct device-resident batches per GPU "
                f"(seeded permutations of the workload's frames at distinct addresses), step k reads batch k mod {R}",
        "config": {
            "workload": {"B": "B: 1M x 64B untagged IPv4/UDP, 1 ns / 1 client",
                         "D": "D: 2M mixed dot1q/QinQ IPv4/IPv6 per GPU (16M over 8), 32K ns / 1M clients",
                         "C": "C: 1M mixed dot1q/QinQ IPv4/IPv6, 4K ns / 64K clients",
                         "E": "E: IMIX 64/594/1518 TCP/UDP, 4K ns / 64K clients"}[cfg],
            "frames_per_gpu": n,
            "frame_bytes_per_gpu": w["nbytes"],
            "parallelism": par,
            "tables": mode if mode != "none" else "replicated",
            "descriptors": "unkeyed" if a.unkeyed else "keyed (EMURX_DESC_KEYED owner keys, as the device framing walk writes them)",
            "table_bytes_per_gpu": ts["table_bytes"],
            "streams": S,
            "batches": R,
            "input_bytes_per_batch": in_bytes,
            "input_reuse_distance_bytes": R * in_bytes,  # > 256 MiB: not served by the Infinity Cache
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": pmc_src,
            "copy_ceiling_gbs": round(copy_gbs, 1),  # a streaming copy on this GPU, measured here
            "frac_of_copy_ceiling": round(achieved / copy_gbs, 4) if copy_gbs > 0 else None,
            "kernel": "k_rx" + (" (parse + lookup keys)" if mode == "partitioned" else ""),
            "alg_bytes_per_launch": alg_bytes,
            "alg_bytes_per_frame": round(alg_bytes / n, 2),
            "alg_bytes_note": "frame + 8-B descriptor + 32-B record (SURVEY.md §8d) + the 4-B queue entry k_rx also "
                              "writes" + ("; the 32-B lookup head (+ the batch's 16-B tail units) instead of the record"
                                          if mode == "partitioned" else ""),
            "table_probe_bytes_per_launch": probed * 128 if mode != "partitioned" else 0,
            "kernel_ms_mean": round(parse_s * 1e3, 5),
            "kernel_launches_timed": max(steps, 100) if region else int(len(pk)),
            "kernel_time_source": ("one HIP event pair on the launch stream around max(--steps, 100) launches back "
                                   f"to back on one stream, rotating over the {R} batch slots, right after the timed "
                                   "region: elapsed / launches = each launch alone (what rocprofv3's kernel "
                                   "trace times, plus the ~1 us dispatch gap between launches)" if region else
                                   f"HIP events on the launch stream around every {a.time_stride}-th "
                                   "k_rx launch of a second pass of the timed region's steps (the timed region "
                                   "itself carries no events)"),
        },
        "warmup_seconds": round(warm_s, 3),
        "host_submit_ms_per_step": round(t_submit / steps * 1e3, 5),
    }
    if interval is not None:
        out["roofline"]["pipelined"] = {
            "interval_ms": round(interval, 5), "achieved": round(alg_bytes / (interval * 1e-3) / 1e9, 1),
            "frac": round(alg_bytes / (interval * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "streams": S,
            "source": f"a second region of the timed region's steps right after it: a HIP event pair on each of the "
                      f"{S} streams (no cross-stream waits), earliest start to latest end / launches = the launch "
                      "interval in steady state (each launch overlaps its neighbours); the wall-timed region itself "
                      "carries no events"}
    if mode == "none" and cfg == "D" and world == 1 and pmc.exists():
        # D classification (k_rx probing 1.75 GB of sparse tables) against the random-line bound,
        # as the owner's k_lookup: the excess FETCH of the calibrated PMC is probe lines
        # (pmc_summary.py's rule for this config), per launch, at the measured random-line rate of an
        # HBM-sized table, plus the algorithmic bytes at the copy ceiling (additive)
        try:
            pj = json.loads(pmc.read_text())
            lines = pj["excess_fetch_bytes"] / 64 * n / (1 << 21)
            rate = 48.8e9  # profiles/r05/probe_rate/rates.txt, 512 MB table
            floor_ms = (lines / rate + alg_bytes / (copy_gbs * 1e9)) * 1e3
            look = parse_s * 1e3
            out["roofline"]["random_line"] = {
                "kernel": "k_rx (parse + classify, full tables)", "probe_lines_per_launch": int(lines),
                "line_rate_glines_per_s": rate / 1e9, "stream_bytes_per_launch": int(alg_bytes),
                "floor_ms": round(floor_ms, 5), "measured_ms": round(look, 5), "frac": round(floor_ms / look, 4),
                "source": f"{pmc.relative_to(ROOT)} (excess FETCH as 64-byte probe lines), "
                          "profiles/r05/probe_rate/rates.txt (line rate), this run's copy ceiling and kernel_ms_mean "
                          "(one launch); frac >= 1 where probe lines hit the Infinity Cache"}
        except Exception as e:  # noqa: BLE001
            out["roofline"]["random_line"] = {"error": repr(e)[:200]}
    if replay is not None:
        out["roofline"]["cache_resident_replay"] = {
            "interval_ms": round(replay, 5), "value": round(n / (replay * 1e-3) / 1e6, 2),
            "frac": round(alg_bytes / (replay * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "source": f"the round-2 measurement: {S} streams each replaying one batch slot (its input stays in the "
                      "256 MiB Infinity Cache); same event pairs, not the metric"}
    if xch is not None:
        xm = [e0.elapsed_time(e1) for e0, e1 in xch["ev"]]
        step_ms = float(np.mean(xm)) if xm else float("nan")
        out["exchange"] = {
            "mode": mode,
            "step_device_ms_mean": round(step_ms, 5),
            "beyond_k_rx_ms_mean": round(step_ms - parse_s * 1e3, 5),
            "steps_timed": len(xm),
            "records_per_region_cap": xch["cap"],
            "record_bytes": xch["rb"],
            "tail_units_per_shard": xch["tcap"],
            "region_bytes": xch["region"],
            "collective": (("emurx_exchange_dev over the library's own RCCL communicator (emurx_comm_init; "
                            "ncclSend / ncclRecv to every peer in one group), " if xch["lib"] else
                            f"torch.distributed ({a.backend}): ") +
                           ("counts, host waits, then the spans that carry data" if xch["payload"]
                            else "whole regions, no host synchronisation")) if world > 1 else "none (1 rank)",
            "transfer_mode": ("payload" if xch["payload"] else "equal") if world > 1 else None,
            "comm_fallback": xch.get("comm_fallback"),
            "comm_library": xch.get("comm_library"),
            "a2a_choice": xch.get("a2a_choice"),
            "overlapped": overlapped,  # batch k's all-to-all beside batch k+1's parse (two buffer sets)
            "includes": ("k_rx + group scan + pack" + (" + all-to-all" if world > 1 else "") +
                         (" + owner lookups (k_lookup)" if mode == "partitioned" else "")),
            "phases": phases,
        }
        pmc_x = ROOT / "profiles" / "pmc_exchangeD.json"
        # the PMC calibration is of one owner holding every table (N = 1, 2M frames): the block is
        # reported for that step only (an owner of N holds 1/N of the tables: other line rates)
        if (mode == "partitioned" and cfg == "D" and world == 1 and pmc_x.exists() and phases
                and phases.get("owner_lookup_kernel_ms")):
            # the owner's k_lookup against ITS roofline: random 64-B probe lines that leave L2
            # (calibrated PMC, per launch, scaled to this batch) at the measured random-line rate
            # of an HBM-sized table, plus its streamed records at the copy ceiling (additive, as
            # the calibration's stream + probes mode measured)
            try:
                px = json.loads(pmc_x.read_text())
                lines = px["k_lookup"]["probe_lines_per_launch"] * n / (1 << 21)
                rate = px["line_rate_glines_per_s"]["hbm_sized_table"] * 1e9
                stream_b = (32 + 0.8 + 40) * n
                floor_ms = (lines / rate + stream_b / (copy_gbs * 1e9)) * 1e3
                look = phases["owner_lookup_kernel_ms"]
                out["exchange"]["random_line"] = {
                    "kernel": "k_lookup", "probe_lines_per_launch": int(lines), "line_rate_glines_per_s": rate / 1e9,
                    "stream_bytes_per_launch": int(stream_b), "floor_ms": round(floor_ms, 5), "measured_ms": look,
                    "frac": round(floor_ms / look, 4),
                    "hbm_frac_alg_bytes": round(stream_b / (look * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "source": f"{pmc_x.relative_to(ROOT)} (probe lines), profiles/r05/probe_rate/rates.txt (line rate), "
                              "this run's copy ceiling and phases.owner_lookup_kernel_ms (launches back to back); "
                              "frac >= 1 where probe lines hit the Infinity Cache, which the HBM-sized table's rate "
                              "does not credit"}
            except Exception as e:  # noqa: BLE001
                out["exchange"]["random_line"] = {"error": repr(e)[:200]}
        if pipelined is not None:
            # N = 1: the line's value is the pipelined rate, as for the one-launch steps of
            # B / C / E; the back-to-back steps above stay beside it
            out["exchange"]["pipelined"] = pipelined
            out["exchange"]["one_stream_steps"] = {"value": out["value"], "ms_per_step": out["ms_per_step"]}
            out["value"], out["ms_per_step"] = pipelined["value"], pipelined["ms_per_step"]
        if mode == "partitioned" and not a.unkeyed:
            # the owner keys the timed steps read from the descriptors are derived by the device
            # framing walk: what that derivation costs the walk is added to every step (VERDICT
            # r04 item 2), so the value covers every byte of parse work the step depends on
            kd = key_derivation(rx, w, torch, dev, stream, inputs[0][1])
            t = torch.tensor([kd["key_ms"]], dtype=torch.float64)
            if world > 1:
                t = t.to(dev) if a.backend == "nccl" else t
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
            key_ms = float(t.cpu().item())
            kd["key_ms_max_over_ranks"] = round(key_ms, 5)
            out["exchange"]["key_derivation"] = kd
            out["exchange"]["without_key_derivation"] = {"value": out["value"], "ms_per_step": out["ms_per_step"]}
            ms = out["ms_per_step"] + key_ms
            out["value"], out["ms_per_step"] = round(n * world / (ms * 1e-3) / 1e6, 2), round(ms, 4)
            one = out["exchange"].get("one_stream_steps")
            if one is not None:  # the same key cost on the one-stream figure (n1_twin compares the two)
                one["without_key_derivation"] = {"value": one["value"], "ms_per_step": one["ms_per_step"]}
                ms1 = one["ms_per_step"] + key_ms
                one["value"], one["ms_per_step"] = round(n * world / (ms1 * 1e-3) / 1e6, 2), round(ms1, 4)
    return out, rx, w


def a2a_choice_block(res, k_steps):
    """The namespace_exchange line's record of --a2a auto: both transfers' rates (frames over all
    ranks / the slowest rank's time), their host submit time per step, and the one chosen (the
    lower ms_per_step; ties keep the sync-free whole regions)."""
    chosen = "payload" if res["payload"]["ms_per_step"] < res["equal"]["ms_per_step"] else "equal"
    return dict(res, chosen=chosen, steps_each=k_steps,
                source="after the warmup: 4 untimed + steps_each timed steps of each transfer over the timed steps' "
                       "pipeline, wall clock, max over ranks; the faster runs the timed steps")


def key_derivation(rx, w, torch, dev, stream, keyed_desc, per_msg=64, reps=30):
    """Device time the Namespace-owner keys add to the framing walk (k_zmq_walk, emurx_zmq_walk_dev)
    on this batch packed as ZMQ messages of `per_msg` frames (veth_zmq.go:36-37,277-320): the walk
    with the keys and without (EMURX_WALK_NO_KEYS), alternated, `reps` launches each, each timed
    by its own event pair on the launch stream; key_ms = the difference of the medians (>= 0).
    The keyed descriptors are checked against the untimed emurx_desc_keys_dev ones."""
    import numpy as np
    from emurx import abi
    from emurx import frames as F
    n = len(w["desc"])
    zs, msgs = F.zmq_messages(w["buf"], w["desc"], per_msg)
    nmsg = len(msgs)
    per = np.minimum(per_msg, n - per_msg * np.arange(nmsg)).astype(np.uint32)
    base = np.zeros(nmsg + 1, np.uint32)
    base[1:] = np.cumsum(per)
    ctl = np.concatenate([np.ascontiguousarray(msgs).view(np.uint32).reshape(-1), base])
    d_buf = torch.from_numpy(np.concatenate([zs, np.zeros(64, np.uint8)])).to(dev)
    d_ctl = torch.from_numpy(ctl.view(np.int32)).to(dev)
    d_desc = torch.empty(n * 8, dtype=torch.uint8, device=dev)
    d_stat = torch.empty(nmsg, dtype=torch.int32, device=dev)
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(2 * reps)]
    sc = stream.cuda_stream
    for k in range(6):
        rx.zmq_walk_dev(d_buf, d_ctl, nmsg, d_desc, d_stat, keys=bool(k & 1), stream=sc)
    for k in range(2 * reps):
        ev[k][0].record(stream)
        rx.zmq_walk_dev(d_buf, d_ctl, nmsg, d_desc, d_stat, keys=bool(k & 1), stream=sc)
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    ms = np.array([e0.elapsed_time(e1) for e0, e1 in ev])
    plain, keyed = float(np.median(ms[0::2])), float(np.median(ms[1::2]))
    got = d_desc.cpu().numpy().view(abi.DESC_DTYPE)
    st = d_stat.cpu().numpy()
    assert (st >> 24 == 0).all() and int((st & 0xFFFFFF).sum()) == n, "framing walk of the bench batch"
    want = keyed_desc.cpu().numpy()[: n * 8].view(abi.DESC_DTYPE)  # emurx_desc_keys_dev's keys
    assert np.array_equal(got["pad"], want["pad"]), "the walk's owner keys equal emurx_desc_keys_dev's"
    return {"key_ms": round(max(0.0, keyed - plain), 5), "walk_keyed_ms": round(keyed, 5),
            "walk_plain_ms": round(plain, 5), "messages": nmsg, "frames_per_msg": per_msg,
            "source": "k_zmq_walk (emurx_zmq_walk_dev) on this batch as ZMQ messages, with and without the owner "
                      f"keys, medians of {reps} launches each (HIP events); key_ms is added to every timed step"}


def dump_exchange(a, xch, inputs, R, rank, world, dist, torch, step_overlapped, drain, k_steps=4):
    """--dump-exchange: k_steps more steps of the overlapped pipeline exactly as timed (batch k's
    all-to-all started, then the previous batch's owner lookups), each step's records saved
    when its consume() has run; then the batch slots' frames and descriptors.  Untimed."""
    import numpy as np
    d = Path(a.dump_exchange)
    d.mkdir(parents=True, exist_ok=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    xch["k"] = 0
    xch["dump"] = []
    for _ in range(k_steps):
        step_overlapped()
    drain()
    torch.cuda.synchronize()
    for e in xch["dump"]:
        np.savez(d / f"rank{rank}_step{e['k']}.npz", cnt=e["cnt"], recs=e["recs"], slot=e["k"] % R,
                 cap=xch["cap"], mode=xch["rb"], tcap=xch["tcap"] or 0)
    for j in range(R):
        np.savez(d / f"rank{rank}_slot{j}.npz", buf=inputs[j][0].cpu().numpy(), desc=inputs[j][1].cpu().numpy())
    xch["dump"] = None
    if world > 1:
        dist.barrier()


def table_update_cost(a, rx, w, torch, rounds=8):
    """Cost of table mutations between batches (the incremental shipment, include/emu_rx.h
    emurx_sync): before every batch, K calls of a mix of CNSCtx.UpdateClientIpv4, AddClient and
    RemoveClient (ns_ctx.go:332-471) on the workload's tables, then one classify_dev.  Device
    time per batch from CUDA events around the call (the delta copy and k_apply run on the
    batch's stream ahead of k_rx), host time of the call itself (gathering the edited blocks);
    the mutation calls are not timed.  Last: the cost of a full rebuild + upload of every
    table, what any mutation cost before the incremental path."""
    import numpy as np
    from emurx import abi
    n = len(w["desc"])
    dev = torch.device("cuda", torch.cuda.current_device())
    buf = torch.from_numpy(w["buf"]).to(dev)
    desc = torch.from_numpy(w["desc"].view(np.uint8).copy()).to(dev)
    d_rec = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    qcap = abi.queue_cap(n)
    qlist = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device=dev)
    tile_cnt = torch.empty(abi.ntiles(n) * 16, dtype=torch.int32, device=dev)
    hist = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)
    call = rx.classify_call(buf, desc, n, d_rec, qlist, qcap, tile_cnt, hist, stream=st)
    c = w["clients"]
    ncl = len(c["cid"])
    spare = int(rx.cfg.max_clients) - ncl
    out = {"frames": n, "clients": ncl, "rounds": rounds}

    def one(k, r):
        # k mutations: a third IPv4 updates, a third AddClient of spare ids, a third RemoveClient
        # of the spare clients added by the previous round
        for j in range(k):
            op, idx = j % 3, j // 3
            if op == 0:
                cid = int(c["cid"][(idx * 7919 + r) % ncl])
                rx.client_update_ipv4(cid, bytes([172, 16 + (r & 7), (idx >> 8) & 0xFF, idx & 0xFF]))
            elif spare > idx:
                ns = int(c["ns"][idx % ncl])
                mac = bytes([6, 0xEE, (idx >> 16) & 0xFF, (idx >> 8) & 0xFF, idx & 0xFF, 1])
                if op == 1 and r % 2 == 0:
                    rx.client_add(ns, ncl + idx, mac, None, None, None, 0x7FF)
                elif op == 2 and r % 2 == 1:
                    rx.client_remove(ns, mac)

    for k in (0, 1, 64, 4096):
        dev_ms, host_ms = [], []
        for r in range(rounds + 2):
            one(k, r)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            t0 = time.perf_counter()
            call()
            t1 = time.perf_counter()
            e1.record(st)
            torch.cuda.synchronize()
            if r >= 2:
                dev_ms.append(e0.elapsed_time(e1))
                host_ms.append((t1 - t0) * 1e3)
        out[f"k{k}"] = {"device_ms_per_batch": round(float(np.median(dev_ms)), 4),
                        "host_ms_in_call": round(float(np.median(host_ms)), 4)}
    blocks, whole, nbytes = (rx.table_stats()[x] for x in ("delta_blocks", "whole_tables", "table_bytes"))
    out["delta_blocks_total"], out["table_bytes"] = blocks, nbytes
    # a full rebuild + whole upload (set_partition(1, 0) rebuilds every table)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rx.set_partition(1, 0)
    call()
    torch.cuda.synchronize()
    out["full_rebuild_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    return out


def copy_ceiling(torch, dev, stream, mib=1024, reps=8):
    """HBM ceiling as this GPU runs it: a 1 GiB streaming copy (emurx_copy_ceiling_dev: 16-byte
    non-temporal loads and stores, 4 in flight per lane over 16,384 workgroups), read + write bytes over the
    HIP-event time of `reps` copies."""
    try:
        from emurx import abi
        lib = abi.load()
        n = mib << 20
        src = torch.empty(n, dtype=torch.uint8, device=dev)
        dst = torch.empty_like(src)

        def once():
            abi.check(lib.emurx_copy_ceiling_dev(dst.data_ptr(), src.data_ptr(), n, stream.cuda_stream), "copy")
        once()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            once()
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        del src, dst
        return 2 * n / (ms * 1e-3) / 1e9
    except Exception:  # noqa: BLE001 - a reported context figure, never the metric
        return 0.0


def exchange_overflow(xch, world, dist, torch, dev):
    """Did any rank's region overflow (send_count > cap, or a tail shard past tcap) in the last
    step? (every step routes the same batch, so the last step's counts are every step's)"""
    c = xch["send_count"].cpu()
    over = (c[0::xch["cs"]] > xch["cap"]).any()
    if xch["cs"] == 2:
        over = over or (c[1::2] > xch["tcap"]).any()
    over = torch.tensor([int(over)], dtype=torch.int64)
    if world > 1:
        over = over.to(dev) if dist.get_backend() == "nccl" else over
        dist.all_reduce(over, op=dist.ReduceOp.MAX)
    return bool(over.cpu().item())


def grow_cap(xch, world, dist, torch, dev):
    """(cap, tcap) after an overflow, the same on every rank."""
    from emurx import exchange as X
    c = xch["send_count"].cpu()
    m = torch.tensor([int(c[0::xch["cs"]].max()), int(c[1::2].max()) if xch["cs"] == 2 else 0], dtype=torch.int64)
    if world > 1:
        m = m.to(dev) if dist.get_backend() == "nccl" else m
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
    m = m.cpu().tolist()
    tcap = X.grow_tail(xch["tcap"], [m[1]]) if xch["cs"] == 2 else None
    return X.grow(xch["cap"], [m[0]]), tcap


def xcheck(xch, rec, n, world, rank, dist, torch, dev, mode):
    """Exchange sanity (counts only; the packing is parity-tested in tests/): every routed
    record arrives once, within capacity (replicated: records with a Namespace; partitioned:
    every frame's lookup record)."""
    import numpy as np
    from emurx import abi
    cnt = xch["recv_count"].cpu().numpy().astype(np.int64)[0::xch["cs"]]
    assert (cnt <= xch["cap"]).all(), f"exchange overflow {cnt} > {xch['cap']}"
    sent = (rec.cpu().numpy().view(abi.REC_DTYPE)["ns_id"] != abi.ID_NONE).sum() if mode == "replicated" else n
    routed = torch.tensor([int(sent), int(cnt.sum())], dtype=torch.int64)
    if world > 1:
        routed = routed.to(dev) if dist.get_backend() == "nccl" else routed
        dist.all_reduce(routed)
    routed = routed.cpu().numpy()
    assert routed[0] == routed[1], f"sent {routed[0]} != received {routed[1]}"


class ReceiveFill:
    """Stands in for the ZMQ receive (veth_zmq.go:132-143 rxThread: RecvBytes per message): the
    batch's messages land straight in the slot's pinned staging buffer that emurx_ingest_buffer
    handed out, written by `threads` receiver threads over disjoint message ranges (ctypes.memmove
    drops the GIL, as a cgo zmq_recv into the slot does).  threads = 1 is the
    round-5 single np.copyto."""

    def __init__(self, threads):
        from concurrent.futures import ThreadPoolExecutor
        self.threads = max(1, int(threads))
        self.pool = ThreadPoolExecutor(self.threads) if self.threads > 1 else None

    def fill(self, dst, src):
        import ctypes
        import numpy as np
        if self.pool is None:
            np.copyto(dst[: src.size], src)
            return
        n = src.nbytes
        chunk = ((n + self.threads - 1) // self.threads + 4095) & ~4095
        d, s = dst.ctypes.data, src.ctypes.data
        futs = [self.pool.submit(ctypes.memmove, d + o, s + o, min(chunk, n - o)) for o in range(0, n, chunk)]
        for f in futs:
            f.result()

    def close(self):
        if self.pool is not None:
            self.pool.shutdown()


def fill_threads():
    """Receiver threads of the host-inclusive passes: the job's cores, at most 16
    (EMURX_BENCH_FILL_THREADS overrides, for the measurement of the choice)."""
    e = os.environ.get("EMURX_BENCH_FILL_THREADS")
    return max(1, int(e)) if e and e.isdigit() else max(1, min(16, host_cores()))


def host_inclusive_block(rx, w, rank, world, dist, torch, backend, per_msg=64, budget_s=1.0, slots=2):
    """The host-inclusive rate of the default line, at every N: the
    headline batch as ZMQ messages of `per_msg` frames (veth_zmq.go:36-37,132-143,277-320)
    through the batched ingest (emurx_ingest_*), both slots alternating: pinned staging -> H2D
    -> framing walk -> k_rx -> queue packing -> D2H of records, descriptors, queues and
    counters.  Passes of `budget_s` each, every rank at once after a barrier: with the messages
    received into the slot's pinned staging by the receiver threads (ReceiveFill: the receive
    copy the caller makes anyway, straight into the slot), the same with one thread, and with
    the staging prefilled (PCIe + GPU only).  The batches rotate over `slots` ingest slots: a
    slot is filled while the others' batches are in flight.  Per pass the node's aggregate = all ranks' frames / the slowest rank's time
    (max over ranks, as the headline)."""
    from emurx import abi
    slots = max(2, min(int(slots), abi.INGEST_SLOTS))
    import numpy as np
    from emurx import frames as F
    zs, msgs = F.zmq_messages(w["buf"], w["desc"], per_msg)
    n, total = len(w["desc"]), len(zs)
    bufs = [rx.ingest_buffer(s, total) for s in range(slots)]
    for s in range(slots):  # warm every slot
        np.copyto(bufs[s], zs)
        rx.ingest_submit(s, msgs)
        assert rx.ingest_wait(s, copy=False)["n"] == n
    out = {"frames_per_batch": n, "frames_per_msg": per_msg, "msgs_per_batch": len(msgs), "bytes_per_batch": total,
           "budget_s_per_pass": budget_s, "slots": slots}

    def one_pass(fill):
        if world > 1:
            dist.barrier()
        pending, k, t0 = [False] * slots, 0, time.perf_counter()
        while True:
            s = k % slots
            if pending[s]:
                rx.ingest_wait(s, copy=False)
            if fill is not None:
                fill.fill(bufs[s], zs)
            rx.ingest_submit(s, msgs)
            pending[s] = True
            k += 1
            if time.perf_counter() - t0 > budget_s and k >= 2 * slots:
                break
        for s in range(slots):
            if pending[s]:
                rx.ingest_wait(s, copy=False)
        el = time.perf_counter() - t0
        t = torch.tensor([el, float(k * n), float(k * total)], dtype=torch.float64)
        per_rank = k * n / el / 1e6
        if world > 1:
            dev = torch.device("cuda", torch.cuda.current_device())
            mx = t[:1].clone().to(dev) if backend == "nccl" else t[:1].clone()
            sm = t[1:].clone().to(dev) if backend == "nccl" else t[1:].clone()
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            dist.all_reduce(sm, op=dist.ReduceOp.SUM)
            t = torch.cat([mx.cpu(), sm.cpu()])
        el_max, frames, nbytes = (float(x) for x in t)
        return {"mpkts": round(frames / el_max / 1e6, 2), "gbs_in": round(nbytes / el_max / 1e9, 2),
                "rank0_mpkts": round(per_rank, 2), "batches_rank0": k}

    fills = [ReceiveFill(fill_threads()), ReceiveFill(1)]
    out["with_host_copy"] = one_pass(fills[0])
    out["with_host_copy"]["fill_threads"] = fills[0].threads
    out["with_host_copy_1_thread"] = one_pass(fills[1])
    out["prefilled"] = one_pass(None)
    for f in fills:
        f.close()
    out["n_gpus"] = world
    out["source"] = (f"emurx_ingest_submit/wait over {slots} slots of every rank, wall clock per rank after a barrier; "
                     "node aggregate = all ranks' frames / the slowest rank's time; with_host_copy: the messages "
                     "received straight into the slot's pinned buffer (emurx_ingest_buffer) by fill_threads receiver "
                     "threads while the other slots are in flight")
    return out


def host_path_rate(rx, w, per_msg=64, budget_s=3.0, slots=2):
    """Host-inclusive rate of the batched ingest (emurx_ingest_*): the batch as ZMQ messages
    of `per_msg` frames (TRex sends at most 64 per message, veth_zmq.go:36-37), `slots` slots in
    rotation.  Timed per batch: copy of the messages into the slot's pinned staging (the
    receive copy the caller makes anyway) + H2D + framing walk + k_rx + queue packing + D2H
    of records, descriptors, queues and counters.  Also timed with the staging pre-filled
    (PCIe + GPU only), and one message per call through emurx_rx_stream."""
    import numpy as np
    from emurx import frames as F
    stream, msgs = F.zmq_messages(w["buf"], w["desc"], per_msg)
    from emurx import abi
    total, n = len(stream), len(w["desc"])
    slots = max(2, min(int(slots), abi.INGEST_SLOTS))
    bufs = [rx.ingest_buffer(s, total) for s in range(slots)]
    out = {"frames_per_batch": n, "frames_per_msg": per_msg, "msgs_per_batch": len(msgs),
           "bytes_per_batch": total, "slots": slots}

    fill = ReceiveFill(fill_threads())
    out["fill_threads"] = fill.threads

    def run(copy):
        pending = [False] * slots
        for s in range(slots):  # warm
            np.copyto(bufs[s], stream)
            rx.ingest_submit(s, msgs)
            res = rx.ingest_wait(s, copy=False)
            assert res["n"] == n
        k, t0 = 0, time.perf_counter()
        while True:
            s = k % slots
            if pending[s]:
                rx.ingest_wait(s, copy=False)
            if copy:
                fill.fill(bufs[s], stream)
            rx.ingest_submit(s, msgs)
            pending[s] = True
            k += 1
            if time.perf_counter() - t0 > budget_s and k >= 2 * slots:
                break
        for s in range(slots):
            if pending[s]:
                rx.ingest_wait(s, copy=False)
        el = time.perf_counter() - t0
        return k, el

    k, el = run(True)
    out["mpkts_with_host_copy"] = round(k * n / el / 1e6, 2)
    out["gbs_in_with_host_copy"] = round(k * total / el / 1e9, 2)
    k, el = run(False)
    fill.close()
    out["mpkts_prefilled"] = round(k * n / el / 1e6, 2)
    out["gbs_in_prefilled"] = round(k * total / el / 1e9, 2)
    # latency of one batch by its size in messages (one slot, nothing else in flight): submit
    # (batches that fit it: the one-launch path k_ingest_small, zero-copy in and out; larger
    # ones: H2D + framing walk + k_rx + queue packing + D2H) until wait returns; raw C calls
    # (no Python-side views), the staging already filled.  And the rate of such batches with
    # both slots alternating (one submitted while the other is in flight)
    import ctypes as C
    from emurx import abi
    lib, h = rx.lib, rx.h
    res = abi.IngestResult()
    mt = np.ascontiguousarray(np.asarray(msgs)).view(np.uint32).reshape(-1, 2)
    np.copyto(bufs[0], stream)
    np.copyto(bufs[1], stream)
    lat, thr = {}, {}
    for nm in (1, 2, 4, 8, 16, 32, 64, 256, 1024, 4096, len(msgs)):
        if nm > len(msgs) or str(nm) in lat:
            continue
        tab = np.ascontiguousarray(mt[:nm])
        ptr = tab.ctypes.data
        ts = []
        for rep in range(25 if nm <= 1024 else 7):
            t0 = time.perf_counter()
            abi.check(lib.emurx_ingest_submit(h, 0, ptr, nm), "ingest_submit")
            abi.check(lib.emurx_ingest_wait(h, 0, C.byref(res)), "ingest_wait")
            ts.append(time.perf_counter() - t0)
        ts = np.array(ts[3:]) * 1e6
        lat[str(nm)] = {"frames": nm * per_msg, "us_median": round(float(np.median(ts)), 1),
                        "us_p10": round(float(np.percentile(ts, 10)), 1),
                        "mpkts": round(nm * per_msg / float(np.median(ts)), 3)}
        if nm <= 1024:  # two slots in flight
            k, t0 = 0, time.perf_counter()
            while k < 400 and (k < 8 or time.perf_counter() - t0 < 0.5):
                sl = k & 1
                if k >= 2:
                    abi.check(lib.emurx_ingest_wait(h, sl, C.byref(res)), "ingest_wait")
                abi.check(lib.emurx_ingest_submit(h, sl, ptr, nm), "ingest_submit")
                k += 1
            for sl in range(2):
                abi.check(lib.emurx_ingest_wait(h, sl, C.byref(res)), "ingest_wait")
            el = time.perf_counter() - t0
            thr[str(nm)] = {"frames": nm * per_msg, "mpkts": round(k * nm * per_msg / el / 1e6, 3),
                            "us_per_batch": round(el / k * 1e6, 1)}
    out["batch_latency_by_msgs"] = lat
    out["two_slot_rate_by_msgs"] = thr
    # one ZMQ message per call (the unbatched OnRxStream shape)
    one = [stream[m["off"]:m["off"] + m["len"]].tobytes() for m in msgs[:300]]
    rx.on_rx_stream(one[0])
    t0 = time.perf_counter()
    for m in one:
        rx.on_rx_stream(m, cap=per_msg)
    out["mpkts_one_msg_per_call"] = round(len(one) * per_msg / (time.perf_counter() - t0) / 1e6, 4)
    return out


def crossover(hp, cpu_mpkts):
    """The smallest batch (frames) at which the host-inclusive ingest beats one core of the CPU
    restatement on the same frames: by latency (frames / the batch's submit-to-wait time) and
    by rate with both slots in flight."""
    def first(table):
        for k in sorted(table, key=lambda x: table[x]["frames"]):
            if table[k]["mpkts"] >= cpu_mpkts:
                return table[k]["frames"]
        return None
    return {"cpu_one_core_mpkts": cpu_mpkts, "frames_by_latency": first(hp["batch_latency_by_msgs"]),
            "frames_by_two_slot_rate": first(hp["two_slot_rate_by_msgs"]),
            "note": "smallest batch whose GPU path (pinned staging -> results in pinned memory) processes frames "
                    "at least as fast as one host core running the oracle's rx_batch"}


def tx_zmq_rate(rx, w, torch, reps=50):
    """Device tx framing (VethIFZmq.Send x n + FlushTx as emurx_tx_zmq_dev) of the batch's
    frames, device-resident in and out; CUDA events on torch's stream around `reps` calls.
    Bytes moved per call: the frames read + the messages written (+ descriptors)."""
    import numpy as np

    def to_dev(a):
        b = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        t = torch.zeros(b.size + 64, dtype=torch.uint8, device="cuda")
        t[: b.size] = torch.from_numpy(b.copy()).to("cuda")
        return t
    n = len(w["desc"])
    fb = int(w["desc"]["len"].astype(np.int64).sum())
    need = 8 * n + fb
    tb, td = to_dev(w["buf"]), to_dev(w["desc"])
    out = torch.empty(need, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    info = torch.empty(2, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream()
    for _ in range(3):
        rx.tx_zmq_dev(tb, td, n, out, need, off, info, stream=st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        rx.tx_zmq_dev(tb, td, n, out, need, off, info, stream=st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nm, total = (int(x) for x in info.cpu().numpy())
    moved = fb + total + 8 * n
    return {"frames": n, "msgs": nm, "bytes_out": total, "ms_per_call": round(ms, 4),
            "mpkts": round(n / ms / 1e3, 1), "gbs_moved": round(moved / ms / 1e6, 1),
            "note": "two launches per call: k_txz_chain (leaf tables + the up-sweep) + k_txz_emit (the write)"}


def tx_csum_rate(rx, w, torch, reps=50):
    """Device tx checksum generation (emurx_tx_checksum_dev: the IPv4 header checksum and the
    L4 checksum of TCP / UDP / ICMP over IPv4 and IPv6, as the plugins' send paths rewrite
    them) over the batch's frames, in place on a device copy, device-resident in and out; the
    tx descriptors come from the library's own parse of the same frames (its records' L3 / L4
    offsets and next header).  CUDA events on torch's stream around `reps` calls.  Bytes per
    call: the frames read (every byte of a checksummed frame) + the 16-byte descriptors."""
    import numpy as np
    from emurx import abi
    n = len(w["desc"])
    buf = torch.from_numpy(np.ascontiguousarray(w["buf"]).view(np.uint8).copy()).to("cuda")
    desc = torch.from_numpy(np.ascontiguousarray(w["desc"]).view(np.uint8).copy()).to("cuda")
    rec = torch.empty(n * abi.REC_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    qcap = abi.queue_cap(n)
    ql = torch.empty(abi.NUM_QUEUES * qcap, dtype=torch.int32, device="cuda")
    tc = torch.empty(((n + 255) // 256) * 16, dtype=torch.int32, device="cuda")
    hist = torch.zeros(abi.HIST_SHARDS * 2 * abi.HIST_BINS, dtype=torch.int64, device="cuda")
    rx.classify_dev(buf, desc, n, rec, ql, qcap, tc, hist, classify=False)
    torch.cuda.synchronize()
    r = rec.cpu().numpy().view(abi.REC_DTYPE)
    d = w["desc"]
    ok = (r["status"] == 0) & (r["l3"] > 0) & (r["l4"] > 0)
    ver = np.asarray(w["buf"])[d["off"].astype(np.int64) + r["l3"].astype(np.int64)] >> 4
    nh = r["next_hdr"].astype(np.int64)
    v4, v6 = ok & (ver == 4), ok & (ver == 6)
    kind = np.zeros(n, np.int64)
    kind[v4 & (nh == 6)], kind[v4 & (nh == 17)], kind[v4 & (nh == 1)] = abi.TX_L4_TCP4, abi.TX_L4_UDP4, abi.TX_L4_ICMP4
    kind[v6 & (nh == 6)], kind[v6 & (nh == 17)], kind[v6 & (nh == 58)] = abi.TX_L4_TCP6, abi.TX_L4_UDP6, abi.TX_L4_ICMP6
    sel = np.nonzero(kind > 0)[0]
    td = np.zeros(len(sel), abi.TX_DESC_DTYPE)
    td["off"], td["len"] = d["off"][sel], d["len"][sel]
    td["l3"], td["l4"] = r["l3"][sel], r["l4"][sel]
    td["osize"] = np.where(v6[sel], r["l4"][sel].astype(np.int64) - r["l3"][sel] - 40, 0)
    td["ops"] = (kind[sel] << abi.TX_L4_SHIFT) | np.where(v4[sel], abi.TX_IPV4_HDR, 0)
    m = len(sel)
    tdd = torch.from_numpy(td.view(np.uint8).copy()).to("cuda")
    st = torch.cuda.current_stream()
    for _ in range(3):
        rx.tx_checksum_dev(buf, tdd, m, stream=st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        rx.tx_checksum_dev(buf, tdd, m, stream=st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    moved = int(d["len"][sel].astype(np.int64).sum()) + 16 * m
    # the in-place field writes dirty whole lines: the 64-byte sectors that hold a checksum
    # field's bytes go back to HBM whatever their other bytes (each field's two bytes; the
    # IPv4 header field where the header checksum is rewritten)
    base = td["off"].astype(np.int64)
    kd = td["ops"].astype(np.int64) >> abi.TX_L4_SHIFT
    fld = np.where((kd == abi.TX_L4_TCP4) | (kd == abi.TX_L4_TCP6), 16,
                   np.where((kd == abi.TX_L4_UDP4) | (kd == abi.TX_L4_UDP6), 6, 2))
    a4 = base + td["l4"].astype(np.int64) + fld
    a3 = (base + td["l3"].astype(np.int64) + 10)[(td["ops"] & abi.TX_IPV4_HDR) != 0]
    sectors = np.unique(np.concatenate([a4 >> 6, (a4 + 1) >> 6, a3 >> 6, (a3 + 1) >> 6]))
    wb = 64 * len(sectors)
    return {"frames": m, "ms_per_call": round(ms, 4), "mpkts": round(m / ms / 1e3, 1),
            "gbs_moved": round(moved / ms / 1e6, 1), "frac_of_8tbs": round(moved / ms / 1e6 / 8000.0, 4),
            "written_sector_bytes": wb, "gbs_with_writeback": round((moved + wb) / ms / 1e6, 1),
            "frac_with_writeback": round((moved + wb) / ms / 1e6 / 8000.0, 4),
            "note": "one k_tx_csum launch per call, in place; descriptors from the library's parse; "
                    "gbs_moved counts the frames read and the descriptors, gbs_with_writeback adds the "
                    "64-byte sectors the in-place field writes dirty (written back to HBM whole)"}


if __name__ == "__main__":
    main()
