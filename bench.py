#!/usr/bin/env python3
"""Benchmark of the north-star path: device-resident Reed-Solomon Encode.

BASELINE.json metric: "Encode GiB/s device-resident ((k+m)*vec/cost),
10+4 @1MiB, 1/2/4/8 GPU; %HBM peak".

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A step = one launch of the HIP encode over one batch of S synthetic stripes
(default S=256 stripes of 10+4 x 1 MiB = 3.5 GiB per GPU, far beyond the
256 MiB Infinity Cache) that are already resident in HBM.  Stripes are
independent, so N GPUs each encode their own S stripes with no collective on
the data path (weak scaling); the only collectives are the timing barrier,
the max-over-ranks of the elapsed time, the rank count and the per-rank
device list, all on a gloo group over the host (RSAMD_BENCH_BACKEND=nccl opts
in to RCCL; the line's `backend` and `rank_devices` say which ran).

`--gpus N` without a launcher starts N ranks itself (torch.distributed.run
as a child process, before any GPU call); under a launcher WORLD_SIZE must
equal N and every rank must join, or the run exits non-zero (`ranks_seen`).

Order per rank: self-check (encode -> erase -> reconst), pre-warm until the
launch time has settled (at least 250 launches; 20 consecutive within 3 %
and within 0.5 % of the 20 before; `prewarm` in the line), W counted
warm-up steps queued right behind it, K timed steps; then (`cold`) 50
launches after a 100 ms idle, the rate a bursty caller sees.

Rank 0 prints ONE JSON line.  `value` = (k+m)*vec*S*N*K / max-rank time in
GiB/s.  `roofline` prices the encode kernel itself: algorithmic bytes per
launch / mean launch time from HIP events on the launch stream, against
8 TB/s HBM3E.  `cpu_baseline` times the oracle's AVX2 restatement of the
reference's split-nibble path on one host core over a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md), GB/s
CONFIGS = {
    # name: (k, m, vector bytes, stripes per GPU)
    "10+4@1MiB": (10, 4, 1 << 20, 256),
    "12+4@1MiB": (12, 4, 1 << 20, 256),
    "10+4@8KiB": (10, 4, 8 << 10, 32768),
    # secondary shapes (profiling of the > 4-parity kernels; not the headline)
    "10+8@1MiB": (10, 8, 1 << 20, 256),
    "16+8@1MiB": (16, 8, 1 << 20, 256),
}


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="10+4@1MiB", choices=sorted(CONFIGS))
    ap.add_argument("--stripes", type=int, default=0, help="stripes per GPU (default: per config)")
    ap.add_argument("--layout", default=os.environ.get("RSAMD_BENCH_LAYOUT", "split"), choices=("split", "interleaved"),
                    help="split: data [S][k][vec] and parity [S][m][vec] in separate buffers; "
                         "interleaved: one [S][k+m][vec] buffer")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--verify", type=int, default=1, help="encode->erase->reconst self-check of one stripe per rank")
    ap.add_argument("--e2e-stripes", type=int, default=128,
                    help="stripes per GPU for the host-resident end-to-end leg (0 = skip)")
    ap.add_argument("--e2e-reps", type=int, default=10)
    ap.add_argument("--prewarm-min", type=int, default=250,
                    help="pre-warm: at least this many launches before the counted warm-up")
    ap.add_argument("--prewarm-max", type=int, default=2000, help="pre-warm: at most this many launches")
    ap.add_argument("--cold", type=int, default=1,
                    help="after the timed region: 50 launches after a 100 ms idle (`cold` in the line)")
    ap.add_argument("--group", type=int, default=0,
                    help="one process drives N device-resident codecs through a device group "
                         "(rs_group_codec; the topology of a Go storage server), instead of one rank per GPU; "
                         "members share RSAMD_BENCH_DEVICE when it is set (rehearsal on fewer GPUs)")
    ap.add_argument("--rehearse-cpu", action="store_true",
                    help="TEST ONLY: rehearse the launcher / rank / timing protocol on CPU (gloo, no GPU, "
                         "no kernel); the line it prints is not a measurement")
    return ap.parse_args(argv)


# ---------------------------------------------------------------- distributed plumbing

def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def stripe_range(rank: int, stripes_per_rank: int):
    """Global ids of the stripes a rank owns (weak scaling: fixed per rank)."""
    return rank * stripes_per_rank, (rank + 1) * stripes_per_rank


def timing_backend(env=None) -> str:
    """Process-group backend of the timing collectives.  The data path has no
    collective: the group only carries the timing barrier, the
    max over ranks, the rank count and the per-rank device list, none of which
    needs a GPU transport, so the default is gloo over the host's loopback /
    TCP, and RCCL is not on the SCALE path at all.  RSAMD_BENCH_BACKEND=nccl
    opts in to RCCL (one process per GPU, device_id bound)."""
    env = os.environ if env is None else env
    b = env.get("RSAMD_BENCH_BACKEND", "gloo")
    if b not in ("gloo", "nccl"):
        raise SystemExit(f"bench: RSAMD_BENCH_BACKEND={b!r}: gloo (default) or nccl")
    return b


def gloo_env(env=None) -> None:
    """The timing group is single-node by the bench's contract (N GPUs of one
    node, MASTER_ADDR 127.0.0.1): gloo on the loopback interface, so the run
    does not depend on the host name resolving (gloo picks its interface from
    it otherwise).  An explicit GLOO_SOCKET_IFNAME wins."""
    env = os.environ if env is None else env
    env.setdefault("GLOO_SOCKET_IFNAME", "lo")


def rank_devices(pg, me: dict) -> list:
    """Every rank's device record, in rank order (all_gather_object over the
    timing group; [me] without one)."""
    if pg is None:
        return [me]
    out = [None] * pg.get_world_size()
    pg.all_gather_object(out, me)
    return out


def make_collectives(pg, device):
    """barrier() and max_over(x) for the timing protocol (no data-path collective).
    pg: torch.distributed module (nccl on GPUs, gloo in the CPU tests) or None."""
    import torch

    if pg is None:
        return (lambda: None), (lambda x: x)

    def barrier():
        pg.barrier()

    if pg.get_backend() == "gloo":
        device = torch.device("cpu")

    def max_over(x):
        t = torch.tensor([float(x)], dtype=torch.float64, device=device)
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        return float(t.item())

    return barrier, max_over


def throughput(bytes_per_step_rank: int, n_ranks: int, steps: int, elapsed: float) -> float:
    """Whole-job GiB/s: every rank's bytes over the max-over-ranks time."""
    return bytes_per_step_rank * n_ranks * steps / elapsed / 2 ** 30


def timed_region(step_fn, steps: int, barrier, sync, max_over_ranks):
    """barrier + sync, time exactly `steps` steps, sync + barrier; max over ranks."""
    barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step_fn(i)
    sync()
    t1 = time.perf_counter()
    barrier()
    return max_over_ranks(t1 - t0)


# ---------------------------------------------------------------- CPU baseline

def cpu_baseline(k, m, vec, seconds):
    """The oracle's AVX2 restatement of the reference's encode path
    (gmu_amd64.s split-nibble + rs.go:141-203 chunking): one core (the
    reference's published convention, README.md:129-138) and, beside it, all
    cores of this process's CPU share with stripes partitioned over threads
    (SURVEY.md 8d)."""
    import concurrent.futures as cf
    import threading

    import numpy as np

    from oracle import oracle

    oracle.build()
    rng = np.random.default_rng(0x5EED)

    def make(n):
        return [[rng.integers(0, 256, vec, dtype=np.uint8) for _ in range(k)] +
                [np.zeros(vec, np.uint8) for _ in range(m)] for _ in range(n)]

    def run(stripes, deadline):
        n = 0
        while True:
            oracle.encode_avx2(k, m, stripes[n % len(stripes)])  # ctypes drops the GIL
            n += 1
            if time.perf_counter() >= deadline:
                return n

    # one stripe encoded over and over, as the reference's own benchmark does
    # (benchEnc, rs_test.go:436-456: the README.md figures come from it)
    stripes = make(1)
    used_avx2 = oracle.has_avx2()
    t0 = time.perf_counter()
    n = run(stripes, t0 + seconds)
    el = time.perf_counter() - t0
    gibs = n * (k + m) * vec / el / 2 ** 30

    try:
        threads = len(os.sched_getaffinity(0))
    except AttributeError:
        threads = os.cpu_count() or 1
    threads = max(1, min(threads, int(os.environ.get("OMP_NUM_THREADS", threads)), 64))
    per = [make(2) for _ in range(threads)]
    mt_seconds = max(1.0, seconds / 6)
    best = None
    for _rep in range(2):  # best of two passes (the first can catch host-side noise)
        start = threading.Barrier(threads + 1, timeout=120)
        t1 = [0.0]

        def worker(st):
            for x in st:  # untimed: first touch of the parity pages happens here
                oracle.encode_avx2(k, m, x)
            start.wait()
            start.wait()  # main thread has stamped t1
            return run(st, t1[0] + mt_seconds)

        with cf.ThreadPoolExecutor(threads) as ex:
            futs = [ex.submit(worker, st) for st in per]
            start.wait()
            t1[0] = time.perf_counter()
            start.wait()
            c = [f.result() for f in futs]
            e = time.perf_counter() - t1[0]
        if best is None or sum(c) / e > sum(best[0]) / best[1]:
            best = (c, e)
    counts, el_mt = best
    mt = sum(counts) * (k + m) * vec / el_mt / 2 ** 30
    del per, stripes

    # BASELINE.json config 1: 10+4 @ 8 KiB on the scalar table path
    # (mulVectNoSIMD, gmu.go:11-23), the reference's no-SIMD row (README.md:135).
    small = make(1)[0]
    small = [x[:8192].copy() for x in small]
    small = [x for x in small[:10]] + [np.zeros(8192, np.uint8) for _ in range(4)]
    n_ns, t2 = 0, time.perf_counter()
    while time.perf_counter() - t2 < max(0.5, seconds / 10):
        oracle.encode(10, 4, small)
        n_ns += 1
    ns = n_ns * 14 * 8192 / (time.perf_counter() - t2) / 2 ** 30

    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    kern = "AVX2 split-nibble" if used_avx2 else "scalar table"
    return {
        "value": round(gibs, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": f"{n} encodes of one {k}+{m} x {vec} B stripe (host memory; the same stripe each time, as "
                  f"benchEnc rs_test.go:436-456) in {el:.1f} s, "
                  f"{kern} restatement of gmu_amd64.s, 1 thread on {cpu}",
        "multi_thread": {"value": round(mt, 3), "unit": "GiB/s", "cores": threads,
                         "sample": f"{sum(counts)} encodes over {threads} threads (2 stripes each) "
                                   f"in {el_mt:.1f} s (best of 2 passes), same kernel"},
        "no_simd_10_4_8KiB": {"value": round(ns, 3), "unit": "GiB/s", "cores": 1,
                              "sample": f"{n_ns} encodes of 10+4 x 8 KiB, scalar mulTbl path (gmu.go:11-23); "
                                        "reference i7-12700K: 1.26 GiB/s (README.md:135)"},
    }


def end_to_end(codec, data, parity, k, m, vec, S, reps, n_gpus, barrier, max_over, sync):
    """Host-resident leg (north star: the path starts and ends in host memory):
    S stripes per rank in pinned host memory, encoded in place by
    rs_encode_host_batch, all ranks at once; max over ranks.  Two paths:
    zero-copy (default for pinned memory: the kernel reads and writes host
    memory over PCIe) and the H2D -> kernel -> D2H hipMemcpyAsync pipeline.
    The stripes are the first S of the device run, so the returned parity is
    checked against the device-resident result."""
    import numpy as np
    import torch

    import reedsolomon_amd as rs

    host = torch.empty((S, k + m, vec), dtype=torch.uint8, pin_memory=True)
    host[:, :k].copy_(data[:S])
    L = rs.lib()
    res = {}
    for name, zc in (("zero_copy", 1), ("dma_pipeline", 0)):
        assert L.rs_tune(b"host_batch_zc", zc) == 0
        host[:, k:].fill_(0xA5)
        codec.encode_host_batch(host, 4, 3)  # warm
        if not torch.equal(host[:2, k:].cuda(), parity[:2]):
            raise SystemExit(f"end-to-end ({name}) parity differs from the device-resident encode")
        sync()
        barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            codec.encode_host_batch(host, 4, 3)
        el = max_over(time.perf_counter() - t0)
        barrier()
        res[name] = round(n_gpus * S * (k + m) * vec * reps / el / 2 ** 30, 2)
    L.rs_tune(b"host_batch_zc", 1)
    # ordinary (pageable) memory, what a caller that registers nothing hands
    # over: staged through the handle's pinned mirror by the host copy threads
    pg = host.numpy().copy()
    pg[:, k:] = 0xA5
    codec.encode_host_batch(pg)  # warm
    ref = torch.empty((2, m, vec), dtype=torch.uint8, pin_memory=True)
    ref.copy_(parity[:2])
    if not np.array_equal(pg[:2, k:], ref.numpy()):
        raise SystemExit("end-to-end (pageable_staged) parity differs from the device-resident encode")
    barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        codec.encode_host_batch(pg)
    el = max_over(time.perf_counter() - t0)
    barrier()
    pageable = round(n_gpus * S * (k + m) * vec * reps / el / 2 ** 30, 2)
    del host, pg, ref
    return {"value": max(res.values()), "unit": "GiB/s", "zero_copy": res["zero_copy"],
            "dma_pipeline": res["dma_pipeline"], "pageable_staged": pageable, "stripes_per_gpu": S, "reps": reps,
            "path": "pinned host stripes in, parity back in pinned host memory (rs_encode_host_batch); "
                    "zero_copy = kernel over host memory via PCIe, dma_pipeline = H2D / encode / D2H "
                    "hipMemcpyAsync on 3 streams, 4 stripes per step; pageable_staged = the same stripes in "
                    "ordinary memory, staged through the pinned mirror by host copy threads (not in value); "
                    "all GPUs at once; wall clock, max over ranks"}


def load_traffic(config: str, algorithmic_bytes: int):
    """(HBM bytes per launch, source) from the committed rocprofv3 PMC summary
    (profiles/traffic.json: FETCH_SIZE / WRITE_SIZE passes of this same
    launch, corrected per MI355X_MICROARCH.md), or (None, None) when there is
    none for this launch (another stripe count measures another launch).  The
    counters are not collected inside this run: `traffic_source` names the file."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        ent = json.load(open(path)).get(config, {})
        b = ent.get("hbm_bytes_per_launch")
        alg = ent.get("algorithmic_bytes_per_launch")
        if not b or (alg is not None and alg != algorithmic_bytes) or not (0.5 < b / algorithmic_bytes < 2.0):
            return None, None
        return b, f"profiles/traffic.json <- {ent.get('source')}"
    except (OSError, ValueError, ZeroDivisionError):
        return None, None


# ---------------------------------------------------------------- launcher

def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv) -> int:
    """`--gpus N` without a launcher: start N ranks (one process per GPU)
    with torch.distributed.run as a CHILD process and return its exit code.
    Runs before this process touches the GPU (no torch import yet), so no
    GPU-initialised process is ever replaced (exec) by another."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    print("bench: --gpus %d without a launcher: %s" % (n, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def check_world(args, world: int, launched: bool) -> None:
    """A line claiming N GPUs must come from N ranks: refuse any mismatch."""
    if launched and world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if not launched and args.gpus != 1:
        raise SystemExit("bench: internal error: multi-GPU run without a launcher")


# ---------------------------------------------------------------- pre-warm

def prewarm(step, stream, min_launches: int, max_launches: int, window: int = 20, tol: float = 0.03,
            drift: float = 0.005, depth: int = 4, max_seconds: float = 5.0):
    """Run the step until the GPU has reached its steady state.  After an idle
    period of a few ms the encode runs 0.57 -> 0.87 -> 0.57 ms per launch over
    ~30-50 launches (power management; rocprof trace), so a short
    warm-up would time that transient.  Each launch is bracketed by HIP events
    on the launch stream; the host waits only on the launch `depth` back, so
    the GPU never idles and the counted warm-up is queued right behind (no
    sync at the end).  Converged = at least `min_launches`, the last `window`
    launches within `tol` (max/min) and their mean within `drift` of the
    window before.  Returns (launches, wall ms, last window's mean ms,
    converged)."""
    import torch

    t0 = time.perf_counter()
    evs = []
    durs = []
    n = 0
    converged = False
    while n < max_launches:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        step(0)
        e1.record(stream)
        evs.append((e0, e1))
        n += 1
        done = n - depth  # launches whose events are read (older ones have finished)
        if done > len(durs):
            a, b = evs[done - 1]
            b.synchronize()
            durs.append(a.elapsed_time(b))
            # release the pair now: destroying ~4,000 events at once when the
            # list dies took longer than the 4 queued launches (a 1.6 ms idle
            # gap before the warm-up, whose power transient then landed on the
            # timed region; profiles/r05/driver_cmd)
            evs[done - 1] = None
            del a, b
            if len(durs) >= max(min_launches, 2 * window) and len(durs) % 2 == 0:
                last, prev = durs[-window:], durs[-2 * window:-window]
                m1, m0 = sum(last) / window, sum(prev) / window
                if max(last) <= min(last) * (1 + tol) and abs(m1 - m0) <= drift * m0:
                    converged = True
                    break
            if time.perf_counter() - t0 > max_seconds:
                break
    last_mean = sum(durs[-window:]) / min(window, len(durs)) if durs else None
    return n, (time.perf_counter() - t0) * 1e3, last_mean, converged, durs


def spread(ms) -> dict | None:
    """min / median / p90 / max / mean of launch times (ms), so a box whose
    clocks never settle can be told from a slower kernel."""
    if not ms:
        return None
    x = sorted(ms)
    n = len(x)

    def q(f):
        return x[min(n - 1, int(round(f * (n - 1))))]

    return {"n": n, "min_ms": round(x[0], 4), "median_ms": round(q(0.5), 4), "p90_ms": round(q(0.9), 4),
            "max_ms": round(x[-1], 4), "mean_ms": round(sum(x) / n, 4)}


def prewarm_summary(n, ms, last_mean, converged, durs, min_launches) -> dict:
    """The line's `prewarm` object: what the pre-warm ran and the spread of
    its last 100 launch times."""
    return {"launches": n, "ms": round(ms, 1), "converged": converged,
            "last20_mean_ms": round(last_mean, 4) if last_mean else None,
            "last100": spread(durs[-100:]),
            "rule": f"untimed launches (>= {min_launches}) until 20 consecutive agree within 3 % "
                    "and their mean within 0.5 % of the 20 before; the counted warm-up is queued "
                    "behind them with no idle gap; last100 = spread of the last 100 pre-warm launches "
                    "(HIP events per launch)"}


def launch_spread(step, stream, n: int):
    """Per-launch times of n launches queued right behind the timed region
    (GPU warm, no idle gap), each bracketed by HIP events on the launch
    stream: the spread of the steady state the timed window averages (events
    inside the timed window itself would add gaps between its kernels)."""
    import torch

    evs = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        step(0)
        e1.record(stream)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


def cold_launches(step, stream, nbytes: int, max_over, idle_s: float = 0.1, n: int = 50):
    """What a bursty caller sees: after `idle_s` of GPU idle,
    `n` launches back to back, each bracketed by HIP events on the launch
    stream; mean / max launch time over them (max over ranks) against the
    steady state the timed region measures.  Runs after the timed region."""
    import torch

    torch.cuda.synchronize()
    time.sleep(idle_s)
    evs = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        step(0)
        e1.record(stream)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in evs]
    mean = max_over(sum(ms) / n)
    return {"idle_ms": idle_s * 1e3, "launches": n, "mean_ms": round(mean, 4), "max_ms": round(max_over(max(ms)), 4),
            "first10_ms": [round(x, 4) for x in ms[:10]],
            "GiBps_per_gpu": round(nbytes / (mean / 1e3) / 2 ** 30, 1),
            "rule": "after the timed region: GPU idle for idle_ms, then `launches` launches back to back, each "
                    "bracketed by HIP events; mean over them (max over ranks)"}


def metric_name(k: int, m: int, vec: int) -> str:
    """BASELINE.json's metric, with the shape of the config actually run."""
    size = f"{vec >> 20}MiB" if vec % (1 << 20) == 0 else f"{vec >> 10}KiB"
    return f"Encode GiB/s device-resident ((k+m)*vec/cost), {k}+{m} @{size}, 1/2/4/8 GPU; %HBM peak"


# ---------------------------------------------------------------- CPU rehearsal (tests only)

def rehearse_cpu(args, world: int, rank: int) -> dict | None:
    """The launcher / rank / timing protocol without a GPU (gloo): what
    tests/test_dist.py drives as `bench.py --gpus 2 --rehearse-cpu`.  The step
    is a numpy XOR over a small buffer; the printed line is marked as a
    rehearsal and carries no measurement."""
    import numpy as np
    import torch
    import torch.distributed as dist

    pg = None
    backend = timing_backend()
    if world > 1:
        if backend != "gloo":
            raise SystemExit("bench: --rehearse-cpu runs on gloo only (no GPU)")
        gloo_env()
        dist.init_process_group("gloo")
        pg = dist
    ranks_seen = count_ranks(pg, torch.device("cpu"))
    devices = rank_devices(pg, {"rank": rank, "device": "cpu", "pid": os.getpid()})
    if ranks_seen != args.gpus:
        raise SystemExit(f"bench: {ranks_seen} ranks joined, --gpus {args.gpus}")
    barrier, max_over = make_collectives(pg, torch.device("cpu"))
    buf = np.random.default_rng(rank).integers(0, 256, (4, 14, 4096), dtype=np.uint8)

    def step(_i):
        np.bitwise_xor.reduce(buf[:, :10], axis=1)

    def host_times(n):  # (the pre-warm's and the spread pass's per-launch times, on the host clock)
        out = []
        for _ in range(n):
            t0 = time.perf_counter()
            step(0)
            out.append((time.perf_counter() - t0) * 1e3)
        return out

    pw = host_times(max(args.warmup, 3))
    el = timed_region(step, args.steps, barrier, lambda: None, max_over)
    after = spread(host_times(max(args.steps, 20)))
    out = None
    if rank == 0:
        out = {"metric": "REHEARSAL (no GPU, no kernel)", "value": None, "n_gpus": world, "ranks_seen": ranks_seen,
               "backend": backend if pg is not None else None, "rank_devices": devices,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3,
               "data": "rehearsal: numpy XOR stand-in, not a measurement",
               "prewarm": prewarm_summary(len(pw), sum(pw), sum(pw[-20:]) / len(pw[-20:]), True, pw, 0),
               "timed_spread": after}
        print(json.dumps(out), flush=True)
    if pg is not None:
        pg.barrier()
        pg.destroy_process_group()
    return out


def count_ranks(pg, device) -> int:
    """Ranks that actually joined the process group (1 without one)."""
    import torch

    if pg is None:
        return 1
    if pg.get_backend() == "gloo":
        device = torch.device("cpu")
    t = torch.ones(1, dtype=torch.float64, device=device)
    pg.all_reduce(t)
    return int(t.item())


# ---------------------------------------------------------------- one process, N devices

def group_devices(n: int, visible: int, pinned: int | None) -> list:
    """Device ordinals of a --group N run: 0..N-1, or N members sharing
    `pinned` (RSAMD_BENCH_DEVICE) to rehearse the topology on fewer GPUs."""
    if n < 1:
        raise SystemExit("bench: --group needs N >= 1")
    if pinned is not None:
        return [pinned] * n
    if visible < n:
        raise SystemExit(f"bench: --group {n} but only {visible} visible GPUs (set RSAMD_BENCH_DEVICE to rehearse)")
    return list(range(n))


def group_main(args) -> dict:
    """`--group N`: ONE process drives N device-resident codecs (rs_group_new,
    rs_group_codec), the way a Go storage server holding several GPUs would
    (contiguous stripe slices, tables replicated, aggregate =
    total bytes / wall time).  Each member owns S stripes in its device's HBM
    (weak scaling, as with one rank per GPU) and its own stream; a step
    launches every member's encode back to back from this one host thread
    (launches are asynchronous), and the step ends when every device is done.
    Every member's stripes are self-checked (encode -> erase -> reconst)."""
    import torch

    import reedsolomon_amd as rs

    k, m, vec, S = CONFIGS[args.config]
    if args.stripes:
        S = args.stripes
    pin = os.environ.get("RSAMD_BENCH_DEVICE")
    devs = group_devices(args.group, torch.cuda.device_count(), int(pin) if pin is not None else None)
    g = rs.NewGroup(k, m, devs)
    members = []
    for i, (dv, codec) in enumerate(zip(devs, g.members)):
        dev = torch.device("cuda", dv)
        gen = torch.Generator(device=dev).manual_seed(0x5EED + i)
        data = torch.empty((S, k, vec), dtype=torch.uint8, device=dev)
        parity = torch.empty((S, m, vec), dtype=torch.uint8, device=dev)
        for s0 in range(0, S, 32):
            data[s0:s0 + 32].random_(0, 256, generator=gen)
        parity.fill_(0xA5)
        members.append((codec, dev, torch.cuda.Stream(dev), data, parity))
    distinct = sorted(set(devs))

    def sync():
        for dv in distinct:
            torch.cuda.synchronize(dv)

    def step(_i):
        for codec, _dev, st, data, parity in members:
            codec.encode_batch_split(data, parity, stream=st)

    sync()
    step(0)
    if args.verify:
        for i, (codec, _dev, st, data, parity) in enumerate(members):
            sl = slice(S // 2, S // 2 + 1)
            ref_d, ref_p = data[sl].clone(), parity[sl].clone()
            data[sl, 1] = 0
            parity[sl, m - 1] = 0
            codec.reconst_batch_split(data[sl], parity[sl], [], [1, k + m - 1], stream=st)
            st.synchronize()
            if not (torch.equal(data[sl], ref_d) and torch.equal(parity[sl], ref_p)):
                raise SystemExit(f"group member {i} (cuda:{devs[i]}): encode/reconst round trip failed")

    # pre-warm: every member's device to its steady state (the same launch count
    # as one rank's pre-warm minimum), then the counted warm-up behind it
    for _ in range(max(args.prewarm_min, 1)):
        step(0)
    for _ in range(args.warmup):
        step(0)
    sync()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in members]

    def timed_step(i):
        for (codec, _dev, st, data, parity), (e0, e1) in zip(members, evs):
            if i == 0:
                e0.record(st)
            codec.encode_batch_split(data, parity, stream=st)
            if i == args.steps - 1:
                e1.record(st)

    elapsed = timed_region(timed_step, args.steps, lambda: None, sync, lambda x: x)
    per_member_ms = [e0.elapsed_time(e1) / args.steps for e0, e1 in evs]
    bytes_per_member = S * (k + m) * vec
    value = throughput(bytes_per_member, len(members), args.steps, elapsed)
    shared = len(distinct) < len(devs)
    kern = max(per_member_ms)
    e2e = None
    if args.e2e_stripes > 0:
        e2e = group_end_to_end(g, members, k, m, vec, min(args.e2e_stripes, S), args.e2e_reps)
    out = {
        "metric": metric_name(k, m, vec) + " [one process, device group]",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": len(distinct), "group_members": len(devs),
        "devices": devs, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (uniform random bytes, seeded per member; parity pre-filled 0xA5)",
        "config": {"workload": f"RS encode {k}+{m}, {vec} B vectors, {S} stripes per member, device-resident",
                   "k": k, "m": m, "vector_bytes": vec, "stripes_per_member": S,
                   "topology": "one process, rs_group_new over the listed devices, one stream per member, "
                               "all launches from one host thread; no collective"},
        "rehearsal": shared,
        "per_member_kernel_ms": [round(x, 4) for x in per_member_ms],
        "roofline": {"bound": "hbm", "achieved": round(bytes_per_member / (kern / 1e3) / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(bytes_per_member / (kern / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                     "kernel_timing": "slowest member: HIP event pair on its stream around the K timed launches / K"
                                      + ("; members SHARE a device, so each launch competes for one HBM"
                                         if shared else "")},
        "end_to_end": e2e,
        "build": rs.build_info(),
    }
    print(json.dumps(out), flush=True)
    return out


def group_end_to_end(g, members, k, m, vec, E, reps) -> dict:
    """Host-resident leg of --group: one pinned host batch of E stripes per
    member, encoded in place by rs_group_encode_host_batch (the group splits
    it with rs_group_slice and runs the slices on their devices concurrently).
    Slice i holds member i's first E stripes, so the parity that comes back is
    checked against that member's device-resident encode."""
    import torch

    n = len(members)
    host = torch.empty((n * E, k + m, vec), dtype=torch.uint8, pin_memory=True)
    for i, (_c, _d, _st, data, _p) in enumerate(members):
        lo, hi = g.slice(n * E, i)
        assert hi - lo == E
        host[lo:hi, :k].copy_(data[:E])
    host[:, k:].fill_(0xA5)
    g.encode_host_batch(host)
    for i, (_c, _d, _st, _data, parity) in enumerate(members):
        lo, _hi = g.slice(n * E, i)
        if not torch.equal(host[lo:lo + 2, k:], parity[:2].cpu()):
            raise SystemExit(f"group end-to-end: member {i} parity differs from its device-resident encode")
    t0 = time.perf_counter()
    for _ in range(reps):
        g.encode_host_batch(host)
    el = time.perf_counter() - t0
    del host
    return {"value": round(n * E * (k + m) * vec * reps / el / 2 ** 30, 2), "unit": "GiB/s",
            "stripes_per_member": E, "reps": reps,
            "path": "one pinned host batch split over the group's members (rs_group_encode_host_batch), "
                    "parity back in host memory; wall clock"}


# ---------------------------------------------------------------- main

def main(argv=None):
    raw = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(raw)
    world, rank, local = dist_env()
    launched = "WORLD_SIZE" in os.environ
    if args.group:
        if launched or args.gpus != 1:
            raise SystemExit("bench: --group N runs in one process (no launcher, no --gpus)")
        return group_main(args)
    if not launched and args.gpus > 1:
        raise SystemExit(spawn_ranks(args.gpus, raw))
    check_world(args, world, launched)
    n_gpus = world
    if args.rehearse_cpu:
        return rehearse_cpu(args, world, rank)

    import torch

    import reedsolomon_amd as rs

    # One process per GPU.  RSAMD_BENCH_DEVICE pins every rank to one device
    # (used only to rehearse the multi-rank path on a 1-GPU box, ranks sharing
    # cuda:0).  The timing collectives run on gloo unless RSAMD_BENCH_BACKEND
    # asks for nccl (timing_backend): no RCCL call is on the SCALE path.
    dev_idx = int(os.environ.get("RSAMD_BENCH_DEVICE", local))
    backend = timing_backend()
    if "RSAMD_BENCH_DEVICE" not in os.environ and torch.cuda.device_count() < world:
        raise SystemExit(f"bench: {world} ranks but only {torch.cuda.device_count()} visible GPUs")
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    pg = None
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            gloo_env()
            dist.init_process_group(backend)
        pg = dist

    if world > 1:
        # one rank per GPU: keep this process (and the threads it starts) on
        # the GPU's NUMA node, so the host-resident leg's pinned buffers are
        # local to its PCIe link (best effort; no-op where sysfs is absent)
        rs.lib().rs_bind_thread_to_device(dev_idx)

    k, m, vec, S = CONFIGS[args.config]
    if args.stripes:
        S = args.stripes
    lo, hi = stripe_range(rank, S)

    codec = rs.New(k, m, device=dev_idx)
    stream = torch.cuda.current_stream(dev)

    # Synthetic stripes: uniform random data seeded per (seed, rank); parity
    # pre-filled with 0xA5 so an encode that skipped a byte would show.
    g = torch.Generator(device=dev).manual_seed(0x5EED + rank)
    if args.layout == "interleaved":
        buf = torch.empty((S, k + m, vec), dtype=torch.uint8, device=dev)
        data, parity = buf[:, :k], buf[:, k:]
    else:
        data = torch.empty((S, k, vec), dtype=torch.uint8, device=dev)
        parity = torch.empty((S, m, vec), dtype=torch.uint8, device=dev)
    for s0 in range(0, S, 32):
        data[s0:s0 + 32].random_(0, 256, generator=g)
    parity.fill_(0xA5)
    torch.cuda.synchronize(dev)

    if args.layout == "interleaved":
        def step(_i):
            codec.encode_batch(buf, stream=stream)
    else:
        def step(_i):
            codec.encode_batch_split(data, parity, stream=stream)

    if args.verify:
        # Self-check without the oracle (bench must not run it outside the
        # CPU-baseline leg): encode, erase 4 vectors of one stripe, rebuild,
        # compare.  Done before the warm-up so no idle gap separates the
        # warm-up from the timed region.
        step(0)
        sl = slice(S // 2, S // 2 + 1)
        ref_d, ref_p = data[sl].clone(), parity[sl].clone()
        lost = [0, 3, k, k + m - 1]
        data[sl, 0] = 0
        data[sl, 3] = 0
        parity[sl, 0] = 0
        parity[sl, m - 1] = 0
        if args.layout == "interleaved":
            codec.reconst_batch(buf[sl], [], lost, stream=stream)
        else:
            codec.reconst_batch_split(data[sl], parity[sl], [], lost, stream=stream)
        torch.cuda.synchronize(dev)
        if not (torch.equal(data[sl], ref_d) and torch.equal(parity[sl], ref_p)):
            raise SystemExit(f"rank {rank}: encode/reconst round trip failed (stripe {lo + S // 2})")

    # Initialise the timing collectives now (the first NCCL call builds the
    # communicator) so nothing slow sits between the warm-up and the timed region.
    barrier, max_over = make_collectives(pg, dev)
    ranks_seen = count_ranks(pg, dev)
    if ranks_seen != args.gpus:
        raise SystemExit(f"bench: {ranks_seen} ranks joined the process group, --gpus {args.gpus}")
    props = torch.cuda.get_device_properties(dev)
    devices = rank_devices(pg, {"rank": rank, "local_rank": local, "device": dev_idx,
                                "pci_bus_id": getattr(props, "pci_bus_id", None), "host": socket.gethostname()})
    barrier()
    max_over(0.0)

    # Pre-warm until launch times settle, then the counted warm-up and the
    # timed region follow back to back (no idle gap, no per-launch events).
    pw_n, pw_ms, pw_mean, pw_ok, pw_durs = prewarm(step, stream, args.prewarm_min, args.prewarm_max)
    for _ in range(args.warmup):
        step(0)
    torch.cuda.synchronize(dev)

    # Kernel time: one HIP event pair on the launch stream around the K timed
    # launches (per-launch event records add ~10 us bubbles between kernels).
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed_step(i):
        if i == 0:
            ev0.record(stream)
        step(i)
        if i == args.steps - 1:
            ev1.record(stream)

    elapsed = timed_region(timed_step, args.steps, barrier, lambda: torch.cuda.synchronize(dev), max_over)
    kern_mean_s = max_over(ev0.elapsed_time(ev1) / args.steps / 1e3)

    bytes_per_step_rank = S * (k + m) * vec
    value = throughput(bytes_per_step_rank, n_gpus, args.steps, elapsed)
    after = spread(launch_spread(step, stream, max(args.steps, 20)))
    cold = cold_launches(step, stream, bytes_per_step_rank, max_over) if args.cold else None

    e2e = None
    if args.e2e_stripes > 0:
        e2e = end_to_end(codec, data, parity, k, m, vec, min(args.e2e_stripes, S), args.e2e_reps, n_gpus,
                         barrier, max_over, lambda: torch.cuda.synchronize(dev))
    achieved = bytes_per_step_rank / kern_mean_s / 1e9

    result = None
    if rank == 0:
        traffic, traffic_src = load_traffic(args.config, bytes_per_step_rank)
        result = {
            "metric": metric_name(k, m, vec),
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": n_gpus,
            "ranks_seen": ranks_seen,
            "backend": backend if pg is not None else None,
            "rank_devices": devices,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (uniform random bytes, seeded per rank; parity pre-filled 0xA5)",
            "config": {
                "workload": f"RS encode {k}+{m}, {vec} B vectors, {S} stripes per GPU, device-resident",
                "k": k, "m": m, "vector_bytes": vec, "stripes_per_gpu": S,
                "layout": ("data [S][k][vec] and parity [S][m][vec] in separate HBM buffers"
                           if args.layout == "split" else "one [S][k+m][vec] HBM buffer"),
                "parallelism": f"stripes partitioned over {n_gpus} GPU(s), no collective",
                "kernel": _kernel_name(k, m),
            },
            "pct_hbm_peak": round(bytes_per_step_rank * n_gpus * args.steps / elapsed / 1e9 / n_gpus
                                  / HBM_PEAK_GBS * 100, 2),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": bytes_per_step_rank,
                "kernel_ms_mean": round(kern_mean_s * 1e3, 4),
                "kernel_timing": "HIP event pair on the launch stream around the K timed launches / K",
            },
            "prewarm": prewarm_summary(pw_n, pw_ms, pw_mean, pw_ok, pw_durs, args.prewarm_min),
            "timed_spread": dict(after or {}, rule="rank 0: per-launch HIP-event times of max(K, 20) launches "
                                 "queued right behind the timed region (same steady state; the timed window "
                                 "itself has one event pair, no per-launch events)"),
        }
        result["cold"] = cold
        result["end_to_end"] = e2e
        result["build"] = rs.build_info()
        if n_gpus == 1 and args.cpu_seconds > 0:
            result["cpu_baseline"] = cpu_baseline(k, m, vec, args.cpu_seconds)
        else:
            result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)
    if pg is not None:
        pg.barrier()
        pg.destroy_process_group()
    return result


def _kernel_name(k, m):
    return f"gf_matmul_vec1<{k},true,4,false,0,8B,128 lanes> (buffer nt dwordx2 loads/stores, paired-column " \
        "xor3, 64-bit-shift bit groups)" if (k, m) in ((10, 4), (12, 4)) else "gf_matmul_vec1"


if __name__ == "__main__":
    main()
