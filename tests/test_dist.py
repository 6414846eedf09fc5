"""N>1 path of bench.py on CPU: world_size-2 gloo ranks run the same timing
protocol (barrier + sync, exactly K steps, max over ranks), own disjoint
stripe ranges, and report whole-job throughput.  No GPU needed."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import time

    import torch
    import torch.distributed as dist

    import bench
    from oracle import oracle

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w, r, local = bench.dist_env()
        assert (w, r, local) == (world, rank, rank)
        S, k, m, n = 4, 10, 4, 256
        lo, hi = bench.stripe_range(rank, S)
        # each rank encodes only its own stripes (CPU stand-in for the device step)
        rng = np.random.default_rng(1000 + rank)
        data = rng.integers(0, 256, (S, k, n), dtype=np.uint8)
        gen = oracle.gen_matrix(k, m).reshape(m, k)

        def step(_i):
            oracle.encode_numpy(gen, data)
            time.sleep(0.01 * (rank + 1))  # uneven ranks: the slow one sets the time

        barrier, max_over = bench.make_collectives(dist, torch.device("cpu"))
        steps = 5
        el = bench.timed_region(step, steps, barrier, lambda: None, max_over)
        value = bench.throughput(S * (k + m) * n, world, steps, el)
        q.put((rank, lo, hi, el, value))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rank_gloo_timing_protocol():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(150)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    (r0, lo0, hi0, el0, v0), (r1, lo1, hi1, el1, v1) = res
    assert el0 == el1, "every rank must report the max-over-ranks time"
    assert el0 >= 5 * 0.02, "the slowest rank (rank 1) bounds the timed region"
    assert (lo0, hi0, lo1, hi1) == (0, 4, 4, 8), "ranks own disjoint, adjacent stripe ranges"
    assert abs(v0 - 4 * 14 * 256 * 2 * 5 / el0 / 2 ** 30) < 1e-9


def _bench_env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    env["HIP_VISIBLE_DEVICES"] = ""  # CPU only: the rehearsal never touches a GPU
    return env


def _last_json(out: str) -> dict:
    import json

    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # rank 0 prints exactly one line
    return json.loads(lines[0])


@pytest.mark.timeout(240)
def test_bench_spawns_ranks_without_launcher():
    """`bench.py --gpus 2` with no launcher starts 2 ranks itself (the driver's
    SCALE runs must never silently measure one GPU): the line reports
    n_gpus 2 and 2 ranks that joined the process group."""
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1", "--rehearse-cpu"], capture_output=True, text=True, env=_bench_env(),
                       timeout=220, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2, line


@pytest.mark.timeout(240)
def test_bench_under_torchrun_like_the_driver():
    """The driver's own command shape: torch.distributed.run --nproc-per-node 2
    ... bench.py --gpus 2."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--rehearse-cpu"]
    r = subprocess.run(cmd, capture_output=True, text=True, env=_bench_env(), timeout=220, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2, line


@pytest.mark.timeout(120)
def test_bench_refuses_world_mismatch():
    """WORLD_SIZE != --gpus exits non-zero before any work."""
    import subprocess

    env = _bench_env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--rehearse-cpu"],
                       capture_output=True, text=True, env=env, timeout=100, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=2" in (r.stderr + r.stdout)
