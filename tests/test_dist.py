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
