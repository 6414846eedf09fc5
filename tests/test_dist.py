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
    # the line carries the launch-time spread of the pre-warm's last 100
    # launches and of a pass right behind the timed region (verdict round 3:
    # tell a box that never settles from a slower kernel)
    for obj in (line["prewarm"]["last100"], line["timed_spread"]):
        assert {"n", "min_ms", "median_ms", "p90_ms", "max_ms", "mean_ms"} <= set(obj), obj
        assert obj["min_ms"] <= obj["median_ms"] <= obj["p90_ms"] <= obj["max_ms"], obj


def test_bench_spread_summary():
    """bench.spread: order statistics of launch times."""
    sys.path.insert(0, ROOT)
    import bench

    s = bench.spread([float(x) for x in range(1, 101)])
    assert s["n"] == 100 and s["min_ms"] == 1 and s["max_ms"] == 100 and s["median_ms"] in (50, 51)
    assert s["p90_ms"] in (90, 91) and s["mean_ms"] == 50.5
    assert bench.spread([]) is None
    pw = bench.prewarm_summary(300, 170.0, 0.57, False, [0.6] * 150 + [0.57] * 150, 250)
    assert pw["last100"]["n"] == 100 and pw["converged"] is False


@pytest.mark.timeout(120)
def test_bench_refuses_world_mismatch():
    """WORLD_SIZE != --gpus exits non-zero before any work."""
    import subprocess

    env = _bench_env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--rehearse-cpu"],
                       capture_output=True, text=True, env=env, timeout=100, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE=2" in (r.stderr + r.stdout)


def _group_worker(rank, world, port, q):
    """One rank of a 2-rank job that drives 2 GPUs per rank through a device
    group (rs_group_*), the way an N-GPU storage node splits its stripes:
    distinct device ordinals per rank (2r, 2r+1; no device call is made on
    CPU, the handles bind lazily), the group's slice rule over this rank's
    global stripe range, and the cross-GPU placement plan computed on every
    rank from the same erasure masks."""
    sys.path.insert(0, ROOT)
    import hashlib

    import torch.distributed as dist

    import bench
    import reedsolomon_amd as rs
    from reedsolomon_amd import placement

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d, p, S = 10, 4, 37
        devs = [2 * rank, 2 * rank + 1]
        g = rs.NewGroup(d, p, devs)
        assert len(g) == 2
        assert [m.device_ordinal() for m in g.members] == devs
        lo, hi = bench.stripe_range(rank, S)
        slices = [g.slice(S, i) for i in range(len(g))]
        assert slices[0][0] == 0 and slices[-1][1] == S
        assert all(a[1] == b[0] for a, b in zip(slices, slices[1:]))  # contiguous, in member order
        assert max(h - l_ for l_, h in slices) - min(h - l_ for l_, h in slices) <= 1
        # (global stripe range, device) per member; every rank collects all of them
        mine = [(lo + a, lo + b, devs[i]) for i, (a, b) in enumerate(slices)]
        allm = [None] * world
        dist.all_gather_object(allm, mine)
        # the placement plan every rank derives from the same masks
        rng = np.random.default_rng(99)
        n_total = S * world
        masks = [0] * n_total
        for s in range(n_total):
            lost = rng.choice(d + p, int(rng.integers(0, p + 1)), replace=False)
            masks[s] = sum(1 << int(v) for v in lost)
        pl = placement.Placement(d, p, world, n_total)
        plan = placement._plan(pl, np.asarray(masks, dtype=np.uint64))
        digest = hashlib.sha256(repr(sorted(plan.items())).encode()).hexdigest()
        digests = [None] * world
        dist.all_gather_object(digests, digest)
        owned = sorted(s for s in plan if pl.owner(s) == rank)
        q.put((rank, allm, digests, len(owned), len(pl.local_shards(rank))))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_two_rank_gloo_device_groups_and_placement():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_group_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(150)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    allm0, allm1 = res[0][1], res[1][1]
    assert allm0 == allm1  # both ranks see the same assignment
    members = [m for per_rank in allm0 for m in per_rank]
    # every global stripe is taken by exactly one member, every member is on its own device
    covered = sorted((a, b) for a, b, _ in members)
    assert covered[0][0] == 0 and covered[-1][1] == 2 * 37
    assert all(x[1] == y[0] for x, y in zip(covered, covered[1:]))
    assert sorted(dv for _, _, dv in members) == [0, 1, 2, 3]
    # the decode plan is identical on every rank; owners split the stripes with erasures
    assert res[0][2] == res[1][2] and res[0][2][0] == res[0][2][1]
    assert res[0][3] > 0 and res[1][3] > 0
    assert res[0][4] + res[1][4] == 2 * 37 * 14  # every shard has exactly one home


@pytest.mark.timeout(400)
def test_bench_eight_ranks_rehearsal():
    """The driver's 8-GPU SCALE shape rehearsed on CPU: `bench.py --gpus 8`
    with no launcher starts 8 gloo ranks, all join, rank 0 alone prints the
    line with n_gpus 8 and ranks_seen 8."""
    import subprocess

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "3",
                        "--warmup", "1", "--rehearse-cpu"], capture_output=True, text=True, env=_bench_env(),
                       timeout=380, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _last_json(r.stdout)
    assert line["n_gpus"] == 8 and line["ranks_seen"] == 8, line
    # the timing group is the default backend (gloo: no RCCL on the SCALE
    # path), and every rank's device record came back in rank order
    assert line["backend"] == "gloo", line
    assert [d["rank"] for d in line["rank_devices"]] == list(range(8)), line
    assert len({d["pid"] for d in line["rank_devices"]}) == 8, line


def test_gloo_env_defaults_to_loopback():
    """Single-node timing group: gloo on the loopback interface unless the
    caller names one (the host name need not resolve)."""
    sys.path.insert(0, ROOT)
    import bench

    env = {}
    bench.gloo_env(env)
    assert env["GLOO_SOCKET_IFNAME"] == "lo"
    env = {"GLOO_SOCKET_IFNAME": "eth0"}
    bench.gloo_env(env)
    assert env["GLOO_SOCKET_IFNAME"] == "eth0"


def test_timing_backend_default_is_gloo():
    """the driver's first 8-GPU run must not depend on an RCCL
    init that never ran on hardware; the timing collectives default to gloo,
    nccl is an explicit opt-in, anything else is refused."""
    sys.path.insert(0, ROOT)
    import bench

    assert bench.timing_backend({}) == "gloo"
    assert bench.timing_backend({"RSAMD_BENCH_BACKEND": "nccl"}) == "nccl"
    with pytest.raises(SystemExit):
        bench.timing_backend({"RSAMD_BENCH_BACKEND": "mpi"})


def _eight_rank_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import time

    import torch
    import torch.distributed as dist

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        barrier, max_over = bench.make_collectives(dist, torch.device("cpu"))
        el = bench.timed_region(lambda _i: time.sleep(0.002 * (rank + 1)), 4, barrier, lambda: None, max_over)
        q.put((rank, bench.stripe_range(rank, 256), el))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_eight_rank_gloo_timing_protocol():
    """World 8: every rank reports the same max-over-ranks time, bounded by the
    slowest rank, and the 8 stripe ranges tile [0, 8*S) with no overlap."""
    world = 8
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_eight_rank_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(250)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(world))
    times = {el for _, _, el in res}
    assert len(times) == 1 and times.pop() >= 4 * 0.016
    ranges = [rg for _, rg, _ in res]
    assert ranges[0][0] == 0 and ranges[-1][1] == 8 * 256
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))


def test_group_devices_rule():
    """bench.py --group N: members on devices 0..N-1, or all on the pinned
    device of a rehearsal; too few GPUs without a pin is refused."""
    sys.path.insert(0, ROOT)
    import bench

    assert bench.group_devices(4, 8, None) == [0, 1, 2, 3]
    assert bench.group_devices(8, 1, 0) == [0] * 8
    with pytest.raises(SystemExit):
        bench.group_devices(8, 1, None)
    with pytest.raises(SystemExit):
        bench.group_devices(0, 8, None)


def test_group_refuses_launcher():
    import subprocess

    env = _bench_env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--group", "2"], capture_output=True,
                       text=True, env=env, timeout=100, cwd=ROOT)
    assert r.returncode != 0 and "one process" in (r.stderr + r.stdout)
