#!/usr/bin/env python3
"""Cross-GPU stripe placement end to end, one process per GPU:

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        tools/placement_demo.py [--backend nccl|gloo] [--stripes S] [--vec BYTES]

Every rank encodes its share of the stripes on its GPU, the shards are
rotated over the ranks (shard v of stripe s on rank (s+v) % N), a random 1-4
shards of most stripes are destroyed, and gather_reconst rebuilds them:
survivors -> owner over all_to_all (RCCL/xGMI with nccl), one multi-pattern
HIP decode per owner, rebuilt shards -> home.  Each rank checks its shards
against the originals and prints "placement_demo ok" with the exchange time.
RSAMD_BENCH_DEVICE pins every rank to one device (rehearsal on a 1-GPU box,
with --backend gloo).  --dump DIR writes each rank's stripes, masks, rebuilt
shards and the transfer plan to DIR/rank<r>.npz, so tests/test_placement.py
can check every rebuilt shard against the CPU oracle's Reconst of the same
stripe and the plan's survivors against the oracle's checkReconst."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--stripes", type=int, default=64)
    ap.add_argument("--vec", type=int, default=65536)
    ap.add_argument("--dump", default="", help="directory for rank<r>.npz (stripes, masks, rebuilt shards, plan)")
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist

    import reedsolomon_amd as rs
    from reedsolomon_amd.placement import Placement, _plan, gather_reconst

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev_idx = int(os.environ.get("RSAMD_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(args.backend)
    d, p, S, vec = 10, 4, args.stripes, args.vec
    codec = rs.New(d, p, device=dev_idx)
    # every rank builds the same stripes (seeded) and encodes them on its GPU
    g = torch.Generator(device=dev).manual_seed(1234)
    full = torch.empty((S, d + p, vec), dtype=torch.uint8, device=dev)
    full[:, :d].random_(0, 256, generator=g)
    codec.encode_batch(full)
    rng = np.random.default_rng(99)
    masks = np.zeros(S, np.uint64)
    for s in range(S):
        if s % 7 == 6:
            continue
        for v in rng.choice(d + p, int(rng.integers(1, p + 1)), replace=False):
            masks[s] |= np.uint64(1) << np.uint64(int(v))
    pl = Placement(d, p, world, S)
    mine = pl.local_shards(rank)
    rows = torch.tensor([s * (d + p) + v for s, v in mine], device=dev)
    orig = full.view(-1, vec).index_select(0, rows)
    local = orig.clone()
    lost_rows = [i for i, (s, v) in enumerate(mine) if int(masks[s]) >> v & 1]
    if lost_rows:
        local[torch.tensor(lost_rows, device=dev)] = 0xEE
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    rebuilt = gather_reconst(codec, local, pl, masks, rank)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ok = torch.equal(local, orig) and all(torch.equal(t, full[s, v]) for (s, v), t in rebuilt.items())
    if not ok:
        raise SystemExit(f"rank {rank}: rebuilt shards differ")
    if args.dump:
        keys = sorted(rebuilt)
        plan = _plan(pl, masks)
        ps = sorted(plan)
        np.savez(os.path.join(args.dump, f"rank{rank}.npz"), full=full.cpu().numpy(), masks=masks,
                 keys=np.array(keys, np.int64).reshape(-1, 2),
                 vals=(torch.stack([rebuilt[x] for x in keys]).cpu().numpy() if keys
                       else np.zeros((0, vec), np.uint8)),
                 plan_stripes=np.array(ps, np.int64),
                 plan_surv=np.array([plan[x][0] for x in ps], np.int64).reshape(len(ps), d),
                 plan_lost=np.array([sum(1 << v for v in plan[x][1]) for x in ps], np.uint64))
    print(f"placement_demo ok rank={rank} world={world} rebuilt={len(rebuilt)} time_ms={el * 1e3:.2f}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
