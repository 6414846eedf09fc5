#!/usr/bin/env python3
"""Planning cost of rs_reconst_batch_multi with many distinct erasure
patterns (1-4 erasures each), host planner (rs_tune("multi_gpu_plan", 0):
the d x d inverse through the cache, combined_matrix and perm tables per
pattern) against the GPU planner (gf_plan_multi, one wave per pattern).
Wall time of the synchronous call (launch + sync) and the device-resident
rate it amounts to, per shape; cold = first call on a fresh handle, warm =
the same masks again (median of 8 calls).  Writes gpurun_out/multi_host_cost.json.
--small: 4-128 patterns per call; --split: the GPU planner's host time, Python
mirror vs the bare C call.
"""
import json
import os
import sys
import time
from itertools import combinations
from math import comb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402


def masks_for(d, p, n, seed, kmax=4):
    """n distinct masks of 1-kmax erasures (all of them when n is their count)."""
    kmax = min(kmax, p)
    total = sum(comb(d + p, k) for k in range(1, kmax + 1))
    if n >= total:
        return [sum(1 << v for v in c) for k in range(1, kmax + 1) for c in combinations(range(d + p), k)]
    rng = np.random.default_rng(seed)
    seen, out = set(), []
    while len(out) < n:
        lost = rng.choice(d + p, int(rng.integers(1, kmax + 1)), replace=False)
        mk = sum(1 << int(v) for v in lost)
        if mk not in seen:
            seen.add(mk)
            out.append(mk)
    return out


def main():
    res = {}
    L = rs.lib()
    shapes = ((10, 4, 1470, 8192, 4), (10, 4, 1470, 1024, 4), (20, 12, 4096, 1024, 4),
              (32, 32, 4096, 1024, 4), (100, 28, 1000, 4096, 4), (10, 8, 4096, 8192, 8),
              (20, 12, 4096, 1024, 8))
    if "--split" in sys.argv:  # where the GPU planner's host time goes: Python mirror vs the C call
        return split(shapes)
    if "--small" in sys.argv:  # where the GPU planner starts to pay (rs_tune("multi_gpu_plan") threshold)
        shapes = tuple((d, p, n, vec, 4) for d, p, vec in ((10, 4, 8192), (20, 12, 1024), (32, 32, 1024))
                       for n in (4, 8, 16, 32, 64, 128))
    for d, p, npat, vec, kmax in shapes:
        masks = masks_for(d, p, npat, d * 100 + p, kmax)
        S = len(masks)
        arg = masks if d + p > 64 else np.array(masks, dtype=np.uint64)
        nbytes = sum((d + bin(m).count("1")) * vec for m in masks)
        data = torch.zeros((S, d, vec), dtype=torch.uint8, device="cuda")
        parity = torch.zeros((S, p, vec), dtype=torch.uint8, device="cuda")
        row = {"stripes": S, "distinct_patterns": S, "vec": vec}
        for plan, name in ((0, "host"), (1, "gpu")):
            assert L.rs_tune(b"multi_gpu_plan", plan) == 0
            r = rs.New(d, p)
            walls, hosts = [], []
            for _ in range(9):  # the first call cold (fresh handle), then 8 warm ones (the upload ring holds 4 slots)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r.reconst_batch_multi(data, parity, arg)
                hosts.append(time.perf_counter() - t0)  # host side: the call returns once its work is queued
                torch.cuda.synchronize()
                walls.append(time.perf_counter() - t0)
            row[f"{name}_cold_ms"] = round(walls[0] * 1e3, 3)
            # (planner forced: 1 = the GPU whatever the count, 0 = the host)
            warm = sorted(walls[1:])
            med = warm[len(warm) // 2]
            row[f"{name}_warm_median_ms"] = round(med * 1e3, 3)
            row[f"{name}_warm_min_ms"] = round(warm[0] * 1e3, 3)
            row[f"{name}_warm_host_median_ms"] = round(sorted(hosts[1:])[len(hosts[1:]) // 2] * 1e3, 3)
            row[f"{name}_warm_GiBps"] = round(nbytes / med / 2 ** 30, 1)
            row[f"{name}_us_per_pattern_warm"] = round(med * 1e6 / S, 3)
        L.rs_tune(b"multi_gpu_plan", -1)
        key = f"{d}+{p} {S} patterns of 1-{kmax} lost @ {vec}"
        res[key] = row
        print(key, row, flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/multi_host_cost" + ("_small" if "--small" in sys.argv else "") + ".json", "w"),
              indent=1)


def split(shapes):
    """Host time of one GPU-planned call through the Python mirror
    (r.reconst_batch_multi) against the bare C ABI call with its layout,
    mask pointer and stream prepared once (rs_reconst_batch_multi), and the
    C call's wall time to completion; medians of 50 warm calls."""
    import ctypes

    from reedsolomon_amd._lib import RSLayout

    L = rs.lib()
    assert L.rs_tune(b"multi_gpu_plan", 1) == 0
    out = {}
    for d, p, npat, vec, kmax in shapes:
        masks = masks_for(d, p, npat, d * 100 + p, kmax)
        S = len(masks)
        data = torch.zeros((S, d, vec), dtype=torch.uint8, device="cuda")
        parity = torch.zeros((S, p, vec), dtype=torch.uint8, device="cuda")
        r = rs.New(d, p)
        arg = masks if d + p > 64 else np.array(masks, dtype=np.uint64)
        m, fn = rs.rs._masks_for(arg, S, d + p, "rs_reconst_batch_multi")
        lay = RSLayout(data.data_ptr(), data.stride(0), data.stride(1), parity.data_ptr(), parity.stride(0),
                       parity.stride(1))
        mp = m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        cfn = getattr(L, fn)
        h = r._h
        t = {"wrapper_host": [], "c_host": [], "c_wall": []}
        for i in range(51):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.reconst_batch_multi(data, parity, arg)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            assert cfn(h, ctypes.byref(lay), S, vec, mp, st) == 0
            t3 = time.perf_counter()
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            if i:
                t["wrapper_host"].append(t1 - t0)
                t["c_host"].append(t3 - t2)
                t["c_wall"].append(t4 - t2)
        row = {k: round(sorted(v)[len(v) // 2] * 1e6, 1) for k, v in t.items()}
        key = f"{d}+{p} {S} patterns @ {vec}"
        out[key] = row
        print(key, "median us:", row, flush=True)
    L.rs_tune(b"multi_gpu_plan", -1)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/multi_host_split.json", "w"), indent=1)


if __name__ == "__main__":
    main()
