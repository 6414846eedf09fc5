#!/usr/bin/env python3
"""Host-side cost of rs_reconst_batch_multi: many distinct erasure patterns,
1-4 erasures each, tiny vectors (the kernel is negligible), wall time of the synchronous call.
Cold = first call on a fresh handle (every inverse computed), warm = the
same masks again (inverses from the cache where the reference would cache).
Usage: python tools/multi_host_cost.py   (writes gpurun_out/multi_host_cost.json)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402


def masks_for(d, p, n, seed):
    rng = np.random.default_rng(seed)
    seen, out = set(), []
    while len(out) < n:
        lost = rng.choice(d + p, int(rng.integers(1, min(p, 4) + 1)), replace=False)
        if not any(v < d for v in lost):
            continue
        mk = sum(1 << int(v) for v in lost)
        if mk not in seen:
            seen.add(mk)
            out.append(mk)
    return np.array(out, dtype=np.uint64)


def main():
    res = {}
    vec = 1024
    for d, p, npat in ((10, 4, 1000), (20, 12, 4096), (32, 32, 4096)):
        masks = masks_for(d, p, npat, d * 100 + p)
        S = len(masks)
        data = torch.zeros((S, d, vec), dtype=torch.uint8, device="cuda")
        parity = torch.zeros((S, p, vec), dtype=torch.uint8, device="cuda")
        r = rs.New(d, p)
        row = {}
        for phase in ("cold", "warm"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.reconst_batch_multi(data, parity, masks)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            row[phase + "_ms"] = round(dt * 1e3, 2)
            row[phase + "_us_per_pattern"] = round(dt * 1e6 / S, 2)
        key = f"{d}+{p} {S} patterns"
        res[key] = row
        print(key, row, flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/multi_host_cost.json", "w"), indent=1)


if __name__ == "__main__":
    main()
