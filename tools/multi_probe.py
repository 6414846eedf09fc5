#!/usr/bin/env python3
"""Multi-pattern Reconst cost breakdown (device-resident, 10+4).

For one erasure pattern applied to every stripe, compares
  single   rs_reconst_batch_layout (one pattern, vec1 kernel)
  multi1   rs_reconst_batch_multi with every stripe on that same pattern
and then multi16 (16 distinct patterns).  Wall time per call comes from HIP
events around back-to-back calls; run under `rocprofv3 --kernel-trace
--stats` to split it into kernel time and host/launch gaps.
Writes gpurun_out/multi_probe.json.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402

GiB = 2 ** 30


def dev_time(fn, iters=40, warm=10):
    st = torch.cuda.current_stream()
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(st)
    for _ in range(iters):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters / 1e3


def main():
    k, m = 10, 4
    out = {}
    g = torch.Generator(device="cuda").manual_seed(3)
    for vec, S in ((8 << 10, 32768), (1 << 20, 256)):
        r = rs.New(k, m)
        data = torch.randint(0, 256, (S, k, vec), dtype=torch.uint8, device="cuda", generator=g)
        parity = torch.empty((S, m, vec), dtype=torch.uint8, device="cuda")
        r.encode_batch_split(data, parity)
        for lost in ([0], [0, 11], [1, 4, 7], [0, 2, 5, 9]):
            mask = sum(1 << v for v in lost)
            masks = np.full(S, mask, np.uint64)
            nb = S * (k + len(lost)) * vec
            t1 = dev_time(lambda: r.reconst_batch_split(data, parity, [], lost))
            t2 = dev_time(lambda: r.reconst_batch_multi(data, parity, masks))
            key = f"{vec >> 10}KiB x{S} lost={lost}"
            out[key] = {"single_us": round(t1 * 1e6, 1), "multi1_us": round(t2 * 1e6, 1),
                        "single_GiBps": round(nb / t1 / GiB, 1), "multi1_GiBps": round(nb / t2 / GiB, 1)}
            print(key, out[key], flush=True)
        rng = np.random.default_rng(5)
        pats = []
        for _ in range(16):
            lost = rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False)
            pats.append(sum(1 << int(v) for v in lost))
        masks = np.array([pats[i % 16] for i in range(S)], dtype=np.uint64)
        nrec = sum(bin(int(x)).count("1") for x in masks)
        t = dev_time(lambda: r.reconst_batch_multi(data, parity, masks))
        key = f"{vec >> 10}KiB x{S} 16 patterns"
        out[key] = {"multi16_us": round(t * 1e6, 1), "GiBps": round((S * k + nrec) * vec / t / GiB, 1)}
        print(key, out[key], flush=True)
        del data, parity
        torch.cuda.empty_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/multi_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
