#!/usr/bin/env python3
"""rs_encode_host_batch / rs_reconst_host_batch_multi on PAGEABLE numpy
memory (staged through the pinned mirror up to 16 MiB stripes, the DMA
pipeline's 1-D copies above): GiB/s, 10+4, dense and padded layouts."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402


def main():
    torch.cuda.init()
    r = rs.New(10, 4)
    for vec, S, pad in ((1 << 20, 64, 0), (65536, 512, 0), (8192, 2048, 0), (8195, 2048, 0), (1 << 20, 64, 64)):
        full = np.random.default_rng(1).integers(0, 256, (S, 14, vec + pad), dtype=np.uint8)
        buf = full[:, :, :vec]
        r.encode_host_batch(buf, 8, 3)
        t0 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            r.encode_host_batch(buf, 8, 3)
        dt = (time.perf_counter() - t0) / reps
        print(f"pageable {vec} B x {S} pad {pad}: {S * 14 * vec / dt / 2**30:.1f} GiB/s", flush=True)
        # multi-pattern Reconst, 16 patterns of 1-4 erasures, (k + lost) * vec per stripe
        rng = np.random.default_rng(5)
        pats = [sum(1 << int(v) for v in rng.choice(14, int(rng.integers(1, 5)), replace=False)) for _ in range(16)]
        masks = np.array([pats[i % 16] for i in range(S)], dtype=np.uint64)
        nrec = sum(bin(int(x)).count("1") for x in masks)
        r.reconst_host_batch_multi(buf, masks)
        t0 = time.perf_counter()
        for _ in range(reps):
            r.reconst_host_batch_multi(buf, masks)
        dt = (time.perf_counter() - t0) / reps
        print(f"  reconst 16 patterns: {(S * 10 + nrec) * vec / dt / 2**30:.1f} GiB/s", flush=True)


if __name__ == "__main__":
    main()
