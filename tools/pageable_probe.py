#!/usr/bin/env python3
"""rs_encode_host_batch on PAGEABLE numpy memory (the DMA pipeline's 1-D copy
path): GiB/s of (k+m)*vec, 10+4, dense and padded layouts."""
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


if __name__ == "__main__":
    main()
