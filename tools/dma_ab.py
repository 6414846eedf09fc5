#!/usr/bin/env python3
"""A/B of the host-batch DMA pipeline's copy shape (rs_encode_host_batch with
zero-copy off): 1-D per-stripe copies vs one 2-D copy per chunk, by stripes
per chunk.  10+4 @ 1 MiB x 128 pinned stripes; wall clock, GiB/s of (k+m)*vec."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402

k, m, vec, S = 10, 4, 1 << 20, 128
r = rs.New(k, m)
L = rs.lib()
host = torch.randint(0, 256, (S, k + m, vec), dtype=torch.uint8).pin_memory()
L.rs_tune(b"host_batch_zc", 0)
res = {}
for rnd in range(3):
    for one_d in (1, 0):
        for spc, nst in ((2, 3), (4, 3), (8, 3), (4, 4)):
            L.rs_tune(b"host_dma_1d", one_d)
            r.encode_host_batch(host, spc, nst)
            t0 = time.perf_counter()
            for _ in range(3):
                r.encode_host_batch(host, spc, nst)
            t = (time.perf_counter() - t0) / 3
            key = f"dma_1d={one_d} spc={spc} streams={nst}"
            res.setdefault(key, []).append(S * (k + m) * vec / t / 2 ** 30)
for key, v in res.items():
    print(f"{key:32s} {max(v):7.2f} GiB/s (best of {len(v)}; all {', '.join(f'{x:.1f}' for x in v)})", flush=True)
