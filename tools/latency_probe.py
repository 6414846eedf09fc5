#!/usr/bin/env python3
"""Per-call latency of the host-memory Go-API entry points (10+4 @ 8 KiB).
Run under `rocprofv3 --hip-trace --kernel-trace --stats` to split one call
into API time (launch, synchronize) and kernel time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402

vec = int(os.environ.get("LAT_VEC", 8192))
n = int(os.environ.get("LAT_N", 300))
r = rs.New(10, 4)
rng = np.random.default_rng(1)
v = [rng.integers(0, 256, vec, dtype=np.uint8) for _ in range(10)] + [np.zeros(vec, np.uint8) for _ in range(4)]
for _ in range(20):
    r.Encode(v)
t0 = time.perf_counter()
for _ in range(n):
    r.Encode(v)
print(f"Encode 10+4 {vec} B: {(time.perf_counter() - t0) / n * 1e6:.1f} us/call", flush=True)
