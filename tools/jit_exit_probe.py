#!/usr/bin/env python3
"""Exit while the first background compile of the run-time kernels is in
flight (the process must still exit cleanly: jit.cpp exit handler order).
    python tools/jit_exit_probe.py <seed>"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reedsolomon_amd as rs  # noqa: E402

L = rs.lib(); L.rs_tune(b"jit_min_bytes", 0); L.rs_tune(b"jit_min_launches", 1)
r = rs.New(10, 4)
mat = np.random.default_rng(int(sys.argv[1])).integers(0, 256, (8, 32), dtype=np.uint8)
src = torch.randint(0, 256, (2, 32, 4096), dtype=torch.uint8, device="cuda")
dst = torch.empty((2, 8, 4096), dtype=torch.uint8, device="cuda")
r.gf_matmul_batch(mat, src, None, dst, None)
torch.cuda.synchronize()
print("queued; exiting", flush=True)
