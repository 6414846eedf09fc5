#!/usr/bin/env python3
"""Time of a run-time kernel from first sight to loaded on the device
(rs_jit_prepare, wait=1: generate + code object + hipModuleLoadData), per
backend (2: machine code in a template, 1: assembly through comgr), for
fresh random matrices of several shapes.  The on-disk cache is off, so
every matrix is generated from scratch.  Prints one JSON line per shape."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import reedsolomon_amd as rs

    torch.cuda.init()
    L = rs.lib()
    assert L.rs_tune(b"jit_disk_cache", 0) == 0
    r = rs.New(10, 4)
    rng = np.random.default_rng(int(time.time()))
    shapes = [(5, 10), (8, 10), (16, 16), (12, 20), (28, 100), (32, 32), (64, 64), (56, 200), (128, 128)]
    for backend in (2, 1):
        assert L.rs_tune(b"jit_backend", backend) == 0
        for rows, cols in shapes:
            ts = []
            for k in range(3 if backend == 2 else 2):
                m = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
                t0 = time.perf_counter()
                r.jit_prepare(m)
                ts.append((time.perf_counter() - t0) * 1e3)
            print(json.dumps({"backend": backend, "rows": rows, "cols": cols,
                              "prepare_ms": [round(x, 3) for x in ts]}), flush=True)
    L.rs_tune(b"jit_backend", 2)


if __name__ == "__main__":
    main()
