#!/usr/bin/env python3
"""Diagnose Update mismatches: host API vs device API vs oracle over shapes and sizes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def first_diff(a, b):
    bad = np.flatnonzero(a != b)
    return None if not len(bad) else (int(bad[0]), int(bad[-1]), len(bad))


def main():
    rng = np.random.default_rng(1)
    for d, p in ((25, 3), (10, 4), (10, 3), (5, 1), (5, 2)):
        for size in (1027, 4096, 131072, 131073, 140000, 236667, 262144, 300000):
            r = rs.New(d, p)
            row = 1 % d
            enc = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(d)] + \
                [np.zeros(size, np.uint8) for _ in range(p)]
            assert orc.encode(d, p, enc) == 0
            new = rng.integers(0, 256, size, dtype=np.uint8)
            ora = [x.copy() for x in enc]
            assert orc.update(d, p, ora[row], new, row, ora[d:]) == 0
            act = [x.copy() for x in enc]
            r.Update(act[row], new, row, act[d:])
            host = [first_diff(act[d + j], ora[d + j]) for j in range(p)]
            dv = [torch.from_numpy(x.copy()).cuda() for x in enc]
            r.update_dev(dv[row], torch.from_numpy(new).cuda(), row, dv[d:])
            torch.cuda.synchronize()
            dev = [first_diff(dv[d + j].cpu().numpy(), ora[d + j]) for j in range(p)]
            ok = all(x is None for x in host + dev)
            print(f"{d}+{p} size={size}: {'ok' if ok else 'MISMATCH'} host={host} dev={dev}", flush=True)


if __name__ == "__main__":
    main()
