#!/usr/bin/env python3
"""Diagnostics for the assembly-generated kernels (jit_asm.cpp) on the GPU:
per output row, is the result right, untouched (the launch never wrote it),
or equal to another row's expected bytes (a row / wave mix-up)?  Which byte
ranges and stripes differ?  (Its own GF(2^8)/0x11d table, numpy.)

    python tools/asm_diag.py [rows,cols ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def mul_table():
    t = np.zeros((256, 256), np.uint8)
    e = np.arange(256)
    for a in range(256):
        row, y = np.zeros(256, np.int64), a
        for bit in range(8):
            if bit:
                y = ((y << 1) ^ 0x11D) if y & 0x80 else (y << 1)
            row ^= np.where((e >> bit) & 1, y, 0)
        t[a] = row.astype(np.uint8)
    return t


def product(T, mat, src):  # src [S][cols][n] -> [S][rows][n]
    S, cols, n = src.shape
    out = np.zeros((S, mat.shape[0], n), np.uint8)
    for r in range(mat.shape[0]):
        for c in range(cols):
            out[:, r] ^= T[mat[r, c]][src[:, c]]
    return out


def diag(rs, torch, T, rows, cols, S, n):
    rng = np.random.default_rng(rows * 7000 + cols)
    mat = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
    r = rs.New(10, 4)
    hsrc = rng.integers(0, 256, (S, cols, n), dtype=np.uint8)
    hdst = rng.integers(0, 256, (S, rows, n), dtype=np.uint8)
    src, dst = torch.from_numpy(hsrc).cuda(), torch.from_numpy(hdst).cuda()
    r.gf_matmul_batch(mat, src, None, dst, None)
    torch.cuda.synchronize()
    got = dst.cpu().numpy()
    exp = product(T, mat, hsrc)
    bad = []
    for s in range(S):
        for row in range(rows):
            g, e = got[s, row], exp[s, row]
            if np.array_equal(g, e):
                continue
            diff = np.nonzero(g != e)[0]
            what = "untouched" if np.array_equal(g, hdst[s, row]) else ""
            for o in range(rows):
                if o != row and np.array_equal(g, exp[s, o]):
                    what = f"= expected row {o}"
            # the bytes differ where? lane pieces of 8 B, 512 B apart per piece slot
            bad.append(f"s{s} r{row}: {diff.size} bytes differ, first {diff[0]} last {diff[-1]} {what}")
    print(f"{rows}x{cols} S={S} n={n}: {'OK' if not bad else f'{len(bad)} bad (stripe,row)'}")
    for b in bad[:40]:
        print("   ", b)
    return not bad


def main(shapes):
    import torch

    import reedsolomon_amd as rs

    L = rs.lib()
    assert L.rs_tune(b"jit", 2) == 0 and L.rs_tune(b"jit_backend", 1) == 0
    T = mul_table()
    assert T[2, 0x80] == 0x1D and T[3, 7] == 9
    ok = True
    for sh in shapes:
        rows, cols = (int(x) for x in sh.split(","))
        for S, n in ((3, 2048), (2, 4096)):
            ok = diag(rs, torch, T, rows, cols, S, n) and ok
    print("jit stats", rs.jit_stats())
    print("ALL OK" if ok else "SOME BAD")


if __name__ == "__main__":
    main(sys.argv[1:] or ["17,5", "16,5", "20,4", "32,8", "33,3", "24,33", "9,10"])
