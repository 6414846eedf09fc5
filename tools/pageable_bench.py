#!/usr/bin/env python3
"""Pageable host batches (rs_encode_host_batch / rs_reconst_host_batch_multi
on ordinary numpy memory): the staged pipeline's rate per size, with the
copy pool size taken from RSAMD_HOST_THREADS (read once per process, so run
this once per setting), with the staging copies' non-temporal stores on and
off (rs_tune "host_copy_nt"), alternating in one process.  Every result is
checked against the device-resident Encode of the same stripes.

Usage: RSAMD_HOST_THREADS=8 python tools/pageable_bench.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import reedsolomon_amd as rs

    d, p = 10, 4
    r = rs.New(d, p)
    threads = os.environ.get("RSAMD_HOST_THREADS", "4 (default)")
    rng = np.random.default_rng(5)
    for vec, S, nt in [(v, s_, nt) for v, s_ in ((8 << 10, 2048), (64 << 10, 512), (1 << 20, 64), ((2 << 20) + 40, 24))
                       for nt in (1, 0, 1, 0)]:
        rs.lib().rs_tune(b"host_copy_nt", nt)
        if os.environ.get("RSAMD_BENCH_COALESCE"):  # alternate run coalescing instead of nt
            rs.lib().rs_tune(b"host_copy_nt", 1)
            rs.lib().rs_tune(b"host_copy_coalesce", nt)
        slot = int(os.environ.get("RSAMD_BENCH_SLOTS", "0"))  # alternate the chunk size instead of nt
        if slot:
            rs.lib().rs_tune(b"host_copy_nt", 1)
            rs.lib().rs_tune(b"host_pageable_slot", (8 << 20) if nt else (slot << 20))
        host = rng.integers(0, 256, (S, d + p, vec), dtype=np.uint8)
        pin = torch.from_numpy(host).pin_memory()  # (the reference through pinned memory: no runtime pageable copy)
        dev = pin.cuda()
        r.encode_batch(dev)
        pin.copy_(dev)
        ref = pin.numpy().copy()
        del dev, pin
        host[:, d:] = 0
        r.encode_host_batch(host)  # warm (mirror allocation)
        assert np.array_equal(host, ref), "encode mismatch"
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            r.encode_host_batch(host)
        te = (time.perf_counter() - t0) / reps
        assert np.array_equal(host, ref), "encode mismatch"
        masks = np.zeros(S, np.uint64)
        for s in range(S):
            for v in rng.choice(d + p, p, replace=False):
                masks[s] |= np.uint64(1) << np.uint64(int(v))
        lost = host.copy()
        bits = ((masks[:, None] >> np.arange(d + p, dtype=np.uint64)) & np.uint64(1)).astype(bool)
        lost[bits] = 0
        work = lost.copy()
        r.reconst_host_batch_multi(work, masks)  # warm (first sight of the patterns)
        tr = 0.0  # the reconst calls alone, not the copies that reset the input
        for _ in range(reps):
            work = lost.copy()
            t1 = time.perf_counter()
            r.reconst_host_batch_multi(work, masks)
            tr += time.perf_counter() - t1
        tr /= reps
        assert np.array_equal(work, ref), "reconst mismatch"
        gib = S * (d + p) * vec / 2**30
        tag = f"slot {(8 if nt else slot):>2} MiB" if slot else \
            f"coalesce {nt}" if os.environ.get("RSAMD_BENCH_COALESCE") else f"nt {nt}"
        print(f"threads {threads:>12} {tag}  10+4 {vec:>8} B x{S:<5} pageable: encode {gib / te:6.1f} GiB/s "
              f"({te * 1e3:7.2f} ms), reconst 4 lost {gib / tr:6.1f} GiB/s ({tr * 1e3:7.2f} ms)", flush=True)
        del host, lost, work, ref


if __name__ == "__main__":
    main()
