#!/usr/bin/env python3
"""The synchronous host API (Encode / Reconst on pageable numpy vectors, what
the cgo binding calls per stripe) against the column chunk of its zero-copy
pipeline (rs_tune "host_chunk", bytes per vector per chunk), alternating
settings in one process; median of `reps` calls per point, every result
checked against the device-resident Encode of the same data.

Usage: python tools/host_chunk_sweep.py [knob value ...]   (default: host_chunk 64-512 KiB)
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

    knob = sys.argv[1] if len(sys.argv) > 1 else "host_chunk"
    chunks = [int(a) for a in sys.argv[2:]] or [64 << 10, 128 << 10, 256 << 10, 512 << 10]
    if knob != "host_chunk_split":
        L0 = rs.lib()
        L0.rs_tune(b"host_chunk_split", 0)  # host_chunk alone
    d, p = 10, 4
    r = rs.New(d, p)
    L = rs.lib()
    rng = np.random.default_rng(9)
    sizes = [int(x) for x in os.environ.get("RSAMD_SWEEP_SIZES", "").split(",") if x] or \
        [256 << 10, 1 << 20, 4 << 20, 16 << 20]
    rounds = int(os.environ.get("RSAMD_SWEEP_ROUNDS", "2"))
    for size in sizes:
        v = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(d)] + [np.zeros(size, np.uint8) for _ in range(p)]
        pin = torch.from_numpy(np.stack(v)).pin_memory()  # the reference through pinned memory
        dev = pin.cuda().unsqueeze(0)
        r.encode_batch(dev)
        pin.copy_(dev[0])
        exp = pin.numpy()[d:].copy()
        del dev, pin
        reps = 30 if size <= (1 << 20) else 12 if size <= (4 << 20) else 5
        for rnd in range(rounds):
            for c in chunks:
                assert L.rs_tune(knob.encode(), c) == 0
                ts = []
                for _ in range(reps):
                    for j in range(p):
                        v[d + j][:] = 0
                    t0 = time.perf_counter()
                    r.Encode(v)
                    ts.append(time.perf_counter() - t0)
                    assert all(np.array_equal(v[d + j], exp[j]) for j in range(p)), (size, c)
                t = sorted(ts)[len(ts) // 2]
                print(f"round {rnd} 10+4 Encode {size >> 10:>5} KiB pageable, {knob} {c:>7}: "
                      f"{t * 1e6:8.1f} us  {(d + p) * size / t / 2**30:6.2f} GiB/s", flush=True)
    L.rs_tune(b"host_chunk", 128 << 10)
    L.rs_tune(b"host_chunk_split", 4)


if __name__ == "__main__":
    main()
