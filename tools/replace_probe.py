#!/usr/bin/env python3
"""Replace 10+4 @ 8 KiB x 32768 for rn = 1..6, alternating rounds in one
process (ops_bench's config-5 rows, tools/ops_bench.py): GiB/s per rn and
round, so one slow rn can be told from box noise.  Measurement tool only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import reedsolomon_amd as rs

    k, m, vec, S = 10, 4, 8 << 10, 32768
    g = torch.Generator(device="cuda").manual_seed(3)
    r = rs.New(k, m)
    buf = torch.randint(0, 256, (S, k + m, vec), dtype=torch.uint8, device="cuda", generator=g)
    r.encode_batch(buf)
    data = {rn: torch.randint(0, 256, (S, rn, vec), dtype=torch.uint8, device="cuda", generator=g) for rn in range(1, 7)}
    st = torch.cuda.current_stream()
    res = {rn: [] for rn in range(1, 7)}
    for rnd in range(int(os.environ.get("RP_ROUNDS", "6"))):
        for rn in range(1, 7):
            fn = lambda: r.replace_batch(data[rn], list(range(rn)), buf)  # noqa: E731
            for _ in range(20):
                fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(50):
                fn()
            b.record(st)
            torch.cuda.synchronize()
            t = a.elapsed_time(b) / 50 / 1e3
            res[rn].append(S * (rn + 2 * m) * vec / t / 2**30)
    for rn in range(1, 7):
        v = sorted(res[rn])
        print(f"replace rn={rn}: median {v[len(v) // 2]:8.1f} GiB/s  min {v[0]:8.1f}  max {v[-1]:8.1f}")


if __name__ == "__main__":
    main()
