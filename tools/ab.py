#!/usr/bin/env python3
"""In-process A/B of encode-kernel variants (cdna_hip_programming.md §5.4
rule 24): variants are switched with rs_tune() and timed in interleaved
rounds on the same device and buffers; reports median / min kernel time.

    python tools/ab.py "var=12" "var=14" "var=14,layout=inter" ...
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402

K, M, VEC, S = 10, 4, 1 << 20, 256
ROUNDS = int(os.environ.get("AB_ROUNDS", "12"))
ITERS = int(os.environ.get("AB_ITERS", "20"))
DEFAULTS = {"max_grid": 0, "vpt": 1, "nt_store": 1, "var": -1, "lds_pad": 0}


def parse(spec):
    kv = dict(x.split("=") for x in spec.split(",") if x)
    layout = kv.pop("layout", "split")
    return layout, {k: int(v) for k, v in kv.items()}


def main():
    specs = sys.argv[1:] or ["var=12"]
    dev = torch.device("cuda", 0)
    r = rs.New(K, M, device=0)
    L = rs.lib()
    g = torch.Generator(device=dev).manual_seed(1)
    buf = torch.randint(0, 256, (S, K + M, VEC), dtype=torch.uint8, device=dev, generator=g)
    data = torch.randint(0, 256, (S, K, VEC), dtype=torch.uint8, device=dev, generator=g)
    par = torch.empty((S, M, VEC), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    times = {s: [] for s in specs}

    def setup(spec):
        layout, kv = parse(spec)
        for k, v in {**DEFAULTS, **kv}.items():
            assert L.rs_tune(k.encode(), v) == 0, k
        return (lambda: r.encode_batch(buf)) if layout == "inter" else (lambda: r.encode_batch_split(data, par))

    for s in specs:  # warm every variant
        f = setup(s)
        for _ in range(30):
            f()
    torch.cuda.synchronize()
    for _ in range(ROUNDS):
        for s in specs:
            f = setup(s)
            f()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(ITERS):
                f()
            b.record(st)
            torch.cuda.synchronize()
            times[s].append(a.elapsed_time(b) / ITERS)
    nbytes = S * (K + M) * VEC
    for s in specs:
        med, mn = statistics.median(times[s]), min(times[s])
        print(f"{s:40s} median {med:.4f} ms ({nbytes / med / 1e9:7.1f} TB/s)  min {mn:.4f} ms "
              f"({nbytes / mn / 1e9:7.1f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
