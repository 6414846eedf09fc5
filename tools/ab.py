#!/usr/bin/env python3
"""In-process A/B of encode-kernel variants (cdna_hip_programming.md §5.4
rule 24): variants are switched with rs_tune() and timed in interleaved
rounds on the same device and buffers; reports median / min kernel time.

    python tools/ab.py "var=12" "var=14" "var=14,layout=inter" ...   (experiments build)
    python tools/ab.py "op=rec1" "op=rec1,block8=256" "op=multi16" ...

jit: 2 (default here: run-time bit-sliced kernels compiled before timing) | 0 (perm-table kernels).
op: enc (Encode, default) | rec1 / rec2 / rec4 / rec5 / rec6 / rec8 (Reconst of
1 / 2 / 4 / 5 / 6 / 8 lost data vectors, split layout; rec8p: 4 data + 4
parity, needs AB_M >= 8) | multi16 (rs_reconst_batch_multi, 16 patterns) |
upd (Update of one row) | repN (Replace of N rows, e.g. rep1, rep3), both on the interleaved
[S][d+p][len] buffer.
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# "var=..." code-shape experiments live only in the experiments build
# (librsamd_exp.so, -DRSAMD_EXPERIMENTS); the product library rejects "var".
EXPERIMENTS = any("var=" in s or "jit_nobar=" in s for s in sys.argv[1:])
if EXPERIMENTS:
    os.environ["RSAMD_LIB_VARIANT"] = "experiments"

import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402

K, M = int(os.environ.get("AB_K", "10")), int(os.environ.get("AB_M", "4"))
VEC = int(os.environ.get("AB_VEC", str(1 << 20)))  # bytes per vector; stripes keep ~3.5 GiB per launch
S = int(os.environ.get("AB_S", str(256 * (1 << 20) // VEC)))  # stripes per launch
ROUNDS = int(os.environ.get("AB_ROUNDS", "12"))
ITERS = int(os.environ.get("AB_ITERS", "20"))
DEFAULTS = {"max_grid": 0, "vpt": 1, "nt_store": 1, "lds_pad": 0, "lane_bytes": 8, "block8": 128,
            "bitslice": 1, "bs_block": 0, "bs_waves": 2, "wide_block": 256, "jit": 2, "jit_pf": 3, "jit_sync": 0, "jit_waves": 2, "jit_min_acc_cols": 1, "jit_min_rows": 5,
            "jit_backend": 2, "jit_layout": 2, "jit_group_waves": 4, "jit_path_rows": 16,
            "jit_wide_pf": 2, "jit_wide_waves": 3, "jit_share": 1, "jit_share_deep": 0, "jit_split_cols": 0, "jit_share_cols": 1, "jit_share_dma": 0,
            "jit_share_ahead": 0, "jit_gray": 0}
LOST = {"rec1": [0], "rec2": [0, 11], "rec4": [0, 2, 5, 9], "rec5": [0, 2, 4, 6, 8], "rec6": [0, 1, 3, 5, 7, 9],
        "rec8": [0, 1, 2, 3, 4, 5, 6, 7], "rec8p": [0, 2, 4, 6, 10, 12, 14, 16], "rec12": list(range(12)),
        "rec16": list(range(16)), "rec24": list(range(24)), "rec32": list(range(32))}


def parse(spec):
    kv = dict(x.split("=") for x in spec.split(",") if x)
    layout = kv.pop("layout", "split")
    op = kv.pop("op", "enc")
    return layout, op, {k: int(v) for k, v in kv.items()}


if EXPERIMENTS:
    DEFAULTS["var"] = -1
    DEFAULTS["jit_nobar"] = 0


def main():
    if EXPERIMENTS:
        from reedsolomon_amd import build as rsbuild
        rsbuild.build(experiments=True)
    specs = sys.argv[1:] or ["jit=2"]
    dev = torch.device("cuda", 0)
    r = rs.New(K, M, device=0)
    L = rs.lib()
    g = torch.Generator(device=dev).manual_seed(1)
    buf = torch.randint(0, 256, (S, K + M, VEC), dtype=torch.uint8, device=dev, generator=g)
    data = torch.randint(0, 256, (S, K, VEC), dtype=torch.uint8, device=dev, generator=g)
    par = torch.empty((S, M, VEC), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    times = {s: [] for s in specs}

    import numpy as np

    rng = np.random.default_rng(5)
    # multi16 patterns over the first 64 vectors (64-bit masks)
    pats = [sum(1 << int(v) for v in rng.choice(min(K + M, 64), int(rng.integers(1, min(M, 64 - K) + 1)),
                                                replace=False))
            for _ in range(16)] if K < 64 else [1] * 16
    masks = np.array([pats[i % 16] for i in range(S)], dtype=np.uint64)
    masks_sorted = np.array([pats[i * 16 // S] for i in range(S)], dtype=np.uint64)  # runs of one pattern
    nrec16 = sum(bin(int(x)).count("1") for x in masks)
    r.encode_batch_split(data, par)

    def setup(spec):
        layout, op, kv = parse(spec)
        for k, v in {**DEFAULTS, **kv}.items():
            assert L.rs_tune(k.encode(), v) == 0, k
        if op in LOST:
            lost = LOST[op]
            if layout == "inter":  # in place in the [S][K+M][VEC] buffer
                return (lambda: r.reconst_batch(buf, [], lost)), S * (K + len(lost)) * VEC
            return (lambda: r.reconst_batch_split(data, par, [], lost)), S * (K + len(lost)) * VEC
        if op == "upd":  # Update row 3 of every stripe: reads old, new, 4 parity; writes 4 parity
            return (lambda: r.update_batch(data[:, 0], data[:, 1], 3, buf)), S * (2 + 2 * M) * VEC
        if op.startswith("rep"):  # Replace of n rows (1, 4, 7, ...): reads n data + m parity, writes m parity
            rn = int(op[3:])
            rows = [1 + 3 * i for i in range(rn)]
            return (lambda: r.replace_batch(data[:, :rn], rows, buf)), S * (rn + 2 * M) * VEC
        if op == "multi16s":
            return (lambda: r.reconst_batch_multi(data, par, masks_sorted)), (S * K + nrec16) * VEC
        if op == "multi16":
            return (lambda: r.reconst_batch_multi(data, par, masks)), (S * K + nrec16) * VEC
        if layout == "inter":
            return (lambda: r.encode_batch(buf)), S * (K + M) * VEC
        return (lambda: r.encode_batch_split(data, par)), S * (K + M) * VEC

    nbytes = {}
    for s in specs:  # warm every variant
        f, nbytes[s] = setup(s)
        for _ in range(30):
            f()
    torch.cuda.synchronize()
    for _ in range(ROUNDS):
        for s in specs:
            f, _ = setup(s)
            f()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(ITERS):
                f()
            b.record(st)
            torch.cuda.synchronize()
            times[s].append(a.elapsed_time(b) / ITERS)
    for s in specs:
        med, mn = statistics.median(times[s]), min(times[s])
        print(f"{s:40s} median {med:.4f} ms ({nbytes[s] / med / 1e9:7.3f} TB/s)  min {mn:.4f} ms "
              f"({nbytes[s] / mn / 1e9:7.3f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
