#!/usr/bin/env python3
"""Where does the multi-pattern Reconst lose time at 8 KiB?  (10+4, split
layout, device-resident, one rs_reconst_batch_multi launch per call.)

Pattern sets, each assigned to stripes in runs of R consecutive stripes:
  mixed16   16 random patterns, 1-4 lost of 14 (tools/multi_probe.py's set)
  pos16_4   16 patterns, all 4 lost data vectors, different positions
  pos16_1   16 patterns, 1 lost data vector each (positions 0..9, repeated)
  nout4     4 patterns losing data {0}, {0,1}, {0,1,2}, {0,1,2,3}
Rate = (k + lost) * vec bytes per stripe / time.  MIX_LAYOUT=interleaved
uses one [S][k+m][vec] buffer.  Writes gpurun_out/multi_mix_<layout>.json.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402

GiB = 2 ** 30


def dev_time(fn, iters=40, warm=10):
    st = torch.cuda.current_stream()
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(st)
    for _ in range(iters):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters / 1e3


def mask(lost):
    return sum(1 << int(v) for v in lost)


def main():
    k, m = 10, 4
    vec = int(os.environ.get("MIX_VEC", 8 << 10))
    S = int(os.environ.get("MIX_S", (256 << 20) // vec))
    rng = np.random.default_rng(5)
    sets = {"mixed16": [mask(rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False)) for _ in range(16)]}
    rng = np.random.default_rng(7)
    sets["pos16_4"] = [mask(rng.choice(k, 4, replace=False)) for _ in range(16)]
    sets["pos16_1"] = [mask([i % k]) for i in range(16)]
    sets["nout4"] = [mask(range(n)) for n in (1, 2, 3, 4)]
    g = torch.Generator(device="cuda").manual_seed(3)
    r = rs.New(k, m)
    layout = os.environ.get("MIX_LAYOUT", "split")
    if layout == "interleaved":  # one [S][k+m][vec] buffer
        buf = torch.randint(0, 256, (S, k + m, vec), dtype=torch.uint8, device="cuda", generator=g)
        data, parity = buf[:, :k], buf[:, k:]
    else:
        data = torch.randint(0, 256, (S, k, vec), dtype=torch.uint8, device="cuda", generator=g)
        parity = torch.empty((S, m, vec), dtype=torch.uint8, device="cuda")
    r.encode_batch_split(data, parity)
    out = {"vec": vec, "stripes": S, "layout": layout}
    for name, pats in sets.items():
        for run in (1, 8, 64, S // len(pats)):
            masks = np.array([pats[(i // run) % len(pats)] for i in range(S)], dtype=np.uint64)
            nrec = sum(bin(int(x)).count("1") for x in masks)
            best = min(dev_time(lambda: r.reconst_batch_multi(data, parity, masks)) for _ in range(3))
            key = f"{name} run={run}"
            out[key] = {"us": round(best * 1e6, 1), "GiBps": round((S * k + nrec) * vec / best / GiB, 1)}
            print(key, out[key], flush=True)
        # every stripe on one pattern of the set, one launch each, time-weighted
        tot_t = tot_b = 0.0
        for pm in pats:
            masks = np.full(S, pm, np.uint64)
            t = min(dev_time(lambda: r.reconst_batch_multi(data, parity, masks)) for _ in range(2))
            tot_t += t
            tot_b += S * (k + bin(pm).count("1")) * vec
        out[f"{name} separate"] = {"GiBps": round(tot_b / tot_t / GiB, 1)}
        print(f"{name} separate", out[f"{name} separate"], flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open(f"gpurun_out/multi_mix_{layout}.json", "w"), indent=1)


if __name__ == "__main__":
    main()
