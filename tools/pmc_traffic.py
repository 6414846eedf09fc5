#!/usr/bin/env python3
"""HBM traffic per launch of one product shape, for rocprofv3 --pmc passes
(MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE in separate passes).

    python tools/pmc_traffic.py run enc:64+64                  # the workload (5 launches)
    python tools/pmc_traffic.py run rec:16+16:16 --jit 0        # Reconst of 16 lost
    python tools/pmc_traffic.py run inrec:10+8:8                # the same in place (interleaved layout)
    python tools/pmc_traffic.py run enc:128+128@jit_layout=1,jit_group_waves=4   # rs_tune knobs first
    python tools/pmc_traffic.py summarize <tag> <dir_FETCH> <dir_WRITE> <calib_FETCH> <calib_WRITE>

`run` encodes (or rebuilds) ~3.5 GiB of 1 MiB-vector stripes on the split
layout, 5 launches after 2 untimed ones, and prints the algorithmic bytes
per launch ((k+m)*vec*S for Encode, (k+lost)*vec*S for Reconst).
`summarize` reads the counter CSVs of the dominant codec kernel and converts
them with the calibration factors measured over known bytes
(tools/fetch_calib.py, same counters): HBM bytes per launch and their ratio
to the algorithmic bytes.
"""
import csv
import json
import math
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(spec, jit):
    import torch

    import reedsolomon_amd as rs

    spec, _, knobs = spec.partition("@")
    op, shape, *rest = spec.split(":")
    k, m = (int(x) for x in shape.split("+"))
    vec = 1 << 20
    S = max(1, (3584 << 20) // ((k + m) * vec))
    assert rs.lib().rs_tune(b"jit", jit) == 0
    for kv in filter(None, knobs.split(",")):
        name, val = kv.split("=")
        assert rs.lib().rs_tune(name.encode(), int(val)) == 0, kv
    r = rs.New(k, m)
    g = torch.Generator(device="cuda").manual_seed(7)
    data = torch.randint(0, 256, (S, k, vec), dtype=torch.uint8, device="cuda", generator=g)
    par = torch.empty((S, m, vec), dtype=torch.uint8, device="cuda")
    r.encode_batch_split(data, par)
    if op == "enc":
        fn, nbytes = (lambda: r.encode_batch_split(data, par)), S * (k + m) * vec
    elif op == "inrec":  # Reconst in place on the interleaved [S][k+m][vec] buffer
        buf = torch.cat([data, par], dim=1).contiguous()
        del data, par
        lost = list(range(int(rest[0])))
        fn, nbytes = (lambda: r.reconst_batch(buf, [], lost)), S * (k + len(lost)) * vec
    else:
        lost = list(range(int(rest[0])))
        fn, nbytes = (lambda: r.reconst_batch_split(data, par, [], lost)), S * (k + len(lost)) * vec
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    print(json.dumps({"spec": spec, "jit": jit, "stripes": S, "algorithmic_bytes_per_launch": nbytes}))


def counter_rows(d):
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                return list(csv.DictReader(open(os.path.join(root, f))))
    raise SystemExit(f"no counter_collection.csv under {d}")


def per_launch(d, want=("gf_matmul", "rs_bs_jit", "rs_bs_asm", "gf_bitslice")):
    rows = [r for r in counter_rows(d) if any(w in r["Kernel_Name"] for w in want)]
    by = {}
    for r in rows:
        by.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    name = max(by, key=lambda n: len(by[n]) * statistics.median(by[n]))
    return name, by[name]


def calib(d, kernel, nbytes=2 << 30):
    vals = [float(r["Counter_Value"]) for r in counter_rows(d) if kernel in r["Kernel_Name"]]
    raw = nbytes / (statistics.median(vals) * 1024)
    return {"measured": raw, "unit": 2.0 ** round(math.log2(raw))}


def summarize(tag, dfetch, dwrite, cfetch, cwrite, algorithmic):
    kf, fetch = per_launch(dfetch)
    kw, write = per_launch(dwrite)
    # the kernels read and write with 16- or 8-byte lanes: use the
    # calibration of the kernel's width (gf_matmul_wide: 16 B; the bit-sliced
    # and one-chunk kernels: 8 B)
    w = 16 if ("gf_matmul_wide" in kf or "16B" in kf) else 8
    cr, cw = calib(cfetch, f"kc_read{w}"), calib(cwrite, f"kc_write{w}")
    f_b = statistics.median(fetch[2:] or fetch) * 1024 * cr["unit"]
    w_b = statistics.median(write[2:] or write) * 1024 * cw["unit"]
    out = {"tag": tag, "kernel": kf, "lane_bytes": w, "fetch_bytes_per_launch": f_b, "write_bytes_per_launch": w_b,
           "hbm_bytes_per_launch": f_b + w_b, "algorithmic_bytes_per_launch": algorithmic,
           "ratio": round((f_b + w_b) / algorithmic, 5), "calibration": {"read": cr, "write": cw},
           "launches_counted": [len(fetch), len(write)]}
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    if sys.argv[1] == "run":
        jit = int(sys.argv[sys.argv.index("--jit") + 1]) if "--jit" in sys.argv else 2
        run(sys.argv[2], jit)
    else:
        summarize(*sys.argv[2:7], int(sys.argv[7]))
