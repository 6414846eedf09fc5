#!/usr/bin/env python3
"""Reconcile a bench.py line with the rocprofv3 kernel trace of the same run.

    python tools/trace_window.py <kt_kernel_trace.csv> <bench log with the JSON line> [out.json] [out_stats.csv]

Takes the device-resident encode launches (the kernel and grid of the bench's
step: the largest grid of gf_* kernels; the self-check and end-to-end legs use
other grids), splits them into pre-warm, counted warm-up and the K timed
launches (the last K of that grid before the line's `cold` launches), and
reports the timed window's mean launch duration from the trace next to the
line's kernel_ms_mean / ms_per_step and the roofline fraction each implies.
out_stats.csv is a rocprofv3-style stats table (Name, Calls, TotalDurationNs,
AverageNs, MinNs, MaxNs, StdDev) with one row per phase of the bench's encode
launches: its `timed` row alone reproduces the line's frac."""
import csv
import json
import statistics
import sys


def main():
    trace, log = sys.argv[1], sys.argv[2]
    line = next(json.loads(ln) for ln in open(log) if ln.startswith("{"))
    rows = [r for r in csv.DictReader(open(trace)) if "rsamd::gf_" in r["Kernel_Name"]]
    big = max(int(r["Grid_Size_X"]) for r in rows)
    main_rows = [r for r in rows if int(r["Grid_Size_X"]) == big]
    main_rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in main_rows]
    K, W = line["steps"], line["warmup"]
    # launches of the same grid after the timed region: the spread pass queued
    # right behind it (round 4: `timed_spread`), then the `cold` launches
    Sp = (line.get("timed_spread") or {}).get("n", 0) or 0
    C = (line.get("cold") or {}).get("launches", 0)
    end = len(dur) - C - Sp
    timed = dur[end - K:end]
    pre = dur[:end - (K + W)]
    spread_pass = dur[end:end + Sp]
    cold = dur[end + Sp:]
    alg = line["roofline"]["algorithmic_bytes_per_launch"]
    mean_t = statistics.mean(timed)
    out = {
        "kernel": main_rows[0]["Kernel_Name"],
        "grid_size_x": big,
        "launches_of_this_grid": len(dur),
        "timed_window": {"launches": K, "mean_ms": round(mean_t, 4), "min_ms": round(min(timed), 4),
                         "max_ms": round(max(timed), 4),
                         "frac_of_8TBps": round(alg / (mean_t * 1e-3) / 8e12, 4)},
        "warmup_mean_ms": round(statistics.mean(dur[end - (K + W):end - K]), 4) if W else None,
        "cold": {"launches": len(cold), "mean_ms": round(statistics.mean(cold), 4) if cold else None,
                 "line_mean_ms": (line.get("cold") or {}).get("mean_ms")},
        "spread_pass": {"launches": len(spread_pass),
                        "mean_ms": round(statistics.mean(spread_pass), 4) if spread_pass else None,
                        "line_median_ms": (line.get("timed_spread") or {}).get("median_ms")},
        "prewarm": {"launches": len(pre), "first_10_ms": [round(x, 3) for x in pre[:10]],
                    "max_ms": round(max(pre), 4) if pre else None,
                    "last_20_mean_ms": round(statistics.mean(pre[-20:]), 4) if len(pre) >= 20 else None},
        "bench_line": {"ms_per_step": line["ms_per_step"], "kernel_ms_mean": line["roofline"]["kernel_ms_mean"],
                       "frac": line["roofline"]["frac"], "value_GiBps": line["value"],
                       "prewarm": line.get("prewarm")},
        "agreement": {"ms_per_step_vs_trace_mean": round(line["ms_per_step"] / mean_t - 1, 4),
                      "kernel_ms_mean_vs_trace_mean": round(line["roofline"]["kernel_ms_mean"] / mean_t - 1, 4)},
    }
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")
    if len(sys.argv) > 4:
        name = main_rows[0]["Kernel_Name"]
        with open(sys.argv[4], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Phase", "Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "StdDev",
                        "AlgorithmicBytesPerCall", "FracOf8TBps"])
            for phase, xs in (("timed", timed), ("warmup", dur[end - (K + W):end - K]), ("prewarm", pre),
                              ("spread_pass", spread_pass), ("cold", cold)):
                if not xs:
                    continue
                ns = [x * 1e6 for x in xs]
                avg = statistics.mean(ns)
                w.writerow([phase, name, len(ns), round(sum(ns)), round(avg, 1), round(min(ns)), round(max(ns)),
                            round(statistics.pstdev(ns), 1), alg, round(alg / (avg * 1e-9) / 8e12, 4)])


if __name__ == "__main__":
    main()
