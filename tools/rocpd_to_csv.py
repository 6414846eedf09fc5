#!/usr/bin/env python3
"""Export a rocprofv3 rocpd database (ROCm 7's default output) to the CSV
files the round-1/2 tools read: <prefix>_kernel_trace.csv (Kernel_Name,
Grid_Size_X, Workgroup_Size_X, Start_Timestamp, End_Timestamp) and
<prefix>_kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs, StdDev).

    python tools/rocpd_to_csv.py <results.db> <out_prefix>
"""
import csv
import sqlite3
import statistics
import sys


def main(db, prefix):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, grid_x, workgroup_x, start, end from kernels order by start"))
    with open(prefix + "_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Grid_Size_X", "Workgroup_Size_X", "Start_Timestamp", "End_Timestamp"])
        w.writerows(rows)
    by = {}
    for name, _, _, s, e in rows:
        by.setdefault(name, []).append(e - s)
    total = sum(sum(v) for v in by.values()) or 1
    with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v),
                        statistics.pstdev(v)])
    print(f"{len(rows)} dispatches, {len(by)} kernels -> {prefix}_kernel_trace.csv / _kernel_stats.csv")


if __name__ == "__main__":
    main(*sys.argv[1:3])
