#!/usr/bin/env python3
"""Turn gpurun_out/prof (tools/gpu_profile.sh) into committed summaries:
  profiles/<round>/kernel_stats.csv      rocprofv3 --kernel-trace --stats summary
  profiles/<round>/pmc_summary.json      FETCH_SIZE / WRITE_SIZE per launch
  profiles/traffic.json                  HBM bytes per launch, read by bench.py

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports half
the bytes of a wide 16-B/lane streaming read -> doubled; WRITE_SIZE (KiB) is
exact for 16-B/lane stores."""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
cfg = sys.argv[2] if len(sys.argv) > 2 else "10+4@1MiB"
src = os.path.join(ROOT, "gpurun_out", "prof")
dst = os.path.join(ROOT, "profiles", rnd)
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))


def per_launch(counter):
    rows = list(csv.DictReader(open(os.path.join(src, f"pmc_{counter}", "pmc_counter_collection.csv"))))
    names = [r["Kernel_Name"] for r in rows if "gf_matmul_vec" in r["Kernel_Name"]]
    dom = statistics.mode(names)
    vals = [float(r["Counter_Value"]) for r in rows if r["Kernel_Name"] == dom]
    return vals


fetch = per_launch("FETCH_SIZE")
write = per_launch("WRITE_SIZE")
f_b = statistics.median(fetch) * 1024 * 2
w_b = statistics.median(write) * 1024
trace_all = [r for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_trace.csv")))
             if "gf_matmul_vec" in r["Kernel_Name"]]
dominant = statistics.mode([r["Kernel_Name"] for r in trace_all])
trace = [r for r in trace_all if r["Kernel_Name"] == dominant]
durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace]
steps = int(os.environ.get("BENCH_STEPS", "100"))
summary = {
    "config": cfg,
    "kernel": trace[0]["Kernel_Name"] if trace else None,
    "launches_traced": len(durs),
    "duration_ns_mean_all_launches": statistics.mean(durs) if durs else None,
    "duration_ns_mean_timed_region": statistics.mean(durs[-steps:]) if durs else None,
    "timed_region_note": f"last {steps} launches = bench.py's timed steps (the earlier ones are the self-check "
                         "and warm-up, which include the post-idle power transient)",
    "FETCH_SIZE_KiB_median": statistics.median(fetch),
    "WRITE_SIZE_KiB_median": statistics.median(write),
    "hbm_read_bytes_per_launch (FETCH_SIZE*1024*2)": f_b,
    "hbm_write_bytes_per_launch (WRITE_SIZE*1024)": w_b,
    "hbm_bytes_per_launch": f_b + w_b,
}
json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
tpath = os.path.join(ROOT, "profiles", "traffic.json")
traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
traffic[cfg] = {"hbm_bytes_per_launch": int(f_b + w_b), "source": f"profiles/{rnd}/pmc_summary.json"}
json.dump(traffic, open(tpath, "w"), indent=1)
print(json.dumps(summary, indent=1))
