#!/usr/bin/env python3
"""Turn gpurun_out/prof (tools/gpu_profile.sh) into committed summaries:
  profiles/<round>/kernel_stats.csv      rocprofv3 --kernel-trace --stats summary
  profiles/<round>/pmc_summary.json      FETCH_SIZE / WRITE_SIZE per launch
  profiles/traffic.json                  HBM bytes per launch, read by bench.py

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports half
the bytes of a wide 16-B/lane streaming read and WRITE_SIZE is exact for
16-B/lane stores; other widths are uncalibrated there.  The codec kernel uses
8-byte lanes, so gpu_profile.sh also runs tools/fetch_calib.py (one pass over
a known 2 GiB with 16- and 8-byte buffer loads / stores) under the same
counters, and the factor measured for the kernel's width (bytes per counted
byte) converts its counts."""
import csv
import json
import math
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


def calib(counter, kernel, nbytes=2 << 30):
    """Bytes per counted byte for one calibration kernel (median over its
    launches), as measured and rounded to the counter's unit (a power of two:
    the measured 1.99998 / 0.9989-0.9993 are 2 and 1 plus ~0.1 % of unrelated
    traffic counted during the calibration launch)."""
    path = os.path.join(src, f"calib_{counter}", "pmc_counter_collection.csv")
    if not os.path.exists(path):
        return None
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    if not vals:
        return None
    raw = nbytes / (statistics.median(vals) * 1024)
    return {"measured": raw, "unit": 2.0 ** round(math.log2(raw))}


lane = 8 if os.environ.get("RSAMD_LANE_BYTES", "8") != "16" else 16
cal = {f"read{w}": calib("FETCH_SIZE", f"kc_read{w}") for w in (16, 8)}
cal.update({f"write{w}": calib("WRITE_SIZE", f"kc_write{w}") for w in (16, 8)})
f_fac = cal[f"read{lane}"]["unit"] if cal[f"read{lane}"] else 2.0
w_fac = cal[f"write{lane}"]["unit"] if cal[f"write{lane}"] else 1.0
f_b = statistics.median(fetch) * 1024 * f_fac
w_b = statistics.median(write) * 1024 * w_fac
trace_all = [r for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_trace.csv")))
             if "gf_matmul_vec" in r["Kernel_Name"]]
dominant = statistics.mode([r["Kernel_Name"] for r in trace_all])
trace = [r for r in trace_all if r["Kernel_Name"] == dominant]
durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in trace]
steps = int(os.environ.get("BENCH_STEPS", "1000"))  # tools/gpu_profile.sh runs --steps 1000
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (the config table: algorithmic bytes of this launch)

_k, _m, _vec, _S = bench.CONFIGS[cfg]
summary = {
    "config": cfg,
    "algorithmic_bytes_per_launch": (_k + _m) * _vec * _S,
    "kernel": trace[0]["Kernel_Name"] if trace else None,
    "launches_traced": len(durs),
    "duration_ns_mean_all_launches": statistics.mean(durs) if durs else None,
    "duration_ns_mean_timed_region": statistics.mean(durs[-steps:]) if durs else None,
    "timed_region_note": f"last {steps} launches = bench.py's timed steps (the earlier ones are the self-check "
                         "and warm-up, which include the post-idle power transient)",
    "FETCH_SIZE_KiB_median": statistics.median(fetch),
    "WRITE_SIZE_KiB_median": statistics.median(write),
    "lane_bytes": lane,
    "counter_calibration_bytes_per_counted_byte": cal,
    "hbm_read_bytes_per_launch (FETCH_SIZE*1024*factor)": f_b,
    "hbm_write_bytes_per_launch (WRITE_SIZE*1024*factor)": w_b,
    "hbm_bytes_per_launch": f_b + w_b,
}
json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
tpath = os.path.join(ROOT, "profiles", "traffic.json")
traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
traffic[cfg] = {"hbm_bytes_per_launch": int(f_b + w_b), "source": f"profiles/{rnd}/pmc_summary.json",
                "algorithmic_bytes_per_launch": summary.get("algorithmic_bytes_per_launch")}
json.dump(traffic, open(tpath, "w"), indent=1)
print(json.dumps(summary, indent=1))
