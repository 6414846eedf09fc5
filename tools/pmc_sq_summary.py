#!/usr/bin/env python3
"""Summarise tools/pmc_sq.sh passes: mean per launch of each counter for the
dominant gf_matmul kernel, plus derived issue shares (SQ_* wave-cycle counters
count quad-cycles; MI355X_MICROARCH.md §Per-instruction cycle constants)."""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

out = sys.argv[1]
res = {}
for d in sorted(glob.glob(os.path.join(out, "p*"))):
    if not os.path.isdir(d):
        continue
    files = glob.glob(os.path.join(d, "**", "pmc_counter_collection.csv"), recursive=True)
    if not files:
        continue
    rows = [r for r in csv.DictReader(open(files[0]))
            if any(k in r["Kernel_Name"] for k in ("gf_matmul", "gf_bitslice", "rs_bs_jit", "rs_bs_asm"))]
    if not rows:
        continue
    dom = statistics.mode(r["Kernel_Name"] for r in rows)
    per = defaultdict(lambda: defaultdict(float))
    for r in rows:
        if r["Kernel_Name"] == dom:
            per[r["Counter_Name"]][r.get("Dispatch_Id", r.get("Correlation_Id", ""))] += float(r["Counter_Value"])
    mean = {c: statistics.mean(v.values()) for c, v in per.items()}
    wc = mean.get("SQ_WAVE_CYCLES", 0) or 1
    derived = {
        "valu_insts_per_wave": mean.get("SQ_INSTS_VALU", 0) / max(mean.get("SQ_WAVES", 1), 1),
        "lds_insts_per_wave": mean.get("SQ_INSTS_LDS", 0) / max(mean.get("SQ_WAVES", 1), 1),
        "wave_cycles_per_wave (x4)": 4 * wc / max(mean.get("SQ_WAVES", 1), 1),
        "share_wait_any": mean.get("SQ_WAIT_ANY", 0) / wc,
        "share_wait_inst_any": mean.get("SQ_WAIT_INST_ANY", 0) / wc,
        "share_active_inst_any": mean.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        "share_active_valu": mean.get("SQ_ACTIVE_INST_VALU", 0) / wc,
        "share_wait_inst_lds": mean.get("SQ_WAIT_INST_LDS", 0) / wc,
        "share_active_lds": mean.get("SQ_ACTIVE_INST_LDS", 0) / wc,
        "share_active_misc": mean.get("SQ_ACTIVE_INST_MISC", 0) / wc,
        "lds_bank_conflict_per_lds_inst": mean.get("SQ_LDS_BANK_CONFLICT", 0) / max(mean.get("SQ_INSTS_LDS", 0), 1),
        "valu_simd_cycles_per_valu_inst": mean.get("SQ_INST_CYCLES_VALU", 0) / max(mean.get("SQ_INSTS_VALU", 0), 1),
        "valu_simd_cycles_per_busy_cycle": mean.get("SQ_INST_CYCLES_VALU", 0) / max(mean.get("SQ_BUSY_CYCLES", 0), 1),
        "ifetch_per_wave": mean.get("SQ_IFETCH", 0) / max(mean.get("SQ_WAVES", 1), 1),
        "icache_miss_rate": mean.get("SQC_ICACHE_MISSES", 0) / max(mean.get("SQC_ICACHE_REQ", 0), 1),
        "icache_hit_rate": mean.get("SQC_ICACHE_HITS", 0) / max(mean.get("SQC_ICACHE_REQ", 0), 1),
    }
    setting = open(os.path.join(d, "setting.txt")).read().strip() if os.path.exists(os.path.join(d, "setting.txt")) else ""
    res[os.path.basename(d)] = {"setting": setting, "kernel": dom, "launches": len(next(iter(per.values()))),
                                "mean_per_launch": mean, "derived": derived}
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
for k, v in res.items():
    print(k, v["setting"], v["kernel"][:60])
    print("   ", {a: round(b, 3) for a, b in v["derived"].items()})
