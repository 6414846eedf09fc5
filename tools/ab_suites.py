#!/usr/bin/env python3
"""Named A/B suites for tools/ab.py (round 4: replaces the one-off
tools/ab_*.sh scripts of rounds 1-2).  Each suite is a list of (shape
environment, variant specs); every entry runs tools/ab.py in its own
process under a time limit, and the suite stops at the first failure.

    python tools/ab_suites.py list
    python tools/ab_suites.py layout gap16_4 ...

Specs are tools/ab.py's ("knob=value,..." pairs, op=..., layout=inter);
"var=..." specs need the experiments build (ab.py loads it itself).  The
logs the DESIGN.md tables cite live under profiles/ (ab_<suite>.log)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def shapes(km, specs, **env):
    return [(dict(AB_K=str(k), AB_M=str(m), **env), specs) for k, m in km]


SUITES = {
    # round 1: bit-sliced Encode vs perm-table kernels, split / interleaved (profiles/r01/ab_bitslice*.log)
    "bitslice": shapes([(10, 8), (10, 6), (10, 5), (12, 8), (8, 5), (8, 8)], ["", "bitslice=0"], AB_ROUNDS="8"),
    "bitslice4": shapes([(10, 4), (12, 4)], ["", "bitslice=2", "layout=inter", "bitslice=2,layout=inter"],
                        AB_ROUNDS="10") + [(dict(AB_VEC="8192", AB_ROUNDS="10"), ["", "bitslice=2"])],
    "bitslice_inter": shapes([(10, 8), (10, 6), (12, 8), (8, 5)], ["layout=inter", "bitslice=0,layout=inter"],
                             AB_ROUNDS="8"),
    "bitslice_q": shapes([(10, 8), (10, 6), (8, 5)], ["", "var=202", "bitslice=0"], AB_ROUNDS="8") +
    shapes([(10, 4), (12, 4)], ["", "bitslice=2", "bitslice=2,var=202"], AB_ROUNDS="8"),
    "bs_block": [e for km in [(10, 8), (10, 6), (12, 8), (8, 5), (10, 5), (8, 8)] for e in
                 shapes([km], ["", "bs_block=64", "bs_block=128", "bs_block=256"], AB_ROUNDS="6") +
                 shapes([km], ["layout=inter", "bs_block=64,layout=inter", "bs_block=128,layout=inter",
                               "bs_block=256,layout=inter"], AB_ROUNDS="6")],
    "cols8": shapes([(16, 4), (14, 4), (9, 3), (12, 4), (20, 4), (16, 8)],
                    ["", "var=200", "op=rec1", "op=rec1,var=200"], AB_ROUNDS="8"),
    "lane_generic": shapes([(8, 4), (6, 3), (16, 4), (20, 4), (8, 2), (4, 2)],
                           ["", "lane_bytes=16", "op=rec1", "op=rec1,lane_bytes=16"], AB_ROUNDS="8"),
    "lane_generic2": shapes([(12, 4), (10, 4), (8, 3), (16, 3), (12, 3)],
                            ["", "lane_bytes=16", "op=upd", "op=upd,lane_bytes=16", "op=rep3", "op=rep3,lane_bytes=16"],
                            AB_ROUNDS="8"),
    "rows8": shapes([(10, 8), (12, 8), (8, 5), (16, 8), (20, 6)],
                    ["", "max_grid=1073741824", "var=200", "op=rep3", "op=rep3,var=200", "op=rep3,max_grid=1073741824"],
                    AB_ROUNDS="8"),
    "wide34": shapes([(8, 4), (6, 3), (16, 4), (8, 3), (20, 4), (5, 4), (9, 3)], ["", "var=201"], AB_ROUNDS="8"),
    "wide34_inter": shapes([(16, 4), (8, 4), (6, 3), (20, 4)], ["layout=inter", "var=201,layout=inter"],
                           AB_ROUNDS="8"),
    # round 4: generated kernels of more than 16 rows, rows over waves (jit_layout=0) vs row
    # groups over workgroups (1) with 2-8 waves each (~3.5 GiB per launch)
    "layout": [(dict(AB_K=str(k), AB_M=str(m), AB_S=str(s)),
                ["jit_layout=0", "jit_layout=1,jit_group_waves=2", "jit_layout=1,jit_group_waves=4",
                 "jit_layout=1,jit_group_waves=8"])
               for k, m, s in ((32, 32, 56), (64, 64, 28), (128, 128, 14), (200, 56, 14))],
    # round 4: occupancy of the wide generated kernels (VALU-latency bound at 2 waves per SIMD:
    # profiles/r04/pmc_icache): the 2-wave cap off, fewer columns of loads in flight, fewer rows per path
    "wide_occupancy": [(dict(AB_K=str(k), AB_M=str(m), AB_S=str(s)),
                        ["jit_waves=2", "jit_waves=0", "jit_waves=0,jit_pf=1", "jit_waves=0,jit_path_rows=13,jit_pf=2",
                         "jit_waves=0,jit_path_rows=11,jit_pf=1", "jit_waves=0,jit_path_rows=10,jit_pf=2",
                         "jit_waves=0,jit_path_rows=8"])  # (before jit_wide_*: jit_pf / jit_waves applied to every row count)
                       for k, m, s in ((32, 32, 56), (64, 64, 28), (128, 128, 14), (200, 56, 14))],
    # round 4: 16-row paths in 168 VGPRs at two columns of loads in flight (3 waves per SIMD
    # without the cap) against the capped default
    "wide_waves3": [(dict(AB_K=str(k), AB_M=str(m), AB_S=str(s)),
                     ["jit_waves=2", "jit_waves=0,jit_pf=2", "jit_waves=3,jit_pf=2", "jit_waves=0"])
                    for k, m, s in ((16, 16, 112), (32, 32, 56), (64, 64, 28), (128, 128, 14), (200, 56, 14))] +
                   [(dict(AB_K="16", AB_M="16", AB_S="112"), ["op=rec24,jit_waves=2", "op=rec24,jit_waves=0,jit_pf=2"])],
    # round 4: the 3-wave setting with the row-group layout
    "wide_combo": [(dict(AB_K=str(k), AB_M=str(m), AB_S=str(s)),
                    ["jit_wide_waves=2,jit_wide_pf=3", "", "jit_layout=1,jit_group_waves=2",
                     "jit_layout=1,jit_group_waves=4"])
                   for k, m, s in ((32, 32, 56), (64, 64, 28), (128, 128, 14), (200, 56, 14))] +
                  [(dict(AB_K="32", AB_M="32", AB_S="56"),
                    ["op=rec24,jit_wide_waves=2,jit_wide_pf=3", "op=rec24", "op=rec24,jit_layout=1,jit_group_waves=2",
                     "layout=inter,op=rec24,jit_wide_waves=2,jit_wide_pf=3", "layout=inter,op=rec24",
                     "layout=inter,op=rec24,jit_layout=1,jit_group_waves=2"])],
    # round 4: the waves of a multi-path workgroup share each column's load and transpose
    # through LDS (jit_share=1) against every wave loading and transposing every column
    "share": [(dict(AB_K=str(k), AB_M=str(m), AB_S=str(s)),
               ["", "jit_share=1", "jit_share=1,jit_wide_waves=2", "jit_share=1,jit_wide_waves=0"])
              for k, m, s in ((32, 32, 56), (64, 64, 28), (128, 128, 14), (200, 56, 14))] +
             [(dict(AB_K="32", AB_M="32", AB_S="56"), ["op=rec24", "op=rec24,jit_share=1"])],
    # round 4: shared columns with two steps of loads in flight and LDS reads one column ahead
    "share_deep": [(dict(AB_K=str(k), AB_M=str(m), AB_S=str(s)),
                    ["jit_share_deep=0", "jit_share_deep=1", "jit_share_deep=1,jit_wide_waves=0"])
                   for k, m, s in ((32, 32, 56), (64, 64, 28), (128, 128, 14), (200, 56, 14))],
    # round 4: shared columns with fewer rows per path (more paths, fewer accumulators) and the
    # deep variant, which then fits 3 waves per SIMD
    "share_paths": [(dict(AB_K=str(k), AB_M=str(m), AB_S=str(s)),
                     ["", "jit_path_rows=13", "jit_path_rows=13,jit_share_deep=1", "jit_path_rows=11,jit_share_deep=1",
                      "jit_path_rows=11"])
                    for k, m, s in ((32, 32, 56), (64, 64, 28), (128, 128, 14), (200, 56, 14))],
    # round 4: shared columns, two columns per wave and step (half the barriers, 8 more VGPRs)
    "share_cols": [(dict(AB_K=str(k), AB_M=str(m), AB_S=str(s)),
                    ["", "jit_share_cols=2", "jit_share_cols=2,jit_wide_waves=0"])
                   for k, m, s in ((32, 32, 56), (64, 64, 28), (128, 128, 14), (200, 56, 14))],
    # round 4: 9-16 rows over many columns as two 8-row paths sharing the columns (jit_split_cols)
    "split_small": [(dict(AB_K=str(k), AB_M=str(m), AB_VEC=str(v), **({"AB_S": str(s_)} if s_ else {})),
                     [f"{op}", f"{op},jit_split_cols=16", f"{op},jit_split_cols=16,jit_wide_waves=0",
                      f"{op},jit_split_cols=16,jit_wide_waves=4,jit_wide_pf=1"])
                    for k, m, v, s_, op in ((48, 16, 262144, 224, "op=rec16"), (100, 16, 262144, 112, "op=rec16"),
                                            (200, 16, 1 << 20, 16, "op=enc"), (16, 16, 1 << 20, 112, "op=enc"),
                                            (32, 12, 1 << 20, 72, "op=enc"))],
    # round 4: 3-4 rows over more than 4 runtime columns, 16-byte units on 256 lanes (default since
    # round 1) vs 8-byte units on 128 lanes (var=201, experiments build), split and interleaved
    "wide34_r4": shapes([(16, 4), (20, 4), (8, 4), (6, 3), (9, 3), (16, 3)],
                        ["", "var=201", "layout=inter", "var=201,layout=inter"], AB_ROUNDS="8"),
    # round 4: the weakest 4-row shapes (16+4 Encode, Replace of 1 row, Update at 8 KiB) at the
    # library's lane widths; their XOR-only access-pattern ceilings: hbm_probe.py PROBE_KMG=1
    "gap16_4": [(dict(AB_K="16", AB_M="4"), ["", "layout=inter", "lane_bytes=16", "lane_bytes=16,layout=inter",
                                               "block8=256", "block8=256,layout=inter"]),
                (dict(AB_K="10", AB_M="4", AB_VEC="8192"), ["op=rep1", "op=rep1,lane_bytes=16", "op=upd",
                                                            "op=upd,lane_bytes=16", "op=rep1,block8=256"])],
    # round 5: the low half's subsets built one at a time in Gray-code order (12 subset
    # registers, not 22), which makes room for reading the next column's planes from LDS
    # while one combines (jit_share_ahead) at 3 waves per SIMD, or for 4 waves per SIMD
    # with 11-13-row paths
    "gray_ahead": [(dict(AB_K=str(k), AB_M=str(m), AB_S=str(s)),
                    ["", "jit_gray=1", "jit_share_ahead=1", "jit_gray=1,jit_share_ahead=1",
                     "jit_gray=1,jit_path_rows=12,jit_wide_waves=4",
                     "jit_gray=1,jit_share_ahead=1,jit_path_rows=11,jit_wide_waves=4",
                     "jit_gray=1,jit_share_dma=3,jit_path_rows=13,jit_wide_waves=4"])
                   for k, m, s in ((64, 64, 28), (128, 128, 14), (200, 56, 14), (32, 32, 56))],
}


def main(argv):
    if not argv or argv[0] == "list":
        for k, v in SUITES.items():
            print(f"{k:16s} {len(v)} runs")
        return 0
    for name in argv:
        for env, specs in SUITES[name]:
            print(f"== {name}: {' '.join(f'{a}={b}' for a, b in env.items())}", flush=True)
            rc = subprocess.call([sys.executable, "-u", os.path.join(ROOT, "tools", "ab.py"), *specs],
                                 env=dict(os.environ, **env), timeout=300)
            if rc != 0:
                print(f"== {name}: ab.py exit {rc}; stopping", flush=True)
                return rc
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
