"""Builds librsamd.so (the HIP/CDNA4 engine + C ABI) in-tree for gfx950.

    python -m reedsolomon_amd.build                 # or __graft_entry__.build()
    python -m reedsolomon_amd.build --experiments   # also librsamd_exp.so

The library is written to reedsolomon_amd/_lib/librsamd.so; it is
git-ignored but travels to the GPU box with the repository snapshot.

librsamd_exp.so is the same sources with -DRSAMD_EXPERIMENTS: it adds the
code-shape experiments of tools/ab.py / tools/sweep.sh (rs_tune("var"),
RSAMD_VAR), some of which are XOR-only diagnostics that do not compute the GF
product.  It is loaded only when RSAMD_LIB_VARIANT=experiments is set (tools);
the product library has none of those kernels and rejects "var".
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "_lib")
LIB = os.path.join(LIB_DIR, "librsamd.so")
LIB_EXP = os.path.join(LIB_DIR, "librsamd_exp.so")
SOURCES = [os.path.join(CSRC, f) for f in ("codec.cpp", "host_calls.cpp", "batches.cpp", "host_batches.cpp",
                                           "engine.cpp", "watchdog.cpp", "jit.cpp", "jit_asm.cpp",
                                           "kernels.hip")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("gf256.hpp", "kernels.hpp", "codec_internal.hpp",
                                                  "host_pool.hpp", "watchdog.hpp", "jit.hpp", "jit_asm.hpp",
                                                  "bitslice_gen.inc")] + [
    os.path.join(ROOT, "include", "rs_amd.h")
]
ARCH = os.environ.get("RSAMD_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: librsamd.so cannot be built")


def needs_build(lib: str = LIB) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(p) > t for p in DEPS)


def build(force: bool = False, verbose: bool = False, experiments: bool = False) -> str:
    lib = LIB_EXP if experiments else LIB
    if not force and not needs_build(lib):
        return lib
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = lib + ".tmp"
    cmd = [
        hipcc(), "-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}",
        "-fvisibility=hidden", "-Wall", "-Wno-unused-result",
        *(["-DRSAMD_EXPERIMENTS"] if experiments else []),
        "-I", os.path.join(ROOT, "include"),
        *SOURCES, "-o", tmp, "-lhiprtc", "-lamd_comgr", "-ldl",
    ]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    if "--experiments" in sys.argv:
        print(build(force="--force" in sys.argv, verbose=True, experiments=True))
