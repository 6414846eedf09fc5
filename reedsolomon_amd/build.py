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

import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

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


def _flags(experiments: bool) -> list:
    return ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}",
            "-fvisibility=hidden", "-Wall", "-Wno-unused-result",
            *(["-DRSAMD_EXPERIMENTS"] if experiments else [])]


def source_digest(deps=None, experiments: bool = False) -> str:
    """SHA-256 over every source the library is built from (by path relative to
    the repository, then content), this script, and the compile flags.  It is
    compiled into the library (rs_build_id) and decides whether a rebuild is
    due, so a measured binary always names the sources it came from."""
    h = hashlib.sha256()
    for path in sorted(deps if deps is not None else DEPS + [os.path.abspath(__file__)]):
        rel = os.path.relpath(path, ROOT) if path.startswith(ROOT) else os.path.basename(path)
        h.update(rel.encode() + b"\0")
        with open(path, "rb") as f:
            data = f.read()
        h.update(len(data).to_bytes(8, "little") + data)
    h.update(" ".join(_flags(experiments)).encode())
    return h.hexdigest()


_STAMP = b"RSAMD_BUILD_ID="


def library_digest(lib: str = LIB):
    """The digest stamped into a built library file (read from the file, not
    loaded), or None when the file is missing or unstamped."""
    try:
        with open(lib, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(_STAMP)
    if i < 0:
        return None
    tag = data[i + len(_STAMP):i + len(_STAMP) + 64]
    try:
        tag = tag.decode("ascii")
    except UnicodeDecodeError:
        return None
    return tag if len(tag) == 64 and all(c in "0123456789abcdef" for c in tag) else None


def needs_build(lib: str = LIB, deps=None, experiments=None) -> bool:
    """True unless `lib` carries the digest of the current sources."""
    if experiments is None:
        experiments = lib == LIB_EXP
    return library_digest(lib) != source_digest(deps, experiments)


def build(force: bool = False, verbose: bool = False, experiments: bool = False) -> str:
    lib = LIB_EXP if experiments else LIB
    if not force and not needs_build(lib):
        return lib
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = lib + ".tmp"
    digest = source_digest(experiments=experiments)
    objdir = os.path.join(LIB_DIR, "obj_exp" if experiments else "obj")
    os.makedirs(objdir, exist_ok=True)
    flags = [*_flags(experiments), f'-DRSAMD_BUILD_ID="{digest}"', "-I", os.path.join(ROOT, "include")]
    # One hipcc per source, in parallel (kernels.hip alone takes most of a
    # serial build), then one link.
    objs, cmds = [], []
    for src in SOURCES:
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        objs.append(obj)
        cmds.append([hipcc(), *[f for f in flags if f != "-shared"], "-c", src, "-o", obj])
    if verbose:
        for c in cmds:
            print(" ".join(c), file=sys.stderr)
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with ThreadPoolExecutor(jobs) as pool:
        for r in list(pool.map(lambda c: subprocess.run(c), cmds)):
            if r.returncode != 0:
                raise subprocess.CalledProcessError(r.returncode, r.args)
    link = [hipcc(), *_flags(experiments), *objs, "-o", tmp, "-lhiprtc", "-lamd_comgr", "-ldl"]
    if verbose:
        print(" ".join(link), file=sys.stderr)
    subprocess.run(link, check=True)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    if "--experiments" in sys.argv:
        print(build(force="--force" in sys.argv, verbose=True, experiments=True))
