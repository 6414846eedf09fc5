"""The C ABI from C: tests/c/rs_consumer.c compiled as strict C99 and as C++17
against include/rs_amd.h and the in-tree librsamd.so (what a cgo/FFI
binding links against), then run."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c", "rs_consumer.c")


def _build(rslib, out, cxx=False):
    libdir = os.path.dirname(rslib.LIB_PATH)
    cmd = (["g++", "-x", "c++", "-std=c++17"] if cxx else ["gcc", "-std=c99", "-pedantic", "-Wextra"]) + [
        "-Wall", "-Werror", "-O1", "-I", os.path.join(ROOT, "include"), SRC, "-L", libdir, "-lrsamd",
        f"-Wl,-rpath,{libdir}", "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return str(out)


def _run(exe, mode, timeout):
    r = subprocess.run([exe, mode], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"rs_consumer {mode}: ok" in r.stdout


@pytest.mark.parametrize("cxx", [False, True], ids=["c99", "cxx17"])
def test_c_consumer_host(rslib, tmp_path, cxx):
    _run(_build(rslib, tmp_path / "rs_consumer", cxx), "host", 60)


@pytest.mark.gpu
def test_c_consumer_gpu(rslib, tmp_path):
    _run(_build(rslib, tmp_path / "rs_consumer"), "gpu", 300)
