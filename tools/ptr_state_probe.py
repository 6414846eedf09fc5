#!/usr/bin/env python3
"""What do hipPointerGetAttributes and hsa_amd_pointer_info report for host
memory in each state (pageable, rs_host_register'ed, hipHostRegister'ed
directly, unregistered again, hipHostMalloc'ed, a pool block)?  Calibrates
tests/hip_ptr.py: a page that both layers report the same way whether it is
registered or not would make the tests' "no longer registered" assertions
vacuous.  Host-side queries only.

Usage: python tools/ptr_state_probe.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch

    import hip_ptr
    import reedsolomon_amd as rs

    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]

    def show(label, addr):
        print(f"{label:<48} rocr type/base/size + hip type: {hip_ptr.page_state(addr)}", flush=True)

    a = np.zeros(16 * 4096, np.uint8)
    base = a.ctypes.data + (-a.ctypes.data) % 4096
    pg = base + 4 * 4096
    show("pageable heap page", pg)
    rs.host_register(base, 8 * 4096)
    show("rs_host_register'ed (page 4 of 8)", pg)
    show("  its first page", base)
    rs.host_unregister(base)
    show("after rs_host_unregister", pg)
    rc = hip.hipHostRegister(ctypes.c_void_p(base), 8 * 4096, 3)
    show(f"hipHostRegister'ed directly (rc {rc})", pg)
    rc = hip.hipHostUnregister(ctypes.c_void_p(base))
    show(f"after hipHostUnregister (rc {rc})", pg)
    h = ctypes.c_void_p()
    rc = hip.hipHostMalloc(ctypes.byref(h), 1 << 16, 0)
    show(f"hipHostMalloc'ed (rc {rc})", h.value + 4096)
    blk = rs.host_alloc(1 << 16)
    show("rs_host_alloc pool block", blk.ctypes.data + 4096)
    t = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    show("device memory (torch)", t.data_ptr() + 4096)
    p = torch.empty(1 << 20, dtype=torch.uint8).pin_memory()
    show("torch pinned host memory", p.data_ptr() + 4096)


if __name__ == "__main__":
    main()
