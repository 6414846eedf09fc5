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

    hsa = ctypes.CDLL("libhsa-runtime64.so.1")
    CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p)
    gpus = []

    def on_agent(agent, _data):
        kind = ctypes.c_uint32(0)
        hsa.hsa_agent_get_info(ctypes.c_uint64(agent), 17, ctypes.byref(kind))  # HSA_AGENT_INFO_DEVICE
        if kind.value == 1:  # HSA_DEVICE_TYPE_GPU
            gpus.append(agent)
        return 0

    cb = CB(on_agent)
    hsa.hsa_iterate_agents(cb, None)

    class Pair(ctypes.Structure):
        _fields_ = [("attribute", ctypes.c_uint64), ("value", ctypes.c_uint64)]

    hsa.hsa_amd_svm_attributes_get.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(Pair), ctypes.c_size_t]

    def svm(addr):
        """KFD's SVM view of one page: (status, global flag, GPU access, preferred location)."""
        ps = (Pair * 3)((0, 0), (0x203, gpus[0] if gpus else 0), (4, 0))
        rc = hsa.hsa_amd_svm_attributes_get(ctypes.c_void_p(addr), 4096, ps, 3)
        acc = {0x200: "accessible", 0x201: "in-place", 0x202: "no-access"}.get(ps[1].attribute, hex(ps[1].attribute))
        return rc, ps[0].value, acc, ps[2].value

    def show(label, addr):
        print(f"{label:<48} rocr type/base/size + hip type: {hip_ptr.page_state(addr)}  svm: {svm(addr)}",
              flush=True)

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
    # registered, unregistered, freed, the range handed out again
    import mmap as _mm
    m = _mm.mmap(-1, 16 * 4096)
    mb = np.frombuffer(m, dtype=np.uint8)
    mbase = mb.ctypes.data
    show("fresh mapping, never registered", mbase + 4096)
    rs.host_register(mbase, 8 * 4096)
    show("  registered", mbase + 4096)
    rs.host_unregister(mbase)
    show("  unregistered (still mapped)", mbase + 4096)
    del mb
    m.close()
    c = ctypes.CDLL(None)
    c.mmap.restype = ctypes.c_void_p
    c.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
    again = c.mmap(ctypes.c_void_p(mbase), 16 * 4096, 3, 0x22 | 0x10, -1, 0)  # MAP_FIXED at the same address
    show(f"  unmapped, mapped again at the same address ({again == mbase})", mbase + 4096)
    x = np.full(2 << 20, 7, np.uint8)
    show("pageable 2 MiB array before any copy", x.ctypes.data + 8192)
    tx = torch.from_numpy(x).cuda()
    torch.cuda.synchronize()
    show("  after a pageable H2D copy of it", x.ctypes.data + 8192)
    y = tx.cpu()
    show("  after a pageable D2H copy into a new tensor (dst)", y.data_ptr() + 8192)
    t = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
    show("device memory (torch)", t.data_ptr() + 4096)
    p = torch.empty(1 << 20, dtype=torch.uint8).pin_memory()
    show("torch pinned host memory", p.data_ptr() + 4096)


if __name__ == "__main__":
    main()
