#!/usr/bin/env python3
"""Does the HIP runtime still treat a host range as pinned / device-mapped
after rs_host_unregister + free, when a new allocation reuses the address?
(No kernel is launched and no copy is made: pointer queries only.)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402


def query(L, addr, nbytes):
    dp = ctypes.c_void_p()
    rc = L.rs_host_device_pointer(ctypes.c_void_p(addr), ctypes.c_size_t(nbytes), ctypes.byref(dp))
    return rc, dp.value


def main():
    torch.cuda.init()
    L = rs.lib()
    r = rs.New(10, 4)
    for size in (1 << 20, 16 << 20, 60 << 10):
        arena = np.zeros(size, np.uint8)
        a0 = arena.ctypes.data
        print(f"size {size}: arena at {a0:#x}, before register: {query(L, a0, size)}", flush=True)
        assert L.rs_host_register(ctypes.c_void_p(a0), ctypes.c_size_t(size)) == 0
        print(f"  registered: {query(L, a0, size)}", flush=True)
        v = [arena[i * 4096:(i + 1) * 4096] for i in range(14)]
        r.Encode(v)  # direct zero-copy host call over the registered range (synchronous)
        assert L.rs_host_unregister(ctypes.c_void_p(a0)) == 0
        print(f"  unregistered, still allocated: {query(L, a0, size)}", flush=True)
        del v, arena
        again = np.zeros(size, np.uint8)
        a1 = again.ctypes.data
        print(f"  freed; new array at {a1:#x} (same address: {a1 == a0}): {query(L, a1, size)}", flush=True)
        del again


if __name__ == "__main__":
    main()
