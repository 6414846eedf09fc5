#!/usr/bin/env python3
"""Host facts that decide how often the kernel invalidates CPU mappings of a
process's memory behind the GPU's back (each invalidation of an SVM range
the GPU has mapped in place makes KFD evict and restore the process's queues
when XNACK is off): NUMA balancing, transparent huge pages / khugepaged,
the amdgpu retry (XNACK) setting, and the global NUMA-hinting / THP-collapse
counters of /proc/vmstat around a loop of pageable torch copies of fresh
arrays (every result checked).  Reads files only; no settings are changed.

Usage: python tools/host_vm_facts.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError as e:
        return f"(unreadable: {e.__class__.__name__})"


def vmstat():
    out = {}
    for line in read("/proc/vmstat").splitlines():
        k, _, v = line.partition(" ")
        if k.startswith(("numa_", "thp_", "pgmigrate", "compact_", "pgdemote")) and v.isdigit():
            out[k] = int(v)
    return out


def main():
    print("kernel", os.uname().release)
    for p in ("/proc/sys/kernel/numa_balancing", "/sys/kernel/mm/transparent_hugepage/enabled",
              "/sys/kernel/mm/transparent_hugepage/defrag", "/sys/kernel/mm/transparent_hugepage/khugepaged/defrag",
              "/sys/kernel/mm/transparent_hugepage/khugepaged/scan_sleep_millisecs",
              "/sys/module/amdgpu/parameters/noretry", "/sys/module/amdgpu/parameters/svm_default_granularity",
              "/sys/module/amdgpu/parameters/mtype_local", "/proc/sys/vm/zone_reclaim_mode"):
        print(f"{p}: {read(p)}")
    print("HSA_XNACK", os.environ.get("HSA_XNACK"), "HSA_ENABLE_IPC_MODE_LEGACY",
          os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY"))
    import numpy as np
    import torch

    torch.cuda.init()
    v0, t0 = vmstat(), time.time()
    for i in range(300):
        x = np.full(int(4 << 20) + 4096 * (i % 7), i & 255, np.uint8)
        t = torch.from_numpy(x).cuda()
        y = t.cpu().numpy()
        assert y[0] == (i & 255) and y[-1] == (i & 255)
        del x, t, y
    torch.cuda.synchronize()
    v1 = vmstat()
    print(f"300 pageable H2D + D2H copies of fresh 4 MiB arrays in {time.time() - t0:.2f} s; /proc/vmstat deltas "
          "(whole machine):")
    for k in sorted(v1):
        d = v1[k] - v0.get(k, 0)
        if d:
            print(f"  {k} +{d}")


if __name__ == "__main__":
    main()
