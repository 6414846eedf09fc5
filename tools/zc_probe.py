#!/usr/bin/env python3
"""Zero-copy probe: the encode / multi-pattern reconst kernels run directly on
pinned host memory (the GPU reads and writes it over PCIe), versus the
3-stream DMA pipeline (rs_encode_host_batch).  10+4, several vector sizes.
Writes gpurun_out/zc_probe.json."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402
from reedsolomon_amd._lib import RSLayout  # noqa: E402

GiB = 2 ** 30


def device_pointer(host_ptr: int) -> int:
    """hipHostGetDevicePointer for pinned host memory (the documented way to
    get the address a kernel may use; never hand a kernel a raw host pointer)."""
    hip = ctypes.CDLL("libamdhip64.so.7")  # torch's bundled runtime (same soname, already loaded)
    d = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(host_ptr), 0)
    assert rc == 0 and d.value, rc
    return d.value


def main():
    k, m = 10, 4
    L = rs.lib()
    r = rs.New(k, m, device=0)
    out = {}
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    for vec, S in ((8 << 10, 8192), (64 << 10, 1024), (1 << 20, 64)):
        host = torch.empty((S, k + m, vec), dtype=torch.uint8, pin_memory=True)
        host.random_(0, 256)
        base = device_pointer(host.data_ptr())
        ss, vs = (k + m) * vec, vec
        # device-resident reference parity
        ref = host.cuda()
        r.encode_batch(ref)
        torch.cuda.synchronize()

        def zc_encode():
            rc = L.rs_encode_batch(r._h, ctypes.c_void_p(base), ss, vs, S, vec, sp)
            assert rc == 0, rc

        zc_encode()
        torch.cuda.synchronize()
        assert torch.equal(host[:, k:].cuda(), ref[:, k:]), "zero-copy encode mismatch"
        for _ in range(3):
            zc_encode()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            zc_encode()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        key = f"encode {vec >> 10}KiB x{S}"
        out[key + " zero-copy"] = round(S * (k + m) * vec / t / GiB, 2)
        t0 = time.perf_counter()
        for _ in range(reps):
            r.encode_host_batch(host, 4, 3)
        t = (time.perf_counter() - t0) / reps
        out[key + " DMA pipeline"] = round(S * (k + m) * vec / t / GiB, 2)

        # multi-pattern reconst straight on host memory (16 patterns)
        rng = np.random.default_rng(5)
        pats = [sum(1 << int(v) for v in rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False))
                for _ in range(16)]
        masks = np.array([pats[i % 16] for i in range(S)], dtype=np.uint64)
        nrec = sum(bin(int(x)).count("1") for x in masks)
        lay = RSLayout(base, ss, vs, base + k * vec, ss, vs)
        mp = masks.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))
        for s in range(S):  # garbage in the lost vectors
            for v in range(k + m):
                if int(masks[s]) >> v & 1:
                    host[s, v].fill_(0x5C)
        rc = L.rs_reconst_batch_multi(r._h, ctypes.byref(lay), S, vec, mp, sp)
        assert rc == 0, rc
        torch.cuda.synchronize()
        assert torch.equal(host.cuda(), ref), "zero-copy multi-pattern reconst mismatch"
        t0 = time.perf_counter()
        for _ in range(reps):
            L.rs_reconst_batch_multi(r._h, ctypes.byref(lay), S, vec, mp, sp)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        out[f"reconst_multi {vec >> 10}KiB x{S} zero-copy"] = round((S * k + nrec) * vec / t / GiB, 2)
        print({kk: vv for kk, vv in out.items() if f"{vec >> 10}KiB" in kk}, flush=True)
        del host, ref
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/zc_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
