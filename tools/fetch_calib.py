#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration workload: one read pass and one write
pass over a known 2 GiB (>> the 256 MiB Infinity Cache) with 16- and 8-byte
lanes (kernels kc_read16 / kc_read8 / kc_write16 / kc_write8 in
tools/hbm_probe.hip).  Run under `rocprofv3 --pmc FETCH_SIZE` / `WRITE_SIZE`
(tools/gpu_profile.sh); tools/summarize_profile.py turns the counts into
bytes-per-count factors for each access width.  Measurement tool only."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import hbm_probe  # noqa: E402

BYTES = 2 << 30


def main():
    import torch

    torch.cuda.init()  # HIP up before the probe library registers its kernels
    a = torch.empty(BYTES, dtype=torch.uint8, device="cuda")
    L = ctypes.CDLL(hbm_probe.build())
    L.probe_calib.restype = ctypes.c_int
    a.fill_(1)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for kind in (0, 1, 2, 3):
        for _ in range(3):
            assert L.probe_calib(kind, ctypes.c_void_p(a.data_ptr()), ctypes.c_uint64(BYTES), st) == 0
        torch.cuda.synchronize()
    print(f"calibration passes done: {BYTES} B per launch", flush=True)


if __name__ == "__main__":
    main()
