#!/usr/bin/env python3
"""HBM calibration on the GPU box: plain copy / read / write and the 10+4
encode access pattern (XOR instead of GF math), GB/s from HIP events.
Measurement tool only."""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_build", "libhbmprobe.so")


def build():
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(os.path.join(HERE, "hbm_probe.hip")):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.run(["hipcc", "-O3", "-shared", "-fPIC", "--offload-arch=gfx950",
                        os.path.join(HERE, "hbm_probe.hip"), "-o", SO], check=True)
    return SO


def main():
    build()
    import torch

    L = ctypes.CDLL(SO)
    for f in ("probe_copy", "probe_read", "probe_write", "probe_pattern"):
        getattr(L, f).restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    GB = 3.5 * 2 ** 30
    a = torch.randint(0, 256, (int(GB),), dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    res = {}

    def timeit(name, fn, nbytes, iters=30, warm=5):
        for _ in range(warm):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record(st)
        for _ in range(iters):
            fn()
        e.record(st)
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / iters / 1e3
        res[name] = round(nbytes / t / 1e9, 1)
        print(f"{name:32s} {res[name]:8.1f} GB/s  ({t*1e3:.3f} ms)", flush=True)

    n = a.numel()
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    basic = os.environ.get("PROBE_BASIC", "1") != "0"
    if basic:
        basic_probes(L, a, b, n, vp, sp, timeit)
    pattern_probes(L, a, n, vp, sp, timeit)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/hbm_probe.json", "w"), indent=1)


def basic_probes(L, a, b, n, vp, sp, timeit):
    timeit("copy (read+write)", lambda: L.probe_copy(vp(a), vp(b), ctypes.c_uint64(n // 2), 0, sp), n // 2 * 2)
    timeit("copy nt-store", lambda: L.probe_copy(vp(a), vp(b), ctypes.c_uint64(n // 2), 1, sp), n // 2 * 2)
    timeit("torch copy_", lambda: b.copy_(a), 2 * n)
    for per in (1, 4, 16):
        timeit(f"read-only per={per}", lambda: L.probe_read(vp(a), vp(b), ctypes.c_uint64(n), per, sp), n)
    timeit("write-only", lambda: L.probe_write(vp(b), ctypes.c_uint64(n), 0, sp), n)
    timeit("write-only nt", lambda: L.probe_write(vp(b), ctypes.c_uint64(n), 1, sp), n)


def pattern_probes(L, a, n, vp, sp, timeit):
    if os.environ.get("PROBE_GRAN", "0") == "1":
        # 10+4 split pattern: bytes per vector per workgroup = lanes x bytes/lane
        import torch
        vec, S = 1 << 20, 240
        b = torch.empty(S * 4 * vec, dtype=torch.uint8, device="cuda")
        assert S * 10 * vec <= n, "probe case out of bounds"
        L.probe_buf_g.restype = ctypes.c_int
        for _ in range(3):
            for kind, name in ((0, "64x16B"), (1, "128x16B"), (2, "256x16B"), (3, "512x16B"), (4, "1024x16B"),
                               (5, "256x8B"), (6, "128x8B"), (7, "512x8B")):
                timeit(f"buffer nt 10+4 pattern {name}/vector/WG",
                       lambda: L.probe_buf_g(kind, vp(a), vp(b), ctypes.c_uint64(vec), S, sp), S * 14 * vec)
        return
    if os.environ.get("PROBE_UPL", "0") == "1":
        # 10+4 split pattern: 4/8/16 KiB per vector per workgroup, natural vs XCD-aware order
        import torch
        vec, S = 1 << 20, 240
        b = torch.empty(S * 4 * vec, dtype=torch.uint8, device="cuda")
        assert S * 10 * vec <= n, "probe case out of bounds"
        for _ in range(2):
            for kind, name in ((0, "4KiB"), (1, "8KiB"), (2, "16KiB"), (4, "4KiB xcd"), (5, "8KiB xcd"),
                               (6, "16KiB xcd")):
                timeit(f"buffer nt 10+4 pattern {name}/vector/WG",
                       lambda: L.probe_buf_u(kind, vp(a), vp(b), ctypes.c_uint64(vec), S, sp), S * 14 * vec)
        return
    if os.environ.get("PROBE_RECON", "0") == "1":
        # Reconst ceilings: 10 reads + m writes per stripe, buffer nt, split regions.
        import torch
        b = torch.empty(n // 2, dtype=torch.uint8, device="cuda")
        for vec, S in ((1 << 20, 240), (8 << 10, 30720)):
            for m, kind in ((1, 4), (2, 5), (3, 6), (4, 3)):
                assert S * 10 * vec <= n and S * m * vec <= b.numel(), "probe case out of bounds"
                timeit(f"buffer nt 10+{m} pattern vec={vec >> 10}KiB",
                       lambda: L.probe_buf(kind, vp(a), vp(b), ctypes.c_uint64(0), ctypes.c_uint64(vec), S, sp),
                       S * (10 + m) * vec)
            assert S * 14 * vec <= n, "probe case out of bounds"
            timeit(f"buffer nt 10+1 in place (11-vector stripes) vec={vec >> 10}KiB",
                   lambda: L.probe_buf(7, vp(a), vp(b), ctypes.c_uint64(0), ctypes.c_uint64(vec), S, sp),
                   S * 11 * vec)
            timeit(f"buffer nt 10+4 in place (lost 0-3 of 14) vec={vec >> 10}KiB",
                   lambda: L.probe_buf(8, vp(a), vp(b), ctypes.c_uint64(0), ctypes.c_uint64(vec), S, sp),
                   S * 14 * vec)
        return
    if os.environ.get("PROBE_INPLACE", "0") == "1":
        # in-place Reconst ceilings (interleaved [S][d+p][1 MiB]), XOR for the math:
        # plain, stores deferred behind a far chunk's loads, or behind the next chunk's
        L.probe_inplace.restype = ctypes.c_int
        vec = 1 << 20
        for shape, nv, kr, kw, name in ((0, 18, 10, 8, "10+8 lost 0-7"), (1, 18, 10, 5, "10+8 lost 5 data"),
                                        (2, 14, 10, 4, "10+4 lost 0-3"), (3, 18, 10, 8, "10+8 encode in place")):
            S = min(256, int(n // (nv * vec)) // 2 * 2)
            for _ in range(2):
                for kind, kname in ((0, "plain"), (1, "defer far"), (2, "defer next")):
                    timeit(f"in place {name} {kname}",
                           lambda: L.probe_inplace(kind, shape, vp(a), ctypes.c_uint64(vec), S, sp),
                           S * (kr + kw) * vec, iters=20)
        return
    if os.environ.get("PROBE_GEO", "0") == "1":
        # the assembly kernels' 2 KiB / 64-lane geometry against the 1 KiB /
        # 128-lane one, in place and with the lost vectors written elsewhere
        L.probe_geo.restype = ctypes.c_int
        vec = 1 << 20
        geos = ((0, "1KiB/128"), (1, "2KiB/64 x4"), (2, "2KiB/256"), (3, "2KiB/128 x2"), (4, "512B x 4 stripes/64"),
                (5, "8KiB/256 x4 wave-interleaved"), (6, "4KiB/128 x4 wave-interleaved"),
                (7, "2KiB/64 x2 dwordx4 1KiB apart"), (8, "2KiB/64 x2 dwordx4 contiguous"))
        if os.environ.get("PROBE_GEOS"):
            keep = {int(x) for x in os.environ["PROBE_GEOS"].split(",")}
            geos = tuple(g for g in geos if g[0] in keep)
        for shape, nv, kr, kw, name in ((1, 18, 10, 5, "10+8 lost 5 data"), (0, 18, 10, 8, "10+8 lost 0-7"),
                                        (2, 14, 10, 4, "10+4 lost 0-3")):
            S = min(256, int(n // (nv * vec))) // 4 * 4
            import torch
            b = torch.empty(S * kw * vec, dtype=torch.uint8, device="cuda")
            for _ in range(2):
                for split in (0, 16):
                    for geo, gname in geos:
                        timeit(f"geo {name} {gname} {'split' if split else 'in place'}",
                               lambda: L.probe_geo(geo + split, shape, vp(a), vp(b), ctypes.c_uint64(vec), S, sp),
                               S * (kr + kw) * vec, iters=20)
        return
    if os.environ.get("PROBE_BUF", "0") == "1":
        import torch
        half = (n // 2) // 4096 * 4096
        b = torch.empty(half, dtype=torch.uint8, device="cuda")
        assert half <= n and half <= b.numel()
        for _ in range(2):
            timeit("buffer nt copy (read+write)", lambda: L.probe_buf(0, vp(a), vp(b), ctypes.c_uint64(half),
                                                                       ctypes.c_uint64(0), 0, sp), 2 * half)
            timeit("buffer nt read-only", lambda: L.probe_buf(1, vp(a), vp(b), ctypes.c_uint64(n // 4096 * 4096),
                                                               ctypes.c_uint64(0), 0, sp), n // 4096 * 4096)
            timeit("buffer nt write-only", lambda: L.probe_buf(2, vp(a), vp(b), ctypes.c_uint64(half),
                                                                ctypes.c_uint64(0), 0, sp), half)
            vec, S = 1 << 20, 240
            assert S * 10 * vec <= n and S * 4 * vec <= b.numel()
            timeit("buffer nt 10+4 pattern, split layout", lambda: L.probe_buf(3, vp(a), vp(b), ctypes.c_uint64(0),
                                                                                ctypes.c_uint64(vec), S, sp),
                   S * 14 * vec)
        return
    if os.environ.get("PROBE_SEP", "0") == "1":
        vec = 1 << 20
        S = 240
        import torch
        b = torch.empty(S * 4 * vec + (64 << 20), dtype=torch.uint8, device="cuda")
        for poff in (0, 4096, 1 << 20, 3 << 19, 5 << 18):
            assert poff + S * 4 * vec <= b.numel() and S * 10 * vec <= n
            timeit(f"10+4 separate parity buffer, offset {poff >> 10}K",
                   lambda: L.probe_pattern_sep(vp(a), ctypes.c_void_p(b.data_ptr() + poff), ctypes.c_uint64(vec),
                                               ctypes.c_uint64(10 * vec), ctypes.c_uint64(4 * vec), S, sp),
                   S * 14 * vec, iters=20)
        for dss_pad in (0,):
            need = S * (10 * vec + dss_pad) + S * 4 * vec
            assert need <= n, "probe case out of bounds"
            timeit(f"10+4 same buffer, parity after all data, dss pad {dss_pad >> 10}K",
                   lambda: L.probe_pattern_sep(vp(a), ctypes.c_void_p(a.data_ptr() + S * (10 * vec + dss_pad)),
                                               ctypes.c_uint64(vec), ctypes.c_uint64(10 * vec + dss_pad),
                                               ctypes.c_uint64(4 * vec), S, sp),
                   S * 14 * vec, iters=20)
        assert S * 14 * vec <= n
        timeit("10+4 interleaved layout (reference)",
               lambda: L.probe_pattern_sep(vp(a), ctypes.c_void_p(a.data_ptr() + 10 * vec), ctypes.c_uint64(vec),
                                           ctypes.c_uint64(14 * vec), ctypes.c_uint64(14 * vec), S, sp),
               S * 14 * vec, iters=20)
        return
    if os.environ.get("PROBE_MAP", "0") == "1":
        vec = 1 << 20
        S = 240
        for mapping in (0, 2, 3):
            for pad, sspad in ((0, 0), (0, 1 << 20), (512 << 10, 0), (1 << 20, 0), (128 << 10, 0), (8192, 0),
                               (0, 4096), (2048, 2048), (32 << 10, 0), (192 << 10, 0)):
                pitch = vec + pad
                sstride = 14 * pitch + sspad
                if (S - 1) * sstride + 13 * pitch + vec > n:  # bounds
                    continue
                timeit(f"10+4 map={mapping} pitch=1M+{pad >> 10}K sspad={sspad >> 10}K",
                       lambda: L.probe_pattern(vp(a), ctypes.c_uint64(vec), ctypes.c_uint64(pitch),
                                               ctypes.c_uint64(sstride), S, 1, mapping, sp),
                       S * 14 * vec, iters=20)
        return
    if os.environ.get("PROBE_VEC", "0") == "1":
        half = (n // 2) // 4096 * 4096
        timeit("flat copy, same allocation halves",
               lambda: L.probe_copy(vp(a), ctypes.c_void_p(a.data_ptr() + half), ctypes.c_uint64(half), 0, sp),
               2 * half)
        for k, m in ((1, 1), (10, 4), (10, 0)):
            for vec in (64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20):
                S = int(n // ((k + m) * vec))
                if S < 1:
                    continue
                timeit(f"pattern k={k} m={m} vec={vec >> 10}KiB S={S}",
                       lambda: L.probe_pattern_km(vp(a), ctypes.c_uint64(vec), ctypes.c_uint64(vec),
                                                  ctypes.c_uint64((k + m) * vec), S, k, m, sp),
                       S * (k + m) * vec, iters=20)
        return
    if os.environ.get("PROBE_KMG", "0") == "1":
        # round 4: the 16+4 / 12+4 / 20+4 encode patterns against 10+4, split and interleaved,
        # at the library's two geometries (128 x 8 B, 256 x 16 B) and 256 x 8 B; and the
        # Replace rn=1 / Update read-modify-write pattern at 8 KiB (10+4 stripes)
        import torch
        L.probe_km_g.restype = ctypes.c_int
        L.probe_rmw.restype = ctypes.c_int
        vec = 1 << 20
        b = torch.empty(256 * 4 * vec, dtype=torch.uint8, device="cuda")
        for _ in range(2):
            for k, m in ((10, 4), (12, 4), (16, 4), (20, 4)):
                S = min(256, int(n // ((k + m) * vec)))
                for kind, gname in ((0, "128x8B"), (1, "256x16B"), (2, "256x8B")):
                    timeit(f"{k}+{m} split {gname}",
                           lambda: L.probe_km_g(kind, k, m, vp(a), vp(b), ctypes.c_uint64(vec),
                                                ctypes.c_uint64(k * vec), ctypes.c_uint64(m * vec), S, sp),
                           S * (k + m) * vec, iters=20)
                    timeit(f"{k}+{m} interleaved {gname}",
                           lambda: L.probe_km_g(kind, k, m, vp(a), ctypes.c_void_p(a.data_ptr() + k * vec),
                                                ctypes.c_uint64(vec), ctypes.c_uint64((k + m) * vec),
                                                ctypes.c_uint64((k + m) * vec), S, sp),
                           S * (k + m) * vec, iters=20)
            v8, S8 = 8192, 32768
            assert S8 * 14 * v8 <= n
            for k, name in ((1, "Replace rn=1"), (2, "Update")):
                for kind, gname in ((0, "128x8B"), (1, "256x16B")):
                    timeit(f"{name} 10+4 8KiB read-modify-write {gname}",
                           lambda: L.probe_rmw(kind, k, vp(a), ctypes.c_uint64(v8), ctypes.c_uint64(14 * v8),
                                               ctypes.c_uint64(0), ctypes.c_uint64(10 * v8), S8, sp),
                           S8 * (k + 8) * v8, iters=20)
        return
    if os.environ.get("PROBE_KM", "0") == "1":
        vec = 1 << 20
        for k, m in ((1, 1), (2, 2), (4, 4), (7, 7), (10, 10), (4, 0), (10, 0), (14, 0), (10, 2), (10, 4), (12, 4), (6, 3)):
            S = min(256, int(n // ((k + m) * vec)))
            timeit(f"pattern k={k} m={m}",
                   lambda: L.probe_pattern_km(vp(a), ctypes.c_uint64(vec), ctypes.c_uint64(vec),
                                              ctypes.c_uint64((k + m) * vec), S, k, m, sp),
                   S * (k + m) * vec, iters=20)
        return
    S, vec = 240, 1 << 20
    for pad in (0, 256, 4096, 65536, 3 * 4096 + 256):
        for sspad in (0, 8192 + 512):
            pitch = vec + pad
            sstride = 14 * pitch + sspad
            for mapping in (0, 1):
                for upl in (1, 2):
                    if S * sstride > n:  # bounds: every stripe must fit the buffer
                        continue
                    timeit(f"pattern pad={pad} sspad={sspad} map={mapping} upl={upl}",
                           lambda: L.probe_pattern(vp(a), ctypes.c_uint64(vec), ctypes.c_uint64(pitch),
                                                   ctypes.c_uint64(sstride), S, upl, mapping, sp),
                           S * 14 * vec, iters=20)


if __name__ == "__main__":
    sys.exit(main())
