#!/usr/bin/env python3
"""Per-operation throughput on one MI355X (BASELINE.json configs 2-5) plus
the host-resident end-to-end rate.  Writes gpurun_out/ops_bench.json.

Formulas follow the reference's benchmarks (README.md:129-161,
rs_test.go:450,489,556,598):
  Encode   (k+m)*vec          Reconst  (k+lost)*vec
  Update   (2+2m)*vec         Replace  (rn+2m)*vec
Device-resident numbers time HIP events around back-to-back launches on one
stream; end-to-end numbers time host wall clock around the pinned pipeline.

    python tools/ops_bench.py                    # every section
    python tools/ops_bench.py --only wide,api    # some sections

Sections: encode, shapes, split, rec8, rec4, multi, upd, wide, first, host, api.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import reedsolomon_amd as rs  # noqa: E402

GiB = 2 ** 30
out = {}


def dev_time(fn, iters=50, warm=50):
    st = torch.cuda.current_stream()
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(st)
    for _ in range(iters):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters / 1e3


def rec(name, nbytes, t, **kw):
    out[name] = dict(GiBps=round(nbytes / t / GiB, 2), us_per_call=round(t * 1e6, 2), **kw)
    print(f"{name:44s} {nbytes / t / GiB:10.2f} GiB/s  {t * 1e6:10.2f} us/call", flush=True)


SECTIONS = ["encode", "shapes", "split", "rec8", "rec4", "multi", "upd", "wide", "first", "first_small", "host", "api"]


def want(name):
    only = None
    if "--only" in sys.argv:
        only = sys.argv[sys.argv.index("--only") + 1].split(",")
    return only is None or name in only


def wide(g):
    """> 8 output rows: the single-pass wide kernels (and the run-time
    compiled networks where they apply), ~3.5 GiB of stripes per launch."""
    L = rs.lib()
    for k, m, vec in ((16, 16, 1 << 20), (32, 32, 1 << 20), (64, 64, 1 << 20), (128, 128, 1 << 20), (200, 56, 1 << 20)):
        S = max(1, (3584 << 20) // ((k + m) * vec))
        r = rs.New(k, m)
        data = torch.randint(0, 256, (S, k, vec), dtype=torch.uint8, device="cuda", generator=g)
        par = torch.empty((S, m, vec), dtype=torch.uint8, device="cuda")
        for jit in (0, 2):
            L.rs_tune(b"jit", jit)
            t = dev_time(lambda: r.encode_batch_split(data, par), iters=10, warm=5)
            rec(f"encode {k}+{m} {vec >> 10}KiB x{S} split, jit={jit} (device)", S * (k + m) * vec, t)
        del data, par
    for k, m, vec, lost in ((16, 16, 1 << 20, list(range(16))), (20, 12, 1 << 20, list(range(12))),
                            (48, 16, 256 << 10, list(range(16))), (100, 28, 256 << 10, list(range(0, 40, 2))),
                            (100, 28, 256 << 10, list(range(0, 84, 3)))):
        S = max(1, (3584 << 20) // ((k + m) * vec))
        r = rs.New(k, m)
        data = torch.randint(0, 256, (S, k, vec), dtype=torch.uint8, device="cuda", generator=g)
        par = torch.empty((S, m, vec), dtype=torch.uint8, device="cuda")
        r.encode_batch_split(data, par)
        for jit, sp in ((0, 1), (0, 0), (2, 1)):
            L.rs_tune(b"jit", jit)
            L.rs_tune(b"wide_single_pass", sp)
            t = dev_time(lambda: r.reconst_batch_split(data, par, [], lost), iters=10, warm=5)
            rec(f"reconst {k}+{m} {vec >> 10}KiB lost={len(lost)} x{S} split, jit={jit} single_pass={sp}",
                S * (k + len(lost)) * vec, t)
        del data, par
    L.rs_tune(b"jit", 2)
    L.rs_tune(b"wide_single_pass", 1)


def first_sight(g):
    """A rebuild storm: every launch a different erasure pattern, seen once
    (its decode matrix new to the process), launched back to back with the
    library's default policy (jit=1: the machine-code backend builds a
    pattern's kernel on the launching thread when the launch is large enough
    to pay for it, jit.cpp est_compile_us) - timed on the host clock from the
    first launch to the last one's completion, so every compile is inside the
    window; against the same launches with one pattern already compiled
    (jit=2, repeated) and with no run-time kernels at all (jit=0).  The
    stripes are rebuilt in place from intact survivors, so they must come
    out unchanged: checked after every run."""
    import numpy as np

    L = rs.lib()
    rng = np.random.default_rng(11)
    for k, m, vec, nlost in ((16, 16, 1 << 20, 16), (100, 28, 256 << 10, 20), (100, 28, 256 << 10, 28)):
        S = max(1, (3584 << 20) // ((k + m) * vec))
        r = rs.New(k, m)
        data = torch.randint(0, 256, (S, k, vec), dtype=torch.uint8, device="cuda", generator=g)
        par = torch.empty((S, m, vec), dtype=torch.uint8, device="cuda")
        r.encode_batch_split(data, par)
        ref_d, ref_p = data.clone(), par.clone()
        nbytes = S * (k + nlost) * vec
        n = 20
        pats = [sorted(int(x) for x in rng.choice(k + m, nlost, replace=False)) for _ in range(n)]
        L.rs_tune(b"jit", 2)
        t = dev_time(lambda: r.reconst_batch_split(data, par, [], pats[0]), iters=10, warm=3)
        rec(f"reconst {k}+{m} {vec >> 10}KiB lost={nlost} x{S}, one pattern compiled (jit=2)", nbytes, t)
        for jit, label in ((0, "no run-time kernels (jit=0)"), (1, "default policy (jit=1)")):
            L.rs_tune(b"jit", jit)
            fresh = [sorted(int(x) for x in rng.choice(k + m, nlost, replace=False)) for _ in range(n)]
            r.reconst_batch_split(data, par, [], fresh[0])  # (clocks up; this pattern is not timed again)
            st0 = rs.jit_stats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for pt in fresh[1:]:
                r.reconst_batch_split(data, par, [], pt)
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) / (n - 1)
            st = rs.jit_stats()
            rec(f"reconst {k}+{m} {vec >> 10}KiB lost={nlost} x{S}, {n - 1} new patterns, {label}", nbytes, t,
                compiled=st["compiled"] - st0["compiled"], compiled_launches=st["launches"] - st0["launches"],
                compile_ms=round(st["compile_ms"] - st0["compile_ms"], 2))
            assert torch.equal(data, ref_d) and torch.equal(par, ref_p), "first-sight reconst changed the stripes"
        del data, par, ref_d, ref_p
        torch.cuda.empty_cache()
    L.rs_tune(b"jit", 2)


def first_small(g):
    """Small synchronous Reconst calls"""
    import numpy as np

    L = rs.lib()
    rng = np.random.default_rng(12)
    # Small synchronous Reconst calls (16 stripes of 10+4 @ 8 KiB): a new
    # pattern's first call (its decode matrix, perm tables and their upload)
    # against a repeat of a pattern already seen; wall time per call with the
    # stream synchronised, median of 100 (default policy: too small to compile)
    L.rs_tune(b"jit", 1)
    k, m, vec, S = 10, 4, 8192, 16
    r = rs.New(k, m)
    buf = torch.randint(0, 256, (S, k + m, vec), dtype=torch.uint8, device="cuda", generator=g)
    r.encode_batch(buf)
    ref = buf.clone()
    seen = set()
    fresh = []
    while len(fresh) < 303:
        pt = tuple(sorted(int(x) for x in rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False)))
        if pt not in seen:
            seen.add(pt)
            fresh.append(list(pt))
    def per_call(pats):
        ts = []
        for pt in pats:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.reconst_batch(buf, [], pt)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[len(ts) // 2]
    r.reconst_batch(buf, [], fresh[0])
    up0, ip0 = r.coef_table_stats()
    t_new = per_call(fresh[1:101])  # default: a new matrix's tables read in place (table_inplace_max)
    up1, ip1 = r.coef_table_stats()
    t_rep = per_call([fresh[1]] * 100)
    L.rs_tune(b"table_inplace_max", 0)  # the same with the upload at first sight (round 5's path)
    t_up = per_call(fresh[101:201])
    L.rs_tune(b"table_inplace_max", 2 << 20)
    # in place from host-writable VRAM (the opt-in table_stage_vram 1: a new handle)
    L.rs_tune(b"table_stage_vram", 1)
    r_main, r = r, rs.New(k, m)
    r.reconst_batch(buf, [], fresh[0])
    t_vram = per_call(fresh[201:301])
    r = r_main
    L.rs_tune(b"table_stage_vram", 0)
    assert torch.equal(buf, ref), "small first-sight reconst changed the stripes"
    print(f"first sights read in place: {ip1 - ip0}, uploads: {up1 - up0}", flush=True)
    for label, t in (("first call of a new pattern", t_new), ("a pattern already seen", t_rep),
                     ("first call of a new pattern, upload at first sight", t_up),
                     ("first call of a new pattern, tables in VRAM (table_stage_vram 1)", t_vram)):
        rec(f"reconst 10+4 8KiB x{S}, synchronous, {label}", S * (k + 2) * vec, t)
    L.rs_tune(b"jit", 2)


def main():
    g = torch.Generator(device="cuda").manual_seed(42)
    # run-time bit-sliced kernels (5-8 output rows) compile on first use here,
    # so the timed calls run them (the library's default compiles in the
    # background and uses the perm-table kernels until the code is ready)
    rs.lib().rs_tune(b"jit", 2)
    if want("wide"):
        wide(g)
    if want("first"):
        first_sight(g)
    if want("first_small"):
        first_small(g)
    if want("encode"):
        # ---- encode, device-resident
        for k, m, vec, S in ((10, 4, 1 << 20, 256), (12, 4, 1 << 20, 256), (10, 4, 8 << 10, 32768), (10, 4, 8 << 10, 1)):
            r = rs.New(k, m)
            buf = torch.randint(0, 256, (S, k + m, vec), dtype=torch.uint8, device="cuda", generator=g)
            t = dev_time(lambda: r.encode_batch(buf))
            rec(f"encode {k}+{m} {vec >> 10}KiB x{S} (device)", S * (k + m) * vec, t)
            del buf
    if want("shapes"):
        # ---- other shapes (runtime-column kernels; 5-8 rows are VALU-bound)
        for k, m in ((8, 4), (6, 3), (16, 4), (10, 6), (10, 8), (12, 8), (16, 8)):
            vec, S = 1 << 20, 256 * 14 // (k + m)
            r = rs.New(k, m)
            buf = torch.randint(0, 256, (S, k + m, vec), dtype=torch.uint8, device="cuda", generator=g)
            t = dev_time(lambda: r.encode_batch(buf))
            rec(f"encode {k}+{m} {vec >> 10}KiB x{S} (device)", S * (k + m) * vec, t)
            del buf
    if want("split"):
        # ---- > 4 outputs on the split layout (data [S][k][vec], parity [S][m][vec],
        # as bench.py): 16+8 Encode (no build-time network: run-time compiled) and
        # 10+8 Reconst of 5 / 8 lost data vectors
        for k, m in ((16, 8), (10, 8)):
            vec, S = 1 << 20, 256 * 14 // (k + m)
            r = rs.New(k, m)
            data = torch.randint(0, 256, (S, k, vec), dtype=torch.uint8, device="cuda", generator=g)
            par = torch.empty((S, m, vec), dtype=torch.uint8, device="cuda")
            t = dev_time(lambda: r.encode_batch_split(data, par))
            rec(f"encode {k}+{m} {vec >> 10}KiB x{S} split (device)", S * (k + m) * vec, t)
            if k == 10:
                for lost in ([0, 2, 4, 6, 8], list(range(8))):
                    t = dev_time(lambda: r.reconst_batch_split(data, par, [], lost))
                    rec(f"reconst {k}+{m} 1MiB lost={len(lost)} data x{S} split", S * (k + len(lost)) * vec, t)
            del data, par
    if want("rec8"):
        # ---- reconst of 5-8 lost at 10+8 @ 1 MiB (run-time matrices, > 4 outputs)
        k, m, vec = 10, 8, 1 << 20
        S = 256 * 14 // (k + m)
        r = rs.New(k, m)
        buf = torch.randint(0, 256, (S, k + m, vec), dtype=torch.uint8, device="cuda", generator=g)
        r.encode_batch(buf)
        for lost in ([0, 2, 4, 6, 8], list(range(8)), [0, 2, 4, 6, 10, 12, 14, 16]):
            t = dev_time(lambda: r.reconst_batch(buf, [], lost))
            rec(f"reconst 10+8 1MiB lost={len(lost)} ({'data' if max(lost) < k else 'data+parity'}) x{S}",
                S * (k + len(lost)) * vec, t)
        del buf
    if want("rec4") or want("multi") or want("upd"):
        # ---- reconst 10+4 @ 8 KiB, 1-4 lost data shards (config 3)
        k, m, vec, S = 10, 4, 8 << 10, 32768
        r = rs.New(k, m)
        buf = torch.randint(0, 256, (S, k + m, vec), dtype=torch.uint8, device="cuda", generator=g)
        r.encode_batch(buf)
        for lost in ([0], [0, 5], [0, 5, 9], [0, 3, 5, 9]):
            t = dev_time(lambda: r.reconst_batch(buf, [], lost))
            rec(f"reconst 10+4 8KiB lost={len(lost)} data x{S}", S * (k + len(lost)) * vec, t)
            t1 = dev_time(lambda: r.reconst_batch(buf[:1], [], lost))
            rec(f"reconst 10+4 8KiB lost={len(lost)} data x1", (k + len(lost)) * vec, t1)
        # ---- multi-pattern reconst: every stripe its own 1-4 erasures (16 distinct patterns)
        import numpy as np

        rng = np.random.default_rng(5)
        pats = []
        for _ in range(16):
            lost = rng.choice(k + m, int(rng.integers(1, m + 1)), replace=False)
            pats.append(sum(1 << int(v) for v in lost))
        masks = np.array([pats[i % 16] for i in range(S)], dtype=np.uint64)
        nrec = sum(bin(int(x)).count("1") for x in masks)
        # full warm-up: the single-stripe calls above leave the GPU idle enough to
        # drop its clocks, and 5 warm-up calls did not bring them back (4,934 GiB/s
        # with warm=5 vs ~5,700 in tools/multi_mix.py on the same box)
        t = dev_time(lambda: r.reconst_batch_multi(buf[:, :k], buf[:, k:], masks))
        rec(f"reconst_multi 10+4 8KiB 16 patterns x{S}", (S * k + nrec) * vec, t)
        # ---- update / replace 10+4 @ 8 KiB (config 5)
        old = buf[:, 3].clone()
        new = torch.randint(0, 256, (S, vec), dtype=torch.uint8, device="cuda", generator=g)
        t = dev_time(lambda: r.update_batch(old, new, 3, buf))
        rec(f"update 10+4 8KiB x{S}", S * (2 + 2 * m) * vec, t)
        for rn in range(1, 7):
            data = torch.randint(0, 256, (S, rn, vec), dtype=torch.uint8, device="cuda", generator=g)
            t = dev_time(lambda: r.replace_batch(data, list(range(rn)), buf))
            rec(f"replace 10+4 8KiB rn={rn} x{S}", S * (rn + 2 * m) * vec, t)
        del buf
        torch.cuda.empty_cache()
    if want("host"):
        # ---- host-resident end-to-end (pinned), 10+4 @ 1 MiB
        k, m, vec, S = 10, 4, 1 << 20, 128
        r = rs.New(k, m)
        host = torch.empty((S, k + m, vec), dtype=torch.uint8, pin_memory=True)
        host.copy_(torch.randint(0, 256, (S, k + m, vec), dtype=torch.uint8, device="cuda", generator=g).cpu())
        L = rs.lib()
        r.encode_host_batch(host)  # warm (zero-copy: pinned memory is device-mapped)
        t0 = time.perf_counter()
        for _ in range(3):
            r.encode_host_batch(host)
        rec(f"encode 10+4 1MiB x{S} host->host pinned, zero-copy", S * (k + m) * vec, (time.perf_counter() - t0) / 3)
        L.rs_tune(b"host_batch_zc", 0)
        for spc, nst in ((2, 3), (4, 3), (8, 3), (8, 4), (16, 3)):
            r.encode_host_batch(host, spc, nst)  # warm
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                r.encode_host_batch(host, spc, nst)
            t = (time.perf_counter() - t0) / reps
            rec(f"encode 10+4 1MiB x{S} host->host pinned, DMA pipeline spc={spc} streams={nst}", S * (k + m) * vec, t)
        L.rs_tune(b"host_batch_zc", 1)
        # pageable (ordinary) host memory: staged through the pinned mirror
        for pv, pS in ((8 << 10, 2048), (64 << 10, 512), (1 << 20, 64)):
            pg = np.random.default_rng(3).integers(0, 256, (pS, k + m, pv), dtype=np.uint8)
            r.encode_host_batch(pg)  # warm
            t0 = time.perf_counter()
            for _ in range(3):
                r.encode_host_batch(pg)
            rec(f"encode 10+4 {pv >> 10}KiB x{pS} host->host pageable (staged)", pS * (k + m) * pv,
                (time.perf_counter() - t0) / 3)
            del pg
        # PCIe reference rates (one direction at a time, then both at once)
        dbuf = torch.empty((S * k * vec,), dtype=torch.uint8, device="cuda")
        hflat = host.view(-1)[: S * k * vec]
        t0 = time.perf_counter()
        dbuf.copy_(hflat, non_blocking=True)
        torch.cuda.synchronize()
        rec("H2D pinned copy (torch)", S * k * vec, time.perf_counter() - t0)
        t0 = time.perf_counter()
        hflat.copy_(dbuf, non_blocking=True)
        torch.cuda.synchronize()
        rec("D2H pinned copy (torch)", S * k * vec, time.perf_counter() - t0)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        half = host.numel() // 2
        ha, hb = host.view(-1)[:half], host.view(-1)[half: 2 * half]
        da, db = torch.empty(half, dtype=torch.uint8, device="cuda"), torch.empty(half, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s1):
            da.copy_(ha, non_blocking=True)
        with torch.cuda.stream(s2):
            hb.copy_(db, non_blocking=True)
        torch.cuda.synchronize()
        rec("H2D + D2H concurrently (torch, sum of both)", 2 * half, time.perf_counter() - t0)
        del da, db
        # verify the pipelined parity against a device encode of the same stripes
        chk = host[:4].cuda()
        ref = chk.clone()
        r.encode_batch(ref)
        torch.cuda.synchronize()
        assert torch.equal(chk, ref), "host pipeline parity mismatch"
    if want("api"):
        # ---- host-memory Go-API calls (pageable numpy buffers), per-call latency
        import numpy as np

        L = rs.lib()
        k, m = 10, 4
        r = rs.New(k, m)
        # (label, host_pinned_max, host_zc_max, host_engine); the library's
        # defaults are 256 KiB / no limit / engine on
        modes = (("default: host-call engine up to 1 MiB", 256 << 10, -1, 1),
                 ("engine off: chunked zero-copy pipeline", 256 << 10, -1, 0),
                 ("engine off, staged: pinned mirror + DMA <= 4MiB", 4 << 20, 0, 0),
                 ("engine off, staged: pageable per-vector copies", 0, 0, 0))
        for label, pinned_max, zc_max, engine in modes:
            L.rs_tune(b"host_pinned_max", pinned_max)
            L.rs_tune(b"host_zc_max", zc_max)
            L.rs_tune(b"host_engine", engine)
            for vec in (8 << 10, 64 << 10, 256 << 10, 1 << 20):
                rng = np.random.default_rng(1)
                v = [rng.integers(0, 256, vec, dtype=np.uint8) for _ in range(k)] + [np.zeros(vec, np.uint8)
                                                                                     for _ in range(m)]
                for _ in range(5):
                    r.Encode(v)
                n = 50 if vec > 65536 else 500
                t0 = time.perf_counter()
                for _ in range(n):
                    r.Encode(v)
                t = (time.perf_counter() - t0) / n
                rec(f"Encode() host API 10+4 {vec >> 10}KiB ({label})", (k + m) * vec, t)
                if vec == 8 << 10:
                    full = [x.copy() for x in v]
                    for lost in ([0], [0, 1, 2, 3]):
                        w = [x.copy() for x in full]
                        for _ in range(5):
                            r.Reconst(w, [], lost)
                        t0 = time.perf_counter()
                        for _ in range(n):
                            r.Reconst(w, [], lost)
                        t = (time.perf_counter() - t0) / n
                        assert all(np.array_equal(a, b) for a, b in zip(w, full))
                        rec(f"Reconst() host API 10+4 8KiB lost={len(lost)} ({label})", (k + len(lost)) * vec, t)
        L.rs_tune(b"host_pinned_max", 256 << 10)
        L.rs_tune(b"host_zc_max", -1)
        L.rs_tune(b"host_engine", 1)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    tag = "_".join(sys.argv[sys.argv.index("--only") + 1].split(",")) if "--only" in sys.argv else "all"
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", f"ops_bench_{tag}.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
