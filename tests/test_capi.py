"""C ABI checks that need no GPU: the library loads, exports every symbol of
include/rs_amd.h, and its host-side logic (checks, planning, matrices,
inverse cache) equals the oracle's."""
import itertools
import os
import platform
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "rs_amd.h")).read()
    return sorted(set(re.findall(r"^RS_API\s+[\w\s\*]+?\b(rs_\w+)\s*\(", text, re.M)))


def test_header_declares_api():
    syms = _header_symbols()
    for s in ("rs_new", "rs_encode", "rs_reconst", "rs_update", "rs_replace", "rs_encode_batch"):
        assert s in syms
    assert len(syms) >= 25


def test_library_exports_every_header_symbol(rslib):
    import subprocess

    out = subprocess.run(["nm", "-D", "--defined-only", rslib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (rs_\w+)", out))
    missing = [s for s in _header_symbols() if s not in exported]
    assert not missing, missing
    # ctypes binds each one
    lib = rslib.lib()
    for s in _header_symbols():
        assert hasattr(lib, s)
    # nothing but the C ABI leaks out
    assert all(s.startswith("rs_") for s in exported)


def test_python_binding_covers_header(rslib):
    from reedsolomon_amd._lib import SIGNATURES

    assert sorted(SIGNATURES) == _header_symbols()


def test_error_codes_match_oracle():
    """include/rs_amd.h and oracle/rs_oracle.h number the errors identically."""
    h = open(os.path.join(ROOT, "include", "rs_amd.h")).read()
    o = open(os.path.join(ROOT, "oracle", "rs_oracle.h")).read()
    prod = dict(re.findall(r"RS_ERR_(\w+) = (\d+)", h))
    orac = dict(re.findall(r"ORC_ERR_(\w+) = (\d+)", o))
    assert orac and all(prod[k] == v for k, v in orac.items())


def test_error_text(rslib):
    L = rslib.lib()
    texts = {1: "illegal data/parity number: <= 0 or data+parity > 256", 2: "too few/many vectors given",
             3: "vector size is 0", 4: "vectors size mismatched", 5: "no need reconst", 6: "too many lost",
             7: "parity number mismatched", 8: "illegal vect index", 9: "too many data for replacing",
             10: "number of replaceRows and data mismatch", 11: "not a square matrix", 12: "matrix is singular"}
    for code, t in texts.items():  # rs.go:44,113-117,239-242,451-454,531-534; matrix.go:81-82
        assert L.rs_strerror(code).decode() == t


def test_new_validation(rslib):  # rs.go:61-63
    R = rslib
    for d, p in [(0, 1), (1, 0), (-1, 4), (200, 57), (256, 1)]:
        with pytest.raises(R.ErrIllegalVects):
            R.New(d, p)
    for d, p in [(1, 1), (255, 1), (1, 255), (128, 128), (10, 4)]:
        r = R.New(d, p)
        assert (r.DataNum, r.ParityNum) == (d, p)


@pytest.mark.parametrize("d,p", [(1, 1), (4, 4), (5, 5), (10, 4), (12, 4), (17, 3), (64, 64), (200, 56)])
def test_matrices_match_oracle(rslib, orc, d, p):
    r = rslib.New(d, p)
    assert np.array_equal(r.encMatrix, orc.make_encode_matrix(d, p))
    assert np.array_equal(r.GenMatrix, orc.gen_matrix(d, p))


def test_gf_mul_table(rslib, orc):
    mul = orc.tables()["mul"]
    for a in range(0, 256, 7):
        for b in range(256):
            assert rslib.gf_mul(a, b) == mul[a, b]


def test_invert_kats_and_random(rslib, orc):
    import json

    kats = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")))["matrix_invert"]
    errs = {11: rslib.ErrNotSquare, 12: rslib.ErrSingularMatrix}
    for c in kats["cases"]:
        if c["err"]:
            with pytest.raises(errs[c["err"]]):
                rslib.invert(np.array(c["m"], np.uint8), c["n"])
        else:
            assert rslib.invert(np.array(c["m"], np.uint8), c["n"]).tolist() == c["expect"]
    rng = np.random.default_rng(11)
    for n in (1, 2, 3, 7, 16, 40):
        for _ in range(10):
            m = rng.integers(0, 256, n * n, dtype=np.uint8)
            rc, exp = orc.invert(m, n)
            if rc:
                with pytest.raises(rslib.RSError):
                    rslib.invert(m, n)
            else:
                assert np.array_equal(rslib.invert(m, n), exp)


def test_invert_scalar_path_equals_vector_path(rslib, orc):
    """invert() takes AVX2 row operations where the host has them and the
    byte-table ones otherwise (RSAMD_INVERT_SCALAR=1 forces them): both give
    the oracle's bytes (matrix.go:85-147) on random and singular matrices up
    to 64 x 64, including zero pivots that swap rows."""
    import subprocess
    import sys

    code = (
        "import sys, numpy as np; sys.path.insert(0, %r);"
        "import reedsolomon_amd as rs; from oracle import oracle as orc; orc.build();"
        "rng = np.random.default_rng(31); bad = 0\n"
        "for n in (1, 2, 5, 10, 17, 32, 33, 64):\n"
        "  for k in range(6):\n"
        "    m = rng.integers(0, 256, n * n, dtype=np.uint8)\n"
        "    if k == 0 and n > 1: m[0] = 0\n"
        "    if k == 1 and n > 2: m[n:2 * n] = m[:n]\n"
        "    rc, exp = orc.invert(m, n)\n"
        "    try:\n"
        "      got = rs.invert(m, n); bad += int(rc != 0 or not np.array_equal(got, exp))\n"
        "    except rs.RSError:\n"
        "      bad += int(rc == 0)\n"
        "print('bad', bad)" % ROOT)
    for env in ({}, {"RSAMD_INVERT_SCALAR": "1"}):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                           env=dict(os.environ, **env), timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert r.stdout.strip().endswith("bad 0"), (env, r.stdout)


def test_inverse_cache_key(rslib, orc):
    rng = np.random.default_rng(12)
    for _ in range(200):
        s = sorted(rng.choice(64, int(rng.integers(1, 64)), replace=False).tolist())
        assert rslib.inverse_cache_key(s) == orc.inverse_cache_key(s)
    assert rslib.inverse_cache_key(list(range(64))) == 2 ** 64 - 1


def test_plan_reconst_matches_oracle(rslib, orc):
    d, p = 10, 4
    r = rslib.New(d, p)
    rng = np.random.default_rng(13)
    cases = [([], []), ([], [0]), ([], [13]), ([1, 2, 3], [0, 1]), ([14], [0]), ([0], [-1]),
             ([], [0, 1, 2, 3, 4]), (list(range(1, 14)), [0, 10])]
    for _ in range(500):
        ns, nn = int(rng.integers(0, 15)), int(rng.integers(0, 6))
        cases.append((rng.choice(14, ns, replace=False).tolist(), rng.choice(14, nn, replace=False).tolist()))
    for surv, need in cases:
        rc, vs, nr, dn = orc.check_reconst(d, p, surv, need)
        if rc:
            with pytest.raises(rslib.RSError) as ei:
                r.plan_reconst(surv, need)
            assert ei.value.code == rc
        else:
            assert r.plan_reconst(surv, need) == (vs, nr, dn)


def test_reconst_matrix_and_cache(rslib, orc):
    d, p = 10, 4
    r = rslib.New(d, p)
    em = orc.make_encode_matrix(d, p).reshape(d + p, d)
    n_patterns = 0
    for lost in itertools.combinations(range(d + p), 3):
        surv = [i for i in range(d + p) if i not in lost][:d]
        need = [i for i in lost if i < d]
        if not need:
            continue
        rc, inv = orc.invert(np.ascontiguousarray(em[surv]).ravel(), d)
        assert rc == 0
        exp = inv.reshape(d, d)[need].ravel()
        assert np.array_equal(r.reconst_matrix(surv, need), exp)
        assert np.array_equal(r.reconst_matrix(surv, need), exp)  # cache hit returns the same bytes
        n_patterns += 1
    assert r.inverse_cache_size() == len({tuple([i for i in range(d + p) if i not in lost][:d])
                                          for lost in itertools.combinations(range(d + p), 3)
                                          if any(i < d for i in lost)})


@pytest.mark.parametrize("d,p,nlost", [(40, 30, 30), (100, 28, 28), (100, 28, 3), (200, 56, 56), (129, 127, 100),
                                        (200, 56, 1)])
def test_wide_reconst_matrix_equals_full_inverse(rslib, orc, d, p, nlost):
    """Codes beyond 64 vectors (no reference cache) build Reconst matrices
    from the u x u block that couples the unknown data to the parity
    survivors standing in for them (codec.cpp unknown_data_rows); every row
    equals the full d x d inverse's row (the oracle's restated matrix.go
    Gauss-Jordan), for survivor lists in and out of index order and a needed
    survivor (its unit row); a repeated survivor is singular as before."""
    rng = np.random.default_rng(d * 7 + nlost)
    r = rslib.New(d, p)
    em = orc.make_encode_matrix(d, p).reshape(d + p, d)
    for trial in range(3):
        lost = sorted(int(v) for v in rng.choice(d, nlost, replace=False))
        par = sorted(int(v) for v in rng.choice(np.arange(d, d + p), nlost, replace=False))
        surv = [i for i in range(d) if i not in lost] + par
        if trial == 1:
            surv = [int(v) for v in rng.permutation(surv)]  # any order
        rc, inv = orc.invert(np.ascontiguousarray(em[surv]).ravel(), d)
        assert rc == 0
        need = lost + [min(x for x in surv if x < d)] if nlost < d else lost  # (+ a survivor: its unit row)
        got = r.reconst_matrix(surv, need).reshape(len(need), d)
        exp = inv.reshape(d, d)[need]
        assert np.array_equal(got, exp), (d, p, nlost, trial)
    with pytest.raises(rslib.ErrSingularMatrix):
        r.reconst_matrix([0] + list(range(0, d - 1)), [d - 1])
    assert r.inverse_cache_size() == 0


def test_cache_disabled_when_wide(rslib):  # rs.go:70 (d+p <= 64 only)
    r = rslib.New(40, 30)
    r.reconst_matrix(list(range(1, 41)), [0])
    assert r.inverse_cache_size() == 0


def _z(n):
    return np.zeros(n, np.uint8)


def test_host_checks_before_device(rslib, orc):
    """Malformed calls return the reference's error with no GPU present."""
    R = rslib
    r = R.New(10, 4)
    cases = [
        (lambda: r.Encode([_z(8)] * 13), 2),
        (lambda: r.Encode([_z(0)] + [_z(8)] * 13), 3),
        (lambda: r.Encode([_z(8)] * 13 + [_z(9)]), 4),
        (lambda: r.Reconst([_z(8)] * 14, [14], [0]), 1),
        (lambda: r.Reconst([_z(8)] * 14, [], [0, 1, 2, 3, 4]), 6),
        (lambda: r.Update(_z(8), _z(8), 0, [_z(8)] * 3), 7),
        (lambda: r.Update(_z(8), _z(0), 0, [_z(8)] * 4), 3),
        (lambda: r.Update(_z(7), _z(8), 0, [_z(8)] * 4), 4),
        (lambda: r.Update(_z(8), _z(8), 0, [_z(8)] * 3 + [_z(7)]), 4),
        (lambda: r.Update(_z(8), _z(8), -1, [_z(8)] * 4), 8),
        (lambda: r.Replace([_z(8)] * 11, list(range(11)), [_z(8)] * 4), 9),
        (lambda: r.Replace([_z(8)] * 2, [0], [_z(8)] * 4), 10),
        (lambda: r.Replace([_z(8)] * 2, [0, 1], [_z(8)] * 3), 7),
        (lambda: r.Replace([_z(0)] * 2, [0, 1], [_z(8)] * 4), 3),
        (lambda: r.Replace([_z(8), _z(9)], [0, 1], [_z(8)] * 4), 4),
        (lambda: r.Replace([_z(8)] * 2, [0, 1], [_z(8)] * 3 + [_z(1)]), 4),
        (lambda: r.Replace([_z(8)] * 2, [0, 10], [_z(8)] * 4), 8),
        (lambda: r.Replace([], [], [_z(8)] * 4), 13),
    ]
    for fn, code in cases:
        with pytest.raises(R.RSError) as ei:
            fn()
        assert ei.value.code == code
    # nothing to rebuild: Reconst swallows ErrNoNeedReconst (rs.go:225-228)
    r.Reconst([_z(8)] * 14, [0, 1], [])


def test_host_batch_argument_checks(rslib):
    """rs_encode_host_batch validates its layout before touching a device."""
    import ctypes
    L = rslib.lib()
    r = rslib.New(10, 4)
    buf = (ctypes.c_uint8 * (14 * 256))()
    base = ctypes.cast(buf, ctypes.POINTER(ctypes.c_uint8))
    assert L.rs_encode_host_batch(r._h, base, -14 * 256, 256, 1, 256, 0, 0) == 13  # RS_ERR_INVAL
    assert L.rs_encode_host_batch(r._h, base, 14 * 256, -256, 1, 256, 0, 0) == 13
    assert L.rs_encode_host_batch(r._h, None, 14 * 256, 256, 1, 256, 0, 0) == 13
    assert L.rs_encode_host_batch(r._h, base, 14 * 256, 256, -1, 256, 0, 0) == 13
    assert L.rs_encode_host_batch(r._h, base, 14 * 256, 256, 1, 0, 0, 0) == 3  # ErrZeroVectSize
    assert L.rs_encode_host_batch(r._h, base, 14 * 256, 256, 0, 256, 0, 0) == 0


def test_reconst_matrix_from_cache(rslib):  # TestRS_getReconstMatrixFromCache rs_test.go:355-404
    """The reference force-enables the cache on 64+64 (white-box); here the
    widest shape the cache serves by policy (d+p = 64, rs.go:70) with d = 60,
    so the miss pays a 60x60 Gauss-Jordan."""
    import time

    r = rslib.New(60, 4)
    surv = list(range(4, 64))  # data 0..3 lost
    need = [0, 1, 2, 3]
    t0 = time.perf_counter()
    first = r.reconst_matrix(surv, need)
    t1 = time.perf_counter()
    second = r.reconst_matrix(surv, need)
    t2 = time.perf_counter()
    assert np.array_equal(first, second)
    assert r.inverse_cache_size() == 1
    assert (t2 - t1) < (t1 - t0)  # the hit skips the inverse


def _gf_matmul(mul, a, b):
    """a (n x k) * b (k x m) over GF(2^8) with the mulTbl (gmu.go:26-28)."""
    out = np.zeros((a.shape[0], b.shape[1]), np.uint8)
    for t in range(a.shape[1]):
        out ^= mul[a[:, t][:, None], b[t][None, :]]
    return out


def test_enc_matrix_invertible_random(rslib, orc):  # TestEncMatrixInvertibleRandom matrix_test.go:202-241
    """One random survivor subset for a spread of d+p <= 256 shapes: the
    reconst matrix times the survivors' encoding rows is the identity."""
    mul = orc.tables()["mul"]
    rng = np.random.default_rng(14)
    shapes = [(1, 1), (1, 255), (255, 1), (128, 128), (200, 56), (17, 3)]
    shapes += [(int(d), int(rng.integers(1, 257 - d))) for d in rng.integers(1, 255, 24)]
    for d, p in shapes:
        r = rslib.New(d, p)
        em = r.encMatrix.reshape(d + p, d)
        surv = sorted(rng.choice(d + p, d, replace=False).tolist())
        need = list(range(d))
        inv = r.reconst_matrix(surv, need).reshape(d, d)
        assert np.array_equal(_gf_matmul(mul, inv, em[surv]), np.eye(d, dtype=np.uint8)), (d, p)


def test_group_handles(rslib):
    """rs_group_* (one codec per device) needs no GPU until a call runs."""
    g = rslib.NewGroup(10, 4, [0, 0, 3])
    assert len(g) == 3 and [m.device for m in g.members] == [0, 0, 3]
    assert all(np.array_equal(m.GenMatrix, g.members[0].GenMatrix) for m in g.members)
    for bad in ([], [-1]):
        with pytest.raises(rslib.ErrInvalidArgument):
            rslib.NewGroup(10, 4, bad)
    with pytest.raises(rslib.ErrIllegalVects):
        rslib.NewGroup(200, 57, [0])
    L = rslib.lib()
    assert L.rs_group_codec(g._g, 3) is None and L.rs_group_codec(g._g, -1) is None


def test_ref_l1d_is_per_handle(rslib):
    """rs_set_ref_l1d: per handle, no device call; -1 resolves to this host's
    L1D (rs_host_l1d; 32 KiB when undetectable, rs.go:159-161); values below
    32 are refused; the old process-wide knob is gone."""
    a, b = rslib.New(10, 4), rslib.New(10, 4)
    assert a.ref_l1d == 0 and b.ref_l1d == 0
    a.set_ref_l1d(49152)
    assert a.ref_l1d == 49152 and b.ref_l1d == 0
    host = rslib.host_l1d()
    b.set_ref_l1d(-1)
    assert b.ref_l1d == (host if host > 0 else 32768)
    if platform.machine() in ("x86_64", "AMD64"):
        # CPUID's answer agrees with the kernel's view of this host's L1D
        p = "/sys/devices/system/cpu/cpu0/cache/index0"
        if os.path.exists(p + "/size") and open(p + "/type").read().strip() == "Data":
            txt = open(p + "/size").read().strip()
            assert host == int(txt.rstrip("K")) * 1024, (host, txt)
    for bad in (1, 16, 31, -2):
        with pytest.raises(rslib.ErrInvalidArgument):
            a.set_ref_l1d(bad)
    assert a.ref_l1d == 49152
    a.set_ref_l1d(0)
    assert a.ref_l1d == 0
    assert rslib.lib().rs_tune(b"ref_update_tail", 32768) == 13


def test_tune_accepts_every_documented_knob(rslib):
    """Every knob name the header documents for rs_tune is accepted, and an
    unknown name is RS_ERR_INVAL (run in a child process: rs_tune changes
    process-wide state)."""
    import subprocess
    import sys

    text = open(os.path.join(ROOT, "include", "rs_amd.h")).read()
    doc = text[text.index("Expert launch knobs"):text.index("RS_API int rs_tune")]
    names = sorted(set(re.findall(r'"(\w+)"', doc)))
    assert {"lane_bytes", "block8", "host_coalesce_max", "table_registry_max"} <= set(names)
    code = (
        "import sys, ctypes\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import reedsolomon_amd as rs\n"
        "L = rs.lib()\n"
        f"names = {names!r}\n"
        "bad = [n for n in names if L.rs_tune(n.encode(), 1) != 0]\n"
        "assert not bad, bad\n"
        "assert L.rs_tune(b'no_such_knob', 1) == 13\n"
        "assert L.rs_tune(b'var', 141) == 13  # experiments build only\n"
        "print('ok', len(names))\n"
    )
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.startswith("ok")


def test_multi_pattern_mask_validation_wide(rslib):
    """Multi-pattern Reconst masks are validated on the host before any device
    work (no GPU needed here): the 64-bit API refuses codecs of more than 64
    vectors (RS_ERR_INVAL), the 256-bit API (rs_reconst_batch_multi256, any
    d+p <= 256 as rs.go:61) rejects bits past d+p (ErrIllegalVects) and more
    than p erasures (ErrTooManyLost); the Python mirror picks the API from
    the codec's size and the masks."""
    import ctypes

    from reedsolomon_amd._lib import RSLayout

    L = rslib.lib()
    d, p, S = 100, 28, 3
    h = ctypes.c_void_p()
    assert L.rs_new(d, p, -1, ctypes.byref(h)) == 0
    try:
        lay = RSLayout(0x1000, 1 << 20, 4096, 0x2000, 1 << 20, 4096)  # never dereferenced: validation fails first
        u64p = ctypes.POINTER(ctypes.c_uint64)
        m64 = np.ones(S, np.uint64)
        assert L.rs_reconst_batch_multi(h, ctypes.byref(lay), S, 4096, m64.ctypes.data_as(u64p), None) == 13
        wide = np.zeros((S, 4), np.uint64)
        wide[1, 2] = np.uint64(1) << np.uint64(128 - 128 + 0)  # vector 128: past d+p = 128
        assert L.rs_reconst_batch_multi256(h, ctypes.byref(lay), S, 4096, wide.ctypes.data_as(u64p), None) == 1
        too_many = [sum(1 << v for v in range(0, 29)), 0, 0]  # 29 > p erasures
        m, fn = rslib.rs._masks_for(too_many, S, d + p, "rs_reconst_batch_multi")
        assert fn == "rs_reconst_batch_multi256" and m.shape == (S, 4)
        assert L.rs_reconst_batch_multi256(h, ctypes.byref(lay), S, 4096, m.ctypes.data_as(u64p), None) == 6
        # host batch variant: same validation before any copy
        assert L.rs_reconst_host_batch_multi256(h, ctypes.c_void_p(0x1000), 1 << 20, 4096, S, 4096,
                                                m.ctypes.data_as(u64p)) == 6
    finally:
        L.rs_free(h)
    # 64-bit masks through the hashed grouping (thousands of distinct
    # patterns, repeats, runs): one bad stripe anywhere fails the whole call
    from itertools import combinations

    for d, p in ((10, 4), (32, 32)):
        assert L.rs_new(d, p, -1, ctypes.byref(h)) == 0
        try:
            lay = RSLayout(0x1000, 1 << 20, 4096, 0x2000, 1 << 20, 4096)
            good = [sum(1 << v for v in c) for k in (1, 2, 3) for c in combinations(range(d + p), k)][:3000]
            good = np.array(good + good[::-1] + [good[7]] * 50, dtype=np.uint64)
            for at, bad, rc in ((len(good) - 1, 1 << (d + p), 1), (len(good) // 2, (1 << (p + 1)) - 1, 6), (5, 0, 14)):
                if d + p == 64 and rc == 1:
                    continue  # every bit of a 64-bit mask is a vector of 32+32
                m = good.copy()
                if bad:
                    m[at] = np.uint64(bad)
                # rc 14: every mask valid, so the call gets as far as the device (none here)
                assert L.rs_reconst_batch_multi(h, ctypes.byref(lay), len(m), 4096, m.ctypes.data_as(u64p),
                                                None) in ((rc,) if rc != 14 else (14, 0)), (d, p, at, bad)
        finally:
            L.rs_free(h)
    # small codecs keep the 64-bit API
    m, fn = rslib.rs._masks_for([1, 2, 3], 3, 14, "rs_reconst_batch_multi")
    assert fn == "rs_reconst_batch_multi" and m.dtype == np.uint64 and m.shape == (3,)
    m, fn = rslib.rs._masks_for([1 << 127, 0], 2, 128, "rs_reconst_batch_multi")
    assert fn == "rs_reconst_batch_multi256" and int(m[0, 1]) == 1 << 63


def test_jit_compile_check(rslib, orc):
    """The run-time bit-sliced kernel generators produce code objects for
    gfx950 with no device - machine code in a template (jit_asm.cpp, the
    default backend), assembly through comgr, or C++ through hiprtc (jit.cpp):
    a Reconst-of-8 matrix of 10+8 (overwrite) and
    a 16-column 5-row XOR-accumulate product, plus a 64 x 64 product for the
    assembly backend; shapes outside each backend's bounds are refused
    (assembly: 1-128 rows, 1-256 columns; hiprtc: 5-16 rows, 1-64 columns;
    rs_jit_prepare: from 5 rows)."""
    import numpy as np

    from reedsolomon_amd.rs import ErrInvalidArgument

    L = rslib.lib()
    r = rslib.New(10, 8)
    survived = list(range(8, 18))
    m = r.reconst_matrix(survived, list(range(8))).reshape(8, 10)  # rows of the inverse for data 0..7
    rng = np.random.default_rng(3)
    try:
        for backend, bad, extra in ((2, [(129, 10), (8, 257)], [(64, 64), (128, 128)]),
                                    (1, [(129, 10), (8, 257)], [(64, 64)]), (0, [(17, 10), (8, 65)], [])):
            assert L.rs_tune(b"jit_backend", backend) == 0
            assert rslib.jit_compile_check(m) > 0
            assert rslib.jit_compile_check(rng.integers(0, 256, (5, 16), dtype=np.uint8), accumulate=True) > 0
            for shape in extra:
                assert rslib.jit_compile_check(rng.integers(0, 256, shape, dtype=np.uint8)) > 0
            for shape in bad:
                with pytest.raises(ErrInvalidArgument):
                    rslib.jit_compile_check(np.ones(shape, np.uint8))
            for shape in bad + [(4, 10)]:
                with pytest.raises(ErrInvalidArgument):  # rs_jit_prepare checks the shape before any device work
                    r.jit_prepare(np.ones(shape, np.uint8))
    finally:
        L.rs_tune(b"jit_backend", 2)



def test_host_memory_entry_points_without_device(rslib):
    """rs_host_free / rs_host_unregister / rs_host_pool_stats argument checks
    (no HIP call is made for these): freeing NULL is a no-op, foreign
    pointers and addresses never registered are refused, the pool is empty."""
    import ctypes

    L = rslib.lib()
    assert L.rs_host_free(None) == 0
    junk = np.zeros(64, np.uint8)
    inval = 13  # RS_ERR_INVAL
    assert L.rs_host_free(ctypes.c_void_p(junk.ctypes.data)) == inval
    assert L.rs_host_unregister(ctypes.c_void_p(junk.ctypes.data)) == inval
    assert L.rs_host_unregister(None) == inval
    out = ctypes.c_void_p()
    assert L.rs_host_alloc(0, ctypes.byref(out)) == inval and not out.value
    st = rslib.host_pool_stats()
    assert st["in_use"] == 0 and set(st) == {"mapped", "in_use", "blocks", "spans"}


def test_cauchy_closed_form_inverse(orc):
    """The GPU planner (kernels.hip gf_plan_multi) inverts enc[P][L], the
    block coupling the lost data L to the parity survivors P, by the Cauchy
    closed form instead of Gauss-Jordan: enc[i][j] = 1/(i ^ j) for a parity
    row (matrix.go:37-54), and for x_j = P_j, y_l = L_l
      Minv[l][j] = prod_k (x_j+y_k)(x_k+y_l) / ((x_j+y_l) prod_{k!=j} (x_j+x_k) prod_{k!=l} (y_l+y_k)).
    The same log sums as the kernel, against the oracle's Gauss-Jordan
    (matrix.go:85-147 restated) on random blocks of 1-8 lost data."""
    t = orc.tables()
    lg = t["log"].astype(np.int64)
    ex = np.concatenate([t["exp"], t["exp"]])
    rng = np.random.default_rng(77)
    for _ in range(400):
        d = int(rng.integers(1, 200))
        p = int(rng.integers(1, 257 - d))
        n = int(rng.integers(1, min(8, p, d) + 1))
        x = sorted(int(v) for v in rng.choice(np.arange(d, d + p), n, replace=False))
        y = sorted(int(v) for v in rng.choice(d, n, replace=False))
        em = orc.make_encode_matrix(d, p).reshape(d + p, d)
        block = np.ascontiguousarray(em[np.ix_(x, y)])
        rc, inv = orc.invert(block.ravel(), n)
        assert rc == 0
        want = inv.reshape(n, n)
        for l in range(n):
            for j in range(n):
                num = sum(lg[x[j] ^ y[k]] + lg[x[k] ^ y[l]] for k in range(n))
                den = lg[x[j] ^ y[l]] + sum(lg[x[j] ^ x[k]] for k in range(n) if k != j) + \
                    sum(lg[y[l] ^ y[k]] for k in range(n) if k != l)
                assert ex[(num + 255 * 4 * 8 - den) % 255] == want[l, j], (d, p, x, y, l, j)
