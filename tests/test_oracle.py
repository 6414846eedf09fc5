"""Pins the CPU oracle to the reference (no GPU).

Every check here is one of the reference's own tests restated, run against
oracle/rs_oracle.c, plus the table fixtures extracted from gftbl.go and
gftbl_test.go (tools/extract_reference_fixtures.py).  Seeds are fixed
(the reference seeds from the clock, helper_test.go:146-148).
"""
import hashlib
import itertools
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
KATS = json.load(open(os.path.join(GOLDEN, "reference_kats.json")))


def _fixture(name):
    return np.frombuffer(open(os.path.join(GOLDEN, name), "rb").read(), np.uint8)


# ---------------------------------------------------------------- tables (gftbl_test.go)

def test_tables_match_reference_gftbl(orc):
    t = orc.tables()
    assert t["mul"].tobytes() == _fixture("ref_mul_tbl.bin").tobytes()        # gftbl.go:14
    assert t["low_high"].tobytes() == _fixture("ref_low_high_tbl.bin").tobytes()  # gftbl.go:16
    assert t["inverse"].tobytes() == _fixture("ref_inverse_tbl.bin").tobytes()    # gftbl.go:12


def test_table_sha256_pins(orc):
    # digests of the reference's generated tables.
    t = orc.tables()
    assert hashlib.sha256(t["mul"].tobytes()).hexdigest() == \
        "003d1a609783d2740b9b3f00b0cd9e43e42c4f3eedc5ff54ec1709996d52e1e0"
    assert hashlib.sha256(t["low_high"].tobytes()).hexdigest() == \
        "76dcc4fc27b2bf98f6c0f50e71570101f61cc2ac983c366f6d80d64b655a2f22"
    assert hashlib.sha256(t["inverse"].tobytes()).hexdigest() == \
        "ce85f43612c0a6d03939cc3dfe9ca877032d017fb26aca602b696b74e5600d72"


def test_mul_tbl_equals_isal(orc):  # TestMulTbl gftbl_test.go:10-20
    assert orc.tables()["mul"].tobytes() == _fixture("isal_mul_tbl.bin").tobytes()


def test_inverse_tbl(orc):  # TestInverseTbl gftbl_test.go:22-36
    t = orc.tables()
    assert t["inverse"][0] == 0
    for i in range(1, 256):
        assert t["mul"][t["inverse"][i], i] == 1


def test_low_high_tbl(orc):  # TestLowHighTbl gftbl_test.go:38-53
    t = orc.tables()
    lh = t["low_high"].reshape(256, 32)
    x = np.arange(256)
    for c in range(256):
        assert np.array_equal(lh[c, :16][x & 15] ^ lh[c, 16:][x >> 4], t["mul"][c])


# ---------------------------------------------------------------- matrix.go KATs

def test_make_encode_matrix_kat(orc):  # TestMakeEncodeMatrix matrix_test.go:16-30
    k = KATS["make_encode_matrix_4_4"]
    assert orc.make_encode_matrix(k["d"], k["p"]).tolist() == k["expect"]


def test_gen_matrix_rows(orc):
    k = KATS["gen_matrix_rows"]
    assert orc.gen_matrix(10, 4).reshape(4, 10).tolist() == k["10_4"]
    assert orc.gen_matrix(12, 4)[:12].tolist() == k["12_4_row0"]


@pytest.mark.parametrize("case", KATS["matrix_invert"]["cases"])
def test_matrix_invert_kat(orc, case):  # TestMatrixInvert matrix_test.go:45-134
    rc, out = orc.invert(np.array(case["m"], np.uint8), case["n"])
    assert rc == case["err"]
    if case["expect"] is not None:
        assert out.tolist() == case["expect"]


def _gf_matmul(orc, a, b, n):
    mul = orc.tables()["mul"]
    out = np.zeros((n, n), np.uint8)
    for i in range(n):
        for j in range(n):
            s = 0
            for k in range(n):
                s ^= int(mul[a[i * n + k], b[k * n + j]])
            out[i, j] = s
    return out


def test_matrix_swap_via_invert_pivot(orc):  # TestMatrixSwap matrix_test.go:32-43 (pivot path)
    # The 3x3 KAT with a zero pivot already drives swap(); here a permutation matrix.
    m = np.array([0, 1, 0, 1, 0, 0, 0, 0, 1], np.uint8)
    rc, inv = orc.invert(m, 3)
    assert rc == 0 and inv.tolist() == m.tolist()


def test_make_enc_matrix_for_reconst(orc):  # TestMakeEncMatrixForReconst matrix_test.go:136-151
    d, p = 4, 4
    em = orc.make_encode_matrix(d, p)
    rng = np.random.default_rng(7)
    for _ in range(20):
        surv = sorted(rng.choice(d + p, d, replace=False).tolist())
        sub = np.concatenate([em[i * d:(i + 1) * d] for i in surv])
        rc, inv = orc.invert(sub, d)
        assert rc == 0
        assert np.array_equal(_gf_matmul(orc, inv, sub, d), np.eye(d, dtype=np.uint8))


@pytest.mark.parametrize("d,p", [(10, 4), (15, 4)])
def test_enc_matrix_invertible_all(orc, d, p):  # TestEncMatrixInvertibleAll matrix_test.go:157-200
    em = orc.make_encode_matrix(d, p).reshape(d + p, d)
    cnt = 0
    for surv in itertools.combinations(range(d + p), d):
        if surv == tuple(range(d)):
            continue  # nothing lost (the reference's bitmap range starts past it)
        rc, _ = orc.invert(np.ascontiguousarray(em[list(surv)]).ravel(), d)
        assert rc == 0, surv
        cnt += 1
    assert cnt == len(list(itertools.combinations(range(d + p), d))) - 1


# ---------------------------------------------------------------- rs.go KATs / properties

def test_rs_mul_kat(orc):  # TestRS_mul rs_test.go:24-49
    k = KATS["rs_mul_5_5"]
    vects = [np.array([x], np.uint8) for x in k["data"]] + [np.zeros(1, np.uint8) for _ in range(5)]
    orc.naive_mul(orc.gen_matrix(5, 5), 5, 5, vects)
    assert [int(v[0]) for v in vects[5:]] == k["parity"]
    vects2 = [np.array([x], np.uint8) for x in k["data"]] + [np.zeros(1, np.uint8) for _ in range(5)]
    assert orc.encode(5, 5, vects2) == 0
    assert [int(v[0]) for v in vects2[5:]] == k["parity"]


def test_inverse_cache_key_kat(orc):  # TestMakeInverseCacheKey rs_test.go:139-163
    for c in KATS["inverse_cache_key"]["cases"]:
        surv = list(range(64)) if c["survived"] == "range(64)" else c["survived"]
        assert orc.inverse_cache_key(surv) == int(c["key"])


def test_encode_matches_naive_all_sizes(orc):  # TestRS_Encode rs_test.go:72-137 (sizes 1..1024)
    d, p = 10, 4
    rng = np.random.default_rng(1)
    gen = orc.gen_matrix(d, p)
    for size in range(1, 1025):
        data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(d)]
        act = data + [np.full(size, 0xA5, np.uint8) for _ in range(p)]
        exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        assert orc.encode(d, p, act) == 0
        orc.naive_mul(gen, d, p, exp)
        for j in range(d, d + p):
            assert np.array_equal(act[j], exp[j]), size


def test_avx2_port_matches_table_path(orc):  # TestRS_Encode AVX2 vs no-SIMD leg / TestGMU gmu_test.go
    d, p = 10, 4
    rng = np.random.default_rng(2)
    for size in list(range(1, 300)) + [1024, 4096, 8192, 16384 + 17, 65536]:
        data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(d)]
        a = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        b = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        orc.encode_avx2(d, p, a)
        orc.encode(d, p, b)
        for j in range(d, d + p):
            assert np.array_equal(a[j], b[j]), size


def test_numpy_restatement_matches(orc):
    d, p = 12, 4
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, (3, d, 777), dtype=np.uint8)
    par = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), data)
    for s in range(3):
        v = [data[s, i].copy() for i in range(d)] + [np.zeros(777, np.uint8) for _ in range(p)]
        orc.encode(d, p, v)
        for j in range(p):
            assert np.array_equal(v[d + j], par[s, j])


def _gen_idx(rng, d, p, survived_n, need_n):  # genIdxForTest helper_test.go:24-63
    survived_n = max(survived_n, d)
    need_n = min(need_n, p)
    if survived_n + need_n > d + p:
        survived_n = d
    need = rng.permutation(d + p)[:need_n].tolist()
    full = rng.permutation(d + p).tolist()
    surv = []
    for i in full:
        if len(surv) == survived_n:
            break
        if i not in need:
            surv.append(i)
    return sorted(surv), sorted(need)


def test_reconst_round_trip(orc):  # TestRS_Reconst rs_test.go:165-217
    d, p, size = 10, 4, 1024
    rng = np.random.default_rng(4)
    for _ in range(128):
        exp = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(d)] + \
              [np.zeros(size, np.uint8) for _ in range(p)]
        assert orc.encode(d, p, exp) == 0
        surv, need = _gen_idx(rng, d, p, int(rng.integers(d + p)), int(rng.integers(p + 1)))
        act = [np.zeros(size, np.uint8) for _ in range(d + p)]
        for i in surv:
            act[i][:] = exp[i]
        for n in need:
            if rng.integers(4) == 1:
                act[n][:] = rng.integers(0, 256, size, dtype=np.uint8)
        assert orc.reconst(d, p, act, surv, need) == 0
        for n in need:
            assert np.array_equal(act[n], exp[n])


def test_update_equals_reencode(orc):  # TestRS_Update rs_test.go:219-266
    d, p, size = 10, 4, 1024
    rng = np.random.default_rng(5)
    for row in range(d):
        exp = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(d)] + \
              [np.zeros(size, np.uint8) for _ in range(p)]
        act = [x.copy() for x in exp]
        orc.encode(d, p, act)
        new = rng.integers(0, 256, size, dtype=np.uint8)
        assert orc.update(d, p, act[row], new, row, act[d:]) == 0
        exp[row] = new.copy()
        orc.encode(d, p, exp)
        for j in range(d, d + p):
            assert np.array_equal(act[j], exp[j])


@pytest.mark.parametrize("size", [16384 + 16 * 40 + 7, 49263, 236667, 16384 * 5 + 17])
def test_reference_update_replace_tail_defect(orc, size):
    """The reference's Update / Replace (restated faithfully) equal re-encoding
    everywhere except the body of a last chunk with a >= 16-byte, non-16-multiple
    length, where they keep the old parity (rs.go:190-200 XORs that body twice).
    Pins the analysis behind DESIGN.md §4 "Reference defect"; librsamd computes
    the re-encode result there."""
    d, p, row = 10, 4, 3
    rng = np.random.default_rng(size)
    base = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(d)] + \
           [np.zeros(size, np.uint8) for _ in range(p)]
    orc.encode(d, p, base)
    new = rng.integers(0, 256, size, dtype=np.uint8)
    upd = [x.copy() for x in base]
    assert orc.update(d, p, upd[row], new, row, upd[d:]) == 0
    rep = [x.copy() for x in base]
    delta = np.bitwise_xor(base[row], new)
    assert orc.replace(d, p, [delta], [row], rep[d:]) == 0
    exp = [x.copy() for x in base]
    exp[row] = new.copy()
    orc.encode(d, p, exp)
    lo, hi = orc.update_quirk_range(size)
    for got in (upd, rep):
        for j in range(d, d + p):
            assert np.array_equal(got[j][:lo], exp[j][:lo]) and np.array_equal(got[j][hi:], exp[j][hi:])
            assert np.array_equal(got[j][lo:hi], base[j][lo:hi])  # untouched: the old parity
    for ok_size in (1024, 16384, 16384 * 3 + 5, 16384 * 2 + 32, 40000 - 40000 % 16):
        assert orc.update_quirk_range(ok_size) is None


@pytest.mark.parametrize("to_zero", [True, False])
def test_replace_equals_reencode(orc, to_zero):  # TestRS_Replace rs_test.go:268-331
    d, p, size = 10, 4, 1024
    rng = np.random.default_rng(6 + to_zero)
    for _ in range(128):
        n = int(rng.integers(d + 1))
        rows = []
        while len(rows) < n:
            v = int(rng.integers(d))
            if v not in rows:
                rows.append(v)
        rows = rows or [0]
        exp = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(d)] + \
              [np.zeros(size, np.uint8) for _ in range(p)]
        act = [x.copy() for x in exp]
        data = [exp[r].copy() for r in rows]
        if to_zero:
            for r in rows:
                exp[r] = np.zeros(size, np.uint8)
        orc.encode(d, p, exp)
        if not to_zero:
            for r in rows:
                act[r] = np.zeros(size, np.uint8)
        orc.encode(d, p, act)
        assert orc.replace(d, p, data, rows, act[d:]) == 0
        for j in range(d, d + p):
            assert np.array_equal(act[j], exp[j])


# ---------------------------------------------------------------- error ordering

def test_check_errors(orc):
    z = lambda n: np.zeros(n, np.uint8)  # noqa: E731
    assert orc.lib().orc_new_check(0, 1) == 1 and orc.lib().orc_new_check(200, 57) == 1
    assert orc.encode(10, 4, [z(8)] * 13) == 2                              # ErrMismatchVects
    assert orc.encode(10, 4, [z(0)] + [z(8)] * 13) == 3                     # ErrZeroVectSize
    assert orc.encode(10, 4, [z(8)] * 13 + [z(9)]) == 4                     # ErrMismatchVectSize
    assert orc.check_reconst(10, 4, [], [])[0] == 5                          # ErrNoNeedReconst
    assert orc.check_reconst(10, 4, [14], [0])[0] == 1                       # ErrIllegalVects
    assert orc.check_reconst(10, 4, [], [0, 1, 2, 3, 4])[0] == 6             # ErrTooManyLost
    assert orc.update(10, 4, z(8), z(8), 0, [z(8)] * 3) == 7                 # ErrMismatchParityNum
    assert orc.update(10, 4, z(8), z(0), 0, [z(8)] * 4) == 3
    assert orc.update(10, 4, z(7), z(8), 0, [z(8)] * 4) == 4
    assert orc.update(10, 4, z(8), z(8), 10, [z(8)] * 4) == 8                # ErrIllegalVectIndex
    assert orc.replace(10, 4, [z(8)] * 11, list(range(11)), [z(8)] * 4) == 9  # ErrTooManyReplace
    assert orc.replace(10, 4, [z(8)] * 2, [0], [z(8)] * 4) == 10             # ErrMismatchReplace
    assert orc.replace(10, 4, [z(8)] * 2, [0, 1], [z(8)] * 3) == 7
    assert orc.replace(10, 4, [], [], [z(8)] * 4) == 13                      # reference panics
    assert orc.replace(10, 4, [z(8)] * 2, [0, 10], [z(8)] * 4) == 8


def test_bitslice_generator_matches_oracle(orc):
    """tools/gen_bitslice.py (build tooling for the bit-sliced Encode kernels):
    its generator matrices are the oracle's, its GF(2) bit matrices reproduce
    every product, and the committed bitslice_gen.inc is what it emits."""
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("gen_bitslice", os.path.join(root, "tools", "gen_bitslice.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    mul = orc.tables()["mul"]
    for d, p in gen.SHAPES:
        G = gen.gen_matrix(d, p)
        assert np.array_equal(np.array(G, np.uint8).ravel(), orc.gen_matrix(d, p)), (d, p)
    for c in range(256):
        for x in (1, 2, 3, 0x55, 0x80, 0xFF, 0x9C):
            prod = 0
            for i in range(8):  # bit i of c*x = XOR of bits j of x with bit i of c*(1<<j)
                b = 0
                for j in range(8):
                    if (x >> j) & 1 and (gen.gmul(c, 1 << j) >> i) & 1:
                        b ^= 1
                prod |= b << i
            assert prod == mul[c, x], (c, x)
    with open(gen.OUT) as f:
        assert f.read() == gen.emit(), "bitslice_gen.inc is stale: run python tools/gen_bitslice.py"


def test_oracle_l1d_setting_moves_the_defect(orc):
    """orc_set_l1d (getSplitSize's L1D, rs.go:158-173) moves the Update tail
    defect exactly to update_quirk_range(size, l1d)."""
    d, p, row = 4, 2, 1
    rng = np.random.default_rng(5)
    for l1d, size in [(49152, 24576 + 33), (32768, 24576 + 33), (65536, 3 * 32768 + 47)]:
        data = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(d)]
        enc = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        assert orc.encode(d, p, enc) == 0
        new = rng.integers(0, 256, size, dtype=np.uint8)
        reenc = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        reenc[row] = new.copy()
        assert orc.encode(d, p, reenc) == 0
        orc.set_l1d(l1d)
        try:
            ora = [x.copy() for x in enc]
            assert orc.update(d, p, ora[row], new, row, ora[d:]) == 0
        finally:
            orc.set_l1d(0)
        q = orc.update_quirk_range(size, l1d)
        for j in range(d, d + p):
            diff = np.flatnonzero(ora[j] != reenc[j])
            if q is None:
                assert diff.size == 0, (l1d, size)
            else:
                assert diff.size and diff.min() >= q[0] and diff.max() < q[1], (l1d, size)
                assert np.array_equal(ora[j][q[0]:q[1]], enc[j][q[0]:q[1]])  # stale parity kept
