"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact for every byte (integer GF(2^8) work: no tolerance).  Mirrors
the reference's own tests (rs_test.go) at the sizes the oracle finishes in
seconds, plus size-independent properties (encode -> erase -> reconst round
trips, linearity) at BASELINE.json's full 10+4 / 1 MiB x 256-stripe size.
"""
import itertools
import threading

import numpy as np
import pytest

import hip_ptr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    torch.cuda.init()
    return torch


def _rand(rng, *shape):
    return rng.integers(0, 256, shape, dtype=np.uint8)


def _first_diff(got, exp):
    """(index, got, expected) of the first differing byte, and the count."""
    bad = np.argwhere(got != exp)
    if not len(bad):
        return None
    i = tuple(int(x) for x in bad[0])
    return i, int(got[i]), int(exp[i]), len(bad)


def _oracle_encode(orc, d, p, data_list):
    size = data_list[0].size
    v = [x.copy() for x in data_list] + [np.zeros(size, np.uint8) for _ in range(p)]
    assert orc.encode(d, p, v) == 0
    return v[d:]


# ---------------------------------------------------------------- Encode (host API)

def test_encode_all_sizes_1_to_1024(rslib, orc, torch_dev):  # TestRS_Encode rs_test.go:72-137
    d, p = 10, 4
    r = rslib.New(d, p)
    rng = np.random.default_rng(100)
    gen = orc.gen_matrix(d, p)
    for size in range(1, 1025):
        data = [_rand(rng, size) for _ in range(d)]
        act = [x.copy() for x in data] + [np.full(size, 0xA5, np.uint8) for _ in range(p)]
        r.Encode(act)
        exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        orc.naive_mul(gen, d, p, exp)
        for j in range(d, d + p):
            assert np.array_equal(act[j], exp[j]), (size, j)


@pytest.mark.parametrize("d,p,size", [
    (1, 1, 1000), (2, 2, 4097), (3, 2, 65536 + 3), (5, 5, 8192), (10, 4, 1 << 20), (12, 4, 1 << 20),
    (17, 3, 12345), (28, 4, 8192), (10, 8, 4096), (6, 12, 3000), (64, 64, 2048), (128, 128, 512),
    (200, 56, 300), (255, 1, 1024), (1, 255, 257),
])
def test_encode_shapes(rslib, orc, torch_dev, d, p, size):
    r = rslib.New(d, p)
    rng = np.random.default_rng(d * 1000 + p)
    data = [_rand(rng, size) for _ in range(d)]
    act = [x.copy() for x in data] + [np.full(size, 0x5A, np.uint8) for _ in range(p)]
    r.Encode(act)
    exp = _oracle_encode(orc, d, p, data)
    for j in range(p):
        assert np.array_equal(act[d + j], exp[j]), j


def test_rs_mul_kat_on_gpu(rslib, torch_dev):  # TestRS_mul rs_test.go:24-49
    r = rslib.New(5, 5)
    v = [np.array([x], np.uint8) for x in (0, 4, 2, 6, 8)] + [np.zeros(1, np.uint8) for _ in range(5)]
    r.Encode(v)
    assert [int(x[0]) for x in v[5:]] == [97, 173, 218, 107, 110]


# ---------------------------------------------------------------- Encode (device, batched)

def test_encode_batch_vs_oracle(rslib, orc, torch_dev):
    torch = torch_dev
    rng = np.random.default_rng(101)
    for d, p, S, n in [(10, 4, 64, 8192), (12, 4, 8, 65536), (10, 4, 3, 1000), (4, 2, 5, 48), (10, 4, 2, 1 << 20)]:
        r = rslib.New(d, p)
        host = _rand(rng, S, d + p, n)
        host[:, d:] = 0xA5
        buf = torch.from_numpy(host).cuda()
        r.encode_batch(buf)
        torch.cuda.synchronize()
        got = buf.cpu().numpy()
        exp = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), host[:, :d])
        assert np.array_equal(got[:, d:], exp), (d, p, S, n)
        assert np.array_equal(got[:, :d], host[:, :d])


def _check_every_stripe(orc, d, p, buf, batch=16):
    """Every stripe of a device batch [S, d+p, n] against the oracle's AVX2
    restatement of the reference's encode (orc.encode_avx2, pinned to the
    table path by tests/test_oracle.py), copied back `batch` stripes at a time."""
    S, n = buf.shape[0], buf.shape[2]
    for s0 in range(0, S, batch):
        host = buf[s0:s0 + batch].cpu().numpy()
        for k in range(host.shape[0]):
            v = [np.ascontiguousarray(host[k, i]) for i in range(d)] + [np.zeros(n, np.uint8) for _ in range(p)]
            orc.encode_avx2(d, p, v)
            for j in range(p):
                if not np.array_equal(host[k, d + j], v[d + j]):
                    raise AssertionError(("stripe", s0 + k, "parity", j, _first_diff(host[k, d + j], v[d + j])))


def test_encode_batch_full_size_round_trip(rslib, orc, torch_dev):
    """BASELINE config 2 at full size: 256 stripes x (10+4) x 1 MiB (3.5 GiB),
    every stripe against the oracle, then an erase / rebuild round trip and
    linearity."""
    torch = torch_dev
    d, p, S, n = 10, 4, 256, 1 << 20
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(0x5EED)
    buf = torch.randint(0, 256, (S, d + p, n), dtype=torch.uint8, device="cuda", generator=g)
    buf[:, d:] = 0xA5
    r.encode_batch(buf)
    torch.cuda.synchronize()
    _check_every_stripe(orc, d, p, buf)
    # erase 4 vectors of every stripe (two data, two parity), rebuild, compare
    ref = buf.clone()
    lost = [0, 7, 11, 13]
    buf[:, lost] = 0
    r.reconst_batch(buf, [], lost)
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    # linearity: parity(a ^ b) == parity(a) ^ parity(b) on a slice of stripes
    a = ref[:8].clone()
    b = torch.randint(0, 256, a.shape, dtype=torch.uint8, device="cuda", generator=g)
    c = a ^ b
    r.encode_batch(b)
    r.encode_batch(c)
    torch.cuda.synchronize()
    assert torch.equal(c[:, d:], a[:, d:] ^ b[:, d:])


def test_encode_12_4_full_size_every_stripe(rslib, orc, torch_dev):
    """BASELINE config 4 per GPU at full size: 256 stripes x (12+4) x 1 MiB
    (4 GiB), split layout as bench.py runs it, every stripe against the oracle."""
    torch = torch_dev
    d, p, S, n = 12, 4, 256, 1 << 20
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(0x5EED + 12)
    data = torch.randint(0, 256, (S, d, n), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.full((S, p, n), 0xA5, dtype=torch.uint8, device="cuda")
    r.encode_batch_split(data, parity)
    torch.cuda.synchronize()
    _check_every_stripe(orc, d, p, torch.cat([data, parity], dim=1))


def test_encode_dev_single_stripe(rslib, orc, torch_dev):
    torch = torch_dev
    d, p = 10, 4
    r = rslib.New(d, p)
    rng = np.random.default_rng(102)
    for size in (1, 15, 16, 17, 31, 33, 255, 1024, 8192, 100003):
        data = [_rand(rng, size) for _ in range(d)]
        vecs = [torch.from_numpy(x).cuda() for x in data] + [torch.full((size,), 7, dtype=torch.uint8,
                                                                          device="cuda") for _ in range(p)]
        r.encode_dev(vecs)
        torch.cuda.synchronize()
        exp = _oracle_encode(orc, d, p, data)
        for j in range(p):
            assert np.array_equal(vecs[d + j].cpu().numpy(), exp[j]), (size, j)


def test_vectors_over_2GiB(rslib, orc, torch_dev):
    """Vectors past the 2 GiB buffer-descriptor range take the global-load
    kernel (body >= 2^31) plus the byte kernel for the 37-byte tail; encode
    then rebuild a lost data vector (rs.go accepts any length >= 1)."""
    torch = torch_dev
    d, p, n = 2, 1, (1 << 31) + 37
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(77)
    vecs = [torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(d)]
    vecs.append(torch.full((n,), 7, dtype=torch.uint8, device="cuda"))
    r.encode_dev(vecs)
    torch.cuda.synchronize()
    for lo, hi in ((0, 4096), (1 << 30, (1 << 30) + 4096), ((1 << 31) - 4096, n)):
        data = [v[lo:hi].cpu().numpy() for v in vecs[:d]]
        exp = _oracle_encode(orc, d, p, data)
        assert np.array_equal(vecs[d][lo:hi].cpu().numpy(), exp[0]), (lo, hi)
    keep = vecs[0].clone()
    vecs[0].zero_()
    r.reconst_dev(vecs, [1, 2], [0])
    torch.cuda.synchronize()
    assert torch.equal(vecs[0], keep)
    del vecs, keep
    torch.cuda.empty_cache()


def test_unaligned_device_vectors(rslib, orc, torch_dev):
    """Go slices can start anywhere: odd offsets take the byte-granular kernel."""
    torch = torch_dev
    d, p = 10, 4
    r = rslib.New(d, p)
    rng = np.random.default_rng(103)
    for size in (1, 7, 16, 100, 4099):
        big = torch.from_numpy(_rand(rng, (d + p) * (size + 64) + 64)).cuda()
        vecs = [big[3 + i * (size + 37): 3 + i * (size + 37) + size] for i in range(d + p)]
        data = [v.cpu().numpy().copy() for v in vecs[:d]]
        r.encode_dev(vecs)
        torch.cuda.synchronize()
        exp = _oracle_encode(orc, d, p, data)
        for j in range(p):
            assert np.array_equal(vecs[d + j].cpu().numpy(), exp[j]), (size, j)
        for i in range(d):
            assert np.array_equal(vecs[i].cpu().numpy(), data[i])


# ---------------------------------------------------------------- Reconst

def _gen_idx(rng, d, p, survived_n, need_n):  # genIdxForTest helper_test.go:24-63
    survived_n = max(survived_n, d)
    need_n = min(need_n, p)
    if survived_n + need_n > d + p:
        survived_n = d
    need = rng.permutation(d + p)[:need_n].tolist()
    surv = []
    for i in rng.permutation(d + p).tolist():
        if len(surv) == survived_n:
            break
        if i not in need:
            surv.append(i)
    return sorted(surv), sorted(need)


def test_reconst_host_round_trip(rslib, orc, torch_dev):  # TestRS_Reconst rs_test.go:165-217
    d, p, size = 10, 4, 1024
    r = rslib.New(d, p)
    rng = np.random.default_rng(104)
    for _ in range(128):
        exp = [_rand(rng, size) for _ in range(d)] + [np.zeros(size, np.uint8) for _ in range(p)]
        r.Encode(exp)
        surv, need = _gen_idx(rng, d, p, int(rng.integers(d + p)), int(rng.integers(p + 1)))
        act = [np.zeros(size, np.uint8) for _ in range(d + p)]
        for i in surv:
            act[i][:] = exp[i]
        for n_ in need:
            if rng.integers(4) == 1:
                act[n_][:] = _rand(rng, size)
        ora = [x.copy() for x in act]
        r.Reconst(act, surv, need)
        assert orc.reconst(d, p, ora, surv, need) == 0
        for n_ in need:
            assert np.array_equal(act[n_], exp[n_])
        for i in range(d + p):  # every byte the oracle wrote, we wrote identically
            assert np.array_equal(act[i], ora[i])


def _oracle_stripes(orc, rng, d, p, S, n):
    """[S, d+p, n] host stripes: random data, parity from the oracle's AVX2
    restatement of the reference's encode (pinned to the table path by
    tests/test_oracle.py), one stripe at a time."""
    host = np.empty((S, d + p, n), np.uint8)
    host[:, :d] = rng.integers(0, 256, (S, d, n), dtype=np.uint8)
    host[:, d:] = 0
    for s in range(S):
        v = list(host[s])
        assert orc.encode_avx2(d, p, v) or orc.encode(d, p, v) == 0
    return host


def test_reconst_batch_every_pattern(rslib, orc, torch_dev):
    """All C(14,1..4) = 1470 erasure patterns of 10+4 @ 8 KiB (BASELINE
    config 3) over a 32,768-stripe batch (the ops_bench size): stripe s loses
    pattern s % 1470 (garbage in the lost vectors), one rs_reconst_batch
    launch per pattern over its strided stripe set; every byte of every
    stripe equals the oracle-encoded original, and the oracle's own Reconst
    (rs.go:221-380 restated) of every stripe gives the same bytes."""
    torch = torch_dev
    d, p, S, n = 10, 4, 32768, 8192
    rng = np.random.default_rng(263)
    r = rslib.New(d, p)
    host = _oracle_stripes(orc, rng, d, p, S, n)
    pats = [list(c) for k in range(1, p + 1) for c in itertools.combinations(range(d + p), k)]
    assert len(pats) == 14 + 91 + 364 + 1001
    work = torch.from_numpy(host).cuda()
    for i, lost in enumerate(pats):
        work[i::len(pats), lost] = 0x3C
    for i, lost in enumerate(pats):
        r.reconst_batch(work[i::len(pats)], [], lost)
    torch.cuda.synchronize()
    got = work.cpu().numpy()
    for s0 in range(0, S, 4096):
        assert np.array_equal(got[s0:s0 + 4096], host[s0:s0 + 4096]), s0
    for s in range(S):  # the restated reference, per stripe
        lost = pats[s % len(pats)]
        v = [x.copy() for x in host[s]]
        for i in lost:
            v[i][:] = 0x3C
        assert orc.reconst(d, p, v, [], lost) == 0
        assert all(np.array_equal(v[i], got[s, i]) for i in lost), s


def test_first_sight_tables_in_place(rslib, orc, torch_dev):
    """A matrix's first use in a small launch reads its perm tables in place
    from the mapped staging slot (no upload); its second use uploads them;
    a large launch uploads at first sight; table_inplace_max 0 always
    uploads.  Eight new patterns back to back on one stream with no sync in
    between reuse the four staging slots (each waits for the launch that read
    it).  Every rebuilt stripe equals the oracle's Reconst (rs.go:221-380)."""
    torch = torch_dev
    L = rslib.lib()
    d, p, S, n = 10, 4, 16, 8192
    r = rslib.New(d, p)
    rng = np.random.default_rng(77)
    host = _rand(rng, S, d + p, n)
    for s in range(S):
        v = [x for x in host[s]]
        assert orc.encode(d, p, v) == 0
    buf = torch.from_numpy(host.copy()).cuda()
    pats = [[0], [1, 12], [2, 5, 11], [3, 4, 6, 13], [7], [8, 9], [0, 10], [1, 2, 3], [5, 6]]

    def rebuild(lost, sync=True, b=None, h=None):
        b = buf if b is None else b
        for v in lost:
            b[:, v] = 0x77
        r.reconst_batch(b, [], lost)
        if sync:
            torch.cuda.synchronize()
            assert torch.equal(b.cpu(), torch.from_numpy(host if h is None else h)), lost

    up0, ip0 = r.coef_table_stats()
    rebuild(pats[0])
    up1, ip1 = r.coef_table_stats()
    assert (up1 - up0, ip1 - ip0) == (0, 1)  # first sight: in place
    rebuild(pats[0])
    up2, ip2 = r.coef_table_stats()
    assert (up2 - up1, ip2 - ip1) == (1, 0)  # second sight: uploaded
    rebuild(pats[0])
    assert r.coef_table_stats() == (up2, ip2)  # registry hit
    for lost in pats[1:]:  # 8 new patterns, no sync between them: slots reused behind their launches
        rebuild(lost, sync=False)
    torch.cuda.synchronize()
    assert torch.equal(buf.cpu(), torch.from_numpy(host))
    up3, ip3 = r.coef_table_stats()
    assert (up3 - up2, ip3 - ip2) == (0, 8)
    # a large launch (> table_inplace_max input bytes) uploads at first sight
    big_h = np.concatenate([host] * 2, axis=2)  # 16 KiB vectors: 16 x 10 x 16 KiB = 2.5 MiB of input
    big = torch.from_numpy(big_h.copy()).cuda()
    rebuild([4, 9], b=big, h=big_h)
    assert r.coef_table_stats() == (up3 + 1, ip3)
    assert L.rs_tune(b"table_inplace_max", 0) == 0
    try:
        rebuild([6, 11])
        assert r.coef_table_stats() == (up3 + 2, ip3)
    finally:
        L.rs_tune(b"table_inplace_max", 2 << 20)
    # the oracle rebuilds the same stripe from the same survivors
    v = [x.copy() for x in host[3]]
    for i in (2, 5, 11):
        v[i][:] = 0
    assert orc.reconst(d, p, v, [], [2, 5, 11]) == 0
    assert all(np.array_equal(v[i], host[3, i]) for i in range(d + p))


def test_reconst_dev_and_explicit_survived(rslib, orc, torch_dev):
    torch = torch_dev
    d, p, size = 10, 4, 8192 + 5
    r = rslib.New(d, p)
    rng = np.random.default_rng(105)
    for _ in range(32):
        exp = [_rand(rng, size) for _ in range(d)] + [np.zeros(size, np.uint8) for _ in range(p)]
        r.Encode(exp)
        surv, need = _gen_idx(rng, d, p, int(rng.integers(d + p)), int(rng.integers(1, p + 1)))
        vecs = [torch.from_numpy(x.copy()).cuda() for x in exp]
        for n_ in need:
            vecs[n_].fill_(0)
        r.reconst_dev(vecs, surv, need)
        torch.cuda.synchronize()
        for n_ in need:
            assert np.array_equal(vecs[n_].cpu().numpy(), exp[n_])


def test_reconst_too_many_lost(rslib, torch_dev):
    r = rslib.New(10, 4)
    v = [np.zeros(64, np.uint8) for _ in range(14)]
    with pytest.raises(rslib.ErrTooManyLost):
        r.Reconst(v, [], [0, 1, 2, 3, 4])


# ---------------------------------------------------------------- Update / Replace

def test_update_every_row(rslib, orc, torch_dev):  # TestRS_Update rs_test.go:219-266
    torch = torch_dev
    d, p, size = 10, 4, 1024 + 3
    rng = np.random.default_rng(106)
    r = rslib.New(d, p)
    for row in range(d):
        exp = [_rand(rng, size) for _ in range(d)] + [np.zeros(size, np.uint8) for _ in range(p)]
        act = [x.copy() for x in exp]
        r.Encode(act)
        new = _rand(rng, size)
        ora = [x.copy() for x in act]
        r.Update(act[row], new, row, act[d:])
        assert orc.update(d, p, ora[row], new, row, ora[d:]) == 0
        exp[row] = new.copy()
        r.Encode(exp)
        for j in range(d, d + p):
            assert np.array_equal(act[j], exp[j])
            assert np.array_equal(act[j], ora[j])
        # device single-stripe variant
        dv = [torch.from_numpy(x.copy()).cuda() for x in ora]
        dv_old = torch.from_numpy(exp[row].copy()).cuda()
        dv_new = torch.from_numpy(_rand(rng, size)).cuda()
        r.update_dev(dv_old, dv_new, row, dv[d:])
        torch.cuda.synchronize()
        exp2 = [x.copy() for x in exp]
        exp2[row] = dv_new.cpu().numpy()
        r.Encode(exp2)
        for j in range(p):
            assert np.array_equal(dv[d + j].cpu().numpy(), exp2[d + j])


@pytest.mark.parametrize("S,rows", [(32768, [3]), (4096, list(range(10)))])
def test_update_batch(rslib, orc, torch_dev, S, rows):
    """rs_update_batch (BASELINE config 5, 10+4 @ 8 KiB) at the ops_bench batch
    size for one row and on 4,096 stripes for every row; every stripe's parity
    equals the oracle's Update (rs.go:424-449 restated)."""
    torch = torch_dev
    d, p, n = 10, 4, 8192
    rng = np.random.default_rng(343 + S)
    r = rslib.New(d, p)
    host = _oracle_stripes(orc, rng, d, p, S, n)
    buf = torch.from_numpy(host).cuda()
    for row in rows:
        new = rng.integers(0, 256, (S, n), dtype=np.uint8)
        r.update_batch(buf[:, row].clone(), torch.from_numpy(new).cuda(), row, buf)
        torch.cuda.synchronize()
        got = buf[:, d:].cpu().numpy()
        for s in range(S):
            par = list(host[s, d:])
            assert orc.update(d, p, host[s, row], new[s], row, par) == 0
            assert all(np.array_equal(got[s, j], par[j]) for j in range(p)), (row, s)
        host[:, row] = new
        buf[:, row] = torch.from_numpy(new).cuda()


def _replace_rows(rng, d):  # makeReplaceRowRandom rs_test.go:333-353
    n = int(rng.integers(d + 1))
    s = []
    while len(s) < n:
        v = int(rng.integers(d))
        if v not in s:
            s.append(v)
    return s or [0]


@pytest.mark.parametrize("to_zero", [True, False])
def test_replace_host(rslib, orc, torch_dev, to_zero):  # TestRS_Replace rs_test.go:268-331
    d, p, size = 10, 4, 1024
    rng = np.random.default_rng(107 + to_zero)
    r = rslib.New(d, p)
    for _ in range(128):
        rows = _replace_rows(rng, d)
        exp = [_rand(rng, size) for _ in range(d)] + [np.zeros(size, np.uint8) for _ in range(p)]
        act = [x.copy() for x in exp]
        data = [exp[rr].copy() for rr in rows]
        if to_zero:
            for rr in rows:
                exp[rr] = np.zeros(size, np.uint8)
        r.Encode(exp)
        if not to_zero:
            for rr in rows:
                act[rr] = np.zeros(size, np.uint8)
        r.Encode(act)
        ora = [x.copy() for x in act[d:]]
        r.Replace(data, rows, act[d:])
        assert orc.replace(d, p, data, rows, ora) == 0
        for j in range(p):
            assert np.array_equal(act[d + j], exp[d + j])
            assert np.array_equal(act[d + j], ora[j])


@pytest.mark.parametrize("S,rns", [(32768, [3]), (4096, [1, 2, 3, 4, 5, 6])])
def test_replace_batch_1_to_6_rows(rslib, orc, torch_dev, S, rns):  # BASELINE config 5 (rn = 1..6)
    """rs_replace_batch with 1-6 replaced rows (rs.go:492-529) at the
    ops_bench batch size (rn = 3) and on 4,096 stripes for rn = 1..6: every
    stripe's parity equals the oracle's Replace of the same rows."""
    torch = torch_dev
    d, p, n = 10, 4, 8192
    rng = np.random.default_rng(397 + S)
    r = rslib.New(d, p)
    host = _oracle_stripes(orc, rng, d, p, S, n)
    for rn in rns:
        rows = sorted(int(x) for x in rng.choice(d, rn, replace=False))
        data = rng.integers(0, 256, (S, rn, n), dtype=np.uint8)
        buf = torch.from_numpy(host).cuda()
        r.replace_batch(torch.from_numpy(data).cuda(), rows, buf)
        torch.cuda.synchronize()
        got = buf[:, d:].cpu().numpy()
        del buf
        for s in range(S):
            par = [x.copy() for x in host[s, d:]]
            assert orc.replace(d, p, list(data[s]), rows, par) == 0
            assert all(np.array_equal(got[s, j], par[j]) for j in range(p)), (rn, s)


def test_replace_dev(rslib, torch_dev):
    torch = torch_dev
    d, p, n = 10, 4, 4096 + 9
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(10)
    full = torch.randint(0, 256, (d + p, n), dtype=torch.uint8, device="cuda", generator=g)
    vec = [full[i].contiguous() for i in range(d + p)]
    r.encode_dev(vec)
    rows = [2, 5, 9]
    zero = [v.clone() for v in vec]
    for rr in rows:
        zero[rr].zero_()
    r.encode_dev(zero)
    r.replace_dev([vec[rr] for rr in rows], rows, zero[d:])
    torch.cuda.synchronize()
    for j in range(d, d + p):
        assert torch.equal(zero[j], vec[j])


# ---------------------------------------------------------------- generic product

@pytest.mark.parametrize("rows,cols,acc", [(1, 1, False), (3, 7, True), (9, 5, False), (20, 33, True),
                                           (4, 10, False), (2, 2, True), (8, 3, False)])
def test_gf_matmul_batch(rslib, orc, torch_dev, rows, cols, acc):
    torch = torch_dev
    rng = np.random.default_rng(rows * 100 + cols)
    S, n = 3, 5000
    mat = _rand(rng, rows, cols)
    src = _rand(rng, S, cols, n)
    dst0 = _rand(rng, S, rows, n)
    r = rslib.New(10, 4)
    dsrc = torch.from_numpy(src).cuda()
    ddst = torch.from_numpy(dst0.copy()).cuda()
    r.gf_matmul_batch(mat, dsrc, None, ddst, None, accumulate=acc)
    torch.cuda.synchronize()
    exp = orc.encode_numpy(mat, src)
    if acc:
        exp ^= dst0
    assert np.array_equal(ddst.cpu().numpy(), exp)


def test_table_registry_recycling_under_threads(rslib, orc, torch_dev):
    """The per-handle table registry is recycled (device sync + free) when
    full; with a cap of 3 and 4 threads launching 12 distinct matrices each,
    every product must still be right (no table freed under a launch)."""
    torch = torch_dev
    L = rslib.lib()
    assert L.rs_tune(b"table_registry_max", 3) == 0
    try:
        r = rslib.New(10, 4)
        errors = []

        def worker(t):
            try:
                rng = np.random.default_rng(900 + t)
                for i in range(12):
                    mat = _rand(rng, 3, 5)
                    src = _rand(rng, 2, 5, 4096)
                    dsrc = torch.from_numpy(src).cuda()
                    ddst = torch.zeros((2, 3, 4096), dtype=torch.uint8, device="cuda")
                    st = torch.cuda.Stream()
                    with torch.cuda.stream(st):
                        r.gf_matmul_batch(mat, dsrc, None, ddst, None, stream=st)
                    st.synchronize()
                    if not np.array_equal(ddst.cpu().numpy(), orc.encode_numpy(mat, src)):
                        errors.append((t, i))
            except Exception as e:  # pragma: no cover
                errors.append(repr(e))

        ts = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors, errors
    finally:
        assert L.rs_tune(b"table_registry_max", 1 << 14) == 0


def test_concurrent_host_calls(rslib, orc, torch_dev):
    """*RS is safe for concurrent use (rs.go: immutable but for the cache)."""
    d, p, size = 10, 4, 20000
    r = rslib.New(d, p)
    errors = []

    def worker(seed):
        try:
            rng = np.random.default_rng(seed)
            for _ in range(10):
                data = [_rand(rng, size) for _ in range(d)]
                v = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                r.Encode(v)
                exp = _oracle_encode(orc, d, p, data)
                for j in range(p):
                    if not np.array_equal(v[d + j], exp[j]):
                        errors.append((seed, j))
                lost = sorted(rng.choice(d + p, 3, replace=False).tolist())
                w = [x.copy() for x in v]
                for i in lost:
                    w[i][:] = 0
                r.Reconst(w, [], lost)
                for i in lost:
                    if not np.array_equal(w[i], v[i]):
                        errors.append((seed, "reconst", i))
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(s,)) for s in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors


@pytest.mark.parametrize("direct", [0, 1])
def test_coalesced_host_calls(rslib, orc, torch_dev, direct):
    """Concurrent host calls of several shapes (Encode at two sizes, Update,
    Replace, Reconst) from 16 threads; every result must equal the oracle's
    for that call alone.  direct=0: they share coalesced launches; direct=1
    (the default): each rings the resident engine itself, many in flight."""
    d, p = 10, 4
    r = rslib.New(d, p)
    errors = []
    barrier = threading.Barrier(16)
    L = rslib.lib()
    # a 2 ms group-commit window: concurrent calls reliably share launches
    # even when Python threads arrive staggered (GIL)
    assert L.rs_tune(b"host_coalesce_linger_us", 2000) == 0
    assert L.rs_tune(b"host_engine_direct", direct) == 0

    def worker(t):
        try:
            rng = np.random.default_rng(1000 + t)
            size = 8192 if t % 2 == 0 else 8197
            barrier.wait()
            for it in range(12):
                data = [_rand(rng, size) for _ in range(d)]
                v = [x.copy() for x in data] + [np.full(size, 0xA5, np.uint8) for _ in range(p)]
                r.Encode(v)
                exp = _oracle_encode(orc, d, p, data)
                if any(not np.array_equal(v[d + j], exp[j]) for j in range(p)):
                    errors.append((t, it, "encode"))
                if t % 4 == 1:  # Update one row
                    row = (t + it) % d
                    new = _rand(rng, size)
                    par = [x.copy() for x in v[d:]]
                    r.Update(v[row], new, row, par)
                    data2 = [x.copy() for x in data]
                    data2[row] = new
                    exp2 = _oracle_encode(orc, d, p, data2)
                    if any(not np.array_equal(par[j], exp2[j]) for j in range(p)):
                        errors.append((t, it, "update"))
                elif t % 4 == 3:  # Replace rows 2, 5 from zero
                    zdata = [x.copy() for x in data]
                    zdata[2][:] = 0
                    zdata[5][:] = 0
                    par = _oracle_encode(orc, d, p, zdata)
                    r.Replace([data[2], data[5]], [2, 5], par)
                    if any(not np.array_equal(par[j], exp[j]) for j in range(p)):
                        errors.append((t, it, "replace"))
                lost = [0, 11] if t % 3 else [3, 7, 12]
                w = [x.copy() for x in v]
                for i in lost:
                    w[i][:] = 0
                r.Reconst(w, [], lost)
                if any(not np.array_equal(w[i], v[i]) for i in lost):
                    errors.append((t, it, "reconst"))
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    # (a call after a quiet period would take the launch path, i.e. the
    # coalescer this test counts: keep every call on its path)
    assert L.rs_tune(b"host_engine_cold_launch", 0) == 0
    try:
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    finally:
        assert L.rs_tune(b"host_coalesce_linger_us", 0) == 0
        assert L.rs_tune(b"host_engine_direct", 1) == 0
        assert L.rs_tune(b"host_engine_cold_launch", 1) == 0
    assert not errors, errors[:10]
    launches, calls = r.host_call_stats()
    if direct:
        ecalls, _ = r.host_engine_stats()
        assert ecalls >= 16 * 12 * 2, ecalls  # every Encode and Reconst rang the engine
        assert calls == 0, calls
    else:
        assert calls >= 16 * 12 * 2  # every Encode and Reconst went through the coalescer
        assert launches < calls, (launches, calls)  # concurrent calls shared launches


def test_host_calls_on_registered_memory(rslib, orc, torch_dev):
    """Host calls whose vectors all lie in rs_host_register'ed memory run the
    kernel straight over them; a vector outside it (or misaligned) takes the
    staged path.  Results equal the oracle's either way."""
    d, p = 10, 4
    r = rslib.New(d, p)
    rng = np.random.default_rng(404)
    for size in (4096, 65536, 1 << 20, 1000):
        pitch = (size + 4095) // 4096 * 4096
        arena = np.zeros((d + p + 1) * pitch + 4096, np.uint8)  # an ordinary heap array
        off = (-arena.ctypes.data) % 4096
        base = arena[off: off + (d + p + 1) * pitch]
        rslib.host_register(base.ctypes.data, base.nbytes)
        try:
            v = [base[i * pitch: i * pitch + size] for i in range(d + p)]
            data = [_rand(rng, size) for _ in range(d)]
            for i in range(d):
                v[i][:] = data[i]
            r.Encode(v)
            exp = _oracle_encode(orc, d, p, data)
            for j in range(p):
                assert np.array_equal(v[d + j], exp[j]), (size, j)
            keep = [x.copy() for x in v]
            for i in (1, 12):
                v[i][:] = 0
            r.Reconst(v, [], [1, 12])
            for i in (1, 12):
                assert np.array_equal(v[i], keep[i]), (size, i)
            new = _rand(rng, size)
            r.Update(v[4], new, 4, v[d:])
            data[4] = new
            v[4][:] = new
            exp = _oracle_encode(orc, d, p, data)
            for j in range(p):
                assert np.array_equal(v[d + j], exp[j]), (size, "update", j)
            # one vector outside the registered range: staged path, same bytes
            mixed = v[:d] + [np.zeros(size, np.uint8)] + v[d + 1:]
            r.Encode(mixed)
            assert np.array_equal(mixed[d], exp[0]), (size, "mixed")
        finally:
            rslib.host_unregister(base.ctypes.data)
        assert hip_ptr.known_pages(base.ctypes.data, base.ctypes.data + base.nbytes) == [], size
        del v, base, arena  # freed: its addresses go back to the heap


def test_encode_host_batch_pipeline(rslib, orc, torch_dev):
    """Host-resident stripes: pinned and pageable, ragged chunking."""
    torch = torch_dev
    d, p = 10, 4
    r = rslib.New(d, p)
    rng = np.random.default_rng(108)
    for S, n, spc, st in ((7, 8192 + 3, 3, 2), (20, 65536, 8, 3), (1, 100, 8, 3)):
        host = _rand(rng, S, d + p, n)
        exp = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), host[:, :d])
        a = host.copy()
        r.encode_host_batch(a, spc, st)  # pageable: staged through the pinned mirror
        assert np.array_equal(a[:, d:], exp), ("pageable parity", S, n, _first_diff(a[:, d:], exp))
        assert np.array_equal(a[:, :d], host[:, :d]), ("pageable data", S, n)
        L = rslib.lib()
        assert L.rs_tune(b"host_pageable_stage", 0) == 0
        try:
            a = host.copy()
            r.encode_host_batch(a, spc, st)  # pageable: DMA pipeline, 1-D copies
            assert np.array_equal(a[:, d:], exp), ("pageable DMA parity", S, n, _first_diff(a[:, d:], exp))
            assert np.array_equal(a[:, :d], host[:, :d]), ("pageable DMA data", S, n)
        finally:
            L.rs_tune(b"host_pageable_stage", 1)
        pinned = torch.from_numpy(host.copy()).pin_memory()
        r.encode_host_batch(pinned, spc, st)  # zero-copy: kernels straight over pinned memory
        got = pinned.numpy()[:, d:]
        assert np.array_equal(got, exp), ("zero-copy parity", S, n, _first_diff(got, exp))
        assert L.rs_tune(b"host_batch_zc", 0) == 0
        try:
            pinned = torch.from_numpy(host.copy()).pin_memory()
            r.encode_host_batch(pinned, spc, st)  # DMA pipeline over pinned memory
            got = pinned.numpy()[:, d:]
            assert np.array_equal(got, exp), ("pinned DMA parity", S, n, _first_diff(got, exp))
        finally:
            L.rs_tune(b"host_batch_zc", 1)


def test_host_batch_zero_copy(rslib, orc, torch_dev):
    """Zero-copy host batches: registered numpy memory (rs_host_register),
    multi-pattern Reconst in place on pinned and on pageable memory (single
    and group), mask validation before any copy, and a clean RS_ERR_INVAL (no
    kernel) for pageable memory with staging off."""
    torch = torch_dev
    d, p, S, n = 10, 4, 33, 8192 + 16
    r = rslib.New(d, p)
    rng = np.random.default_rng(122)
    host = _rand(rng, S, d + p, n)
    exp = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), host[:, :d])
    # registered pageable numpy heap buffer -> device-mapped, freed afterwards
    reg = host.copy()
    rslib.host_register(reg.ctypes.data, reg.nbytes)
    try:
        dp = rslib.host_device_pointer(reg.ctypes.data, reg.nbytes)
        assert dp != 0
        r.encode_host_batch(reg)
        assert np.array_equal(reg[:, d:], exp)
    finally:
        rslib.host_unregister(reg.ctypes.data)
    assert hip_ptr.known_pages(reg.ctypes.data, reg.ctypes.data + reg.nbytes) == []
    del reg
    full = host.copy()
    full[:, d:] = exp
    masks = np.zeros(S, np.uint64)
    for s in range(S):
        for v in rng.choice(d + p, int(rng.integers(0, p + 1)), replace=False):
            masks[s] |= np.uint64(1) << np.uint64(int(v))
    broken = full.copy()
    for s in range(S):
        for v in range(d + p):
            if int(masks[s]) >> v & 1:
                broken[s, v] = 0xEE
    pinned = torch.from_numpy(broken.copy()).pin_memory()
    r.reconst_host_batch_multi(pinned, masks)
    assert np.array_equal(pinned.numpy(), full)
    pinned = torch.from_numpy(broken.copy()).pin_memory()
    rslib.NewGroup(d, p, [0, 0]).reconst_host_batch_multi(pinned, masks)
    assert np.array_equal(pinned.numpy(), full)
    # pageable memory: staged through the pinned mirror (single and group)
    pageable = broken.copy()
    r.reconst_host_batch_multi(pageable, masks)
    assert np.array_equal(pageable, full)
    pageable = broken.copy()
    rslib.NewGroup(d, p, [0, 0]).reconst_host_batch_multi(pageable, masks)
    assert np.array_equal(pageable, full)
    # a 5-erasure stripe is rejected before anything is copied or launched
    bad = masks.copy()
    bad[S - 1] = np.uint64(0b11111)
    pageable = broken.copy()
    with pytest.raises(rslib.ErrTooManyLost):
        r.reconst_host_batch_multi(pageable, bad)
    assert np.array_equal(pageable, broken)
    # staging off: a clean RS_ERR_INVAL (no kernel) for pageable memory
    L = rslib.lib()
    assert L.rs_tune(b"host_pageable_stage", 0) == 0
    try:
        with pytest.raises(rslib.ErrInvalidArgument):
            r.reconst_host_batch_multi(pageable, masks)
    finally:
        L.rs_tune(b"host_pageable_stage", 1)
    with pytest.raises(rslib.ErrInvalidArgument):
        rslib.host_device_pointer(pageable.ctypes.data, pageable.nbytes)
    assert np.array_equal(pageable, broken)


def test_host_batch_large_pageable_stripes(rslib, orc, torch_dev):
    """Pageable host batches whose stripes exceed one mirror slot (16 MiB):
    10+4 with 2 MiB + 40 byte vectors (a 28 MiB stripe) and 4+2 with 3 MiB +
    3 bytes, interleaved [S][d+p][len] and with a gap between vectors, are
    staged through the pinned mirror in byte windows of every vector (Encode
    and multi-pattern Reconst, rs.go:104-203 / 221-380): bytes equal the
    oracle's, and no page of the caller's buffer was ever GPU-mapped (KFD
    SVM access stays no-access: the runtime's pageable copies, which map the
    source in place, were not used)."""
    rng = np.random.default_rng(2048)
    for d, p, S, n, gap in ((10, 4, 2, (2 << 20) + 40, 0), (4, 2, 3, (3 << 20) + 3, 4096 + 5)):
        r = rslib.New(d, p)
        vs = n + gap
        buf = np.zeros(S * (d + p) * vs + 64, np.uint8)  # an ordinary heap array
        view = np.lib.stride_tricks.as_strided(buf[64:], shape=(S, d + p, n), strides=((d + p) * vs, vs, 1))
        host = rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)
        view[:] = host
        view[:, d:] = 0xA5
        lo, hi = buf.ctypes.data, buf.ctypes.data + buf.nbytes
        probe = ((lo + 4095) & ~4095) + 4096
        # (a fresh mapping at an address an earlier test's pageable copy used
        # can report in-place already: start from no-access explicitly)
        svm = hip_ptr.gpu_access(probe) != "unknown"  # (the SVM API exists on the box)
        if svm:
            assert hip_ptr.gpu_revoke(lo, hi) and hip_ptr.gpu_access(probe) == "no-access"
        r.encode_host_batch(view)
        exp = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), host[:, :d])
        assert np.array_equal(view[:, d:], exp), (d, p, n, _first_diff(view[:, d:], exp))
        assert np.array_equal(view[:, :d], host[:, :d])
        full = np.concatenate([host[:, :d], exp], axis=1)
        masks = np.zeros(S, np.uint64)
        for s_ in range(S):
            for v in rng.choice(d + p, int(rng.integers(1, p + 1)), replace=False):
                masks[s_] |= np.uint64(1) << np.uint64(int(v))
                view[s_, int(v)] = 0xEE
        r.reconst_host_batch_multi(view, masks)
        assert np.array_equal(view, full), (d, p, n, _first_diff(view, full))
        if svm:
            assert hip_ptr.gpu_mapped_pages(lo, hi) == [], "pageable buffer was handed to the runtime"
        del view, buf


def test_split_layout_encode_reconst(rslib, orc, torch_dev):
    """Data and parity in separate buffers (rs_layout_t)."""
    torch = torch_dev
    d, p, S, n = 10, 4, 6, 8192 + 48
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(11)
    data = torch.randint(0, 256, (S, d, n), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.full((S, p, n), 0xA5, dtype=torch.uint8, device="cuda")
    r.encode_batch_split(data, parity)
    torch.cuda.synchronize()
    exp = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), data.cpu().numpy())
    assert np.array_equal(parity.cpu().numpy(), exp)
    ref_d, ref_p = data.clone(), parity.clone()
    for lost in ([0], [3, 12], [1, 2, 10, 13], [11], [0, 9, 10, 11]):
        data.copy_(ref_d)
        parity.copy_(ref_p)
        for v in lost:
            (data[:, v] if v < d else parity[:, v - d]).fill_(0x77)
        r.reconst_batch_split(data, parity, [], lost)
        torch.cuda.synchronize()
        assert torch.equal(data, ref_d) and torch.equal(parity, ref_p), lost


def test_update_batch_distinct_strides(rslib, torch_dev):
    torch = torch_dev
    d, p, S, n = 10, 4, 5, 4096
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(12)
    buf = torch.randint(0, 256, (S, d + p, n), dtype=torch.uint8, device="cuda", generator=g)
    r.encode_batch(buf)
    old = buf[:, 4].clone()                                   # stride n
    new_big = torch.randint(0, 256, (S, 3, n), dtype=torch.uint8, device="cuda", generator=g)
    new = new_big[:, 1]                                       # stride 3n
    r.update_batch(old, new, 4, buf)
    buf[:, 4] = new
    exp = buf.clone()
    r.encode_batch(exp)
    torch.cuda.synchronize()
    assert torch.equal(buf, exp)


def test_reconst_batch_multi_pattern(rslib, torch_dev):
    """Every stripe with its own erasure set, incl. a ragged tail."""
    torch = torch_dev
    d, p, S, n = 10, 4, 96, 8192 + 5
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(13)
    buf = torch.randint(0, 256, (S, d + p, n), dtype=torch.uint8, device="cuda", generator=g)
    r.encode_batch(buf)
    ref = buf.clone()
    rng = np.random.default_rng(109)
    masks = np.zeros(S, np.uint64)
    for s in range(S):
        k = int(rng.integers(0, p + 1))  # 0 = stripe untouched
        lost = rng.choice(d + p, k, replace=False)
        for v in lost:
            masks[s] |= np.uint64(1) << np.uint64(int(v))
            buf[s, int(v)] = 0x5C
    r.reconst_batch_multi(buf[:, :d], buf[:, d:], masks)
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    # a pattern beyond p erasures is rejected before anything runs
    bad = masks.copy()
    bad[3] = np.uint64(0b11111)
    work = ref.clone()
    with pytest.raises(rslib.ErrTooManyLost):
        r.reconst_batch_multi(work[:, :d], work[:, d:], bad)
    torch.cuda.synchronize()
    assert torch.equal(work, ref)


def test_xor_batch(rslib, torch_dev):
    """xorsimd xor.Encode restated on the device."""
    torch = torch_dev
    r = rslib.New(10, 4)
    g = torch.Generator(device="cuda").manual_seed(14)
    for S, n, L in ((1, 2, 1), (7, 3, 1000), (64, 5, 8192), (4, 16, 65536 + 7)):
        src = torch.randint(0, 256, (S, n, L), dtype=torch.uint8, device="cuda", generator=g)
        dst = torch.full((S, L), 0x33, dtype=torch.uint8, device="cuda")
        r.xor_batch(src, dst)
        exp = src[:, 0].clone()
        for i in range(1, n):
            exp ^= src[:, i]
        torch.cuda.synchronize()
        assert torch.equal(dst, exp), (S, n, L)


@pytest.mark.parametrize("d,p,n", [(10, 4, 8192), (6, 3, 4096), (10, 4, 65536), (8, 6, 4096), (3, 2, 16)])
def test_reconst_batch_multi_single_launch(rslib, torch_dev, d, p, n):
    """Aligned lengths take the single-launch pattern kernel (nout <= 8: 8+6's
    patterns of 5-6 outputs too, in the image with 8 rows per column)."""
    torch = torch_dev
    S = 200
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(d * 100 + p)
    data = torch.randint(0, 256, (S, d, n), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((S, p, n), dtype=torch.uint8, device="cuda")
    r.encode_batch_split(data, parity)
    ref_d, ref_p = data.clone(), parity.clone()
    rng = np.random.default_rng(d + p)
    masks = np.zeros(S, np.uint64)
    for s in range(S):
        lost = rng.choice(d + p, int(rng.integers(0, p + 1)), replace=False)
        for v in lost:
            v = int(v)
            masks[s] |= np.uint64(1) << np.uint64(v)
            (data[s, v] if v < d else parity[s, v - d]).fill_(0xE7)
    r.reconst_batch_multi(data, parity, masks)
    torch.cuda.synchronize()
    assert torch.equal(data, ref_d) and torch.equal(parity, ref_p)


def _distinct_patterns(d, p, count, seed, kmax=4):
    """`count` distinct need masks of 1-kmax erasures (every one of them when
    count is the number that exists), as Python ints."""
    from itertools import combinations
    from math import comb

    n = d + p
    kmax = min(kmax, p)
    total = sum(comb(n, k) for k in range(1, kmax + 1))
    if count >= total:
        return [sum(1 << v for v in c) for k in range(1, kmax + 1) for c in combinations(range(n), k)]
    rng = np.random.default_rng(seed)
    seen, out = set(), []
    while len(out) < count:
        lost = rng.choice(n, int(rng.integers(1, kmax + 1)), replace=False)
        m = sum(1 << int(v) for v in lost)
        if m not in seen:
            seen.add(m)
            out.append(m)
    return out


@pytest.mark.parametrize("d,p,n,npat,kmax", [(10, 4, 8192, 1470, 4), (100, 28, 4096, 300, 4), (6, 3, 16, 129, 4),
                                             (32, 32, 1024, 512, 4), (60, 4, 2048, 9, 4), (10, 8, 4096, 800, 8),
                                             (20, 12, 1024, 600, 8), (40, 30, 2048 + 16, 100, 8), (8, 6, 64, 6475, 6)])
def test_reconst_batch_multi_gpu_planner(rslib, orc, torch_dev, d, p, n, npat, kmax):
    """rs_tune("multi_gpu_plan", n): a batch with at least n distinct erasure
    patterns has its pattern tables and descriptors built on the GPU
    (gf_plan_multi, kernels.hip: the lost data from a dn x dn inverse) instead
    of by the host (the d x d inverse, combined_matrix).  Every pattern of 1-4
    erasures (10+4: all 1,470 of C(14, 1..4), one stripe each; 100+28: 256-bit
    masks reaching past bit 64), and patterns of up to 8 (10+8, 20+12, 40+30;
    8+6: all 6,475 of C(14, 1..6)) in the one launch whose tables hold 8 rows,
    rebuilt bit-exact through both planners, stripes shuffled, a few stripes
    untouched.  A sample of the stripes of every shape (patterns of every
    erasure count, and masks past bit 64 for 100+28) is also rebuilt by the
    oracle from the same survivors (orc.reconst: rs.go:327-373 restated) and
    must equal the GPU planner's bytes, so the planner is pinned to the
    oracle, not only to the HIP encoder's round trip."""
    torch = torch_dev
    L = rslib.lib()
    pats = _distinct_patterns(d, p, npat, d * 1000 + p, kmax)
    assert len(pats) == npat
    S = npat + 3
    rng = np.random.default_rng(npat)
    order = rng.permutation(S)
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(d * 37 + p)
    data = torch.randint(0, 256, (S, d, n), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((S, p, n), dtype=torch.uint8, device="cuda")
    r.encode_batch_split(data, parity)
    torch.cuda.synchronize()
    ref_d, ref_p = data.clone(), parity.clone()
    masks = [0] * S
    for i, m in enumerate(pats):
        masks[int(order[i])] = m   # (the 3 stripes past the patterns stay untouched)
    arg = masks if d + p > 64 else np.array(masks, dtype=np.uint64)
    sample = _planner_sample(pats, order, d + p)
    try:
        for plan in (1, 0):
            assert L.rs_tune(b"multi_gpu_plan", plan) == 0
            for s, m in enumerate(masks):
                for v in range(d + p):
                    if m >> v & 1:
                        (data[s, v] if v < d else parity[s, v - d]).fill_(0x5A)
            broken = _host_stripes(data, parity, sample) if plan == 1 else None
            r.reconst_batch_multi(data, parity, arg)
            torch.cuda.synchronize()
            bad = [s for s in range(S) if not (torch.equal(data[s], ref_d[s]) and torch.equal(parity[s], ref_p[s]))]
            assert not bad, (plan, bad[:5], [bin(masks[s]) for s in bad[:5]])
            if plan == 1:
                _oracle_rebuilds_sample(orc, d, p, broken, masks, data, parity, sample)
    finally:
        L.rs_tune(b"multi_gpu_plan", -1)


def _planner_sample(pats, order, nvec, k=48):
    """Stripes (indexes) of up to k patterns spread over the pattern list (the
    exhaustive lists run by erasure count, so every count is hit), plus up to
    8 whose masks reach past bit 63 when the code is that wide."""
    idx = sorted(set(np.linspace(0, len(pats) - 1, min(len(pats), k)).astype(int).tolist()))
    if nvec > 64:
        idx += [i for i, m in enumerate(pats) if m >> 64][:8]
    return sorted({int(order[i]) for i in idx})


def _host_stripes(data, parity, stripes):
    return {s: ([x.copy() for x in data[s].cpu().numpy()], [x.copy() for x in parity[s].cpu().numpy()])
            for s in stripes}


def _oracle_rebuilds_sample(orc, d, p, broken, masks, data, parity, sample):
    """The oracle rebuilds each sampled stripe from the same survivors the
    GPU saw (the broken copy); every vector must equal the GPU's."""
    for s in sample:
        v = broken[s][0] + broken[s][1]
        lost = [i for i in range(d + p) if masks[s] >> i & 1]
        assert orc.reconst(d, p, v, [], lost) == 0, (s, lost)
        got = np.concatenate([data[s].cpu().numpy(), parity[s].cpu().numpy()])
        bad = [i for i in range(d + p) if not np.array_equal(v[i], got[i])]
        assert not bad, ("GPU planner vs oracle", s, lost, bad[:4])


@pytest.mark.parametrize("d,p,npat", [(10, 4, 300), (32, 32, 700)])
def test_reconst_batch_multi_repeated_patterns(rslib, orc, torch_dev, d, p, npat):
    """The host groups stripes by pattern (batches.cpp group_patterns): the
    previous stripe's pattern, a scan of the first 16, then a hash that grows
    as patterns arrive.  Stripes here repeat their patterns in runs, in
    interleaved order and after the hash has grown (32+32: masks up to bit
    63), with untouched stripes between; both planners rebuild every stripe
    bit-exact and leave the untouched ones alone."""
    torch = torch_dev
    L = rslib.lib()
    n = 1024
    pats = _distinct_patterns(d, p, npat, d * 7 + p, 4)
    rng = np.random.default_rng(npat + d)
    seq = []
    for k in range(npat):  # runs of 1-3 as patterns first appear
        seq += [pats[k]] * int(rng.integers(1, 4))
    seq += [pats[int(i)] for i in rng.integers(0, npat, 2 * npat)]  # repeats after the hash has grown
    seq += [0] * 50
    masks = [seq[int(i)] for i in rng.permutation(len(seq))[:len(seq) // 2]] + seq  # interleaved, then in order
    S = len(masks)
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(d * 11 + p)
    data = torch.randint(0, 256, (S, d, n), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((S, p, n), dtype=torch.uint8, device="cuda")
    r.encode_batch_split(data, parity)
    torch.cuda.synchronize()
    ref_d, ref_p = data.clone(), parity.clone()
    arg = np.array(masks, dtype=np.uint64)
    lossy = [s for s, m in enumerate(masks) if m]
    sample = sorted(set(lossy[i] for i in np.linspace(0, len(lossy) - 1, 40).astype(int).tolist()))
    try:
        for plan in (1, 0):
            assert L.rs_tune(b"multi_gpu_plan", plan) == 0
            for s, m in enumerate(masks):
                for v in range(d + p):
                    if m >> v & 1:
                        (data[s, v] if v < d else parity[s, v - d]).fill_(0x3C)
            broken = _host_stripes(data, parity, sample) if plan == 1 else None
            r.reconst_batch_multi(data, parity, arg)
            torch.cuda.synchronize()
            assert torch.equal(data, ref_d) and torch.equal(parity, ref_p), plan
            if plan == 1:  # pinned to the oracle, not only to the HIP encoder's round trip
                _oracle_rebuilds_sample(orc, d, p, broken, masks, data, parity, sample)
    finally:
        L.rs_tune(b"multi_gpu_plan", -1)


@pytest.mark.parametrize("d,p", [(10, 8), (8, 8), (10, 6)])
def test_reconst_batch_multi_parity_rows_bitsliced(rslib, orc, torch_dev, d, p):
    """Stripes that lose only parity rows p' in 5..p: the grouped fallback's
    combined matrix is then the first p' rows of the generator, which the
    bit-sliced Encode kernels match byte for byte (10+8 losing rows 10..14 =
    BsShape(10, 5)).  Those launches name their stripes through a device id
    list: every listed stripe must be rebuilt and no other stripe touched."""
    torch = torch_dev
    S, n = 48, 65536
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(d * 31 + p)
    data = torch.randint(0, 256, (S, d, n), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.empty((S, p, n), dtype=torch.uint8, device="cuda")
    r.encode_batch_split(data, parity)
    torch.cuda.synchronize()
    # the encode itself against the oracle on two stripes
    for s in (0, S - 1):
        host = data[s].cpu().numpy()
        exp = _oracle_encode(orc, d, p, [host[i].copy() for i in range(d)])
        assert np.array_equal(parity[s].cpu().numpy(), np.stack(exp)), s
    ref_d, ref_p = data.clone(), parity.clone()
    rng = np.random.default_rng(d * 7 + p)
    masks = np.zeros(S, np.uint64)
    for s in range(S):
        kind = s % 6
        if kind in (1, 4):  # untouched, interleaved with the damaged ones
            continue
        if kind == 0:
            lost = list(range(d, d + 5))                 # exactly the first 5 parity rows
        elif kind == 2:
            lost = list(range(d, d + p))                 # every parity row
        elif kind == 3:
            lost = list(range(d, d + int(rng.integers(5, p + 1))))  # a prefix of 5..p rows
        else:
            lost = sorted(int(v) for v in rng.choice(d + p, int(rng.integers(1, p + 1)), replace=False))
        for v in lost:
            masks[s] |= np.uint64(1) << np.uint64(v)
            (data[s, v] if v < d else parity[s, v - d]).fill_(0x3C)
    r.reconst_batch_multi(data, parity, masks)
    torch.cuda.synchronize()
    for s in range(S):
        assert torch.equal(data[s], ref_d[s]) and torch.equal(parity[s], ref_p[s]), (s, int(masks[s]))


# ---------------------------------------------------------------- host-call staging paths

@pytest.mark.parametrize("mode", ["chunked", "fixed_chunks", "small_chunks", "staged_pinned", "staged_pageable"])
def test_host_calls_staging_paths(rslib, orc, torch_dev, mode):
    """The synchronous host-memory calls through every staging path:
    the chunked zero-copy pipeline (default: chunks of a quarter of the
    vectors, 1 MiB + 5 B = 4 ragged chunks, 3 MiB + 48 B = 6 chunks capped at
    8 MiB per slot, around the 3-slot ring twice), fixed 128 KiB chunks
    (host_chunk_split 0), 4 KiB chunks (many trips around the ring), and the
    older staged paths (device staging with pinned DMA / pageable copies)."""
    L = rslib.lib()
    knobs = {"chunked": {}, "fixed_chunks": {"host_chunk_split": 0},
             "small_chunks": {"host_chunk": 4096, "host_chunk_split": 0},
             "staged_pinned": {"host_zc_max": 0, "host_pinned_max": 4 << 20},
             "staged_pageable": {"host_zc_max": 0, "host_pinned_max": 0}}[mode]
    try:
        for k, v in knobs.items():
            assert L.rs_tune(k.encode(), v) == 0
        d, p = 10, 4
        r = rslib.New(d, p)
        rng = np.random.default_rng(120)
        for size in (1, 4099, 65536 * 3 + 7, (1 << 20) + 5) + (((3 << 20) + 48,) if mode == "chunked" else ()):
            data = [_rand(rng, size) for _ in range(d)]
            exp = _oracle_encode(orc, d, p, data)
            act = [x.copy() for x in data] + [np.full(size, 0xA5, np.uint8) for _ in range(p)]
            r.Encode(act)
            for j in range(p):
                assert np.array_equal(act[d + j], exp[j]), (size, j)
            full = [x.copy() for x in act]
            lost = [1, 4, 10, 13]
            for i in lost:
                act[i][:] = 0x77
            r.Reconst(act, [], lost)
            for i in range(d + p):
                assert np.array_equal(act[i], full[i]), (size, i)
            new = _rand(rng, size)
            par = [x.copy() for x in full[d:]]
            r.Update(full[2], new, 2, par)
            ora = [x.copy() for x in full[d:]]
            assert orc.update(d, p, full[2], new, 2, ora) == 0
            for j in range(p):
                assert np.array_equal(par[j], ora[j]), (size, j)
            par = [x.copy() for x in full[d:]]
            r.Replace([full[3], full[7]], [3, 7], par)
            ora = [x.copy() for x in full[d:]]
            assert orc.replace(d, p, [full[3], full[7]], [3, 7], ora) == 0
            for j in range(p):
                assert np.array_equal(par[j], ora[j]), (size, j)
    finally:
        for k, v in {"host_chunk": 128 << 10, "host_chunk_split": 4, "host_zc_max": -1,
                     "host_pinned_max": 256 << 10}.items():
            L.rs_tune(k.encode(), v)


def test_group_encode_host_batch(rslib, torch_dev):
    """rs_group_encode_host_batch: stripes split over the members (here two
    codecs sharing cuda:0, plus a ragged split), parity identical to one
    device-resident encode."""
    torch = torch_dev
    d, p, S, n = 10, 4, 37, 65536 + 256
    g = torch.Generator(device="cuda").manual_seed(21)
    ref = torch.randint(0, 256, (S, d + p, n), dtype=torch.uint8, device="cuda", generator=g)
    host = ref.cpu()
    host[:, d:] = 0xA5
    rslib.New(d, p).encode_batch(ref)
    torch.cuda.synchronize()
    for devs in ([0], [0, 0], [0, 0, 0]):
        h = host.clone()
        grp = rslib.NewGroup(d, p, devs)
        grp.encode_host_batch(h, 4, 3)
        assert torch.equal(h, ref.cpu()), devs


@pytest.mark.parametrize("d,p,n", [(100, 28, 4096), (200, 56, 1024 + 16), (40, 30, 8192 + 5)])
def test_reconst_batch_multi_wide_masks(rslib, orc, torch_dev, d, p, n):
    """Multi-pattern Reconst beyond 64 vectors (256-bit masks,
    rs_reconst_batch_multi256; rs.go:61 allows d+p <= 256): mixed patterns of
    0..p erasures per stripe (data and parity), encode checked against the
    oracle, every stripe rebuilt bit-exact, untouched stripes unchanged; then
    the host-batch variant on pinned and on pageable memory."""
    torch = torch_dev
    S = 24
    r = rslib.New(d, p)
    rng = np.random.default_rng(d * 7 + p)
    host = rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)
    exp = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), host[:2, :d])
    data = torch.from_numpy(np.ascontiguousarray(host[:, :d])).cuda()
    parity = torch.empty((S, p, n), dtype=torch.uint8, device="cuda")
    r.encode_batch_split(data, parity)
    torch.cuda.synchronize()
    assert np.array_equal(parity[:2].cpu().numpy(), exp)
    ref_d, ref_p = data.clone(), parity.clone()
    masks = []
    for s in range(S):
        k = 0 if s % 5 == 1 else int(rng.choice([1, 2, 3, 4, p // 2, p]))
        lost = [int(v) for v in rng.choice(d + p, k, replace=False)]
        if s % 7 == 3:
            lost = sorted(set(lost) | {d + p - 1})[:p]  # the last vector (bit >= 64)
        m = 0
        for v in lost:
            m |= 1 << v
            (data[s, v] if v < d else parity[s, v - d]).fill_(0xC3)
        masks.append(m)
    assert any(m >> 64 for m in masks)
    r.reconst_batch_multi(data, parity, masks)
    torch.cuda.synchronize()
    for s in range(S):
        assert torch.equal(data[s], ref_d[s]) and torch.equal(parity[s], ref_p[s]), (s, bin(masks[s]))
    # host batches: pinned (zero-copy) and pageable (staged)
    full = torch.cat([ref_d, ref_p], dim=1).cpu()
    for pinned in (True, False):
        hb = full.clone().pin_memory() if pinned else full.clone()
        for s, m in enumerate(masks):
            for v in range(d + p):
                if m >> v & 1:
                    hb[s, v] = 0x3C
        r.reconst_host_batch_multi(hb, masks)
        assert torch.equal(hb, full), pinned
