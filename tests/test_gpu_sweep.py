"""Seeded random sweep: shapes, sizes and operations the targeted tests do
not pin one by one, each through the C ABI and compared byte-for-byte with
the CPU oracle (rs_oracle.c restating rs.go / matrix.go / gmu.go).

Host API: Encode / Reconst / Update / Replace on d in 1..40, p in 1..12,
(Update / Replace against re-encoding, and against the restated reference
outside its tail defect: DESIGN.md §4 "Reference defect"),
sizes from 1 B to ~300 KiB (odd sizes take the byte-tail kernel, small
ones the coalesced path, large ones the chunked pipeline).  Device batches:
split-layout Encode and per-stripe-pattern Reconst on random shapes and
stripe counts, every stripe checked against the oracle.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    torch.cuda.init()
    return torch


def _size(rng):
    kind = int(rng.integers(4))
    if kind == 0:
        return int(rng.integers(1, 300))
    if kind == 1:
        return 4096 + int(rng.integers(-17, 18))
    if kind == 2:
        return int(rng.integers(8192, 70000))
    return int(rng.integers(130000, 300000))


def _shape(rng):
    d = int(rng.integers(1, 41))
    p = int(rng.integers(1, 13))
    return d, p


def _rand(rng, n):
    return rng.integers(0, 256, n, dtype=np.uint8)


def _check_update_like(orc, act, ora, exp, d, p, size, tag):
    """Update / Replace: every parity byte equals re-encoding (the reference's
    own definition, rs_test.go:225-331), and equals the restated reference
    byte-for-byte outside its tail defect (rs_oracle.c encode_part)."""
    q = orc.update_quirk_range(size)
    for j in range(d, d + p):
        assert np.array_equal(act[j], exp[j]), tag + (j,)
        if q is None:
            assert np.array_equal(act[j], ora[j]), tag + (j,)
        else:
            lo, hi = q
            assert np.array_equal(act[j][:lo], ora[j][:lo]) and np.array_equal(act[j][hi:], ora[j][hi:]), tag


def test_host_api_random_sweep(rslib, orc, torch_dev):
    rng = np.random.default_rng(2024)
    counts = {"encode": 0, "reconst": 0, "update": 0, "replace": 0}
    for case in range(80):
        d, p = _shape(rng)
        size = _size(rng)
        r = rslib.New(d, p)
        data = [_rand(rng, size) for _ in range(d)]
        enc = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        assert orc.encode(d, p, enc) == 0
        op = ("encode", "reconst", "update", "replace")[case % 4]
        counts[op] += 1
        tag = (case, op, d, p, size)
        if op == "encode":
            act = [x.copy() for x in data] + [np.full(size, 0xA5, np.uint8) for _ in range(p)]
            r.Encode(act)
            for j in range(p):
                assert np.array_equal(act[d + j], enc[d + j]), tag + (j,)
        elif op == "reconst":
            nlost = int(rng.integers(1, p + 1))
            lost = sorted(int(v) for v in rng.choice(d + p, nlost, replace=False))
            surv = [v for v in range(d + p) if v not in lost]
            act = [x.copy() for x in enc]
            for v in lost:
                act[v][:] = _rand(rng, size)  # garbage where the lost vectors were
            ora = [x.copy() for x in act]
            r.Reconst(act, surv, lost)
            assert orc.reconst(d, p, ora, surv, lost) == 0
            for v in range(d + p):
                assert np.array_equal(act[v], ora[v]), tag + (v,)
            for v in lost:
                assert np.array_equal(act[v], enc[v]), tag + (v,)
        elif op == "update":
            row = int(rng.integers(d))
            new = _rand(rng, size)
            act = [x.copy() for x in enc]
            ora = [x.copy() for x in enc]
            r.Update(act[row], new, row, act[d:])
            assert orc.update(d, p, ora[row], new, row, ora[d:]) == 0
            exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
            exp[row] = new.copy()
            assert orc.encode(d, p, exp) == 0
            _check_update_like(orc, act, ora, exp, d, p, size, tag)
        else:
            rn = int(rng.integers(1, d + 1))
            rows = [int(v) for v in rng.choice(d, rn, replace=False)]
            delta = [_rand(rng, size) for _ in range(rn)]
            act = [x.copy() for x in enc]
            ora = [x.copy() for x in enc]
            r.Replace(delta, rows, act[d:])
            assert orc.replace(d, p, [x.copy() for x in delta], rows, ora[d:]) == 0
            exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
            for k_, rr in enumerate(rows):
                exp[rr] = np.bitwise_xor(exp[rr], delta[k_])
            assert orc.encode(d, p, exp) == 0
            _check_update_like(orc, act, ora, exp, d, p, size, tag)
    assert all(v == 20 for v in counts.values())


def test_device_batch_random_sweep(rslib, orc, torch_dev):
    torch = torch_dev
    rng = np.random.default_rng(77)
    for case in range(24):
        d = int(rng.integers(1, 25))
        p = int(rng.integers(1, 9))
        S = int(rng.integers(1, 40))
        n = int(rng.choice([16, 48, 1003, 1024, 4096 + 16 * int(rng.integers(1, 9)), 8192, 20000 * 16]))
        if n > 8192:
            S = min(S, 4)
        r = rslib.New(d, p)
        host = rng.integers(0, 256, (S, d, n), dtype=np.uint8)
        data = torch.from_numpy(host).cuda()
        parity = torch.full((S, p, n), 0xA5, dtype=torch.uint8, device="cuda")
        r.encode_batch_split(data, parity)
        torch.cuda.synchronize()
        par = parity.cpu().numpy()
        exp = []
        for s in range(S):
            v = [host[s, i].copy() for i in range(d)] + [np.zeros(n, np.uint8) for _ in range(p)]
            assert orc.encode(d, p, v) == 0
            exp.append(v)
            for j in range(p):
                assert np.array_equal(par[s, j], v[d + j]), (case, d, p, S, n, s, j)
        if d + p > 64:
            continue
        # a different 1..min(p,4)-erasure pattern per stripe (some stripes intact)
        masks = np.zeros(S, np.uint64)
        for s in range(S):
            if rng.integers(5) == 0:
                continue
            k = int(rng.integers(1, min(p, 4) + 1))
            masks[s] = sum(1 << int(v) for v in rng.choice(d + p, k, replace=False))
        for s in range(S):
            for v in range(d + p):
                if int(masks[s]) >> v & 1:
                    (data[s, v] if v < d else parity[s, v - d]).fill_(int(rng.integers(256)))
        r.reconst_batch_multi(data, parity, masks)
        torch.cuda.synchronize()
        got_d, got_p = data.cpu().numpy(), parity.cpu().numpy()
        for s in range(S):
            for v in range(d + p):
                got = got_d[s, v] if v < d else got_p[s, v - d]
                assert np.array_equal(got, exp[s][v]), (case, d, p, S, n, s, v, int(masks[s]))


@pytest.mark.parametrize("size", [16384 + 16 * 40 + 7, 49263, 236667])
def test_update_replace_at_reference_defect_sizes(rslib, orc, torch_dev, size):
    """Sizes where the reference's Update / Replace keep stale parity in the
    last chunk's body (rs_oracle.c encode_part): the host API and
    the device call equal re-encoding there, and the restated reference
    everywhere else."""
    torch = torch_dev
    d, p, row = 10, 4, 7
    rng = np.random.default_rng(size)
    data = [_rand(rng, size) for _ in range(d)]
    enc = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
    assert orc.encode(d, p, enc) == 0
    new = _rand(rng, size)
    exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
    exp[row] = new.copy()
    assert orc.encode(d, p, exp) == 0
    r = rslib.New(d, p)
    # Update, host API and device call
    act = [x.copy() for x in enc]
    ora = [x.copy() for x in enc]
    r.Update(act[row], new, row, act[d:])
    assert orc.update(d, p, ora[row], new, row, ora[d:]) == 0
    _check_update_like(orc, act, ora, exp, d, p, size, ("update", size))
    dv = [torch.from_numpy(x.copy()).cuda() for x in enc]
    r.update_dev(dv[row], torch.from_numpy(new.copy()).cuda(), row, dv[d:])
    torch.cuda.synchronize()
    for j in range(d, d + p):
        assert np.array_equal(dv[j].cpu().numpy(), exp[j]), ("update_dev", size, j)
    # Replace of the same row (delta = old ^ new)
    act = [x.copy() for x in enc]
    ora = [x.copy() for x in enc]
    delta = np.bitwise_xor(data[row], new)
    r.Replace([delta], [row], act[d:])
    assert orc.replace(d, p, [delta.copy()], [row], ora[d:]) == 0
    _check_update_like(orc, act, ora, exp, d, p, size, ("replace", size))


@pytest.mark.parametrize("l1d,size", [(32768, 17031), (32768, 49263), (32768, 236667), (49152, 24576 + 33),
                                      (49152, 3 * 24576 + 1000 + 5), (32768, 16384 * 3),
                                      (-1, 16384 + 17), (-1, 49152 + 17), (-1, 100000 + 3)])
def test_update_replace_reference_compat_mode(rslib, orc, torch_dev, l1d, size):
    """rs_set_ref_l1d(handle, l1d) reproduces the reference's Update /
    Replace bytes (rs.go:190-200 tail pass, rs_oracle.c encode_part) on a host
    whose L1D is `l1d`: host API, single-stripe device call and device batch,
    byte for byte against the restated reference with the same L1D.  The
    sixth size has no defect range (a whole number of chunks): compat =
    re-encode.  l1d = -1 is the cgo binding's default (its New calls
    rs_set_ref_l1d(h, -1)): THIS host's L1D as rs.go reads it,
    so a Go drop-in gets the reference's bytes at defect sizes such as
    16 KiB + 17 (a defect on 32 KiB-L1D hosts) and 48 KiB + 17 (on both 32 and
    48 KiB hosts)."""
    torch = torch_dev
    L = rslib.lib()
    d, p, row, rows = 10, 4, 3, [1, 6, 9]
    rng = np.random.default_rng(size + l1d)
    data = [_rand(rng, size) for _ in range(d)]
    enc = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
    assert orc.encode(d, p, enc) == 0
    new = _rand(rng, size)
    r = rslib.New(d, p)
    r.set_ref_l1d(l1d)
    if l1d == -1:  # the binding's New: this host's L1D, 32 KiB when CPUID has none (rs.go:159-161)
        host = rslib.host_l1d()
        l1d = host if host > 0 else 32768
        print("host L1D", host, "defect range", orc.update_quirk_range(size, l1d))
    assert r.ref_l1d == l1d
    orc.set_l1d(l1d)
    try:
        # Update: restated reference, then each librsamd entry point
        ora = [x.copy() for x in enc]
        assert orc.update(d, p, ora[row], new, row, ora[d:]) == 0
        q = orc.update_quirk_range(size, l1d)
        if q is not None:  # the defect is real at this size: some parity byte differs from re-encoding
            reenc = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
            reenc[row] = new.copy()
            assert orc.encode(d, p, reenc) == 0
            assert any(not np.array_equal(ora[j], reenc[j]) for j in range(d, d + p))
        act = [x.copy() for x in enc]
        r.Update(act[row], new, row, act[d:])
        dv = [torch.from_numpy(x.copy()).cuda() for x in enc]
        r.update_dev(dv[row], torch.from_numpy(new.copy()).cuda(), row, dv[d:])
        S = 3
        buf = torch.from_numpy(np.stack([np.stack(enc)] * S)).cuda()
        old_b = buf[:, row].clone()
        new_b = torch.from_numpy(np.stack([new] * S)).cuda()
        r.update_batch(old_b, new_b, row, buf)
        torch.cuda.synchronize()
        for j in range(d, d + p):
            assert np.array_equal(act[j], ora[j]), ("Update", l1d, size, j)
            assert np.array_equal(dv[j].cpu().numpy(), ora[j]), ("update_dev", l1d, size, j)
            for s_ in range(S):
                assert np.array_equal(buf[s_, j].cpu().numpy(), ora[j]), ("update_batch", l1d, size, s_, j)
        # Replace of three rows
        delta = [_rand(rng, size) for _ in rows]
        ora = [x.copy() for x in enc]
        assert orc.replace(d, p, [x.copy() for x in delta], rows, ora[d:]) == 0
        act = [x.copy() for x in enc]
        r.Replace([x.copy() for x in delta], rows, act[d:])
        dv = [torch.from_numpy(x.copy()).cuda() for x in enc]
        r.replace_dev([torch.from_numpy(x.copy()).cuda() for x in delta], rows, dv[d:])
        buf = torch.from_numpy(np.stack([np.stack(enc)] * S)).cuda()
        dl = torch.from_numpy(np.stack([np.stack(delta)] * S)).cuda()
        r.replace_batch(dl, rows, buf)
        torch.cuda.synchronize()
        for j in range(d, d + p):
            assert np.array_equal(act[j], ora[j]), ("Replace", l1d, size, j)
            assert np.array_equal(dv[j].cpu().numpy(), ora[j]), ("replace_dev", l1d, size, j)
            for s_ in range(S):
                assert np.array_equal(buf[s_, j].cpu().numpy(), ora[j]), ("replace_batch", l1d, size, s_, j)
    finally:
        orc.set_l1d(0)


def test_update_replace_reference_compat_per_handle_concurrent(rslib, orc, torch_dev):
    """The compat setting belongs to the handle (verdict round 4): three
    handles in one process - re-encode (0), 32 KiB and 48 KiB L1D - run Update
    and Replace concurrently from their own threads over sizes with a defect
    range for both L1D values, and each one's bytes equal the restated
    reference with ITS setting (orc.set_l1d), host API and device batch."""
    import threading

    torch = torch_dev
    d, p, row, rows = 10, 4, 2, [0, 5, 7]
    # last chunk >= 16 B and not a multiple of 16 for both L1Ds, at different offsets
    sizes = [40001, 70003]
    settings = [0, 32768, 49152]
    rng = np.random.default_rng(77)
    cases = []
    for size in sizes:
        data = [_rand(rng, size) for _ in range(d)]
        enc = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        assert orc.encode(d, p, enc) == 0
        new = _rand(rng, size)
        delta = [_rand(rng, size) for _ in rows]
        exp = {}
        for l1d in settings:
            orc.set_l1d(l1d)
            if l1d == 0:  # the re-encode definition
                u = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                u[row] = new.copy()
                assert orc.encode(d, p, u) == 0
                rp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                for i, rr in enumerate(rows):
                    rp[rr] = np.bitwise_xor(rp[rr], delta[i])
                assert orc.encode(d, p, rp) == 0
                exp[l1d] = ([x.copy() for x in u[d:]], [x.copy() for x in rp[d:]])
            else:
                u = [x.copy() for x in enc]
                assert orc.update(d, p, u[row], new, row, u[d:]) == 0
                rp = [x.copy() for x in enc]
                assert orc.replace(d, p, [x.copy() for x in delta], rows, rp[d:]) == 0
                exp[l1d] = (u[d:], rp[d:])
        orc.set_l1d(0)
        # the three expectations really differ pairwise at these sizes
        for a in settings:
            for b in settings:
                if a < b:
                    assert any(not np.array_equal(x, y) for x, y in zip(exp[a][0], exp[b][0])), (size, a, b)
        cases.append((size, enc, new, delta, exp))
    handles = {}
    for l1d in settings:
        h = rslib.New(d, p, device=0)
        h.set_ref_l1d(l1d)
        handles[l1d] = h
    errors = []
    start = threading.Barrier(len(settings))

    def run(l1d):
        try:
            h = handles[l1d]
            stream = torch.cuda.Stream(0)
            start.wait()
            for _rep in range(3):
                for size, enc, new, delta, exp in cases:
                    act = [x.copy() for x in enc]
                    h.Update(act[row], new, row, act[d:])
                    for j in range(p):
                        if not np.array_equal(act[d + j], exp[l1d][0][j]):
                            errors.append(("Update", l1d, size, j))
                    act = [x.copy() for x in enc]
                    h.Replace([x.copy() for x in delta], rows, act[d:])
                    for j in range(p):
                        if not np.array_equal(act[d + j], exp[l1d][1][j]):
                            errors.append(("Replace", l1d, size, j))
                    S = 2
                    with torch.cuda.stream(stream):
                        buf = torch.from_numpy(np.stack([np.stack(enc)] * S)).cuda(0)
                        old_b = buf[:, row].clone()
                        new_b = torch.from_numpy(np.stack([new] * S)).cuda(0)
                    h.update_batch(old_b, new_b, row, buf, stream=stream)
                    stream.synchronize()
                    got = buf.cpu().numpy()
                    for s_ in range(S):
                        for j in range(p):
                            if not np.array_equal(got[s_, d + j], exp[l1d][0][j]):
                                errors.append(("update_batch", l1d, size, s_, j))
        except Exception as e:  # noqa: BLE001
            errors.append(("exception", l1d, repr(e)))

    ts = [threading.Thread(target=run, args=(l1d,)) for l1d in settings]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors[:10]
    assert [handles[x].ref_l1d for x in settings] == settings


def _padded(torch, rng, S, nvec, n, device):
    """[S, nvec, n] view of a larger random buffer (padding between vectors and
    stripes, sometimes an odd vector stride: the unaligned / byte-kernel paths)."""
    vpad = int(rng.choice([0, 16, 5, 256]))
    spad = int(rng.choice([0, 1, 3]))
    full = torch.randint(0, 256, (S, nvec + spad, n + vpad), dtype=torch.uint8,
                         generator=torch.Generator().manual_seed(int(rng.integers(1 << 30))))
    if device == "cuda":
        full = full.cuda()
    elif device == "pinned":
        full = full.pin_memory()
    return full[:, :nvec, :n]


def _encode_expect(orc, host, d, p):
    """Parity of every stripe of host[S, >= d, n] (numpy), per the oracle."""
    S, _, n = host.shape
    out = np.zeros((S, p, n), np.uint8)
    for s in range(S):
        v = [host[s, i].copy() for i in range(d)] + [np.zeros(n, np.uint8) for _ in range(p)]
        assert orc.encode(d, p, v) == 0
        out[s] = np.stack(v[d:])
    return out


def test_batch_update_replace_random_sweep(rslib, orc, torch_dev):
    """rs_update_batch / rs_replace_batch on padded, sometimes unaligned
    layouts: parity equals re-encoding the changed stripes."""
    torch = torch_dev
    rng = np.random.default_rng(91)
    for case in range(16):
        d = int(rng.integers(1, 21))
        p = int(rng.integers(1, 9))
        S = int(rng.integers(1, 17))
        n = int(rng.choice([1, 15, 16, 100, 1024, 4099, 8192, 40000]))
        r = rslib.New(d, p)
        buf = _padded(torch, rng, S, d + p, n, "cuda")
        r.encode_batch(buf)
        host = buf.cpu().numpy()
        assert np.array_equal(host[:, d:], _encode_expect(orc, host, d, p)), (case, "encode")
        if case % 2 == 0:
            row = int(rng.integers(d))
            new = torch.randint(0, 256, (S, n), dtype=torch.uint8, device="cuda")
            old = buf[:, row].clone()
            r.update_batch(old, new, row, buf)
            host2 = host.copy()
            host2[:, row] = new.cpu().numpy()
        else:
            rn = int(rng.integers(1, d + 1))
            rows = [int(v) for v in rng.choice(d, rn, replace=False)]
            delta = torch.randint(0, 256, (S, rn, n), dtype=torch.uint8, device="cuda")
            r.replace_batch(delta, rows, buf)
            host2 = host.copy()
            dh = delta.cpu().numpy()
            for k_, rr in enumerate(rows):
                host2[:, rr] ^= dh[:, k_]
        torch.cuda.synchronize()
        got = buf.cpu().numpy()[:, d:]
        assert np.array_equal(got, _encode_expect(orc, host2, d, p)), (case, d, p, S, n)


def test_host_batch_random_sweep(rslib, orc, torch_dev):
    """rs_encode_host_batch on pageable (DMA pipeline) and pinned (zero-copy)
    padded layouts, and rs_reconst_host_batch_multi on pinned memory."""
    torch = torch_dev
    rng = np.random.default_rng(92)
    for case in range(12):
        d = int(rng.integers(1, 17))
        p = int(rng.integers(1, 7))
        S = int(rng.integers(1, 25))
        n = int(rng.choice([16, 256, 1000, 4096, 65536 + 256]))
        where = "pinned" if case % 2 else "pageable"
        r = rslib.New(d, p)
        buf = _padded(torch, rng, S, d + p, n, where)
        arr = buf if where == "pinned" else buf.numpy()
        r.encode_host_batch(arr, stripes_per_chunk=int(rng.integers(1, 6)), streams=int(rng.integers(1, 4)))
        host = buf.numpy().copy()
        assert np.array_equal(host[:, d:], _encode_expect(orc, host, d, p)), (case, where, d, p, S, n)
        if where != "pinned" or d + p > 64 or n % 16:
            continue
        masks = np.zeros(S, np.uint64)
        for s in range(S):
            k = int(rng.integers(0, min(p, 4) + 1))
            lost = rng.choice(d + p, k, replace=False)
            masks[s] = sum(1 << int(v) for v in lost)
            for v in lost:
                buf[s, int(v)].fill_(0x3C)
        r.reconst_host_batch_multi(buf, masks)
        assert np.array_equal(buf.numpy(), host), (case, "reconst", d, p, S, n)


def test_concurrent_random_host_calls(rslib, orc, torch_dev):
    """8 threads of random host calls (Encode / Reconst / Update / Replace,
    sizes on both sides of the coalescing and chunking thresholds) on ONE
    handle: every result equals the oracle's (re-encoding for Update /
    Replace) for that call made alone."""
    d, p = 10, 4
    r = rslib.New(d, p)
    errors = []
    barrier = threading.Barrier(8)

    def worker(t):
        try:
            rng = np.random.default_rng(5000 + t)
            barrier.wait()
            for it in range(15):
                size = int(rng.choice([100, 4096, 8197, 70000, 200000]))
                data = [_rand(rng, size) for _ in range(d)]
                enc = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                assert orc.encode(d, p, enc) == 0
                op = int(rng.integers(4))
                if op == 0:
                    v = [x.copy() for x in data] + [np.full(size, 0x5A, np.uint8) for _ in range(p)]
                    r.Encode(v)
                    ok = all(np.array_equal(v[d + j], enc[d + j]) for j in range(p))
                elif op == 1:
                    lost = sorted(int(x) for x in rng.choice(d + p, int(rng.integers(1, p + 1)), replace=False))
                    v = [x.copy() for x in enc]
                    for i in lost:
                        v[i][:] = 0
                    r.Reconst(v, [], lost)
                    ok = all(np.array_equal(v[i], enc[i]) for i in lost)
                else:
                    exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                    par = [x.copy() for x in enc[d:]]
                    if op == 2:
                        row = int(rng.integers(d))
                        new = _rand(rng, size)
                        r.Update(data[row], new, row, par)
                        exp[row] = new
                    else:
                        rows = [int(x) for x in rng.choice(d, int(rng.integers(1, 4)), replace=False)]
                        delta = [_rand(rng, size) for _ in rows]
                        r.Replace(delta, rows, par)
                        for k_, rr in enumerate(rows):
                            exp[rr] = np.bitwise_xor(exp[rr], delta[k_])
                    assert orc.encode(d, p, exp) == 0
                    ok = all(np.array_equal(par[j], exp[d + j]) for j in range(p))
                if not ok:
                    errors.append((t, it, op, size))
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:10]


def test_device_single_stripe_random_sweep(rslib, orc, torch_dev):
    """rs_*_dev on vectors at random byte offsets inside one device buffer
    (Go slices start anywhere): Encode / Reconst / Update / Replace against
    the oracle (re-encoding for Update / Replace)."""
    torch = torch_dev
    rng = np.random.default_rng(93)
    for case in range(40):
        d = int(rng.integers(1, 21))
        p = int(rng.integers(1, 9))
        size = int(rng.choice([1, 5, 16, 33, 1000, 4096, 4099, 65536 + 48, 200003]))
        r = rslib.New(d, p)
        gap = int(rng.integers(0, 40))
        start = int(rng.integers(0, 16))
        big = torch.from_numpy(_rand(rng, start + (d + p) * (size + gap))).cuda()
        vecs = [big[start + i * (size + gap): start + i * (size + gap) + size] for i in range(d + p)]
        data = [v.cpu().numpy().copy() for v in vecs[:d]]
        enc = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
        assert orc.encode(d, p, enc) == 0
        r.encode_dev(vecs)
        torch.cuda.synchronize()
        tag = (case, d, p, size, gap, start)
        for j in range(p):
            assert np.array_equal(vecs[d + j].cpu().numpy(), enc[d + j]), tag + ("encode", j)
        op = case % 3
        if op == 0:
            lost = sorted(int(v) for v in rng.choice(d + p, int(rng.integers(1, p + 1)), replace=False))
            for v in lost:
                vecs[v].fill_(0x77)
            r.reconst_dev(vecs, [], lost)
            torch.cuda.synchronize()
            for v in lost:
                assert np.array_equal(vecs[v].cpu().numpy(), enc[v]), tag + ("reconst", v)
        elif op == 1:
            row = int(rng.integers(d))
            new = torch.from_numpy(_rand(rng, size)).cuda()
            r.update_dev(vecs[row], new, row, vecs[d:])
            torch.cuda.synchronize()
            exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
            exp[row] = new.cpu().numpy()
            assert orc.encode(d, p, exp) == 0
            for j in range(p):
                assert np.array_equal(vecs[d + j].cpu().numpy(), exp[d + j]), tag + ("update", j)
        else:
            rows = [int(v) for v in rng.choice(d, int(rng.integers(1, d + 1)), replace=False)]
            delta = [torch.from_numpy(_rand(rng, size)).cuda() for _ in rows]
            r.replace_dev(delta, rows, vecs[d:])
            torch.cuda.synchronize()
            exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
            for k_, rr in enumerate(rows):
                exp[rr] = np.bitwise_xor(exp[rr], delta[k_].cpu().numpy())
            assert orc.encode(d, p, exp) == 0
            for j in range(p):
                assert np.array_equal(vecs[d + j].cpu().numpy(), exp[d + j]), tag + ("replace", j)


@pytest.mark.parametrize("bitslice", [1, 0])
def test_bitsliced_encode_shapes(rslib, orc, torch_dev, bitslice):
    """Every generated bit-sliced shape (tools/gen_bitslice.py) at sizes that
    exercise whole 32-byte units, ragged workgroups and the byte tail, against
    the oracle, with the bit-sliced kernels on and off."""
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location(
        "gen_bitslice", os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "gen_bitslice.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    L = rslib.lib()
    assert L.rs_tune(b"bitslice", bitslice) == 0
    try:
        rng = np.random.default_rng(94 + bitslice)
        for d, p in gen.SHAPES:
            r = rslib.New(d, p)
            for size in (16, 23, 32, 33, 2048 + 16, 4096 + 5, 65536 + 96, 1 << 20):
                data = [_rand(rng, size) for _ in range(d)]
                v = [x.copy() for x in data] + [np.full(size, 0xA5, np.uint8) for _ in range(p)]
                r.Encode(v)
                exp = [x.copy() for x in data] + [np.zeros(size, np.uint8) for _ in range(p)]
                assert orc.encode(d, p, exp) == 0
                for j in range(p):
                    assert np.array_equal(v[d + j], exp[d + j]), (d, p, size, j, bitslice)
    finally:
        L.rs_tune(b"bitslice", 1)


@pytest.mark.parametrize("bs_block", [64, 128, 256])
def test_bitsliced_workgroup_sizes(rslib, orc, torch_dev, bs_block):
    """Every bit-sliced shape at each workgroup size (rs_tune("bs_block")),
    batched device Encode on both layouts (interleaved [S][d+p][n]; data and
    parity in separate buffers), whole-unit, ragged and tail sizes, against
    the oracle."""
    import importlib.util
    import os

    torch = torch_dev
    spec = importlib.util.spec_from_file_location(
        "gen_bitslice", os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "gen_bitslice.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    L = rslib.lib()
    assert L.rs_tune(b"bs_block", bs_block) == 0
    try:
        rng = np.random.default_rng(1000 + bs_block)
        for d, p in gen.SHAPES:
            r = rslib.New(d, p)
            G = orc.gen_matrix(d, p).reshape(p, d)
            for S, n in [(3, 16), (5, 4096 + 5), (4, 65536 + 96)] + ([(3, 1 << 20)] if (d, p) == (10, 8) else []):
                host = rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)
                host[:, d:] = 0xA5
                exp = orc.encode_numpy(G, host[:, :d])
                buf = torch.from_numpy(host).cuda()
                r.encode_batch(buf)
                data = torch.from_numpy(np.ascontiguousarray(host[:, :d])).cuda()
                par = torch.full((S, p, n), 0xA5, dtype=torch.uint8, device="cuda")
                r.encode_batch_split(data, par)
                torch.cuda.synchronize()
                got = buf.cpu().numpy()
                assert np.array_equal(got[:, d:], exp), (d, p, S, n, bs_block, "interleaved")
                assert np.array_equal(got[:, :d], host[:, :d])
                assert np.array_equal(par.cpu().numpy(), exp), (d, p, S, n, bs_block, "split")
    finally:
        L.rs_tune(b"bs_block", 0)


def test_many_row_runtime_matrices(rslib, orc, torch_dev):
    """More than 4 output rows on runtime matrices (the 8-row one-chunk
    kernels and, above 8 rows, the row-group loop), against the oracle: the
    generic product (overwrite and accumulate, 5..20 rows, ragged and tail
    sizes), Encode of shapes with no generated network, Reconst of 5..8 lost
    vectors, Update and Replace with 8 parity rows, and multi-pattern Reconst
    whose > 4-output patterns run over a device stripe-id list."""
    torch = torch_dev
    rng = np.random.default_rng(700)
    r = rslib.New(10, 8)
    for rows, cols, S, n, acc in [(5, 10, 6, 8192, False), (8, 10, 5, 65536 + 16, True), (6, 12, 4, 4096 + 7, False),
                                  (7, 7, 3, 2048, True), (8, 16, 4, 40960, False), (13, 3, 3, 1 << 16, True),
                                  (20, 20, 2, 8192 + 48, False), (9, 1, 7, 16, True)]:
        mat = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
        src = torch.from_numpy(rng.integers(0, 256, (S, cols, n), dtype=np.uint8)).cuda()
        init = rng.integers(0, 256, (S, rows, n), dtype=np.uint8)
        dst = torch.from_numpy(init.copy()).cuda()
        r.gf_matmul_batch(mat, src, None, dst, None, accumulate=acc)
        torch.cuda.synchronize()
        exp = orc.encode_numpy(mat, src.cpu().numpy())
        if acc:
            exp ^= init
        assert np.array_equal(dst.cpu().numpy(), exp), (rows, cols, S, n, acc)
    for d, p in [(16, 8), (7, 6), (20, 5)]:  # no generated network: runtime-matrix Encode
        rs_ = rslib.New(d, p)
        S, n = 5, 65536 + 32
        data = torch.from_numpy(rng.integers(0, 256, (S, d, n), dtype=np.uint8)).cuda()
        par = torch.full((S, p, n), 0xA5, dtype=torch.uint8, device="cuda")
        rs_.encode_batch_split(data, par)
        torch.cuda.synchronize()
        exp = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), data.cpu().numpy())
        assert np.array_equal(par.cpu().numpy(), exp), (d, p)
    for d, p in [(10, 8), (12, 8)]:  # Reconst of 5..8 lost (data and parity)
        rs_ = rslib.New(d, p)
        S, n = 6, 32768 + 48
        buf = torch.from_numpy(rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)).cuda()
        rs_.encode_batch(buf)
        ref = buf.clone()
        for k in range(5, p + 1):
            lost = sorted(int(v) for v in rng.choice(d + p, k, replace=False))
            buf[:, lost] = 0x77
            rs_.reconst_batch(buf, [], lost)
            torch.cuda.synchronize()
            assert torch.equal(buf, ref), (d, p, lost)
        # Update of one row, Replace of 3 rows, against re-encoding
        new = torch.from_numpy(rng.integers(0, 256, (S, n), dtype=np.uint8)).cuda()
        rs_.update_batch(buf[:, 2].clone(), new, 2, buf)
        buf[:, 2] = new
        exp = buf.clone()
        rs_.encode_batch(exp)
        torch.cuda.synchronize()
        assert torch.equal(buf, exp), (d, p, "update")
        rows = [1, 4, 7]
        delta = torch.from_numpy(rng.integers(0, 256, (S, 3, n), dtype=np.uint8)).cuda()
        rs_.replace_batch(delta, rows, buf)
        for k_, rr in enumerate(rows):
            buf[:, rr] ^= delta[:, k_]
        exp = buf.clone()
        rs_.encode_batch(exp)
        torch.cuda.synchronize()
        assert torch.equal(buf, exp), (d, p, "replace")
    # multi-pattern Reconst: stripes losing > 4 vectors run per-pattern
    # launches over a device stripe-id list
    d, p, S, n = 10, 8, 40, 16384
    rs_ = rslib.New(d, p)
    data = torch.from_numpy(rng.integers(0, 256, (S, d, n), dtype=np.uint8)).cuda()
    par = torch.empty((S, p, n), dtype=torch.uint8, device="cuda")
    rs_.encode_batch_split(data, par)
    ref_d, ref_p = data.clone(), par.clone()
    masks = np.zeros(S, np.uint64)
    for s in range(1, S, 3):
        for v in rng.choice(d + p, int(rng.integers(5, p + 1)), replace=False):
            v = int(v)
            masks[s] |= np.uint64(1) << np.uint64(v)
            (data[s, v] if v < d else par[s, v - d]).fill_(0x99)
    rs_.reconst_batch_multi(data, par, masks)
    torch.cuda.synchronize()
    assert torch.equal(data, ref_d) and torch.equal(par, ref_p)

