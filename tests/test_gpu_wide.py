"""Single-pass wide kernels (gf_matmul_wide, kernels.hip): products with more
than 8 output rows over run-time matrices and no compiled network, every
input read once.  The reference encodes any d+p <= 256 in one pass over each
chunk (rs.go:61, encodePart rs.go:175-203); Reconst rebuilds up to p lost
vectors (rs.go:221-380) and Update / Replace XOR into p parity rows
(rs.go:424-570).  Every byte is compared with the CPU oracle (rs_oracle.c,
the restatement of those functions), with the run-time compiler off (jit=0)
so the wide kernels are what runs.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    torch.cuda.init()
    return torch


@pytest.fixture
def no_jit(rslib):
    L = rslib.lib()
    assert L.rs_tune(b"jit", 0) == 0
    assert L.rs_tune(b"wide_single_pass", 1) == 0
    yield L
    L.rs_tune(b"jit", 1)
    L.rs_tune(b"wide_single_pass", 1)


def _padded(torch, rng, S, v, n, pad):
    host = rng.integers(0, 256, (S, v, n + pad), dtype=np.uint8)
    t = torch.from_numpy(host).cuda()
    return t[:, :, :n], host[:, :, :n]


@pytest.mark.parametrize("rows,cols", [(9, 10), (12, 16), (16, 16), (17, 5), (24, 33), (32, 64), (33, 7),
                                       (56, 200), (64, 64), (65, 3), (100, 100), (128, 128), (129, 2),
                                       (200, 56), (255, 1)])
def test_wide_matmul_vs_oracle(rslib, orc, torch_dev, no_jit, rows, cols):
    """The primitive at 9-255 output rows and 1-200 columns (odd and even
    column counts, row counts off every multiple of 4 / 16 / 128), overwrite
    and XOR-accumulate, aligned and ragged sizes."""
    torch = torch_dev
    rng = np.random.default_rng(rows * 1000 + cols)
    mat = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
    r = rslib.New(10, 4)
    for S, n, pad in [(3, 1024, 0), (2, 4096 + 5, 11), (2, 65536 + 48, 16)]:
        src, hsrc = _padded(torch, rng, S, cols, n, pad)
        dst, _ = _padded(torch, rng, S, rows, n, pad)
        r.gf_matmul_batch(mat, src, None, dst, None)
        torch.cuda.synchronize()
        exp = orc.encode_numpy(mat, hsrc)
        assert np.array_equal(dst.cpu().numpy(), exp), (rows, cols, S, n)
        dst2, hdst2 = _padded(torch, rng, S, rows, n, pad)
        r.gf_matmul_batch(mat, src, None, dst2, None, accumulate=True)
        torch.cuda.synchronize()
        assert np.array_equal(dst2.cpu().numpy(), hdst2 ^ exp), (rows, cols, S, n, "acc")


@pytest.mark.parametrize("d,p,n", [(64, 64, 65536), (128, 128, 16384 + 16), (200, 56, 65536), (1, 255, 4096),
                                   (16, 16, 1 << 20)])
def test_wide_encode_vs_oracle(rslib, orc, torch_dev, no_jit, d, p, n):
    """Encode of wide codes (GenMatrix rs.go:65-68 with p > 8 rows), batched on
    the interleaved layout, every stripe against the oracle."""
    torch = torch_dev
    rng = np.random.default_rng(d * 7 + p)
    S = 3
    r = rslib.New(d, p)
    host = rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)
    buf = torch.from_numpy(host).cuda()
    r.encode_batch(buf)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    exp = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), host[:, :d])
    assert np.array_equal(got[:, d:], exp)
    assert np.array_equal(got[:, :d], host[:, :d])


@pytest.mark.parametrize("d,p,lost", [
    (16, 16, list(range(16))),                                   # 16 lost data
    (100, 28, list(range(0, 34, 2))),                            # 17 lost data
    (100, 28, list(range(3, 63, 3))),                            # 20 lost data
    (100, 28, list(range(0, 96, 4)) + [100, 110, 127]),          # 24 data + 3 parity
    (100, 28, list(range(1, 100, 4))[:25] + [101, 105, 120]),    # 25 data + 3 parity = 28
    (40, 30, list(range(0, 40, 2)) + list(range(41, 70, 3))),    # 20 data + 10 parity
])
def test_wide_reconst_vs_oracle(rslib, orc, torch_dev, no_jit, d, p, lost):
    """Reconst of 16-28 lost vectors (data and parity mixed): one pass over
    the first d survivors (rs.go:327-373), rebuilt bytes equal the encoded
    originals and the oracle's two-pass Reconst of the first stripe."""
    torch = torch_dev
    rng = np.random.default_rng(d * 100 + len(lost))
    S, n = 3, 8192 + 48
    r = rslib.New(d, p)
    G = orc.gen_matrix(d, p).reshape(p, d)
    host = rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)
    host[:, d:] = orc.encode_numpy(G, host[:, :d])
    buf = torch.from_numpy(host).cuda()
    buf[:, lost] = 0x5A
    r.reconst_batch(buf, [], lost)
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy(), host), (d, p, len(lost))
    # the oracle's own Reconst (restated rs.go) on stripe 0 gives the same bytes
    v = [host[0, i].copy() for i in range(d + p)]
    for i in lost:
        v[i][:] = 0x5A
    assert orc.reconst(d, p, v, [], lost) == 0
    assert all(np.array_equal(v[i], host[0, i]) for i in range(d + p))


def test_wide_update_replace_vs_oracle(rslib, orc, torch_dev, no_jit):
    """Update and Replace on a 64+64 batch: 64-row XOR-accumulate products
    over 2 and 5 columns (rs.go:424-449, :492-529) against the oracle."""
    torch = torch_dev
    d, p, S, n = 64, 64, 2, 8192
    rng = np.random.default_rng(640)
    r = rslib.New(d, p)
    G = orc.gen_matrix(d, p).reshape(p, d)
    host = rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)
    host[:, d:] = orc.encode_numpy(G, host[:, :d])
    buf = torch.from_numpy(host.copy()).cuda()
    new = rng.integers(0, 256, (S, n), dtype=np.uint8)
    row = 37
    r.update_batch(torch.from_numpy(host[:, row].copy()).cuda(), torch.from_numpy(new).cuda(), row, buf)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    for s in range(S):
        par = [host[s, d + j].copy() for j in range(p)]
        assert orc.update(d, p, host[s, row].copy(), new[s].copy(), row, par) == 0
        assert all(np.array_equal(got[s, d + j], par[j]) for j in range(p)), s
    rows = [1, 9, 22, 40, 63]
    delta = rng.integers(0, 256, (S, len(rows), n), dtype=np.uint8)
    buf = torch.from_numpy(host.copy()).cuda()
    r.replace_batch(torch.from_numpy(delta).cuda(), rows, buf)
    torch.cuda.synchronize()
    got = buf.cpu().numpy()
    for s in range(S):
        par = [host[s, d + j].copy() for j in range(p)]
        assert orc.replace(d, p, [delta[s, k].copy() for k in range(len(rows))], rows, par) == 0
        assert all(np.array_equal(got[s, d + j], par[j]) for j in range(p)), s


def test_wide_multi_pattern_grouped(rslib, orc, torch_dev, no_jit):
    """rs_reconst_batch_multi256 with 9-30-output patterns on a 40+30 code:
    each pattern's grouped launch runs the wide kernel over a device stripe-id
    list; untouched stripes stay bit-identical."""
    torch = torch_dev
    d, p, S, n = 40, 30, 10, 4096
    rng = np.random.default_rng(4030)
    r = rslib.New(d, p)
    G = orc.gen_matrix(d, p).reshape(p, d)
    host = rng.integers(0, 256, (S, d, n), dtype=np.uint8)
    hpar = orc.encode_numpy(G, host)
    pats = [list(range(9)), list(range(0, 60, 2)), [], list(range(40, 70)), list(range(5, 65, 4))]
    masks = []
    for s in range(S):
        m = 0
        for v in pats[s % len(pats)]:
            m |= 1 << v
        masks.append(m)
    data = torch.from_numpy(host.copy()).cuda()
    par = torch.from_numpy(hpar.copy()).cuda()
    for s in range(S):
        for v in pats[s % len(pats)]:
            (data[s, v] if v < d else par[s, v - d]).fill_(0xEE)
    r.reconst_batch_multi(data, par, masks)
    torch.cuda.synchronize()
    assert np.array_equal(data.cpu().numpy(), host) and np.array_equal(par.cpu().numpy(), hpar)


def test_wide_matches_row_groups(rslib, torch_dev, no_jit):
    """wide_single_pass 1 and 0 (the looped kernel in row groups of 8) write
    the same bytes on a 1 MiB 48+16 Reconst-shaped product."""
    torch = torch_dev
    L = rslib.lib()
    rng = np.random.default_rng(4816)
    mat = rng.integers(0, 256, (16, 48), dtype=np.uint8)
    r = rslib.New(10, 4)
    src = torch.from_numpy(rng.integers(0, 256, (2, 48, 1 << 20), dtype=np.uint8)).cuda()
    out = []
    for sp in (1, 0):
        assert L.rs_tune(b"wide_single_pass", sp) == 0
        dst = torch.zeros((2, 16, 1 << 20), dtype=torch.uint8, device="cuda")
        r.gf_matmul_batch(mat, src, None, dst, None)
        torch.cuda.synchronize()
        out.append(dst.cpu())
    assert torch.equal(out[0], out[1])


@pytest.fixture
def asm_jit(rslib):
    L = rslib.lib()
    assert L.rs_tune(b"jit", 2) == 0 and L.rs_tune(b"jit_backend", 2) == 0
    yield L
    L.rs_tune(b"jit", 1)


@pytest.mark.parametrize("rows,cols", [(9, 10), (16, 64), (17, 5), (24, 33), (56, 200), (64, 64), (100, 100),
                                       (128, 128), (128, 1), (40, 1), (33, 7), (128, 9)])
def test_wide_asm_jit_vs_oracle(rslib, orc, torch_dev, asm_jit, rows, cols):
    """The assembly-generated bit-sliced kernels (jit_asm.cpp) for 9-128
    output rows: 1-8 waves per workgroup, each wave up to 16 rows, all over
    the same chunk (columns shared through LDS, the default); overwrite and XOR-accumulate, aligned and ragged
    sizes, against the oracle.  The compiled kernel really runs (launch
    counter)."""
    torch = torch_dev
    rng = np.random.default_rng(rows * 7000 + cols)
    mat = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
    r = rslib.New(10, 4)
    # compiled up front (rs_jit_prepare): a launch that finds the kernel table
    # full takes the table kernels while the worker evicts (by design), which
    # a long test session reaches; preparing makes room on this thread first
    r.jit_prepare(mat)
    r.jit_prepare(mat, accumulate=True)
    before = rslib.jit_stats()["launches"]
    for S, n, pad in [(3, 2048, 0), (2, 4096 + 5, 11), (2, 65536 + 48, 16)]:
        src, hsrc = _padded(torch, rng, S, cols, n, pad)
        dst, _ = _padded(torch, rng, S, rows, n, pad)
        r.gf_matmul_batch(mat, src, None, dst, None)
        torch.cuda.synchronize()
        exp = orc.encode_numpy(mat, hsrc)
        assert np.array_equal(dst.cpu().numpy(), exp), (rows, cols, S, n)
        dst2, hdst2 = _padded(torch, rng, S, rows, n, pad)
        r.gf_matmul_batch(mat, src, None, dst2, None, accumulate=True)
        torch.cuda.synchronize()
        assert np.array_equal(dst2.cpu().numpy(), hdst2 ^ exp), (rows, cols, S, n, "acc")
    st = rslib.jit_stats()
    assert st["launches"] >= before + 6 and st["failed"] == 0, st


@pytest.mark.parametrize("d,p,lost", [(100, 28, list(range(0, 84, 3))), (64, 64, list(range(0, 128, 2))),
                                      (16, 16, list(range(16)))])
def test_wide_asm_jit_reconst(rslib, orc, torch_dev, asm_jit, d, p, lost):
    """Reconst of 16-64 lost vectors through the assembly kernels, in place
    on the interleaved layout and on the split layout."""
    torch = torch_dev
    rng = np.random.default_rng(d + 10 * len(lost))
    S, n = 3, 8192 + 48
    r = rslib.New(d, p)
    G = orc.gen_matrix(d, p).reshape(p, d)
    host = rng.integers(0, 256, (S, d + p, n), dtype=np.uint8)
    host[:, d:] = orc.encode_numpy(G, host[:, :d])
    buf = torch.from_numpy(host).cuda()
    buf[:, lost] = 0x5A
    r.reconst_batch(buf, [], lost)
    torch.cuda.synchronize()
    assert np.array_equal(buf.cpu().numpy(), host), (d, p, len(lost))
    data = torch.from_numpy(np.ascontiguousarray(host[:, :d])).cuda()
    par = torch.from_numpy(np.ascontiguousarray(host[:, d:])).cuda()
    for v in lost:
        (data[:, v] if v < d else par[:, v - d]).fill_(0x33)
    r.reconst_batch_split(data, par, [], lost)
    torch.cuda.synchronize()
    assert np.array_equal(data.cpu().numpy(), host[:, :d]) and np.array_equal(par.cpu().numpy(), host[:, d:])


@pytest.mark.parametrize("rows,cols", [(17, 5), (24, 33), (56, 200), (64, 64), (128, 128), (40, 1), (33, 7)])
def test_wide_asm_jit_unshared_columns(rslib, orc, torch_dev, asm_jit, rows, cols):
    """rs_tune("jit_share", 0): every wave of a multi-wave kernel loads and
    transposes every column itself (the default shares them through LDS, and
    the tests above run that); overwrite and accumulate, aligned and ragged
    sizes, against the oracle."""
    assert asm_jit.rs_tune(b"jit_share", 0) == 0
    try:
        test_wide_asm_jit_vs_oracle(rslib, orc, torch_dev, asm_jit, rows, cols)
    finally:
        asm_jit.rs_tune(b"jit_share", 1)


@pytest.mark.parametrize("rows,cols", [(64, 64), (128, 17), (33, 7)])
def test_wide_asm_jit_shared_deep(rslib, orc, torch_dev, asm_jit, rows, cols):
    """rs_tune("jit_share_deep", 1): shared columns with two steps of loads in
    flight and the next column's planes read from LDS ahead (lgkmcnt(2)),
    against the oracle."""
    assert asm_jit.rs_tune(b"jit_share_deep", 1) == 0
    try:
        test_wide_asm_jit_vs_oracle(rslib, orc, torch_dev, asm_jit, rows, cols)
    finally:
        asm_jit.rs_tune(b"jit_share_deep", 0)


@pytest.mark.parametrize("rows,cols,dma", [(64, 64, 3), (128, 128, 4), (33, 7, 2), (56, 200, 4), (17, 5, 8)])
def test_wide_asm_jit_shared_dma(rslib, orc, torch_dev, asm_jit, rows, cols, dma):
    """rs_tune("jit_share_dma", n): shared columns streamed into per-wave LDS
    rings by LDS-DMA loads (buffer_load_dwordx4 ... lds), n - 1 steps ahead,
    against the oracle on the GPU (overwrite and accumulate, aligned and
    ragged sizes)."""
    assert asm_jit.rs_tune(b"jit_share_dma", dma) == 0
    try:
        test_wide_asm_jit_vs_oracle(rslib, orc, torch_dev, asm_jit, rows, cols)
    finally:
        asm_jit.rs_tune(b"jit_share_dma", 0)


@pytest.mark.parametrize("rows,cols,layout,gray,ahead", [(64, 64, 0, 1, 1), (128, 128, 2, 1, 1), (33, 7, 0, 1, 0),
                                                        (56, 200, 2, 0, 1), (16, 16, 0, 1, 0), (100, 28, 2, 1, 1)])
def test_wide_asm_jit_gray_ahead(rslib, orc, torch_dev, asm_jit, rows, cols, layout, gray, ahead):
    """rs_tune("jit_gray", 1) (low-half subsets built one at a time in
    Gray-code order) and rs_tune("jit_share_ahead", 1) (the next column's
    planes read from LDS while one combines, lgkmcnt(2)), alone and together,
    in layout 0 and the row-group layout 2, against the oracle on the GPU."""
    assert asm_jit.rs_tune(b"jit_layout", layout) == 0
    assert asm_jit.rs_tune(b"jit_gray", gray) == 0 and asm_jit.rs_tune(b"jit_share_ahead", ahead) == 0
    try:
        test_wide_asm_jit_vs_oracle(rslib, orc, torch_dev, asm_jit, rows, cols)
    finally:
        asm_jit.rs_tune(b"jit_layout", 2)
        asm_jit.rs_tune(b"jit_gray", 0)
        asm_jit.rs_tune(b"jit_share_ahead", 0)


@pytest.mark.parametrize("rows,cols,gw,dma", [(128, 128, 4, 0), (100, 28, 4, 0), (64, 64, 2, 0), (56, 200, 2, 0),
                                              (128, 17, 4, 3), (40, 9, 2, 2)])
def test_wide_asm_jit_grouped_shared(rslib, orc, torch_dev, asm_jit, rows, cols, gw, dma):
    """rs_tune("jit_layout", 2): row groups of shared-column workgroups (at
    most `gw` waves each, G workgroups per chunk, XCD-mapped), with and
    without the LDS-DMA rings, against the oracle on the GPU."""
    assert asm_jit.rs_tune(b"jit_layout", 2) == 0 and asm_jit.rs_tune(b"jit_group_waves", gw) == 0
    assert asm_jit.rs_tune(b"jit_share_dma", dma) == 0
    try:
        test_wide_asm_jit_vs_oracle(rslib, orc, torch_dev, asm_jit, rows, cols)
    finally:
        asm_jit.rs_tune(b"jit_layout", 2)
        asm_jit.rs_tune(b"jit_group_waves", 4)
        asm_jit.rs_tune(b"jit_share_dma", 0)


@pytest.mark.parametrize("d,p,S", [(64, 64, 4), (128, 128, 2), (200, 56, 2)])
def test_wide_full_size_round_trip(rslib, orc, torch_dev, asm_jit, d, p, S):
    """Full-size wide stripes (1 MiB vectors) through the compiled shared-column
    kernels: encode, destroy p vectors (data and parity), rebuild, and the
    stripes equal the originals; the first stripe's parity also equals the
    oracle's (size-independent round trip plus one oracle spot check)."""
    torch = torch_dev
    vec = 1 << 20
    rng = np.random.default_rng(d * 31 + p)
    r = rslib.New(d, p)
    g = torch.Generator(device="cuda").manual_seed(d + p)
    buf = torch.empty((S, d + p, vec), dtype=torch.uint8, device="cuda")
    buf[:, :d].random_(0, 256, generator=g)
    r.encode_batch(buf)
    torch.cuda.synchronize()
    G = orc.gen_matrix(d, p).reshape(p, d)
    host0 = buf[0].cpu().numpy()
    assert np.array_equal(host0[d:], orc.encode_numpy(G, host0[None, :d])[0])
    ref = buf.clone()
    lost = sorted(int(v) for v in rng.choice(d + p, p, replace=False))
    buf[:, lost] = 0x5A
    r.reconst_batch(buf, [], lost)
    torch.cuda.synchronize()
    assert torch.equal(buf, ref), (d, p, lost[:8])
