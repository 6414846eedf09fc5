"""The run-time kernel generator's gfx950 assembly (jit_asm.cpp), checked on
the CPU: the source from rs_jit_asm_source is assembled by comgr (as the
library does at run time, no device needed) and executed by a small
emulator of the instructions it uses (tests/asm_emu.py) over random stripes;
every output byte must equal the oracle's product (encodePart rs.go:175-203:
out[r] = XOR_c G[r][c] * in[c], or out[r] ^= ... in accumulate mode).  The
GPU tests (tests/test_gpu_jit.py, tests/test_gpu_wide.py) run the same
kernels on the MI355X."""
import struct

import numpy as np
import pytest

from asm_emu import Emu, Memory

KMAXPTRS = 260


@pytest.fixture(autouse=True)
def _layout0_unless_set(rslib):
    """These tests describe the kernels by layout 0's shape (nw = paths per
    workgroup, one workgroup per chunk) unless they pick a layout themselves;
    the library's default (2) is layout 0 up to jit_group_waves paths."""
    L = rslib.lib()
    assert L.rs_tune(b"jit_layout", 0) == 0
    yield
    L.rs_tune(b"jit_layout", 2)


def _karg(body, stripe0, stripe_ids, ptrs, strides16):
    b = struct.pack("<IIQ", body, stripe0, stripe_ids)
    p = list(ptrs) + [0] * (KMAXPTRS - len(ptrs))
    s = list(strides16) + [0] * (KMAXPTRS - len(strides16))
    b += struct.pack(f"<{KMAXPTRS}Q", *p) + struct.pack(f"<{KMAXPTRS}I", *s)
    assert len(b) == 3136
    return b


@pytest.mark.parametrize("rows,cols,acc", [(5, 10, 0), (8, 10, 1), (3, 7, 0), (16, 16, 0), (12, 5, 1),
                                           (20, 4, 0), (33, 3, 1), (9, 1, 0), (17, 5, 0)])
def test_asm_kernel_matches_oracle(rslib, orc, rows, cols, acc):
    _check_kernel(rslib, orc, rows, cols, acc)


@pytest.mark.parametrize("rows,cols,sync", [(33, 7, 2), (40, 9, 4), (17, 5, 1)])
def test_asm_kernel_with_barriers(rslib, orc, rows, cols, sync):
    """rs_tune("jit_sync", n): the waves of a multi-wave kernel meet at
    s_barrier every n columns; the same number of barriers in every wave."""
    L = rslib.lib()
    assert L.rs_tune(b"jit_sync", sync) == 0 and L.rs_tune(b"jit_share", 0) == 0  # (shared columns: own barriers)
    try:
        src = _check_kernel(rslib, orc, rows, cols, 0)
    finally:
        L.rs_tune(b"jit_sync", 0)
        L.rs_tune(b"jit_share", 1)
    nw = (rows + 15) // 16
    assert src.count("s_barrier") == nw * ((cols - 1) // sync)


@pytest.mark.parametrize("rows,cols,acc,gw", [(33, 3, 1, 2), (17, 5, 0, 1), (40, 9, 0, 4), (9, 1, 0, 2),
                                            (20, 4, 0, 8), (16, 16, 1, 4), (64, 5, 0, 2)])
def test_asm_kernel_row_group_layout(rslib, orc, rows, cols, acc, gw):
    """rs_tune("jit_layout", 1): row groups over workgroups (grid x = chunk
    groups of gw chunks x row groups, laid out 8 chunk groups at a time so
    the row groups of one chunk group share an XCD), every wave of a
    workgroup on its own chunk with the same code; padded workgroups past the
    body leave at once."""
    L = rslib.lib()
    assert L.rs_tune(b"jit_layout", 1) == 0 and L.rs_tune(b"jit_group_waves", gw) == 0
    try:
        _check_kernel(rslib, orc, rows, cols, acc, layout=1, gw=gw)
    finally:
        L.rs_tune(b"jit_layout", 0)
        L.rs_tune(b"jit_group_waves", 4)


def _check_kernel(rslib, orc, rows, cols, acc, layout=0, gw=4, paths=None, edit=None, groups=1):
    rng = np.random.default_rng(rows * 1000 + cols * 10 + acc)
    mat = rng.integers(0, 256, (rows, cols), dtype=np.uint8)
    src = rslib.jit_asm_source(mat, bool(acc))
    if edit:
        src = edit(src)
    assert "rs_bs_asm" in src and "s_endpgm" in src
    if not edit:
        rslib.jit_compile_check(mat, bool(acc))  # assembles and links with comgr (the library's own path)
    S, body, vlen = 3, 4096, 4096 + 32      # two 2 KiB chunks per vector, bytes past the body untouched
    nvec = cols + rows
    mem = Memory(S * nvec * vlen + 65536)
    # every vector in its own region: vector v of stripe s at ptr[v] + s * stride
    stride = vlen * nvec
    region = mem.alloc(S * stride)
    ptrs = [region + v * vlen for v in range(nvec)]
    host = rng.integers(0, 256, (S, nvec, vlen), dtype=np.uint8)
    mem.view(region, S * stride)[:] = host.reshape(-1)
    # launch stripes through a stripe-id list (reversed order), as grouped launches do
    ids = mem.alloc(4 * S)
    mem.view(ids, 4 * S).view(np.uint32)[:] = np.arange(S)[::-1]
    from reedsolomon_amd.rs import lib  # noqa: F401  (library loaded by the fixture)
    if paths is None:
        paths = 1 if rows <= 16 else (rows + 15) // 16
    if layout == 1:  # the library's launch rule (kernels.hip): ceil(chunk groups / 8) * 8 * row groups
        nw, cgs = gw, (body // 2048 + gw - 1) // gw
        grid = ((cgs + 7) // 8 * 8 * paths, S)
    elif layout == 2:  # chunk groups of one chunk, `groups` row groups of gw waves each
        nw, cgs = gw, body // 2048
        grid = ((cgs + 7) // 8 * 8 * groups, S)
    else:
        nw, grid = paths, (body // 2048, S)
    emu = Emu(mem)
    emu.launch(src, _karg(body, 0, ids, ptrs, [stride // 16] * nvec), grid, nw)
    got = mem.view(region, S * stride).reshape(S, nvec, vlen)
    exp = orc.encode_numpy(mat, host[:, :cols, :body])
    if acc:
        exp = exp ^ host[:, cols:, :body]
    assert np.array_equal(got[:, cols:, :body], exp)
    assert np.array_equal(got[:, :cols], host[:, :cols])             # inputs untouched
    assert np.array_equal(got[:, cols:, body:], host[:, cols:, body:])  # past the body untouched
    return src


@pytest.mark.parametrize("waves,vgprs", [(2, 256), (4, 128), (0, None)])
def test_asm_kernel_occupancy_cap(rslib, waves, vgprs):
    """rs_tune("jit_waves", n): the kernel declares 512 / n VGPRs (granule 8,
    at most 256) so at most n waves share a SIMD; 0 declares what it uses."""
    import re

    L = rslib.lib()
    mat = np.random.default_rng(3).integers(0, 256, (5, 10), dtype=np.uint8)
    assert L.rs_tune(b"jit_waves", waves) == 0
    try:
        src = rslib.jit_asm_source(mat, False)
    finally:
        L.rs_tune(b"jit_waves", 2)
    declared = int(re.search(r"\.amdhsa_next_free_vgpr (\d+)", src).group(1))
    if vgprs is None:
        assert declared < 128  # 5 rows x 8 planes + slots + subsets
    else:
        assert declared == vgprs


@pytest.mark.parametrize("rows,cols,acc,pf,sync,layout", [(5, 10, 0, 3, 0, 0), (8, 10, 1, 3, 0, 0), (3, 7, 0, 1, 0, 0),
                                                          (16, 16, 0, 4, 0, 0), (12, 5, 1, 2, 0, 0), (33, 3, 1, 3, 0, 0),
                                                          (17, 5, 0, 3, 1, 0), (40, 9, 0, 3, 4, 0), (9, 1, 0, 3, 0, 0),
                                                          (64, 64, 0, 3, 0, 0), (56, 200, 1, 3, 0, 0),
                                                          (128, 128, 0, 3, 0, 0), (128, 256, 1, 2, 0, 0),
                                                          (33, 3, 1, 3, 0, 1), (128, 128, 0, 3, 0, 1),
                                                          (56, 200, 1, 3, 2, 1), (16, 16, 0, 3, 0, 1)])
def test_machine_code_equals_assembler(rslib, rows, cols, acc, pf, sync, layout):
    """The default backend encodes the kernel straight into gfx950 machine
    code (no assembler at run time); those bytes equal comgr's assembly of the
    generator's text for the same matrix and settings, instruction for
    instruction (rs_jit_encoder_check), so the emulator runs above and the GPU
    tests of the assembly path cover the machine code too."""
    L = rslib.lib()
    mat = np.random.default_rng(rows * 31 + cols).integers(0, 256, (rows, cols), dtype=np.uint8)
    assert L.rs_tune(b"jit_pf", pf) == 0 and L.rs_tune(b"jit_sync", sync) == 0
    assert L.rs_tune(b"jit_layout", layout) == 0
    try:
        n = rslib.jit_encoder_check(mat, bool(acc))
    finally:
        L.rs_tune(b"jit_pf", 3)
        L.rs_tune(b"jit_sync", 0)
        L.rs_tune(b"jit_layout", 0)
    assert n > 0 and n % 4 == 0


@pytest.mark.parametrize("rows,cols,acc,path_rows,layout", [(40, 9, 0, 11, 0), (33, 5, 1, 8, 1), (20, 3, 0, 7, 0)])
def test_asm_kernel_path_rows(rslib, orc, rows, cols, acc, path_rows, layout):
    """rs_tune("jit_path_rows", n): products of more than 16 rows in code
    paths of n rows (fewer VGPRs per wave), either layout, against the oracle."""
    L = rslib.lib()
    assert L.rs_tune(b"jit_path_rows", path_rows) == 0 and L.rs_tune(b"jit_layout", layout) == 0
    try:
        paths = (rows + path_rows - 1) // path_rows
        _check_kernel(rslib, orc, rows, cols, acc, layout=layout, gw=4, paths=paths)
    finally:
        L.rs_tune(b"jit_path_rows", 16)
        L.rs_tune(b"jit_layout", 0)


@pytest.mark.parametrize("rows,cols,acc,share,deep,kc", [(33, 7, 0, 1, -1, 1), (40, 9, 1, 1, -1, 1), (17, 5, 0, 1, -1, 1),
                                                        (64, 5, 1, 1, -1, 1), (20, 1, 0, 1, -1, 1), (48, 12, 0, 1, -1, 1),
                                                        (33, 7, 0, 0, -1, 1), (40, 9, 1, 0, -1, 1), (33, 7, 1, 1, 1, 1),
                                                        (64, 13, 0, 1, 1, 1), (17, 2, 0, 1, 1, 1), (128, 9, 1, 1, -1, 1),
                                                        (128, 17, 0, 1, 0, 1), (33, 7, 0, 1, 0, 2), (40, 13, 1, 1, 0, 2),
                                                        (17, 3, 0, 1, 0, 2), (128, 19, 0, 1, 0, 2), (64, 1, 1, 1, 0, 2)])
def test_asm_kernel_shared_columns(rslib, orc, rows, cols, acc, share, deep, kc):
    """rs_tune("jit_share", 1, the default): the waves of a multi-path workgroup share the
    column work through LDS (step s: wave w loads and transposes column
    s * nw + w into LDS buffer s & 1, barrier, every wave combines the step's
    columns).  Against the oracle, with the emulator's LDS race check (waves
    run between barriers in alternating order; a read of bytes another wave
    wrote in the same round fails); ragged last steps and waves without a
    column included.  share=0: every wave loads and transposes every column,
    no LDS, no barrier.  deep (rs_tune("jit_share_deep"); -1 = 8-wave
    workgroups only): two steps of loads in flight and the next column's
    planes read from LDS while the current one combines (lgkmcnt(2))."""
    L = rslib.lib()
    assert L.rs_tune(b"jit_share", share) == 0 and L.rs_tune(b"jit_share_deep", deep) == 0
    assert L.rs_tune(b"jit_share_cols", kc) == 0
    try:
        src = _check_kernel(rslib, orc, rows, cols, acc)
    finally:
        L.rs_tune(b"jit_share", 1)
        L.rs_tune(b"jit_share_deep", 0)
        L.rs_tune(b"jit_share_cols", 1)
    is_deep = share and kc == 1 and (deep == 1 or (deep == -1 and rows > 112))
    assert ("lgkmcnt(2)" in src) == bool(is_deep and cols > 1)
    nw = (rows + 15) // 16
    steps = (cols + nw * kc - 1) // (nw * kc)
    assert src.count("s_barrier") == (nw * steps if share else 0)
    assert src.count("ds_write_b128") == (2 * cols if share else 0)
    assert f".amdhsa_group_segment_fixed_size {2 * nw * kc * 2048 if share else 0}" in src


@pytest.mark.parametrize("rows,cols,acc,share", [(64, 64, 0, 1), (56, 200, 1, 1), (128, 128, 0, 1), (33, 3, 1, 1),
                                                (17, 5, 0, 1), (64, 64, 0, 0), (128, 256, 1, 0), (64, 64, 1, 2),
                                                (24, 7, 0, 2)])
def test_machine_code_equals_assembler_shared(rslib, rows, cols, acc, share):
    """The shared-column kernels' machine code (ds_write_b128 / ds_read_b128,
    barriers), and the unshared ones', equal comgr's assembly of their text
    (share=2: the deep variant, lgkmcnt(2) included)."""
    L = rslib.lib()
    mat = np.random.default_rng(rows * 37 + cols).integers(0, 256, (rows, cols), dtype=np.uint8)
    assert L.rs_tune(b"jit_share", min(share, 1)) == 0
    assert L.rs_tune(b"jit_share_deep", 1 if share == 2 else 0) == 0
    try:
        n = rslib.jit_encoder_check(mat, bool(acc))
    finally:
        L.rs_tune(b"jit_share", 1)
        L.rs_tune(b"jit_share_deep", 0)
    assert n > 0 and n % 4 == 0


def test_emulator_catches_a_missing_barrier(rslib, orc):
    """The race check is live: the shared-column kernel with its barriers
    removed fails in the emulator (a wave reads LDS bytes another wave wrote
    in the same round)."""
    from asm_emu import LdsRaceError

    L = rslib.lib()
    assert L.rs_tune(b"jit_share", 1) == 0
    try:
        with pytest.raises(LdsRaceError):
            _check_kernel(rslib, orc, 33, 7, 0, edit=lambda s: s.replace("\ts_barrier\n", ""))
    finally:
        L.rs_tune(b"jit_share", 1)


@pytest.mark.parametrize("rows,cols,acc", [(16, 20, 0), (12, 9, 1), (9, 17, 0)])
def test_asm_kernel_split_small(rslib, orc, rows, cols, acc):
    """rs_tune("jit_split_cols", n): products of 9-16 rows over at least n
    columns run as two paths of at most 8 rows in one workgroup, sharing the
    columns through LDS, against the oracle."""
    L = rslib.lib()
    assert L.rs_tune(b"jit_split_cols", 8) == 0
    try:
        src = _check_kernel(rslib, orc, rows, cols, acc, paths=2)
    finally:
        L.rs_tune(b"jit_split_cols", 0)
    assert "ds_write_b128" in src and ".amdhsa_group_segment_fixed_size 8192" in src


@pytest.mark.parametrize("rows,cols,acc,dma", [(33, 7, 0, 3), (40, 9, 1, 2), (17, 5, 0, 4), (64, 13, 0, 3),
                                               (64, 1, 1, 4), (128, 19, 0, 3), (48, 30, 1, 6), (20, 2, 0, 8)])
def test_asm_kernel_shared_columns_dma(rslib, orc, rows, cols, acc, dma):
    """rs_tune("jit_share_dma", n): each wave's columns stream into a private
    LDS ring of n steps through LDS-DMA loads (buffer_load_dwordx4 ... lds,
    n - 1 steps ahead), are read back into the plane registers (ds_read_b64),
    transposed and shared as before.  Against the oracle in the emulator,
    which fails an LDS read of bytes whose DMA was not waited for (vmcnt) and
    the usual cross-wave races; ragged steps and short columns included."""
    L = rslib.lib()
    assert L.rs_tune(b"jit_share_dma", dma) == 0
    try:
        src = _check_kernel(rslib, orc, rows, cols, acc)
    finally:
        L.rs_tune(b"jit_share_dma", 0)
    nw = (rows + 15) // 16
    assert src.count(" lds") == 2 * cols  # two 1 KiB LDS-DMA loads per column
    assert src.count("ds_read_b64") == 4 * cols
    assert f".amdhsa_group_segment_fixed_size {(2 + dma) * nw * 2048}" in src


def test_emulator_catches_an_unwaited_dma(rslib, orc):
    """The DMA wait check is live: the same kernel with every vmcnt wait made
    a no-op reads ring bytes whose LDS-DMA is still outstanding."""
    import re

    from asm_emu import WaitcntError

    L = rslib.lib()
    assert L.rs_tune(b"jit_share_dma", 3) == 0
    try:
        with pytest.raises(WaitcntError):
            _check_kernel(rslib, orc, 33, 7, 0, edit=lambda s: re.sub(r"vmcnt\(\d+\)", "vmcnt(63)", s))
    finally:
        L.rs_tune(b"jit_share_dma", 0)


@pytest.mark.parametrize("rows,cols,acc,dma", [(64, 64, 0, 4), (128, 128, 1, 3), (56, 200, 0, 4), (33, 3, 1, 2)])
def test_machine_code_equals_assembler_dma(rslib, rows, cols, acc, dma):
    """The DMA-ring kernels' machine code (M0 writes, buffer_load_dwordx4 ...
    lds, ds_read_b64) equals comgr's assembly of their text."""
    L = rslib.lib()
    mat = np.random.default_rng(rows * 41 + cols).integers(0, 256, (rows, cols), dtype=np.uint8)
    assert L.rs_tune(b"jit_share_dma", dma) == 0
    try:
        n = rslib.jit_encoder_check(mat, bool(acc))
    finally:
        L.rs_tune(b"jit_share_dma", 0)
    assert n > 0 and n % 4 == 0


def _layout2_shape(rows, gw):
    """asm_shape(rows, layout 2, gw) (jit_asm.hpp): (row groups, waves per workgroup, rows per path)."""
    paths = (rows + 15) // 16
    G = (paths + gw - 1) // gw
    nw = (paths + G - 1) // G
    rw = (rows + G * nw - 1) // (G * nw)
    return G, nw, rw


@pytest.mark.parametrize("rows,cols,acc,gw,dma", [(128, 9, 0, 4, 0), (100, 7, 1, 4, 0), (65, 5, 1, 2, 0),
                                                  (40, 13, 0, 2, 0), (128, 9, 1, 4, 3), (72, 11, 0, 2, 2)])
def test_asm_kernel_grouped_shared_layout(rslib, orc, rows, cols, acc, gw, dma):
    """rs_tune("jit_layout", 2): row groups of shared-column workgroups - a
    workgroup is at most jit_group_waves waves over one 2 KiB chunk, each with
    its own path (g * nw + w) of the rows, sharing the columns through LDS;
    the G row groups of a chunk are G workgroups mapped XCD-aware as in
    layout 1 (grid ceil(chunks / 8) * 8 * G).  Against the oracle in the
    emulator with the LDS race and DMA wait checks; rows spread evenly over
    the paths (100 rows: 8 paths of 13)."""
    L = rslib.lib()
    G, nw, rw = _layout2_shape(rows, gw)
    assert G > 1 and (G * nw - 1) * rw < rows
    assert L.rs_tune(b"jit_layout", 2) == 0 and L.rs_tune(b"jit_group_waves", gw) == 0
    assert L.rs_tune(b"jit_share_dma", dma) == 0
    try:
        src = _check_kernel(rslib, orc, rows, cols, acc, layout=2, gw=nw, groups=G)
    finally:
        L.rs_tune(b"jit_layout", 0)
        L.rs_tune(b"jit_group_waves", 4)
        L.rs_tune(b"jit_share_dma", 0)
    steps = (cols + nw - 1) // nw
    assert src.count("s_barrier") == G * nw * steps  # every path's code has one barrier per step
    assert f".amdhsa_group_segment_fixed_size {(2 + dma) * nw * 2048}" in src


@pytest.mark.parametrize("rows,cols,acc,dma", [(128, 128, 0, 0), (128, 64, 1, 3), (100, 28, 0, 0)])
def test_machine_code_equals_assembler_grouped(rslib, rows, cols, acc, dma):
    """Layout 2's machine code (path dispatch on g * nw + w) equals comgr's
    assembly of its text."""
    L = rslib.lib()
    mat = np.random.default_rng(rows * 43 + cols).integers(0, 256, (rows, cols), dtype=np.uint8)
    assert L.rs_tune(b"jit_layout", 2) == 0 and L.rs_tune(b"jit_share_dma", dma) == 0
    try:
        n = rslib.jit_encoder_check(mat, bool(acc))
    finally:
        L.rs_tune(b"jit_layout", 0)
        L.rs_tune(b"jit_share_dma", 0)
    assert n > 0 and n % 4 == 0


def _vgprs_used(src):
    import re
    return int(re.search(r"\.amdhsa_next_free_vgpr (\d+)", src).group(1))


@pytest.mark.parametrize("rows,cols,acc,layout,gw,dma", [(5, 10, 0, 0, 4, 0), (16, 16, 1, 0, 4, 0), (33, 7, 0, 0, 4, 0),
                                                         (40, 9, 1, 0, 4, 0), (64, 13, 0, 0, 4, 3), (17, 2, 1, 0, 4, 0),
                                                         (128, 9, 0, 2, 4, 0), (100, 7, 1, 2, 4, 0),
                                                         (72, 11, 0, 2, 2, 2), (33, 5, 1, 1, 4, 0)])
@pytest.mark.parametrize("gray,ahead", [(1, 0), (0, 1), (1, 1)])
def test_asm_kernel_gray_subsets_and_read_ahead(rslib, orc, rows, cols, acc, layout, gw, dma, gray, ahead):
    """rs_tune("jit_gray", 1): the low half's subsets are built one at a time
    into one register in Gray-code order (one XOR / xor3 each, from the subset
    before or from the planes) with the outputs they feed updated right after
    - 12 subset registers instead of 22.  rs_tune("jit_share_ahead", 1): a
    shared-column kernel reads the next column's planes from LDS while this
    one combines (lgkmcnt(2) with the staging scalar loads possibly still
    out: LDS reads return in order).  Against the oracle in the emulator
    (LDS races, wait counts) for every layout, accumulate included."""
    L = rslib.lib()
    assert L.rs_tune(b"jit_layout", layout) == 0 and L.rs_tune(b"jit_group_waves", gw) == 0
    assert L.rs_tune(b"jit_share_dma", dma) == 0
    # (no occupancy cap: the kernel declares the VGPRs it uses)
    assert L.rs_tune(b"jit_waves", 0) == 0 and L.rs_tune(b"jit_wide_waves", 0) == 0
    mat = np.random.default_rng(rows * 1000 + cols * 10 + acc).integers(0, 256, (rows, cols), dtype=np.uint8)
    base = _vgprs_used(rslib.jit_asm_source(mat, bool(acc)))
    assert L.rs_tune(b"jit_gray", gray) == 0 and L.rs_tune(b"jit_share_ahead", ahead) == 0
    try:
        paths = 1 if rows <= 16 else (rows + 15) // 16
        if layout == 2:
            G, nw, _rw = _layout2_shape(rows, gw)
            src = _check_kernel(rslib, orc, rows, cols, acc, layout=2, gw=nw, groups=G)
        else:
            src = _check_kernel(rslib, orc, rows, cols, acc, layout=layout, gw=gw, paths=paths)
    finally:
        L.rs_tune(b"jit_gray", 0)
        L.rs_tune(b"jit_share_ahead", 0)
        L.rs_tune(b"jit_layout", 0)
        L.rs_tune(b"jit_group_waves", 4)
        L.rs_tune(b"jit_share_dma", 0)
        L.rs_tune(b"jit_waves", 2)
        L.rs_tune(b"jit_wide_waves", 3)
    shared = layout != 1 and paths > 1
    assert ("lgkmcnt(2)" in src) == bool(ahead and shared and cols > 1)
    # registers: 10 fewer with gray, 8 more with the read-ahead plane set
    # (declared VGPRs round up to 4)
    want = base - (10 if gray else 0) + (8 if ahead and shared else 0)
    assert abs(_vgprs_used(src) - want) <= 3


@pytest.mark.parametrize("rows,cols,acc,layout", [(128, 128, 0, 2), (64, 64, 1, 0), (56, 200, 0, 0), (16, 16, 1, 0)])
def test_machine_code_equals_assembler_gray_ahead(rslib, rows, cols, acc, layout):
    """The gray / read-ahead kernels' machine code equals comgr's assembly of
    their text."""
    L = rslib.lib()
    mat = np.random.default_rng(rows * 47 + cols).integers(0, 256, (rows, cols), dtype=np.uint8)
    assert L.rs_tune(b"jit_layout", layout) == 0
    assert L.rs_tune(b"jit_gray", 1) == 0 and L.rs_tune(b"jit_share_ahead", 1) == 0
    try:
        n = rslib.jit_encoder_check(mat, bool(acc))
    finally:
        L.rs_tune(b"jit_gray", 0)
        L.rs_tune(b"jit_share_ahead", 0)
        L.rs_tune(b"jit_layout", 0)
    assert n > 0 and n % 4 == 0
