"""Every value rs_tune accepts in the product library computes the same bytes.

The reference has no tuning switches: its Encode / Reconst / Update
(rs.go:104-203, :221-380, :424-477) are one definition.  librsamd's rs_tune
knobs choose kernel shapes, staging paths and the host-call engine, so each
accepted value must leave every output byte unchanged.  For every knob the
header documents (the list is parsed from include/rs_amd.h, so a new knob
without a sweep entry fails here) and every value in its sweep, this runs
10+4, 10+8 and 20+12 at 64 KiB through the device batch API (interleaved and split
layouts, in-place Reconst, Update), the synchronous host API (Encode, Reconst,
Update) and a pinned host batch, and compares every byte with the CPU oracle.
"""
import os
import re

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# knob -> values swept (each one set, checked, then the default restored)
SWEEP = {
    "max_grid": [1024, 0],
    "vpt": [2, 1],
    "nt_store": [0, 1],
    "lds_pad": [65536, 0],
    "lane_bytes": [16, 8],
    "block8": [256, 128],
    "bitslice": [0, 1],
    "bs_block": [64, 128, 256, 0],
    "bs_waves": [0, 4, 2],
    "wide_block": [128, 256],
    "wide_single_pass": [0, 1],
    "host_engine": [0, 1],
    "host_engine_waves": [1, 64, 8],
    "host_engine_group_waves": [1, 8],
    "host_engine_direct": [0, 1],
    "host_engine_wg_units": [1, 0],
    "host_engine_poll_gap": [100, 0],
    "host_engine_yield_us": [1, 0],
    "host_engine_idle_us": [20, 2000],
    "host_engine_life_us": [100, 4000],
    "host_engine_vram": [0, 1],
    "host_engine_split_rows": [1, 0, 2],
    "host_engine_cold_launch": [0, 1],
    "host_flag_sync": [0, 1],
    "host_engine_max_bytes": [0, 1 << 20],
    "host_pinned_max": [0, 4 << 20, 256 << 10],
    "host_zc_max": [0, 2 << 20, -1],
    "host_chunk": [4096, 128 << 10],
    "host_chunk_split": [0, 1, 4],
    "host_coalesce_max": [0, 128 << 10],
    "host_coalesce_linger_us": [100, 0],
    "host_coalesce_running": [1, 2],
    "host_batch_zc": [0, 1],
    "host_unregister_revoke": [0, 1],
    "host_dma_1d": [1, 0],
    "host_pageable_stage": [0, 1],
    "host_pageable_slot": [4096, 32 << 20, 8 << 20],
    "host_copy_nt": [0, 1],
    "host_copy_coalesce": [0, 1],
    "bind_numa": [0, 1],
    "jit": [0, 2, 1],
    "jit_min_launches": [1, 2],
    "jit_min_bytes": [0, 8 << 20],
    "jit_min_acc_cols": [8, 1],
    "jit_min_rows": [1, 5],
    "jit_pf": [1, 2, 4, 6, 3],
    "jit_sync": [1, 4, 0],
    "jit_waves": [0, 4, 2],
    "jit_disk_cache": [0, 1],
    "jit_backend": [0, 1, 2],
    "jit_layout": [1, 0, 2],
    "jit_group_waves": [2, 8, 4],
    "jit_path_rows": [5, 11, 16],
    "jit_wide_pf": [1, 3, 2],
    "jit_wide_waves": [0, 2, 3],
    "jit_share": [0, 1],
    "jit_share_deep": [1, -1, 0],
    "jit_share_dma": [3, 0],
    "jit_share_ahead": [1, 0],
    "jit_gray": [1, 0],
    "jit_split_cols": [4, 0],
    "jit_share_cols": [2, -1, 1],
    "table_registry_max": [1, 1 << 14],
    "table_inplace_max": [0, 1 << 30, 2 << 20],
    "table_stage_vram": [1, 0],
    "multi_gpu_plan": [1, 0, 8, -1],
}

# 20+12: 12 output rows (the wide single-pass kernels, or a compiled network)
SHAPES = [(10, 4, [0, 5, 11, 13]), (10, 8, [0, 1, 2, 4, 6, 8, 12, 15]),
          (20, 12, [0, 1, 2, 3, 5, 8, 13, 19, 21, 25, 30, 31])]
S, N = 3, 64 << 10
UPD_ROW = 3


def _documented_knobs():
    text = open(os.path.join(ROOT, "include", "rs_amd.h")).read()
    doc = text[text.index("Expert launch knobs"):text.index("RS_API int rs_tune")]
    return sorted(set(re.findall(r'"(\w+)"', doc)))


def test_sweep_covers_every_documented_knob():
    assert sorted(SWEEP) == _documented_knobs()


@pytest.fixture(scope="module")
def cases(orc):
    """Inputs and oracle outputs per shape (computed once)."""
    out = {}
    for d, p, lost in SHAPES:
        rng = np.random.default_rng(d * 100 + p)
        data = rng.integers(0, 256, (S, d, N), dtype=np.uint8)
        full = np.empty((S, d + p, N), np.uint8)
        full[:, :d] = data
        full[:, d:] = orc.encode_numpy(orc.gen_matrix(d, p).reshape(p, d), data)
        new = rng.integers(0, 256, (S, N), dtype=np.uint8)
        upd = full.copy()
        for s in range(S):
            par = [upd[s, d + j].copy() for j in range(p)]
            assert orc.update(d, p, full[s, UPD_ROW].copy(), new[s].copy(), UPD_ROW, par) == 0
            for j in range(p):
                upd[s, d + j] = par[j]
            upd[s, UPD_ROW] = new[s]
        out[(d, p)] = (full, new, upd, lost)
    return out


def _check_all(rslib, torch, cases, tag):
    for (d, p), (full, new, upd, lost) in cases.items():
        r = rslib.New(d, p)
        # device batch, interleaved [S][d+p][N]
        buf = torch.from_numpy(full).cuda()
        buf[:, d:] = 0xA5
        r.encode_batch(buf)
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy(), full), (tag, d, p, "encode_batch")
        # device batch, split layout
        dat = torch.from_numpy(np.ascontiguousarray(full[:, :d])).cuda()
        par = torch.full((S, p, N), 0x5A, dtype=torch.uint8, device="cuda")
        r.encode_batch_split(dat, par)
        torch.cuda.synchronize()
        assert np.array_equal(par.cpu().numpy(), full[:, d:]), (tag, d, p, "encode_batch_split")
        # in-place Reconst (garbage in the lost vectors)
        buf[:, lost] = 0x77
        r.reconst_batch(buf, [], lost)
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy(), full), (tag, d, p, "reconst_batch")
        # multi-pattern Reconst: a different erasure set per stripe (the
        # single launch up to 8 lost vectors, grouped launches beyond)
        pats = [lost[:1], lost[:max(2, len(lost) // 2)], lost]
        masks = np.array([sum(1 << v for v in pat) for pat in pats], dtype=np.uint64)
        for s, pat in enumerate(pats):
            buf[s, pat] = 0x4D
        r.reconst_batch_multi(buf[:, :d], buf[:, d:], masks)
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy(), full), (tag, d, p, "reconst_batch_multi")
        # Update of one data row
        old_t = buf[:, UPD_ROW].clone()
        new_t = torch.from_numpy(new).cuda()
        r.update_batch(old_t, new_t, UPD_ROW, buf)
        buf[:, UPD_ROW] = new_t
        torch.cuda.synchronize()
        assert np.array_equal(buf.cpu().numpy(), upd), (tag, d, p, "update_batch")
        # synchronous host API on stripe 1
        v = [full[1, i].copy() for i in range(d)] + [np.full(N, 0xA5, np.uint8) for _ in range(p)]
        r.Encode(v)
        assert all(np.array_equal(v[i], full[1, i]) for i in range(d + p)), (tag, d, p, "Encode")
        for i in lost:
            v[i][:] = 0x33
        r.Reconst(v, [], lost)
        assert all(np.array_equal(v[i], full[1, i]) for i in range(d + p)), (tag, d, p, "Reconst")
        pv = [v[d + j] for j in range(p)]
        r.Update(full[1, UPD_ROW].copy(), new[1].copy(), UPD_ROW, pv)
        assert all(np.array_equal(pv[j], upd[1, d + j]) for j in range(p)), (tag, d, p, "Update")
        # host batch: pinned (zero-copy or DMA pipeline) and pageable (staged)
        hb = torch.from_numpy(full.copy()).pin_memory()
        hb[:, d:] = 0
        r.encode_host_batch(hb)
        assert np.array_equal(hb.numpy(), full), (tag, d, p, "encode_host_batch pinned")
        hn = full.copy()
        hn[:, d:] = 0
        r.encode_host_batch(hn)
        assert np.array_equal(hn, full), (tag, d, p, "encode_host_batch pageable")


_DEFAULT = {k: v[-1] for k, v in SWEEP.items()}


@pytest.mark.parametrize("knob", sorted(SWEEP))
def test_every_tune_value_is_bit_exact(rslib, orc, cases, knob):
    import torch

    L = rslib.lib()
    # the jit_* policy knobs only matter with run-time compiles on: compile on
    # the launching thread so the compiled kernels really run in this test
    base = {"jit": 2} if knob.startswith("jit_") else {}
    try:
        for k, v in base.items():
            assert L.rs_tune(k.encode(), v) == 0
        for value in SWEEP[knob]:
            assert L.rs_tune(knob.encode(), value) == 0, (knob, value)
            _check_all(rslib, torch, cases, f"{knob}={value}")
    finally:
        L.rs_tune(knob.encode(), _DEFAULT[knob])
        for k in base:
            L.rs_tune(k.encode(), _DEFAULT[k])


def test_var_knob_absent_from_product(rslib):
    """The code-shape experiments (XOR-only diagnostics among them) are only in
    librsamd_exp.so: the product library refuses the knob and ignores RSAMD_VAR."""
    L = rslib.lib()
    assert L.rs_tune(b"var", 141) == 13
    assert L.rs_tune(b"var", -1) == 13
