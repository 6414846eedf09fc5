"""Golden vectors (tests/golden/vectors.json, made by tests/golden/make_vectors.py).

CPU: the oracle reproduces every committed vector, and an independent numpy
restatement of the product (mulTbl lookups, gmu.go:11-23) agrees with it.
GPU: the HIP path reproduces the same vectors through the C ABI, via the
single-stripe host API (the Go API's shape) and the batched device entry
points (one stripe per golden case).
"""
import hashlib
import importlib.util
import itertools
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
_spec = importlib.util.spec_from_file_location("make_vectors", os.path.join(GOLDEN, "make_vectors.py"))
mv = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mv)
VEC = json.load(open(os.path.join(GOLDEN, "vectors.json")))


def _full_stripe(orc):
    g = VEC["reconst"]
    d, p, size = g["d"], g["p"], g["size"]
    full = mv.stripe_data(d, size) + [np.zeros(size, np.uint8) for _ in range(p)]
    assert orc.encode(d, p, full) == 0
    return d, p, size, full


# ---------------------------------------------------------------- CPU: oracle pinned to the fixtures

def test_stream_is_stable():
    # The input generator itself is part of the fixture: pin its first bytes.
    assert mv.stream(0, 0, 8).tobytes().hex() == mv.stream(0, 0, 64)[:8].tobytes().hex()
    assert mv.stream(0, 0, 16).tobytes() != mv.stream(0, 1, 16).tobytes()
    assert mv.sha([mv.stream(0, 0, 4096)]) == hashlib.sha256(mv.stream(0, 0, 4096).tobytes()).hexdigest()


def test_oracle_reproduces_golden_vectors(orc):
    assert mv.make(orc) == {k: v for k, v in VEC.items()}


@pytest.mark.parametrize("case", [e for e in VEC["encode"] if e["size"] <= 8192],
                         ids=lambda e: f"{e['d']}+{e['p']}@{e['size']}")
def test_numpy_restatement_matches_golden_encode(orc, case):
    d, p, size = case["d"], case["p"], case["size"]
    gen = orc.gen_matrix(d, p).reshape(p, d)
    data = np.stack(mv.stripe_data(d, size))
    par = orc.encode_numpy(gen, data)
    assert mv.sha(list(par)) == case["parity_sha256"]
    if "parity_hex" in case:
        assert [x.tobytes().hex() for x in par] == case["parity_hex"]


# ---------------------------------------------------------------- GPU: HIP path vs the fixtures

@pytest.fixture(scope="module")
def torch_dev():
    import torch

    assert torch.cuda.is_available()
    torch.cuda.init()
    return torch


@pytest.mark.gpu
def test_gpu_encode_golden_host_api(rslib, torch_dev):
    for case in VEC["encode"]:
        d, p, size = case["d"], case["p"], case["size"]
        r = rslib.New(d, p)
        v = mv.stripe_data(d, size) + [np.full(size, 0xA5, np.uint8) for _ in range(p)]
        r.Encode(v)
        assert mv.sha(v[d:]) == case["parity_sha256"], (d, p, size)


@pytest.mark.gpu
def test_gpu_encode_golden_device_batch(rslib, torch_dev):
    torch = torch_dev
    for case in VEC["encode"]:
        d, p, size = case["d"], case["p"], case["size"]
        r = rslib.New(d, p)
        buf = torch.empty((1, d + p, size), dtype=torch.uint8, device="cuda")
        buf[0, :d] = torch.from_numpy(np.stack(mv.stripe_data(d, size))).cuda()
        buf[0, d:] = 0xA5
        r.encode_batch(buf)
        assert mv.sha(list(buf[0, d:].cpu().numpy())) == case["parity_sha256"], (d, p, size)


@pytest.mark.gpu
def test_gpu_reconst_golden_every_pattern(rslib, orc, torch_dev):
    """All 1470 patterns through the host Reconst (garbage in lost vectors)."""
    g = VEC["reconst"]
    d, p, size, full = _full_stripe(orc)
    r = rslib.New(d, p)
    h, n = hashlib.sha256(), 0
    for lost in mv.reconst_patterns(d + p):
        v = [x.copy() for x in full]
        for i in lost:
            v[i] = mv.garbage(i, size)
        r.Reconst(v, [], lost)
        rebuilt = [v[i] for i in lost]
        for x in rebuilt:
            h.update(x.tobytes())
        key = ",".join(map(str, lost))
        if key in g["per_pattern_sha256"]:
            assert mv.sha(rebuilt) == g["per_pattern_sha256"][key], lost
        n += 1
    assert n == g["patterns"]
    assert h.hexdigest() == g["all_sha256"]


@pytest.mark.gpu
def test_gpu_reconst_golden_multi_pattern_batch(rslib, orc, torch_dev):
    """The same 1470 patterns as one batch, one stripe per pattern (rs_reconst_batch_multi)."""
    torch = torch_dev
    g = VEC["reconst"]
    d, p, size, full = _full_stripe(orc)
    pats = mv.reconst_patterns(d + p)
    S = len(pats)
    stripe = torch.from_numpy(np.stack(full)).cuda()
    data = stripe[:d].unsqueeze(0).repeat(S, 1, 1).contiguous()
    parity = stripe[d:].unsqueeze(0).repeat(S, 1, 1).contiguous()
    masks = np.zeros(S, np.uint64)
    for s, lost in enumerate(pats):
        for i in lost:
            masks[s] |= np.uint64(1) << np.uint64(i)
            dst = data[s, i] if i < d else parity[s, i - d]
            dst.copy_(torch.from_numpy(mv.garbage(i, size)))
    r = rslib.New(d, p)
    r.reconst_batch_multi(data, parity, masks)
    both = torch.cat([data, parity], 1).cpu().numpy()
    h = hashlib.sha256()
    for s, lost in enumerate(pats):
        for i in lost:
            h.update(both[s, i].tobytes())
    assert h.hexdigest() == g["all_sha256"]


@pytest.mark.gpu
def test_gpu_update_replace_golden(rslib, orc, torch_dev):
    d, p, size, full = _full_stripe(orc)
    r = rslib.New(d, p)
    for case in VEC["update"]:
        row = case["row"]
        par = [x.copy() for x in full[d:]]
        r.Update(full[row], mv.stream(1, row, size), row, par)
        assert mv.sha(par) == case["parity_sha256"], row
    for case in VEC["replace"]:
        par = [x.copy() for x in full[d:]]
        r.Replace([full[i] for i in case["rows"]], case["rows"], par)
        assert mv.sha(par) == case["parity_sha256"], case["rn"]


@pytest.mark.gpu
def test_gpu_update_replace_golden_batch(rslib, orc, torch_dev):
    torch = torch_dev
    d, p, size, full = _full_stripe(orc)
    r = rslib.New(d, p)
    stripe = torch.from_numpy(np.stack(full)).cuda()
    for case in VEC["update"]:
        row = case["row"]
        buf = stripe.unsqueeze(0).clone()
        old = buf[:, row].clone()
        new = torch.from_numpy(mv.stream(1, row, size)).cuda().unsqueeze(0)
        r.update_batch(old, new, row, buf)
        assert mv.sha(list(buf[0, d:].cpu().numpy())) == case["parity_sha256"], row
    for case in VEC["replace"]:
        buf = stripe.unsqueeze(0).clone()
        rows = case["rows"]
        src = buf[:, rows].clone()
        r.replace_batch(src, rows, buf)
        assert mv.sha(list(buf[0, d:].cpu().numpy())) == case["parity_sha256"], case["rn"]
