"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
import this module; it is the checker, never the thing measured or shipped.
The restated algorithm lives in ``oracle/rs_oracle.c`` (each function cites
the reference file:line it follows).  ``build()`` compiles it with gcc.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liborc.so")

_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or (
        os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "rs_oracle.c"))
    ):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        ip = ctypes.POINTER(ctypes.c_int)
        szp = ctypes.POINTER(ctypes.c_size_t)
        ppu8 = ctypes.POINTER(u8p)
        L.orc_tables.argtypes = [u8p] * 5
        L.orc_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.orc_gf_mul.restype = ctypes.c_uint8
        L.orc_mul_vect.argtypes = [ctypes.c_uint8, u8p, u8p, ctypes.c_size_t]
        L.orc_mul_vect_xor.argtypes = [ctypes.c_uint8, u8p, u8p, ctypes.c_size_t]
        L.orc_make_encode_matrix.argtypes = [ctypes.c_int, ctypes.c_int, u8p]
        L.orc_invert.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int, u8p]
        L.orc_new_check.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_inverse_cache_key.argtypes = [ip, ctypes.c_int]
        L.orc_inverse_cache_key.restype = ctypes.c_uint64
        L.orc_check_reconst.argtypes = [ctypes.c_int, ctypes.c_int, ip, ctypes.c_int, ip,
                                        ctypes.c_int, ip, ip, ip, ip, ip]
        L.orc_encode.argtypes = [ctypes.c_int, ctypes.c_int, ppu8, szp, ctypes.c_int]
        L.orc_encode_gen.argtypes = [ctypes.c_int, ctypes.c_int, u8p, ppu8, szp, ctypes.c_int,
                                     ctypes.c_int]
        L.orc_reconst.argtypes = [ctypes.c_int, ctypes.c_int, ppu8, szp, ctypes.c_int, ip,
                                  ctypes.c_int, ip, ctypes.c_int]
        L.orc_update.argtypes = [ctypes.c_int, ctypes.c_int, u8p, ctypes.c_size_t, u8p,
                                 ctypes.c_size_t, ctypes.c_int, ppu8, szp, ctypes.c_int]
        L.orc_replace.argtypes = [ctypes.c_int, ctypes.c_int, ppu8, szp, ctypes.c_int, ip,
                                  ctypes.c_int, ppu8, szp, ctypes.c_int]
        L.orc_naive_mul.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ppu8, ctypes.c_size_t]
        L.orc_has_avx2.restype = ctypes.c_int
        L.orc_encode_avx2.argtypes = [ctypes.c_int, ctypes.c_int, ppu8, ctypes.c_size_t]
        _lib = L
    return _lib


# ---------------------------------------------------------------- helpers

def _u8p(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _vec_table(vects):
    arr = (ctypes.POINTER(ctypes.c_uint8) * max(1, len(vects)))()
    lens = (ctypes.c_size_t * max(1, len(vects)))()
    for i, v in enumerate(vects):
        arr[i] = _u8p(v) if v.size else ctypes.cast(ctypes.c_void_p(1), ctypes.POINTER(ctypes.c_uint8))
        lens[i] = v.size
    return arr, lens


def _ints(xs):
    xs = list(xs)
    return (ctypes.c_int * max(1, len(xs)))(*xs), len(xs)


# ---------------------------------------------------------------- API

def tables():
    exp = np.zeros(255, np.uint8)
    log = np.zeros(256, np.uint8)
    mul = np.zeros(65536, np.uint8)
    lh = np.zeros(8192, np.uint8)
    inv = np.zeros(256, np.uint8)
    lib().orc_tables(_u8p(exp), _u8p(log), _u8p(mul), _u8p(lh), _u8p(inv))
    return {"exp": exp, "log": log, "mul": mul.reshape(256, 256), "low_high": lh, "inverse": inv}


def gf_mul(a: int, b: int) -> int:
    return int(lib().orc_gf_mul(a, b))


def make_encode_matrix(d: int, p: int) -> np.ndarray:
    m = np.zeros((d + p) * d, np.uint8)
    lib().orc_make_encode_matrix(d, p, _u8p(m))
    return m


def gen_matrix(d: int, p: int) -> np.ndarray:
    return make_encode_matrix(d, p)[d * d:]


def invert(m: np.ndarray, n: int):
    m = np.ascontiguousarray(m, dtype=np.uint8)
    out = np.zeros(n * n, np.uint8)
    rc = lib().orc_invert(_u8p(m), m.size, n, _u8p(out))
    return rc, out


def inverse_cache_key(survived) -> int:
    a, n = _ints(survived)
    return int(lib().orc_inverse_cache_key(a, n))


def check_reconst(d, p, survived, need):
    s, ns = _ints(survived)
    q, nq = _ints(need)
    vs = (ctypes.c_int * 256)()
    nr = (ctypes.c_int * 256)()
    nvs, nnr, dn = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    rc = lib().orc_check_reconst(d, p, s, ns, q, nq, vs, ctypes.byref(nvs), nr,
                                 ctypes.byref(nnr), ctypes.byref(dn))
    return rc, list(vs[: nvs.value]), list(nr[: nnr.value]), dn.value


def encode(d, p, vects) -> int:
    arr, lens = _vec_table(vects)
    return lib().orc_encode(d, p, arr, lens, len(vects))


def encode_gen(d, p, gen, vects, update_only=False) -> int:
    gen = np.ascontiguousarray(gen, dtype=np.uint8)
    arr, lens = _vec_table(vects)
    return lib().orc_encode_gen(d, p, _u8p(gen), arr, lens, len(vects), int(update_only))


def reconst(d, p, vects, survived, need) -> int:
    arr, lens = _vec_table(vects)
    s, ns = _ints(survived)
    q, nq = _ints(need)
    return lib().orc_reconst(d, p, arr, lens, len(vects), s, ns, q, nq)


def update(d, p, old, new, row, parity) -> int:
    arr, lens = _vec_table(parity)
    return lib().orc_update(d, p, _u8p(old) if old.size else None, old.size,
                            _u8p(new) if new.size else None, new.size, row, arr, lens,
                            len(parity))


def replace(d, p, data, rows, parity) -> int:
    darr, dlens = _vec_table(data)
    parr, plens = _vec_table(parity)
    r, nr = _ints(rows)
    return lib().orc_replace(d, p, darr, dlens, len(data), r, nr, parr, plens, len(parity))


def set_l1d(l1d: int) -> None:
    """The L1D size the restated getSplitSize (rs.go:158-173) uses; 0 = 32 KiB."""
    lib().orc_set_l1d(ctypes.c_size_t(int(l1d)))


def update_quirk_range(size: int, l1d: int = 32 * 1024):
    """Byte range [lo, hi) where the reference's Update / Replace keep the old
    parity (rs_oracle.c encode_part: the tail pass of rs.go:190-200 covers the
    whole last chunk, XORing its 16-byte body twice), or None.  getSplitSize
    rs.go:158-173 with the given L1D size."""
    if size < l1d // 2:
        return None  # chunks: 16-byte multiples, then a < 16-byte tail alone
    last = size % (l1d // 2)
    if last >= 16 and last % 16:
        return size - last, size - last + (last & ~15)
    return None


def naive_mul(gen, d, p, vects):
    gen = np.ascontiguousarray(gen, dtype=np.uint8)
    arr, _ = _vec_table(vects)
    lib().orc_naive_mul(_u8p(gen), d, p, arr, vects[0].size)


def has_avx2() -> bool:
    return bool(lib().orc_has_avx2())


def encode_avx2(d, p, vects) -> bool:
    arr, _ = _vec_table(vects)
    return bool(lib().orc_encode_avx2(d, p, arr, vects[0].size))


def encode_numpy(gen: np.ndarray, data: np.ndarray) -> np.ndarray:
    """Vectorised restatement of the same byte-wise product for big inputs:
    parity[j] = XOR_i mulTbl[G[j][i]][data[i]] (gmu.go:11-23 semantics).
    data: [..., k, n] uint8; gen: [m, k]."""
    mul = tables()["mul"]
    m, k = gen.shape
    out = np.zeros(data.shape[:-2] + (m, data.shape[-1]), np.uint8)
    for j in range(m):
        acc = np.zeros(data.shape[:-2] + (data.shape[-1],), np.uint8)
        for i in range(k):
            acc ^= mul[gen[j, i]][data[..., i, :]]
        out[..., j, :] = acc
    return out
