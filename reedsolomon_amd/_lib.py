"""ctypes binding of librsamd.so (include/rs_amd.h).

There is no fallback: if the HIP library is missing the import of any codec
operation fails loudly (RuntimeError), so a test or benchmark can never pass
on a silent CPU path.
"""
from __future__ import annotations

import ctypes
import os
import threading

from . import build as _build

# RSAMD_LIB_VARIANT=experiments loads librsamd_exp.so, the build with the A/B
# code-shape experiments (tools/ab.py, tools/sweep.sh); never the product path.
LIB_PATH = _build.LIB_EXP if os.environ.get("RSAMD_LIB_VARIANT") == "experiments" else _build.LIB

_lock = threading.Lock()
_lib = None

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u8pp = ctypes.POINTER(c_u8p)
c_intp = ctypes.POINTER(ctypes.c_int)
c_sizep = ctypes.POINTER(ctypes.c_size_t)
c_void = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_sz = ctypes.c_size_t
c_int = ctypes.c_int


class RSLayout(ctypes.Structure):
    """rs_layout_t (include/rs_amd.h)."""
    _fields_ = [("data_base", ctypes.c_void_p), ("data_stripe_stride", ctypes.c_int64),
                ("data_vect_stride", ctypes.c_int64), ("parity_base", ctypes.c_void_p),
                ("parity_stripe_stride", ctypes.c_int64), ("parity_vect_stride", ctypes.c_int64)]


c_layoutp = ctypes.POINTER(RSLayout)

# name -> (restype, argtypes); mirrors include/rs_amd.h
SIGNATURES = {
    "rs_strerror": (ctypes.c_char_p, [c_int]),
    "rs_version": (c_int, []),
    "rs_build_id": (ctypes.c_char_p, []),
    "rs_device_count": (c_int, []),
    "rs_new": (c_int, [c_int, c_int, c_int, ctypes.POINTER(c_void)]),
    "rs_free": (None, [c_void]),
    "rs_data_num": (c_int, [c_void]),
    "rs_parity_num": (c_int, [c_void]),
    "rs_gen_matrix": (c_int, [c_void, c_u8p]),
    "rs_enc_matrix": (c_int, [c_void, c_u8p]),
    "rs_encode": (c_int, [c_void, c_u8pp, c_sizep, c_int]),
    "rs_reconst": (c_int, [c_void, c_u8pp, c_sizep, c_int, c_intp, c_int, c_intp, c_int]),
    "rs_update": (c_int, [c_void, c_u8p, c_sz, c_u8p, c_sz, c_int, c_u8pp, c_sizep, c_int]),
    "rs_replace": (c_int, [c_void, c_u8pp, c_sizep, c_int, c_intp, c_int, c_u8pp, c_sizep, c_int]),
    "rs_encode_dev": (c_int, [c_void, c_u8pp, c_sizep, c_int, c_void]),
    "rs_reconst_dev": (c_int, [c_void, c_u8pp, c_sizep, c_int, c_intp, c_int, c_intp, c_int, c_void]),
    "rs_update_dev": (c_int, [c_void, c_u8p, c_sz, c_u8p, c_sz, c_int, c_u8pp, c_sizep, c_int, c_void]),
    "rs_replace_dev": (c_int, [c_void, c_u8pp, c_sizep, c_int, c_intp, c_int, c_u8pp, c_sizep, c_int, c_void]),
    "rs_encode_batch": (c_int, [c_void, c_void, c_i64, c_i64, c_int, c_sz, c_void]),
    "rs_encode_batch_layout": (c_int, [c_void, c_layoutp, c_int, c_sz, c_void]),
    "rs_reconst_batch_layout": (c_int, [c_void, c_layoutp, c_int, c_sz, c_intp, c_int, c_intp, c_int, c_void]),
    "rs_reconst_batch_multi": (c_int, [c_void, c_layoutp, c_int, c_sz, ctypes.POINTER(ctypes.c_uint64), c_void]),
    "rs_reconst_batch_multi256": (c_int, [c_void, c_layoutp, c_int, c_sz, ctypes.POINTER(ctypes.c_uint64), c_void]),
    "rs_reconst_batch": (c_int, [c_void, c_void, c_i64, c_i64, c_int, c_sz, c_intp, c_int, c_intp, c_int,
                                 c_void]),
    "rs_update_batch": (c_int, [c_void, c_void, c_i64, c_void, c_i64, c_int, c_void, c_i64, c_i64, c_int, c_sz,
                                c_void]),
    "rs_replace_batch": (c_int, [c_void, c_void, c_i64, c_i64, c_intp, c_int, c_void, c_i64, c_i64, c_int, c_sz,
                                 c_void]),
    "rs_encode_host_batch": (c_int, [c_void, c_void, c_i64, c_i64, c_int, c_sz, c_int, c_int]),
    "rs_group_new": (c_int, [c_int, c_int, c_intp, c_int, ctypes.POINTER(c_void)]),
    "rs_group_free": (None, [c_void]),
    "rs_group_size": (c_int, [c_void]),
    "rs_group_codec": (c_void, [c_void, c_int]),
    "rs_group_slice": (c_int, [c_void, c_int, c_int, c_intp, c_intp]),
    "rs_device": (c_int, [c_void]),
    "rs_set_ref_l1d": (c_int, [c_void, c_int]),
    "rs_ref_l1d": (c_int, [c_void]),
    "rs_host_l1d": (c_int, []),
    "rs_group_encode_host_batch": (c_int, [c_void, c_void, c_i64, c_i64, c_int, c_sz, c_int, c_int]),
    "rs_group_reconst_host_batch_multi": (c_int, [c_void, c_void, c_i64, c_i64, c_int, c_sz,
                                                  ctypes.POINTER(ctypes.c_uint64)]),
    "rs_reconst_host_batch_multi": (c_int, [c_void, c_void, c_i64, c_i64, c_int, c_sz,
                                            ctypes.POINTER(ctypes.c_uint64)]),
    "rs_reconst_host_batch_multi256": (c_int, [c_void, c_void, c_i64, c_i64, c_int, c_sz,
                                               ctypes.POINTER(ctypes.c_uint64)]),
    "rs_group_reconst_host_batch_multi256": (c_int, [c_void, c_void, c_i64, c_i64, c_int, c_sz,
                                                     ctypes.POINTER(ctypes.c_uint64)]),
    "rs_host_device_pointer": (c_int, [c_void, c_sz, ctypes.POINTER(c_void)]),
    "rs_host_register": (c_int, [c_void, c_sz]),
    "rs_host_unregister": (c_int, [c_void]),
    "rs_host_alloc": (c_int, [c_sz, ctypes.POINTER(c_void)]),
    "rs_host_free": (c_int, [c_void]),
    "rs_host_pool_stats": (c_int, [ctypes.POINTER(c_sz)] * 4),
    "rs_bind_thread_to_device": (c_int, [c_int]),
    "rs_last_device_error": (ctypes.c_char_p, []),
    "rs_xor_batch": (c_int, [c_void, c_void, c_i64, c_i64, c_int, c_void, c_i64, c_int, c_sz, c_void]),
    "rs_gf_matmul_batch": (c_int, [c_void, c_u8p, c_int, c_int, c_void, c_i64, c_i64, c_intp, c_void, c_i64,
                                   c_i64, c_intp, c_int, c_sz, c_int, c_void]),
    "rs_plan_reconst": (c_int, [c_void, c_intp, c_int, c_intp, c_int, c_intp, c_intp, c_intp, c_intp, c_intp]),
    "rs_reconst_matrix": (c_int, [c_void, c_intp, c_intp, c_int, c_u8p]),
    "rs_matrix_invert": (c_int, [c_u8p, c_sz, c_int, c_u8p]),
    "rs_inverse_cache_key": (ctypes.c_uint64, [c_intp, c_int]),
    "rs_inverse_cache_size": (c_i64, [c_void]),
    "rs_host_call_stats": (c_int, [c_void, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "rs_host_engine_stats": (c_int, [c_void, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "rs_gf_mul": (ctypes.c_uint8, [ctypes.c_uint8, ctypes.c_uint8]),
    "rs_jit_stats": (c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64),
                             ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_double)]),
    "rs_jit_cache_stats": (c_int, [ctypes.POINTER(ctypes.c_uint64)] * 4),
    "rs_jit_table_stats": (c_int, [ctypes.POINTER(ctypes.c_uint64)] * 2),
    "rs_coef_table_stats": (c_int, [c_void, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "rs_jit_prepare": (c_int, [c_void, ctypes.c_void_p, c_int, c_int, c_int, c_int]),
    "rs_jit_compile_check": (c_int, [ctypes.c_void_p, c_int, c_int, c_int, ctypes.POINTER(ctypes.c_double)]),
    "rs_jit_encoder_check": (c_int, [ctypes.c_void_p, c_int, c_int, c_int, ctypes.POINTER(c_sz)]),
    "rs_jit_asm_source": (c_i64, [ctypes.c_void_p, c_int, c_int, c_int, ctypes.c_char_p, c_sz]),
    "rs_tune": (c_int, [ctypes.c_char_p, c_int]),
}


def lib():
    """Load librsamd.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"librsamd.so not found at {LIB_PATH}: build it with "
                    "`python -m reedsolomon_amd.build` (hipcc, gfx950). There is no CPU fallback."
                )
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib
