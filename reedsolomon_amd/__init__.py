"""reedsolomon_amd — MI355X-native Reed-Solomon erasure coding.

A drop-in for templexxx/reedsolomon's hot path (New / Encode / Reconst /
Update / Replace over GF(2^8), identity + Cauchy encoding matrix), with every
vector byte processed by hand-written CDNA4 HIP kernels (librsamd.so).
See DESIGN.md and include/rs_amd.h.
"""
from .rs import (  # noqa: F401
    RS, New, Group, NewGroup, RSError, ErrIllegalVects, ErrMismatchVects, ErrZeroVectSize, ErrMismatchVectSize,
    ErrNoNeedReconst, ErrTooManyLost, ErrMismatchParityNum, ErrIllegalVectIndex, ErrTooManyReplace,
    ErrMismatchReplace, ErrNotSquare, ErrSingularMatrix, ErrInvalidArgument, ErrDevice, ErrNoMemory,
    invert, inverse_cache_key, host_l1d, gf_mul, device_count, host_register, host_unregister, host_device_pointer,
    host_alloc, host_free, host_pool_stats,
    jit_stats, jit_cache_stats, jit_table_stats, jit_compile_check, jit_asm_source, jit_encoder_check,
)
from ._lib import lib, LIB_PATH  # noqa: F401


def build_id() -> str:
    """Source digest compiled into the loaded librsamd.so (rs_build_id)."""
    return lib().rs_build_id().decode()


def build_info() -> dict:
    """The loaded library's digest next to the digest of the sources in this
    tree: `matches_tree` is False when the binary was built from other
    sources (a stale .so)."""
    from . import build as _b
    lib_id = build_id()
    tree_id = _b.source_digest(experiments=LIB_PATH == _b.LIB_EXP)
    return {"build_id": lib_id, "tree_digest": tree_id, "matches_tree": lib_id == tree_id}

__version__ = "0.1.0"
