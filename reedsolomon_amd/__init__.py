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
    invert, inverse_cache_key, gf_mul, device_count, host_register, host_unregister, host_device_pointer,
    host_alloc, host_free, host_pool_stats,
    jit_stats, jit_cache_stats, jit_compile_check, jit_asm_source, jit_encoder_check,
)
from ._lib import lib, LIB_PATH  # noqa: F401

__version__ = "0.1.0"
