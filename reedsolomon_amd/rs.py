"""Python mirror of templexxx/reedsolomon's public API on top of librsamd.

    import reedsolomon_amd as reedsolomon
    r = reedsolomon.New(10, 4)            # rs.go:54
    r.Encode(vects)                       # rs.go:104  (vects: 14 writable uint8 buffers)
    r.Reconst(vects, survived, need)      # rs.go:221
    r.Update(old, new, row, parity)       # rs.go:424
    r.Replace(data, rows, parity)         # rs.go:492

Same names, argument meaning, in-place outputs and error behaviour as the
Go methods: every reference sentinel error is an exception class here
(ErrMismatchVects, ErrTooManyLost, ...) raised where the Go method returns
it.  Host buffers are numpy uint8 arrays, bytearrays or writable
memoryviews.  The *_dev / *_batch methods take torch uint8 tensors that live
on the GPU and run asynchronously on torch's current stream.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from ._lib import RSLayout, c_u8p, c_u8pp, lib


# ---------------------------------------------------------------- errors

class RSError(Exception):
    """Base of every codec error; ``code`` is the C ABI return code."""

    code = -1

    def __init__(self, msg: str | None = None):
        super().__init__(msg if msg is not None else lib().rs_strerror(self.code).decode())


class ErrIllegalVects(RSError):        # rs.go:44
    code = 1


class ErrMismatchVects(RSError):       # rs.go:114
    code = 2


class ErrZeroVectSize(RSError):        # rs.go:115
    code = 3


class ErrMismatchVectSize(RSError):    # rs.go:116
    code = 4


class ErrNoNeedReconst(RSError):       # rs.go:240 (swallowed by Reconst)
    code = 5


class ErrTooManyLost(RSError):         # rs.go:241
    code = 6


class ErrMismatchParityNum(RSError):   # rs.go:452
    code = 7


class ErrIllegalVectIndex(RSError):    # rs.go:453
    code = 8


class ErrTooManyReplace(RSError):      # rs.go:532
    code = 9


class ErrMismatchReplace(RSError):     # rs.go:533
    code = 10


class ErrNotSquare(RSError):           # matrix.go:81
    code = 11


class ErrSingularMatrix(RSError):      # matrix.go:82
    code = 12


class ErrInvalidArgument(RSError):     # inputs the reference panics on
    code = 13


class ErrDevice(RSError):              # HIP runtime failure
    code = 14


class ErrNoMemory(RSError):
    code = 15


_ERRORS = {cls.code: cls for cls in (
    ErrIllegalVects, ErrMismatchVects, ErrZeroVectSize, ErrMismatchVectSize, ErrNoNeedReconst,
    ErrTooManyLost, ErrMismatchParityNum, ErrIllegalVectIndex, ErrTooManyReplace, ErrMismatchReplace,
    ErrNotSquare, ErrSingularMatrix, ErrInvalidArgument, ErrDevice, ErrNoMemory)}


def _check(rc: int) -> None:
    if rc:
        cls = _ERRORS.get(rc, RSError)
        if cls is ErrDevice:  # say which HIP call failed
            raise cls(f"HIP device error: {lib().rs_last_device_error().decode(errors='replace')}")
        raise cls()


# ---------------------------------------------------------------- marshalling

_U8 = np.dtype(np.uint8)


def _host_array(buf, writable: bool) -> np.ndarray:
    a = buf if type(buf) is np.ndarray else np.frombuffer(buf, dtype=np.uint8)
    if a.dtype != _U8 or a.ndim != 1 or not a.flags.c_contiguous:
        raise TypeError("vectors must be 1-D contiguous uint8 buffers")
    if writable and not a.flags.writeable:
        raise TypeError("output vector is read-only")
    return a


_addr_of = ctypes.addressof
_char_from = ctypes.c_char.from_buffer


def _data_ptr(a: np.ndarray) -> int:
    # a ctypes view of a writable buffer gives its address ~2.5x faster than
    # __array_interface__ (which builds a dict per call); read-only arrays
    # (and empty ones) take the interface
    try:
        return _addr_of(_char_from(a))
    except (TypeError, ValueError):
        return a.__array_interface__["data"][0]


def _host_vecs(bufs: Sequence, writable: bool):
    arrs = [_host_array(b, writable) for b in bufs]
    n = len(arrs)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[_data_ptr(a) for a in arrs])
    lens = (ctypes.c_size_t * max(n, 1))(*[a.size for a in arrs])
    return arrs, ctypes.cast(ptrs, c_u8pp), lens, n


def _dev_vecs(tensors: Sequence):
    n = len(tensors)
    ptrs = (c_u8p * max(n, 1))()
    lens = (ctypes.c_size_t * max(n, 1))()
    for i, t in enumerate(tensors):
        _check_tensor(t)
        ptrs[i] = ctypes.cast(ctypes.c_void_p(t.data_ptr()), c_u8p)
        lens[i] = t.numel()
    return ptrs, lens, n


def _check_tensor(t) -> None:
    import torch

    if not isinstance(t, torch.Tensor) or t.dtype != torch.uint8 or not t.is_cuda:
        raise TypeError("device vectors must be torch.uint8 tensors on a GPU")
    if not t.is_contiguous():
        raise TypeError("device vectors must be contiguous")


def _ints(xs):
    xs = [int(x) for x in (xs or [])]
    return (ctypes.c_int * max(len(xs), 1))(*xs), len(xs)




# ---------------------------------------------------------------- codec

class RS:
    """Reed-Solomon encoder/decoder (rs.go:22-42).  Create with :func:`New`."""

    def __init__(self, handle: ctypes.c_void_p, device: int, owner=None):
        self._h = handle
        self.device = device
        self._owner = owner  # a Group keeps borrowed member handles alive
        L = lib()
        self.DataNum = L.rs_data_num(handle)
        self.ParityNum = L.rs_parity_num(handle)
        d, p = self.DataNum, self.ParityNum
        g = np.zeros(d * p, np.uint8)
        _check(L.rs_gen_matrix(handle, g.ctypes.data_as(c_u8p)))
        e = np.zeros((d + p) * d, np.uint8)
        _check(L.rs_enc_matrix(handle, e.ctypes.data_as(c_u8p)))
        self.GenMatrix = g            # p x d, row-major: G[j*d+i]   (rs.go:31)
        self.encMatrix = e            # (d+p) x d                      (rs.go:30)

    def set_ref_l1d(self, l1d: int) -> None:
        """Reference-compat Update / Replace for this codec (rs_set_ref_l1d):
        0 = re-encode definition (default), n = rs.go's bytes on a host whose
        L1D is n bytes, -1 = this host's L1D (rs.go:158-173, 190-200)."""
        _check(lib().rs_set_ref_l1d(self._h, int(l1d)))

    @property
    def ref_l1d(self) -> int:
        """The codec's reference-compat L1D setting in bytes (0 = off)."""
        return int(lib().rs_ref_l1d(self._h))

    def device_ordinal(self) -> int:
        """The device the handle launches on (rs_device; -1 = not bound yet)."""
        return int(lib().rs_device(self._h))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and getattr(self, "_owner", None) is None:
            try:
                lib().rs_free(h)
            except Exception:
                pass
            self._h = None

    def _stream(self, stream, *tensors) -> ctypes.c_void_p:
        """The HIP stream to launch on, on the codec's device.  Every tensor
        must live on that device (the C side switches to the handle's device
        and would otherwise get another device's pointers); stream=None means
        torch's current stream OF THAT DEVICE, not of the current device."""
        import torch

        dev = self.device
        if dev is None or dev < 0:  # New(..., device=-1): the current device (rs_new)
            dev = torch.cuda.current_device()
        for t in tensors:
            if t.device.index != dev:
                raise TypeError(f"tensor on {t.device} but the codec runs on cuda:{dev}")
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        elif isinstance(stream, torch.cuda.Stream) and stream.device.index != dev:
            raise TypeError(f"stream on {stream.device} but the codec runs on cuda:{dev}")
        if hasattr(stream, "cuda_stream"):
            stream = stream.cuda_stream
        return ctypes.c_void_p(int(stream))

    # ------------------------------------------------ host memory (Go API)

    def Encode(self, vects: Sequence) -> None:
        """rs.go:104 — vects[d:] = GenMatrix x vects[:d]."""
        _, ptrs, lens, n = _host_vecs(vects, writable=False)
        _check(lib().rs_encode(self._h, ptrs, lens, n))

    def Reconst(self, vects: Sequence, survived: Sequence[int] | None, needReconst: Sequence[int] | None) -> None:
        """rs.go:221 — rebuild vects[needReconst] from vects[survived]."""
        _, ptrs, lens, n = _host_vecs(vects, writable=False)
        s, ns = _ints(survived)
        q, nq = _ints(needReconst)
        _check(lib().rs_reconst(self._h, ptrs, lens, n, s, ns, q, nq))

    def Update(self, oldData, newData, row: int, parity: Sequence) -> None:
        """rs.go:424 — parity[j] ^= G[j][row] x (oldData ^ newData)."""
        o = _host_array(oldData, False)
        w = _host_array(newData, False)
        _, ptrs, lens, n = _host_vecs(parity, writable=True)
        _check(lib().rs_update(self._h, o.ctypes.data_as(c_u8p), o.size, w.ctypes.data_as(c_u8p), w.size,
                               int(row), ptrs, lens, n))

    def Replace(self, data: Sequence, replaceRows: Sequence[int], parity: Sequence) -> None:
        """rs.go:492 — parity[j] ^= sum_k G[j][replaceRows[k]] x data[k]."""
        _, dptrs, dlens, nd = _host_vecs(data, writable=False)
        r, nr = _ints(replaceRows)
        _, pptrs, plens, np_ = _host_vecs(parity, writable=True)
        _check(lib().rs_replace(self._h, dptrs, dlens, nd, r, nr, pptrs, plens, np_))

    # ------------------------------------------------ device memory, one stripe

    def encode_dev(self, vects: Sequence, stream=None) -> None:
        ptrs, lens, n = _dev_vecs(vects)
        _check(lib().rs_encode_dev(self._h, ptrs, lens, n, self._stream(stream, *vects)))

    def reconst_dev(self, vects: Sequence, survived, needReconst, stream=None) -> None:
        ptrs, lens, n = _dev_vecs(vects)
        s, ns = _ints(survived)
        q, nq = _ints(needReconst)
        _check(lib().rs_reconst_dev(self._h, ptrs, lens, n, s, ns, q, nq, self._stream(stream, *vects)))

    def update_dev(self, oldData, newData, row: int, parity: Sequence, stream=None) -> None:
        _check_tensor(oldData)
        _check_tensor(newData)
        ptrs, lens, n = _dev_vecs(parity)
        _check(lib().rs_update_dev(
            self._h, ctypes.cast(ctypes.c_void_p(oldData.data_ptr()), c_u8p), oldData.numel(),
            ctypes.cast(ctypes.c_void_p(newData.data_ptr()), c_u8p), newData.numel(), int(row), ptrs, lens, n,
            self._stream(stream, oldData, newData, *parity)))

    def replace_dev(self, data: Sequence, replaceRows, parity: Sequence, stream=None) -> None:
        dptrs, dlens, nd = _dev_vecs(data)
        r, nr = _ints(replaceRows)
        pptrs, plens, np_ = _dev_vecs(parity)
        _check(lib().rs_replace_dev(self._h, dptrs, dlens, nd, r, nr, pptrs, plens, np_,
                                    self._stream(stream, *data, *parity)))

    # ------------------------------------------------ device memory, batched stripes

    @staticmethod
    def _stripes(buf, nvec: int):
        """buf: uint8 GPU tensor [S, nvec, len] (any strides with unit inner stride)."""
        _check_tensor_any(buf)
        if buf.dim() != 3 or buf.shape[1] < nvec or buf.stride(2) != 1:
            raise TypeError(f"expected a [stripes, >= {nvec}, len] uint8 GPU tensor with unit inner stride")
        return ctypes.c_void_p(buf.data_ptr()), buf.stride(0), buf.stride(1), buf.shape[0], buf.shape[2]

    def encode_batch(self, buf, stream=None) -> None:
        """Encode every stripe of buf[S, d+p, len] (the north-star hot path)."""
        base, ss, vs, S, n = self._stripes(buf, self.DataNum + self.ParityNum)
        _check(lib().rs_encode_batch(self._h, base, ss, vs, S, n, self._stream(stream, buf)))

    def _split_layout(self, data, parity):
        _check_tensor_any(data)
        _check_tensor_any(parity)
        d, p = self.DataNum, self.ParityNum
        if data.dim() != 3 or parity.dim() != 3 or data.shape[0] != parity.shape[0] or \
                data.shape[2] != parity.shape[2] or data.shape[1] < d or parity.shape[1] < p or \
                data.stride(2) != 1 or parity.stride(2) != 1:
            raise TypeError("expected data [S, >=d, len] and parity [S, >=p, len] uint8 GPU tensors")
        L = RSLayout(data.data_ptr(), data.stride(0), data.stride(1), parity.data_ptr(), parity.stride(0),
                     parity.stride(1))
        return L, data.shape[0], data.shape[2]

    def encode_batch_split(self, data, parity, stream=None) -> None:
        """Encode S stripes whose data [S, d, len] and parity [S, p, len] live in separate buffers."""
        L, S, n = self._split_layout(data, parity)
        _check(lib().rs_encode_batch_layout(self._h, ctypes.byref(L), S, n, self._stream(stream, data, parity)))

    def reconst_batch_split(self, data, parity, survived, needReconst, stream=None) -> None:
        L, S, n = self._split_layout(data, parity)
        s, ns = _ints(survived)
        q, nq = _ints(needReconst)
        _check(lib().rs_reconst_batch_layout(self._h, ctypes.byref(L), S, n, s, ns, q, nq,
                                             self._stream(stream, data, parity)))

    def reconst_batch_multi(self, data, parity, need_masks, stream=None) -> None:
        """Per-stripe erasure patterns: need_masks[s] = bitmap of vectors of stripe s to rebuild
        (data in [S, d, len], parity in [S, p, len]; the interleaved buffer can be passed as
        data=buf[:, :d], parity=buf[:, d:])."""
        L, S, n = self._split_layout(data, parity)
        masks, fn = _masks_for(need_masks, S, self.DataNum + self.ParityNum, "rs_reconst_batch_multi")
        _check(getattr(lib(), fn)(self._h, ctypes.byref(L), S, n, masks.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                  self._stream(stream, data, parity)))

    def reconst_batch(self, buf, survived, needReconst, stream=None) -> None:
        base, ss, vs, S, n = self._stripes(buf, self.DataNum + self.ParityNum)
        s, ns = _ints(survived)
        q, nq = _ints(needReconst)
        _check(lib().rs_reconst_batch(self._h, base, ss, vs, S, n, s, ns, q, nq, self._stream(stream, buf)))

    def update_batch(self, old, new, row: int, buf, stream=None) -> None:
        """old/new: [S, len] GPU tensors; parity rows of buf[S, d+p, len] are updated."""
        base, ss, vs, S, n = self._stripes(buf, self.DataNum + self.ParityNum)
        for t in (old, new):
            _check_tensor_any(t)
            if t.dim() != 2 or t.shape[0] != S or t.shape[1] != n or t.stride(1) != 1:
                raise TypeError("old/new must be [stripes, len] uint8 GPU tensors")
        _check(lib().rs_update_batch(self._h, ctypes.c_void_p(old.data_ptr()), old.stride(0),
                                     ctypes.c_void_p(new.data_ptr()), new.stride(0), int(row), base, ss, vs, S, n,
                                     self._stream(stream, old, new, buf)))

    def replace_batch(self, data, replaceRows, buf, stream=None) -> None:
        """data: [S, rn, len] GPU tensor of replacement vectors."""
        base, ss, vs, S, n = self._stripes(buf, self.DataNum + self.ParityNum)
        _check_tensor_any(data)
        if data.dim() != 3 or data.shape[0] != S or data.shape[2] != n or data.stride(2) != 1:
            raise TypeError("data must be a [stripes, rn, len] uint8 GPU tensor")
        r, nr = _ints(replaceRows)
        if data.shape[1] != nr:
            raise ErrMismatchReplace()
        _check(lib().rs_replace_batch(self._h, ctypes.c_void_p(data.data_ptr()), data.stride(0), data.stride(1),
                                      r, nr, base, ss, vs, S, n, self._stream(stream, data, buf)))

    def encode_host_batch(self, buf, stripes_per_chunk: int = 8, streams: int = 3) -> None:
        """Encode stripes held in HOST memory: buf is a [S, d+p, len] uint8
        numpy array or CPU torch tensor (pin it for full PCIe rate).  Pipelined
        H2D -> encode -> D2H; returns when parity is back in host memory."""
        ptr, ss, vs, S, n = _host_batch(buf, self.DataNum + self.ParityNum)
        _check(lib().rs_encode_host_batch(self._h, ctypes.c_void_p(ptr), ss, vs, S, n, int(stripes_per_chunk),
                                          int(streams)))

    def reconst_host_batch_multi(self, buf, need_masks) -> None:
        """Reconst a host batch [S, d+p, len] in place, need_masks[s] = bitmap of
        the vectors of stripe s to rebuild (zero-copy kernels over pinned
        memory; pageable memory is staged through a pinned mirror)."""
        ptr, ss, vs, S, n = _host_batch(buf, self.DataNum + self.ParityNum)
        masks, fn = _masks_for(need_masks, S, self.DataNum + self.ParityNum, "rs_reconst_host_batch_multi")
        _check(getattr(lib(), fn)(self._h, ctypes.c_void_p(ptr), ss, vs, S, n,
                                  masks.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))

    def xor_batch(self, src, dst, stream=None) -> None:
        """dst[s] = src[s, 0] ^ src[s, 1] ^ ... (xorsimd xor.Encode) for [S, n, len] / [S, len] GPU tensors."""
        _check_tensor_any(src)
        _check_tensor_any(dst)
        if src.dim() != 3 or dst.dim() != 2 or src.shape[0] != dst.shape[0] or src.shape[2] != dst.shape[1] or \
                src.stride(2) != 1 or dst.stride(1) != 1:
            raise TypeError("expected src [S, n, len] and dst [S, len] uint8 GPU tensors")
        _check(lib().rs_xor_batch(self._h, ctypes.c_void_p(src.data_ptr()), src.stride(0), src.stride(1),
                                  src.shape[1], ctypes.c_void_p(dst.data_ptr()), dst.stride(0), src.shape[0],
                                  src.shape[2], self._stream(stream, src, dst)))

    def gf_matmul_batch(self, mat: np.ndarray, src, in_map, dst, out_map, accumulate=False, stream=None) -> None:
        """dst[:, out_map[r]] (=|^=) sum_c mat[r, c] x src[:, in_map[c]] for every stripe."""
        mat = np.ascontiguousarray(mat, dtype=np.uint8)
        rows, cols = mat.shape
        _check_tensor_any(src)
        _check_tensor_any(dst)
        if src.dim() != 3 or dst.dim() != 3 or src.shape[0] != dst.shape[0] or src.shape[2] != dst.shape[2]:
            raise TypeError("src/dst must be [stripes, vectors, len] uint8 GPU tensors")
        im, _ = _ints(in_map if in_map is not None else range(cols))
        om, _ = _ints(out_map if out_map is not None else range(rows))
        _check(lib().rs_gf_matmul_batch(
            self._h, mat.ctypes.data_as(c_u8p), rows, cols, ctypes.c_void_p(src.data_ptr()), src.stride(0),
            src.stride(1), im, ctypes.c_void_p(dst.data_ptr()), dst.stride(0), dst.stride(1), om,
            src.shape[0], src.shape[2], int(bool(accumulate)), self._stream(stream, src, dst)))

    # ------------------------------------------------ host-side planning

    def plan_reconst(self, survived, needReconst):
        """checkReconst rs.go:264-325 -> (survived, needReconst(sorted, data first), dataNeedReconstN)."""
        s, ns = _ints(survived)
        q, nq = _ints(needReconst)
        vs = (ctypes.c_int * 256)()
        nr = (ctypes.c_int * 256)()
        nvs, nnr, dn = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib().rs_plan_reconst(self._h, s, ns, q, nq, vs, ctypes.byref(nvs), nr, ctypes.byref(nnr),
                                     ctypes.byref(dn)))
        return list(vs[: nvs.value]), list(nr[: nnr.value]), dn.value

    def reconst_matrix(self, survived, needReconst) -> np.ndarray:
        """getReconstMatrix rs.go:382-412 (through the inverse cache)."""
        s, ns = _ints(survived)
        q, nq = _ints(needReconst)
        out = np.zeros(max(nq, 1) * self.DataNum, np.uint8)
        _check(lib().rs_reconst_matrix(self._h, s, q, nq, out.ctypes.data_as(c_u8p)))
        return out[: nq * self.DataNum]

    def inverse_cache_size(self) -> int:
        return int(lib().rs_inverse_cache_size(self._h))

    def jit_prepare(self, mat=None, accumulate: bool = False, wait: bool = True) -> None:
        """Compile the run-time bit-sliced kernel for `mat` (rows x cols,
        5 <= rows <= 128, cols <= 256) on this codec's device now
        (rs_jit_prepare; a full kernel table is made room in first); default
        mat = GenMatrix, i.e. this code's Encode."""
        m = (self.GenMatrix.reshape(self.ParityNum, self.DataNum) if mat is None
             else np.ascontiguousarray(mat, dtype=np.uint8))
        _check(lib().rs_jit_prepare(self._h, m.ctypes.data, m.shape[0], m.shape[1], int(bool(accumulate)),
                                    int(bool(wait))))

    def host_engine_stats(self) -> tuple:
        """(calls, launches) of the resident host-call engine since New (rs_host_engine_stats)."""
        a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(lib().rs_host_engine_stats(self._h, ctypes.byref(a), ctypes.byref(b)))
        return int(a.value), int(b.value)

    def coef_table_stats(self) -> tuple:
        """(uploads, in-place first sights) of this codec's coefficient tables (rs_coef_table_stats)."""
        a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(lib().rs_coef_table_stats(self._h, ctypes.byref(a), ctypes.byref(b)))
        return int(a.value), int(b.value)

    def host_call_stats(self) -> tuple:
        """(launches, calls) of coalesced host calls since New (see rs_host_call_stats)."""
        a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(lib().rs_host_call_stats(self._h, ctypes.byref(a), ctypes.byref(b)))
        return int(a.value), int(b.value)


def _check_tensor_any(t) -> None:
    import torch

    if not isinstance(t, torch.Tensor) or t.dtype != torch.uint8 or not t.is_cuda:
        raise TypeError("expected a torch.uint8 tensor on a GPU")


def _host_batch(buf, nvec: int):
    """(address, stripe stride, vector stride, stripes, len) of a [S, >=nvec, len]
    uint8 host array (numpy, or a CPU torch tensor)."""
    if isinstance(buf, np.ndarray):
        if buf.dtype != np.uint8 or buf.ndim != 3 or buf.strides[2] != 1:
            raise TypeError("expected a [stripes, d+p, len] uint8 array with unit inner stride")
        ptr, ss, vs, S, n = buf.ctypes.data, buf.strides[0], buf.strides[1], buf.shape[0], buf.shape[2]
    else:
        if str(buf.dtype) != "torch.uint8" or buf.is_cuda or buf.dim() != 3 or buf.stride(2) != 1:
            raise TypeError("expected a [stripes, d+p, len] uint8 CPU tensor with unit inner stride")
        ptr, ss, vs, S, n = buf.data_ptr(), buf.stride(0), buf.stride(1), buf.shape[0], buf.shape[2]
    if buf.shape[1] < nvec:
        raise TypeError("buffer holds fewer than d+p vectors per stripe")
    return ptr, ss, vs, S, n


def _masks(need_masks, S: int) -> np.ndarray:
    masks = np.ascontiguousarray(np.asarray(need_masks, dtype=np.uint64))
    if masks.shape != (S,):
        raise TypeError("need_masks must hold one mask per stripe")
    return masks


def _masks_for(need_masks, S: int, nvec: int, fn64: str):
    """(mask array, entry point): 64-bit masks through `fn64` when the codec
    has <= 64 vectors and every mask fits in 64 bits, else [S, 4] words
    through the *_multi256 variant (d+p <= 256).  need_masks: one int per
    stripe (Python ints may exceed 64 bits), a uint64 [S] array, or a uint64
    [S, 4] array of 256-bit masks (vector v at bit v % 64 of word v // 64)."""
    if isinstance(need_masks, np.ndarray) and need_masks.ndim == 2:
        m = np.ascontiguousarray(need_masks, dtype=np.uint64)
        if m.shape != (S, 4):
            raise TypeError("256-bit need_masks must be a [stripes, 4] uint64 array")
        return m, fn64 + "256"
    if isinstance(need_masks, np.ndarray):
        if nvec <= 64:
            return _masks(need_masks, S), fn64
        need_masks = [int(x) for x in need_masks]
    vals = [int(x) for x in need_masks]
    if len(vals) != S:
        raise TypeError("need_masks must hold one mask per stripe")
    if nvec <= 64 and all(0 <= v < (1 << 64) for v in vals):
        return np.asarray(vals, dtype=np.uint64), fn64
    try:  # 32 little-endian bytes per mask = 4 words, vector v at bit v % 64 of word v // 64
        raw = b"".join(v.to_bytes(32, "little") for v in vals)
    except OverflowError:  # negative, or a bit past 255
        raise ErrIllegalVects() from None
    return np.frombuffer(raw, dtype="<u8").astype(np.uint64).reshape(S, 4), fn64 + "256"


def host_device_pointer(ptr: int, nbytes: int) -> int:
    """Device address of a pinned / registered host range (rs_host_device_pointer)."""
    d = ctypes.c_void_p()
    _check(lib().rs_host_device_pointer(ctypes.c_void_p(int(ptr)), int(nbytes), ctypes.byref(d)))
    return int(d.value)


class Group:
    """One codec per device for a process that drives several GPUs
    (rs_group_*).  Create with :func:`NewGroup`."""

    def __init__(self, handle: ctypes.c_void_p, devices):
        self._g = handle
        self.devices = list(devices)
        L = lib()
        self.members = [RS(ctypes.c_void_p(L.rs_group_codec(handle, i)), dv, owner=self)
                        for i, dv in enumerate(self.devices)]
        self.DataNum, self.ParityNum = self.members[0].DataNum, self.members[0].ParityNum

    def __len__(self) -> int:
        return lib().rs_group_size(self._g)

    def slice(self, nstripes: int, i: int) -> tuple:
        """(lo, hi): the stripes of a batch of `nstripes` that member i takes
        in the group's batched calls (rs_group_slice)."""
        lo, hi = ctypes.c_int(), ctypes.c_int()
        _check(lib().rs_group_slice(self._g, int(nstripes), int(i), ctypes.byref(lo), ctypes.byref(hi)))
        return lo.value, hi.value

    def encode_host_batch(self, buf, stripes_per_chunk: int = 4, streams: int = 3) -> None:
        """RS.encode_host_batch with the stripes split across the group's devices."""
        ptr, ss, vs, S, n = _host_batch(buf, self.DataNum + self.ParityNum)
        _check(lib().rs_group_encode_host_batch(self._g, ctypes.c_void_p(ptr), ss, vs, S, n,
                                                int(stripes_per_chunk), int(streams)))

    def reconst_host_batch_multi(self, buf, need_masks) -> None:
        """RS.reconst_host_batch_multi with the stripes split across the group's devices."""
        ptr, ss, vs, S, n = _host_batch(buf, self.DataNum + self.ParityNum)
        masks, fn = _masks_for(need_masks, S, self.DataNum + self.ParityNum, "rs_group_reconst_host_batch_multi")
        _check(getattr(lib(), fn)(self._g, ctypes.c_void_p(ptr), ss, vs, S, n,
                                  masks.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))

    def __del__(self):
        g = getattr(self, "_g", None)
        if g:
            for m in getattr(self, "members", []):
                m._h = None
            try:
                lib().rs_group_free(g)
            except Exception:
                pass
            self._g = None


def NewGroup(dataNum: int, parityNum: int, devices) -> Group:
    devs = [int(x) for x in devices]
    arr = (ctypes.c_int * max(len(devs), 1))(*devs)
    h = ctypes.c_void_p()
    _check(lib().rs_group_new(int(dataNum), int(parityNum), arr, len(devs), ctypes.byref(h)))
    return Group(h, devs)


def New(dataNum: int, parityNum: int, device: int = -1) -> RS:
    """rs.go:54 — validates d>0, p>0, d+p<=256 (else ErrIllegalVects)."""
    h = ctypes.c_void_p()
    _check(lib().rs_new(int(dataNum), int(parityNum), int(device), ctypes.byref(h)))
    return RS(h, device)


# ---------------------------------------------------------------- free helpers

def host_l1d() -> int:
    """cpu.X86.Cache.L1D of this host as rs.go:158-159 reads it (rs_host_l1d)."""
    return int(lib().rs_host_l1d())


def invert(m, n: int) -> np.ndarray:
    """matrix.go:85-147 (raises ErrNotSquare / ErrSingularMatrix)."""
    m = np.ascontiguousarray(np.frombuffer(bytes(m), np.uint8) if not isinstance(m, np.ndarray) else m,
                             dtype=np.uint8)
    out = np.zeros(max(n * n, 1), np.uint8)
    _check(lib().rs_matrix_invert(m.ctypes.data_as(c_u8p), m.size, int(n), out.ctypes.data_as(c_u8p)))
    return out[: n * n]


def inverse_cache_key(survived) -> int:
    s, ns = _ints(survived)
    return int(lib().rs_inverse_cache_key(s, ns))


def jit_stats() -> dict:
    """Run-time compiled bit-sliced kernels (rs_jit_stats): code objects
    compiled, failures, launches, total compile time (ms)."""
    c, f, n, ms = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_double()
    _check(lib().rs_jit_stats(ctypes.byref(c), ctypes.byref(f), ctypes.byref(n), ctypes.byref(ms)))
    return {"compiled": c.value, "failed": f.value, "launches": n.value, "compile_ms": ms.value}


def jit_table_stats() -> dict:
    """Compiled run-time kernels held and evictions so far (rs_jit_table_stats)."""
    e, v = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().rs_jit_table_stats(ctypes.byref(e), ctypes.byref(v)))
    return {"entries": e.value, "evictions": v.value}


def jit_cache_stats() -> dict:
    """The run-time kernels' on-disk code-object cache (rs_jit_cache_stats)."""
    v = [ctypes.c_uint64(0) for _ in range(4)]
    _check(lib().rs_jit_cache_stats(*[ctypes.byref(x) for x in v]))
    return dict(zip(("hits", "misses", "writes", "rejects"), (int(x.value) for x in v)))


def jit_asm_source(mat, accumulate: bool = False) -> str:
    """The gfx950 assembly of the run-time kernel for `mat` (rs_jit_asm_source)."""
    m = np.ascontiguousarray(mat, dtype=np.uint8)
    n = lib().rs_jit_asm_source(m.ctypes.data, m.shape[0], m.shape[1], int(bool(accumulate)), None, 0)
    if n < 0:
        _check(int(-n))
    buf = ctypes.create_string_buffer(int(n))
    lib().rs_jit_asm_source(m.ctypes.data, m.shape[0], m.shape[1], int(bool(accumulate)), buf, int(n))
    return buf.value.decode()


def jit_compile_check(mat, accumulate: bool = False) -> float:
    """Generate and compile (no device needed) the run-time kernel for `mat`
    (rows x cols, 5 <= rows <= 8); returns the compile time in ms."""
    m = np.ascontiguousarray(mat, dtype=np.uint8)
    ms = ctypes.c_double()
    _check(lib().rs_jit_compile_check(m.ctypes.data, m.shape[0], m.shape[1], int(bool(accumulate)), ctypes.byref(ms)))
    return ms.value


def jit_encoder_check(mat, accumulate: bool = False) -> int:
    """The run-time kernel's directly encoded machine code equals comgr's
    assembly of its text (rs_jit_encoder_check); returns the code size in
    bytes, raises ErrDevice on a difference."""
    m = np.ascontiguousarray(mat, dtype=np.uint8)
    n = ctypes.c_size_t(0)
    _check(lib().rs_jit_encoder_check(m.ctypes.data, m.shape[0], m.shape[1], int(bool(accumulate)), ctypes.byref(n)))
    return int(n.value)


def gf_mul(a: int, b: int) -> int:
    return int(lib().rs_gf_mul(a, b))


def host_register(ptr: int, nbytes: int) -> None:
    _check(lib().rs_host_register(ctypes.c_void_p(ptr), nbytes))


def host_unregister(ptr: int) -> None:
    _check(lib().rs_host_unregister(ctypes.c_void_p(ptr)))


def host_alloc(nbytes: int) -> np.ndarray:
    """A uint8 array of `nbytes` over a library-owned page-locked block
    (rs_host_alloc): host calls and host batches on it run zero-copy.  Give
    it back with :func:`host_free` (the block stays registered for reuse)."""
    p = ctypes.c_void_p()
    _check(lib().rs_host_alloc(int(nbytes), ctypes.byref(p)))
    buf = (ctypes.c_uint8 * int(nbytes)).from_address(int(p.value))
    return np.frombuffer(buf, dtype=np.uint8, count=int(nbytes))


def host_free(buf) -> None:
    """Return a block from :func:`host_alloc` (the array, or its address)."""
    ptr = buf if isinstance(buf, int) else buf.ctypes.data
    _check(lib().rs_host_free(ctypes.c_void_p(int(ptr))))


def host_pool_stats() -> dict:
    """rs_host_pool_stats: pool bytes mapped / in use, pool blocks, registered page spans."""
    v = [ctypes.c_size_t(0) for _ in range(4)]
    _check(lib().rs_host_pool_stats(*[ctypes.byref(x) for x in v]))
    return dict(zip(("mapped", "in_use", "blocks", "spans"), (int(x.value) for x in v)))


def device_count() -> int:
    return int(lib().rs_device_count())
