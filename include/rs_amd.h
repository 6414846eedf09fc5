/*
 * rs_amd.h — C ABI of the MI355X-native Reed-Solomon engine (librsamd.so).
 *
 * This is the drop-in boundary for templexxx/reedsolomon's public Go API
 * (reference: /root/reference/rs.go).  Every entry point below names the
 * reference function it replaces.  A Go caller binds these through cgo
 * (see INTEGRATION.md); Python binds them through ctypes
 * (reedsolomon_amd/_lib.py).  No torch or HIP C++ types appear in the
 * signatures: device memory is passed as plain pointers and streams as
 * `void*` (a hipStream_t, NULL = the legacy default stream).
 *
 * Conventions (same as the reference, rs.go:101-111, 205-237, 422-529):
 *   - The caller owns every buffer; outputs are written in place.
 *   - A vector is (pointer, length).  Lengths are passed per vector so that
 *     the reference's size checks (ErrZeroVectSize, ErrMismatchVectSize) are
 *     reproduced exactly.
 *   - Host-memory entry points (rs_encode, rs_reconst, rs_update, rs_replace)
 *     are synchronous, like the Go methods.
 *   - Device entry points (*_dev, *_batch) are asynchronous on `stream`.
 *   - An rs_t handle is safe for concurrent use from several threads, like
 *     *RS (its only mutable state, the inverse-matrix cache, is locked).
 *   - Return value: RS_OK (0) or one of the RS_ERR_* codes; codes 1..12 map
 *     1:1 to the reference's sentinel errors (rs_strerror gives the exact Go
 *     error text, so a cgo wrapper can return errors that compare equal).
 */
#ifndef RS_AMD_H
#define RS_AMD_H

#include <stddef.h>
#include <stdint.h>

#if defined(__GNUC__)
#define RS_API __attribute__((visibility("default")))
#else
#define RS_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes: rs.go:44,113-117,239-242,451-454,531-534; matrix.go:81-82 ---- */
enum {
    RS_OK = 0,
    RS_ERR_ILLEGAL_VECTS = 1,       /* ErrIllegalVects      rs.go:44  */
    RS_ERR_MISMATCH_VECTS = 2,      /* ErrMismatchVects     rs.go:114 */
    RS_ERR_ZERO_VECT_SIZE = 3,      /* ErrZeroVectSize      rs.go:115 */
    RS_ERR_MISMATCH_VECT_SIZE = 4,  /* ErrMismatchVectSize  rs.go:116 */
    RS_ERR_NO_NEED_RECONST = 5,     /* ErrNoNeedReconst     rs.go:240 (swallowed by Reconst) */
    RS_ERR_TOO_MANY_LOST = 6,       /* ErrTooManyLost       rs.go:241 */
    RS_ERR_MISMATCH_PARITY_NUM = 7, /* ErrMismatchParityNum rs.go:452 */
    RS_ERR_ILLEGAL_VECT_INDEX = 8,  /* ErrIllegalVectIndex  rs.go:453 */
    RS_ERR_TOO_MANY_REPLACE = 9,    /* ErrTooManyReplace    rs.go:532 */
    RS_ERR_MISMATCH_REPLACE = 10,   /* ErrMismatchReplace   rs.go:533 */
    RS_ERR_NOT_SQUARE = 11,         /* ErrNotSquare         matrix.go:81 */
    RS_ERR_SINGULAR_MATRIX = 12,    /* ErrSingularMatrix    matrix.go:82 */
    /* Misuse the reference does not return an error for but panics on
     * (index out of range: Replace with empty data rs.go:549, Reconst with
     * fewer than d+p vectors rs.go:343,346,366,369). */
    RS_ERR_INVAL = 13,
    RS_ERR_DEVICE = 14,             /* a HIP runtime call failed (no GPU, OOM, ...) */
    RS_ERR_NOMEM = 15               /* host allocation failed */
};

typedef struct rs_codec rs_t;

/* Text of the reference's error for `code` ("" for RS_OK). */
RS_API const char* rs_strerror(int code);

/* Library / device information. */
RS_API int rs_version(void);                /* 100*major + minor */
RS_API int rs_device_count(void);           /* number of visible HIP devices, <0 on error */
/* SHA-256 (64 hex digits) of the sources and compile flags this library was
 * built from (reedsolomon_amd/build.py source_digest), so a measurement names
 * the exact tree it ran; "unstamped" for a build outside build.py. */
RS_API const char* rs_build_id(void);

/* ------------------------------------------------------------------------
 * Codec lifetime.  Replaces New(dataNum, parityNum) rs.go:54-85.
 * Validates d>0, p>0, d+p<=256 (RS_ERR_ILLEGAL_VECTS), builds the
 * identity+Cauchy encoding matrix (matrix.go:37-54), sets GenMatrix = rows
 * d..d+p-1, and enables the inverse-matrix cache when d+p<=64
 * (rs.go:70-74).  `device` selects the HIP device the handle launches on
 * (-1 = the calling thread's current device at first use).  No device work
 * happens here: the handle can be created on a host without a GPU.
 * ------------------------------------------------------------------------ */
RS_API int  rs_new(int data_num, int parity_num, int device, rs_t** out);
RS_API void rs_free(rs_t* rs);
RS_API int  rs_data_num(const rs_t* rs);                 /* RS.DataNum   rs.go:24 */
RS_API int  rs_parity_num(const rs_t* rs);               /* RS.ParityNum rs.go:25 */
/* The HIP device ordinal the handle launches on: the one given to rs_new,
 * or -1 while it is "the current device at first use" and no call has bound
 * it yet.  No device call. */
RS_API int  rs_device(const rs_t* rs);
/* Reference-compat Update / Replace, per handle (DESIGN.md §4 "Reference
 * defect").  rs.go's encodePart runs its sub-16-byte tail pass over the whole
 * last chunk of getSplitSize (rs.go:158-173, 190-200), so under updateOnly
 * the body of a last chunk whose length is >= 16 and not a multiple of 16 is
 * XORed twice and keeps its old parity; which bytes those are depends on the
 * host's L1D size (cpu.X86.Cache.L1D).  l1d = 0 (rs_new's setting): Update /
 * Replace compute the re-encode definition (rs_test.go:219-331) everywhere.
 * The cgo binding's New sets -1, so a Go drop-in returns
 * rs.go's bytes on its host by default.
 * l1d > 0 (>= 32): the bytes rs.go produces on a host with that L1D.
 * l1d = -1: this host's L1D as rs_host_l1d reports it, 32 KiB when unknown
 * (rs.go:159-161).  Affects only this handle's Update / Replace calls (host,
 * device and batch forms) that start after the call.  RS_ERR_INVAL for other
 * values. */
RS_API int rs_set_ref_l1d(rs_t* rs, int l1d);
/* The handle's current setting in bytes (0 = off). */
RS_API int rs_ref_l1d(const rs_t* rs);
/* cpu.X86.Cache.L1D on this host as the reference's getSplitSize reads it
 * (rs.go:158-159): the L1 data cache bytes from CPUID, -1 when undetectable,
 * 0 on a non-x86 host.  No device call. */
RS_API int rs_host_l1d(void);
/* Copies GenMatrix (p x d, row-major, G[j*d+i]) into out[p*d]. rs.go:31,65-68 */
RS_API int  rs_gen_matrix(const rs_t* rs, uint8_t* out);
/* Copies the (d+p) x d encoding matrix into out[(d+p)*d]. rs.go:30 */
RS_API int  rs_enc_matrix(const rs_t* rs, uint8_t* out);

/* ------------------------------------------------------------------------
 * Host-memory operations (synchronous; the drop-in for the Go methods).
 * vects[i] is a host pointer of length lens[i].
 * ------------------------------------------------------------------------ */

/* (*RS).Encode rs.go:104-111: vects[d..d+p) = GenMatrix * vects[0..d). */
RS_API int rs_encode(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n);

/* (*RS).Reconst rs.go:221-237 with checkReconst rs.go:264-325.  survived /
 * need are index lists (ns / nn entries; ns==0 means "all survived").  The
 * reconstructed vectors are written into vects[need...] (and, when any
 * parity is rebuilt, every data vector that is neither survived nor needed,
 * exactly like the reference rs.go:297-303). Returns RS_OK when nn==0. */
RS_API int rs_reconst(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n,
               const int* survived, int ns, const int* need, int nn);

/* (*RS).Update rs.go:424-449: parity[j] ^= G[j][row] * (old ^ new). */
RS_API int rs_update(rs_t* rs, const uint8_t* old_data, size_t old_len,
              const uint8_t* new_data, size_t new_len, int row,
              uint8_t* const* parity, const size_t* parity_lens, int np);

/* (*RS).Replace rs.go:492-529: parity[j] ^= sum_k G[j][rows[k]] * data[k]. */
RS_API int rs_replace(rs_t* rs, const uint8_t* const* data, const size_t* data_lens, int nd,
               const int* replace_rows, int nr,
               uint8_t* const* parity, const size_t* parity_lens, int np);

/* ------------------------------------------------------------------------
 * Device-memory operations, one stripe, asynchronous on `stream`.
 * Same semantics and checks as the host versions; pointers are device
 * pointers (hipMalloc / torch CUDA tensors) on the handle's device.
 * ------------------------------------------------------------------------ */
RS_API int rs_encode_dev(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n, void* stream);
RS_API int rs_reconst_dev(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n,
                   const int* survived, int ns, const int* need, int nn, void* stream);
RS_API int rs_update_dev(rs_t* rs, const uint8_t* old_data, size_t old_len,
                  const uint8_t* new_data, size_t new_len, int row,
                  uint8_t* const* parity, const size_t* parity_lens, int np, void* stream);
RS_API int rs_replace_dev(rs_t* rs, const uint8_t* const* data, const size_t* data_lens, int nd,
                   const int* replace_rows, int nr,
                   uint8_t* const* parity, const size_t* parity_lens, int np, void* stream);

/* ------------------------------------------------------------------------
 * Batched device-resident operations over `nstripes` independent stripes
 * laid out with fixed strides: vector v of stripe s lives at
 *     base + s*stripe_stride + v*vect_stride       (bytes)
 * with v in [0, d+p), each vector `len` bytes.  This is the layout the
 * benchmark uses (one [S][d+p][len] allocation) and the unit the multi-GPU
 * path partitions (stripes are independent: no collective).
 * ------------------------------------------------------------------------ */

/* Encode every stripe (the north-star hot path). */
RS_API int rs_encode_batch(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                    int nstripes, size_t len, void* stream);

/* A batch layout with data and parity in possibly separate regions:
 * data vector i (< d) of stripe s:   data_base   + s*data_stripe_stride   + i*data_vect_stride
 * parity vector j (< p) of stripe s: parity_base + s*parity_stripe_stride + j*parity_vect_stride
 * (rs_encode_batch's interleaved [S][d+p][len] layout is the special case
 * parity_base = base + d*vect_stride with equal strides). */
typedef struct rs_layout {
    uint8_t* data_base;
    int64_t data_stripe_stride;
    int64_t data_vect_stride;
    uint8_t* parity_base;
    int64_t parity_stripe_stride;
    int64_t parity_vect_stride;
} rs_layout_t;

RS_API int rs_encode_batch_layout(rs_t* rs, const rs_layout_t* layout, int nstripes, size_t len, void* stream);
RS_API int rs_reconst_batch_layout(rs_t* rs, const rs_layout_t* layout, int nstripes, size_t len,
                                   const int* survived, int ns, const int* need, int nn, void* stream);

/* Reconst a batch where every stripe has its own erasure pattern (SURVEY
 * §8f.1): need_masks[s] has bit v set when vector v of stripe s must be
 * rebuilt (all other vectors of that stripe are survivors, i.e. Reconst's
 * "empty survived" form, rs.go:281-285); 0 skips the stripe.  Stripes are
 * grouped by pattern on the host; each distinct pattern costs one inverse
 * (cached) and one or two launches over its stripes.  Requires d+p <= 64.
 * Every pattern is validated (RS_ERR_TOO_MANY_LOST, ...) before any launch. */
RS_API int rs_reconst_batch_multi(rs_t* rs, const rs_layout_t* layout, int nstripes, size_t len,
                                  const uint64_t* need_masks, void* stream);

/* The same for any d+p <= 256 (rs.go:61; the reference's Reconst has no
 * 64-vector limit, only its inverse cache does, rs.go:70-74): stripe s's
 * mask is the 256-bit set need_masks[4*s .. 4*s+3], vector v at bit v % 64
 * of word v / 64.  The *_multi256 host-batch and group variants below take
 * masks the same way. */
RS_API int rs_reconst_batch_multi256(rs_t* rs, const rs_layout_t* layout, int nstripes, size_t len,
                                     const uint64_t* need_masks, void* stream);

/* Reconst every stripe with the same survived/need pattern
 * (one host plan + one cached matrix, then at most two device passes). */
RS_API int rs_reconst_batch(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                     int nstripes, size_t len, const int* survived, int ns,
                     const int* need, int nn, void* stream);

/* Update: old/new vectors of stripe s at old_base + s*old_stride and
 * new_base + s*new_stride; parity vectors are vectors d..d+p of the stripe
 * layout above. */
RS_API int rs_update_batch(rs_t* rs, const uint8_t* old_base, int64_t old_stride,
                    const uint8_t* new_base, int64_t new_stride, int row,
                    uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                    int nstripes, size_t len, void* stream);

/* Replace: replacement data vector r of stripe s at
 * data_base + s*data_stripe_stride + r*data_vect_stride; parity as above. */
RS_API int rs_replace_batch(rs_t* rs, const uint8_t* data_base, int64_t data_stripe_stride,
                     int64_t data_vect_stride, const int* replace_rows, int nr,
                     uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                     int nstripes, size_t len, void* stream);

/* ------------------------------------------------------------------------
 * Host-resident batches (the path storage callers see: stripes arrive in
 * host memory from disk or the network).  Layout as for rs_encode_batch but
 * `base` is a HOST pointer.  Pinned / registered memory: one zero-copy launch
 * straight over it.  Pageable memory: staged through a pinned mirror by host
 * copy threads, zero-copy kernels on the mirror (stripes above 16 MiB in byte
 * windows of every vector), so no pageable byte reaches the runtime's own
 * pageable copies.  With rs_tune("host_batch_zc" / "host_pageable_stage",
 * 0): H2D copies of the data vectors, the device encode and D2H copies of the
 * parity vectors pipelined over `streams` HIP streams with
 * `stripes_per_chunk` stripes per step.  Returns when every parity byte is
 * back in host memory.  Strides are non-negative (RS_ERR_INVAL otherwise).
 * Pin the memory (rs_host_register) for the full PCIe rate.
 * ------------------------------------------------------------------------ */
RS_API int rs_encode_host_batch(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                                int nstripes, size_t len, int stripes_per_chunk, int streams);

/* ------------------------------------------------------------------------
 * Several GPUs from one process: a group holds one codec per
 * device.  Batched calls split the stripes into contiguous slices, one per
 * device, and run the slices concurrently (one host thread per device); they
 * return when every device is done, with the first error seen.  Stripes are
 * independent, so there is no inter-GPU traffic.  A device may be listed
 * more than once (two codecs sharing it).
 * ------------------------------------------------------------------------ */
typedef struct rs_group rs_group_t;
RS_API int  rs_group_new(int data_num, int parity_num, const int* devices, int ndev, rs_group_t** out);
RS_API void rs_group_free(rs_group_t* g);
RS_API int  rs_group_size(const rs_group_t* g);
/* The codec of member i (borrowed; valid until rs_group_free), for
 * device-resident calls on that member's device. */
RS_API rs_t* rs_group_codec(rs_group_t* g, int i);
/* The slice [*lo, *hi) of stripes [0, nstripes) that member i takes in the
 * group's batched calls: contiguous, in member order, sizes differing by at
 * most one (lo = nstripes*i/n, hi = nstripes*(i+1)/n).  Device-resident
 * callers splitting their own batches over rs_group_codec(g, i) use the same
 * rule.  No device call. */
RS_API int rs_group_slice(const rs_group_t* g, int nstripes, int i, int* lo, int* hi);
/* rs_encode_host_batch over the group: stripes [0, nstripes) of one host
 * buffer split across the members. */
RS_API int rs_group_encode_host_batch(rs_group_t* g, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                                      int nstripes, size_t len, int stripes_per_chunk, int streams);

/* Page-lock / unlock caller memory (hipHostRegister, mapped + portable).
 * Registered (or hipHostMalloc'd) memory is device-addressable: the host
 * batch entry points then run their kernels straight over it (zero-copy,
 * no staging): 72 GiB/s for 10+4 encode on one MI355X vs 20-57 GiB/s for
 * pageable memory (staged through a pinned mirror by host threads).
 * Any address and length: the range is rounded out to whole pages, and pages
 * already registered by an earlier call (a neighbouring buffer sharing a
 * page) are shared by reference rather than registered twice.
 * rs_host_unregister(ptr) takes the address given to rs_host_register
 * (RS_ERR_INVAL for any other); a page leaves the runtime when the last
 * registration holding it goes, after every device this process launched on
 * has been drained.  The library then holds nothing of the range, the
 * runtime reports no page of it registered any more (hipPointerGetAttributes),
 * and the GPUs' in-place mapping of the caller's whole pages, which the
 * runtime's own unregister leaves in KFD's shared-virtual-memory ranges, is
 * revoked (rs_tune("host_unregister_revoke"); checked after every unregister
 * of the GPU tests): the caller may free the memory and the
 * allocator may reuse the addresses (the reference retains nothing after a
 * call: rs.go:101-111).
 * No rs_host_register equivalent exists in the reference; it replaces the
 * pinning a cgo caller would otherwise do per call. */
RS_API int rs_host_register(void* ptr, size_t bytes);
/* Library-owned page-locked buffers (mmap + hipHostRegister), for callers
 * that allocate and release stripe buffers continually (a Go server's
 * per-request buffers): rs_host_alloc hands out a block of at least `bytes`
 * (page-aligned; size classes of powers of two from 64 KiB, carved from
 * 2 MiB-aligned slabs of whole 2 MiB granules that no other mapping shares),
 * device-mapped like registered memory; rs_host_free returns it to the library, which keeps
 * it registered and mapped for reuse and never gives the pages back while the
 * process runs (no per-buffer register / unregister cost).  A reused block holds its
 * previous bytes.  rs_host_free(NULL) is a no-op; any other pointer that is
 * not a live block gives RS_ERR_INVAL.  Thread-safe. */
RS_API int rs_host_alloc(size_t bytes, void** out);
RS_API int rs_host_free(void* ptr);
/* Pool bytes mapped / handed out, pool blocks, and registered page spans
 * (pool blocks and caller registrations); any pointer may be NULL. */
RS_API int rs_host_pool_stats(size_t* mapped, size_t* in_use, size_t* blocks, size_t* spans);
/* Bind the calling thread to the CPUs local to `device` (its PCI function's
 * NUMA node, from sysfs), within the process's affinity, so page-locked
 * buffers and staging copies stay near the GPU.  Device-group workers do
 * this themselves (rs_tune "bind_numa", default 1).  RS_ERR_INVAL when the
 * topology cannot be read. */
RS_API int rs_bind_thread_to_device(int device);
RS_API int rs_host_unregister(void* ptr);
/* Device address of host range [host_ptr, host_ptr+bytes) if all of it is
 * pinned / registered and device-mapped; RS_ERR_INVAL for pageable memory.
 * The result may be passed to every device / batch entry point above. */
RS_API int rs_host_device_pointer(const void* host_ptr, size_t bytes, void** dev_ptr);

/* Reconst of a host-resident batch, a different erasure set per stripe
 * (need_masks as in rs_reconst_batch_multi): stripe s, vector v at
 * base + s*stripe_stride + v*vect_stride (data 0..d-1, then parity).
 * Pinned / registered memory is processed in place (zero-copy); pageable
 * memory is staged through a pinned mirror (the first d survivors in, the
 * rebuilt vectors out; stripes above 16 MiB in byte windows of every
 * vector); with rs_tune("host_pageable_stage", 0) pageable memory gives
 * RS_ERR_INVAL.  Every mask is
 * validated before anything is copied or launched.  Synchronous. */
RS_API int rs_reconst_host_batch_multi(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                                       int nstripes, size_t len, const uint64_t* need_masks);
RS_API int rs_group_reconst_host_batch_multi(rs_group_t* g, uint8_t* base, int64_t stripe_stride,
                                             int64_t vect_stride, int nstripes, size_t len,
                                             const uint64_t* need_masks);
RS_API int rs_reconst_host_batch_multi256(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                                          int nstripes, size_t len, const uint64_t* need_masks);
RS_API int rs_group_reconst_host_batch_multi256(rs_group_t* g, uint8_t* base, int64_t stripe_stride,
                                                int64_t vect_stride, int nstripes, size_t len,
                                                const uint64_t* need_masks);

/* ------------------------------------------------------------------------
 * Generic GF(2^8) matrix product over device vectors — the primitive all of
 * the above reduce to (rs.go:175-203 encodePart, gmu.go:4-9):
 *   out[r] (=|^=) sum_c mat[r*cols+c] (x) in[c]        byte-wise, for every stripe
 * in/out vector c of stripe s at in_base + s*in_stripe_stride + in_map[c]*in_vect_stride
 * (same for out).  accumulate=0 overwrites, 1 XORs into out (updateOnly).
 * ------------------------------------------------------------------------ */
RS_API int rs_gf_matmul_batch(rs_t* rs, const uint8_t* mat, int rows, int cols,
                       const uint8_t* in_base, int64_t in_stripe_stride, int64_t in_vect_stride,
                       const int* in_map,
                       uint8_t* out_base, int64_t out_stripe_stride, int64_t out_vect_stride,
                       const int* out_map,
                       int nstripes, size_t len, int accumulate, void* stream);

/* XOR of vectors (templexxx/xorsimd xor.Encode(dst, src), used by Update
 * rs.go:432-433 and by templexxx/xrs): dst = src[0] ^ src[1] ^ ... for every
 * stripe.  Vector c of stripe s at src_base + s*src_stripe_stride +
 * c*src_vect_stride; dst at dst_base + s*dst_stripe_stride.  Runs as the
 * GF(2^8) product with an all-ones 1 x nsrc matrix (multiplication by 1 is the
 * identity table), so it shares the tuned kernel. */
RS_API int rs_xor_batch(rs_t* rs, const uint8_t* src_base, int64_t src_stripe_stride, int64_t src_vect_stride,
                        int nsrc, uint8_t* dst_base, int64_t dst_stripe_stride, int nstripes, size_t len,
                        void* stream);

/* ------------------------------------------------------------------------
 * Host-side planning helpers (no device work; exported for tests and for
 * callers that batch many erasure patterns themselves).
 * ------------------------------------------------------------------------ */

/* checkReconst rs.go:264-325.  Writes sorted survived indexes (vs, up to
 * d+p), indexes to rebuild (nr, data first; up to d+p) and the count of data
 * indexes among them.  Returns RS_OK, RS_ERR_NO_NEED_RECONST,
 * RS_ERR_ILLEGAL_VECTS or RS_ERR_TOO_MANY_LOST. */
RS_API int rs_plan_reconst(const rs_t* rs, const int* survived, int ns, const int* need, int nn,
                    int* vs, int* nvs, int* nr, int* nnr, int* dn);

/* getReconstMatrix rs.go:382-412 (through the inverse cache when enabled):
 * rows `need` (data indexes) of inv(encMatrix rows survived[0..d)).
 * out has nn*d bytes. */
RS_API int rs_reconst_matrix(rs_t* rs, const int* survived_d, const int* need, int nn, uint8_t* out);

/* invert matrix.go:85-147: n x n inverse over GF(2^8); m has m_len bytes. */
RS_API int rs_matrix_invert(const uint8_t* m, size_t m_len, int n, uint8_t* out);

/* makeInverseCacheKey rs.go:414-420 */
RS_API uint64_t rs_inverse_cache_key(const int* survived, int ns);

/* Number of inverse matrices currently cached (rs.go:33-39). */
RS_API int64_t rs_inverse_cache_size(const rs_t* rs);

/* Host-call coalescing counters since rs_new: kernel launches made for
 * coalesced batches, and the host calls they carried (calls > launches
 * when concurrent calls shared a launch).  Either pointer may be NULL. */
RS_API int rs_host_call_stats(const rs_t* rs, uint64_t* launches, uint64_t* calls);

/* Host-call engine counters since rs_new: calls served by the resident
 * engine kernel (doorbell in host memory instead of a launch + stream sync
 * per call) and the engine instances launched for them (a new one after each
 * idle period).  Either pointer may be NULL. */
RS_API int rs_host_engine_stats(const rs_t* rs, uint64_t* calls, uint64_t* launches);

/* Run-time compiled bit-sliced kernels (products with 5-16 output rows over a
 * matrix known only at run time: Reconst of 5-16 lost vectors, Encode of codes
 * without a build-time network, Update / Replace with 5-16 parity rows; see
 * DESIGN.md §3).  Process-wide counters: code objects compiled, compiles or
 * loads that failed (the perm-table kernels then stay in use), launches of
 * compiled kernels, and the total compile time in ms.  Any pointer may be
 * NULL. */
RS_API int rs_jit_stats(uint64_t* compiled, uint64_t* failed, uint64_t* launches, double* compile_ms);

/* The run-time kernels' in-process table, process-wide: compiled kernels
 * held now (at most 256) and evictions so far (each drops the older half;
 * a launch never waits for one: it is queued on the library's worker thread,
 * which drains the devices that ran the evicted kernels before unloading
 * them).  Either pointer may be NULL. */
RS_API int rs_jit_table_stats(uint64_t* entries, uint64_t* evictions);

/* A handle's coefficient tables (the perm-table kernels' per-matrix tables):
 * uploads to device memory so far, and launches that read a new matrix's
 * tables in place from a mapped staging slot (the first sight of a matrix in
 * a launch of at most rs_tune("table_inplace_max") input bytes, default
 * 2 MiB; its second use uploads).  Either pointer may be NULL.  No device
 * call. */
RS_API int rs_coef_table_stats(const rs_t* rs, uint64_t* uploads, uint64_t* inplace);

/* The run-time kernels' on-disk code-object cache (RSAMD_JIT_CACHE_DIR,
 * default $XDG_CACHE_HOME/rsamd/jit or ~/.cache/rsamd/jit; knob
 * "jit_disk_cache"), process-wide: first sights of a matrix whose code object
 * was on disk (loaded, no compile), first sights that found none, code
 * objects written, files rejected on load (corrupt or stale: recompiled).
 * The directory must be the user's own and not group / world-writable (the
 * library creates it 0700 and its files 0600), since the cache holds GPU code
 * the process runs; otherwise it is neither read nor written.  Any pointer
 * may be NULL. */
RS_API int rs_jit_cache_stats(uint64_t* hits, uint64_t* misses, uint64_t* writes, uint64_t* rejects);

/* Compile the run-time kernel for a rows x cols matrix (row-major, 5 <= rows
 * <= 128 and 1 <= cols <= 256 with the assembly backend, <= 16 x 64 with
 * hiprtc; accumulate 1 = the XOR-into-outputs form Update /
 * Replace use) for the handle's device now, instead of on the matrix's
 * second large launch: wait 1 compiles and loads it on the calling thread
 * (RS_OK, or RS_ERR_DEVICE if the compile failed), wait 0 queues the compile
 * on the library's worker and returns.  For servers that know their codes at
 * start-up, e.g. the Encode of a code without a build-time network
 * (mat = GenMatrix, rows = p, cols = d) or a common rebuild pattern
 * (rs_reconst_matrix).  RS_ERR_INVAL for shapes outside those bounds. */
RS_API int rs_jit_prepare(rs_t* rs, const uint8_t* mat, int rows, int cols, int accumulate, int wait);

/* Generate and compile (comgr / hiprtc, no device needed) the run-time kernel
 * for a rows x cols matrix (row-major, bounds as rs_jit_prepare), overwrite
 * (accumulate 0) or XOR-into-outputs (1) mode.  RS_OK, RS_ERR_INVAL (shape)
 * or RS_ERR_DEVICE (compile failed: the log goes to stderr).  ms may be NULL.
 * For tests and warm-up. */
RS_API int rs_jit_compile_check(const uint8_t* mat, int rows, int cols, int accumulate, double* ms);

/* The run-time kernel generator's two outputs agree: the machine code it
 * encodes directly (the default backend) equals, byte for byte, comgr's
 * assembly of the assembly text it prints for the same rows x cols matrix
 * (bounds as rs_jit_asm_source).  RS_OK, RS_ERR_DEVICE (the first difference
 * goes to stderr) or RS_ERR_INVAL.  *code_bytes (may be NULL) receives the
 * kernel's size.  For tests; no device needed. */
RS_API int rs_jit_encoder_check(const uint8_t* mat, int rows, int cols, int accumulate, size_t* code_bytes);

/* The gfx950 assembly the run-time kernel generator emits for a rows x cols
 * matrix (row-major, 1 <= rows <= 128, 1 <= cols <= 256), overwrite
 * (accumulate 0) or XOR-into-outputs (1): copied NUL-terminated into
 * buf[len] (truncated if short).  Returns the length needed including the
 * NUL, or -RS_ERR_INVAL.  For tests (a CPU emulator runs it against the
 * oracle) and inspection; no device needed. */
RS_API int64_t rs_jit_asm_source(const uint8_t* mat, int rows, int cols, int accumulate, char* buf, size_t len);

/* Expert launch knobs, process-wide (for A/B experiments; defaults are the
 * tuned values; every setting computes the same bytes, which
 * tests/test_gpu_tune_sweep.py checks against the oracle): "max_grid", "vpt",
 * "nt_store", "lds_pad", "lane_bytes" (8 default | 16), "block8" (lanes
 * per workgroup of the 8-byte-lane kernels: 128 default | 256), "bitslice"
 * (1 default: bit-sliced Encode for the generated 5-8-parity shapes | 0),
 * "multi_gpu_plan" (rs_reconst_batch_multi and its host-batch / group
 * variants: from this many distinct patterns in one call the pattern tables
 * are planned on the GPU, one wave per pattern, instead of on the host;
 * -1 default = when patterns x d >= 160, where the GPU planner starts to
 * pay; 0 = always on the host; patterns of 1-8 erasures on the
 * single-launch path only),
 * "bs_block" (lanes per workgroup of the bit-sliced kernels: 64 | 128 | 256;
 * 0 default = 64, or 256 for interleaved stripes of d+p >= 18), "bs_waves"
 * (bit-sliced kernels hold at most n waves per SIMD, 1..7, through LDS
 * padding of at most 64 KiB per workgroup, so 256-lane workgroups keep at
 * least 2; 0 = as many as fit; default 2), "wide_block" (128 | 256),
 * "wide_single_pass" (1 default: products with more than 8 output rows and
 * no compiled network read every input once, all rows of a chunk in one
 * workgroup | 0: the looped kernel in row groups of 8, for A/B),
 * "host_engine" (1 default: small synchronous host calls, coalesced or
 * alone, are served by a resident kernel through a doorbell in host memory |
 * 0: one launch + stream sync per call), "host_engine_waves" (1..64
 * workgroups, each polling the doorbell with its first wave; default 8),
 * "host_engine_group_waves" (1..8 waves per workgroup; default 8),
 * "host_engine_direct" (1 default: small calls the engine takes stage their
 * stripe in a pinned block of their own and ring the engine directly, several
 * callers' calls in flight at once | 0: they join coalesced batches),
 * "host_engine_wg_units" (16-byte units per workgroup a call is spread over;
 * 0 default = adaptive: a lone call spreads over the first wave of every
 * workgroup, calls that overlap others take one unit per lane of one
 * workgroup, so calls in flight run on different workgroups),
 * "host_engine_split_rows" (2 default: a lone call of >= 3 rows and >= 4
 * columns small enough for one 64-lane group per workgroup has its rows
 * computed by separate waves from inputs loaded once into LDS | 0: every
 * row by the first wave of each workgroup | 1: by separate waves, each
 * reading every input again; measured 2x slower over host memory),
 * "host_engine_poll_gap" (0 default: the engine reads the doorbell once per
 * PCIe round trip | n: two reads in flight, n x 10 ns apart),
 * "host_engine_yield_us" (a caller waiting longer than this on its engine
 * call yields its core between polls; 0 default = always spin),
 * "host_engine_idle_us" (the engine leaves after this long without a call,
 * default 2000), "host_engine_cold_launch" (1 default: a call that finds the
 * engine gone, with no call pending, takes the launch path and the engine is
 * relaunched while that call's kernel runs | 0: the call waits for the
 * relaunch), "host_flag_sync" (1 default: a host call served by a kernel
 * launch waits for it through a pinned flag the stream writes after the
 * kernel | 0: hipStreamSynchronize), "host_engine_life_us" (the engine also leaves once it has run
 * this long, even while calls keep coming: a device-wide synchronisation waits at most about
 * this long for it; default 4000), "host_engine_max_bytes" (larger batches
 * launch; default 1 MiB), "host_engine_vram" (1: the engine's call slots and
 * the small calls' input staging live in device memory the host writes
 * through the BAR, where the platform maps it for the CPU | 0 default: pinned
 * host memory, measured faster; taken by handles whose engine starts after
 * the change),
 * "host_pinned_max", "host_zc_max" (bytes, -1 = no limit, the default since
 * round 4: every synchronous host call takes the chunked zero-copy pipeline),
 * "host_chunk" (bytes per vector per chunk of the host-memory call pipeline,
 * at least; default 128 KiB), "host_chunk_split" (n: chunks of at least 1/n
 * of the vectors, within 8 MiB per chunk of all vectors; default 4, 0 =
 * host_chunk alone), "host_coalesce_max" (bytes per vector up to which
 * concurrent host calls of one shape share a launch; 0 = off),
 * "host_coalesce_linger_us" (a ready shared batch waits this long for more
 * callers before it launches; default 0), "host_coalesce_running" (shared
 * batches in flight at once: 1 | 2 default),
 * "host_batch_zc" (0/1), "host_dma_1d" (0/1), "host_pageable_stage" (0/1:
 * pageable host batches staged through a pinned mirror), "host_pageable_slot"
 * (bytes of stripes per chunk of that staging, at least one stripe; default
 * 8 MiB), "host_copy_nt" (1
 * default: the host threads' staging copies of large batches store
 * non-temporally | 0: memcpy), "host_copy_coalesce" (1 default: vectors back
 * to back in both source and destination are copied as one run | 0: one
 * piece per vector at least), "bind_numa" (0/1),
 * "host_unregister_revoke" (1 default: rs_host_unregister takes back the
 * GPUs' in-place mapping of the caller's whole pages, ~0.18 ms per call on
 * MI355X | 0: leave the runtime's state; env RSAMD_UNREGISTER_REVOKE),
 * "jit" (run-time bit-sliced kernels for 5-16 output rows: 1 default = compile
 * in the background on first sight, perm-table kernels until ready | 2 =
 * compile on the launching thread | 0 = off), "jit_min_launches" (background
 * mode compiles a matrix from its n-th launch on; default 2: one-off erasure
 * patterns are never compiled), "jit_min_bytes" (... and once its launches
 * moved this many bytes; default 8 MiB), "jit_min_acc_cols" (XOR-accumulate
 * products over fewer columns stay on the table kernels; default 1),
 * "jit_min_rows" (launches with fewer output rows stay on the table kernels;
 * default 5),
 * "jit_pf" (columns loaded ahead in
 * the compiled kernels, 1..6 (1..4 for assembly kernels), default 3),
 * "jit_sync" (assembly kernels of more than 16 rows: the waves of a
 * workgroup meet at a barrier every n columns, 0 = never; default 0),
 * "jit_waves" (assembly kernels hold at most n waves per SIMD, 2..8, by
 * declaring more registers; 0 = as many as fit; default 2),
 * "jit_layout" (generated kernels of more than 16 rows: 0 = the
 * rows over the waves of a workgroup, all on the same 2 KiB chunk | 1 = row
 * groups of up to 16 rows over workgroups whose waves take consecutive
 * chunks with the same code, the row groups of a chunk on one XCD | 2 =
 * with shared columns and more paths than jit_group_waves: workgroups of at
 * most jit_group_waves waves, one path each, over one chunk, sharing its
 * columns through LDS, G such workgroups per chunk on one XCD; layout 0 up
 * to jit_group_waves paths; the default),
 * "jit_group_waves" (layout 1: waves per workgroup, 1, 2, 4 or 8 - other
 * values round down; layout 2: at most this many waves per workgroup,
 * 2..8; default 4),
 * "jit_path_rows" (generated kernels of more than 16 rows: rows per code
 * path, 1..16, each row 8 VGPR accumulators; default 16),
 * "jit_share" (generated kernels of several waves, layout 0: 1 = each column
 * is loaded and bit-transposed by one wave and shared with the others
 * through LDS, one barrier per nw columns, the default | 0: every wave
 * loads and transposes every column), "jit_share_deep" (shared columns with
 * two steps of loads in flight and the next column's planes read ahead, 24
 * more VGPRs: 0 default | 1 | -1 = for 8-wave workgroups only),
 * "jit_share_cols" (shared columns: columns each wave loads per step, one
 * barrier per nw x n columns: 1 default | 2 | -1 = 2 for 8-wave workgroups),
 * "jit_share_dma" (shared columns: 0 = each wave loads its next column into
 * registers one step ahead | n = 2..8: each wave's columns stream into a
 * private LDS ring of n steps through LDS-DMA loads, n - 1 steps ahead, with
 * no load registers),
 * "jit_share_ahead" (shared columns: 1 = the next column's planes are read
 * from LDS while the current one combines, 8 more VGPRs; 0 default),
 * "jit_gray" (1 = the low half's subsets are built one at a time in
 * Gray-code order, 12 subset VGPRs instead of 22; 0 default; with
 * jit_share_ahead the 16-row paths keep 3 waves per SIMD; both measured
 * within -1..+1 %),
 * "jit_split_cols" (n > 0: products of 9-16 rows over at least n columns run
 * as two 8-row paths sharing the columns; 0 default: one path; measured
 * within -4..+4 %),
 * "jit_wide_pf", "jit_wide_waves" (jit_pf and jit_waves of the generated
 * kernels of more than 16 rows; defaults 2 and 3: their 16-row paths fit 168
 * VGPRs, so 3 waves share a SIMD; jit_pf / jit_waves apply to 1-16 rows),
 * "jit_backend" (2 default: kernels generated as gfx950 machine code and
 * copied into a code-object template, up to 128 output rows x 256 columns |
 * 1: the same kernels as assembly text assembled by comgr, 12 ms - 1.7 s per
 * matrix | 0: C++ compiled by hiprtc, seconds per matrix, up to 16 x 64),
 * "jit_disk_cache" (1 default: compiled
 * code objects are kept in an on-disk cache shared by processes, see
 * rs_jit_cache_stats | 0: compile in every process),
 * "table_registry_max" (distinct coefficient matrices
 * kept on the device per handle before the registry is recycled),
 * "table_inplace_max" (bytes of input vectors up to which a launch reads a
 * matrix it sees for the first time with its tables in place from a mapped
 * staging slot, the matrix's second use uploading them; default 2 MiB, 0 =
 * upload at first sight; see rs_coef_table_stats), "table_stage_vram" (0,
 * the default: coherent pinned host memory slots, read across PCIe, with an
 * event per launch; 1: first-sight tables written by the host through the
 * BAR into device memory (a 1 MiB arena per handle, then the staging slots),
 * where the platform maps it, so the launch reads them from HBM and no
 * upload call or event is made; slots allocated after the change; env
 * RSAMD_TAB_VRAM).  Returns
 * RS_OK, or RS_ERR_INVAL for an unknown name.  The code-shape experiments of
 * earlier rounds (the knob named var, env RSAMD_VAR; some are XOR-only
 * diagnostics) exist only in the separate experiments build librsamd_exp.so:
 * this library returns RS_ERR_INVAL for var and ignores RSAMD_VAR. */
RS_API int rs_tune(const char* name, int value);

/* The calling thread's last RS_ERR_DEVICE cause ("where: hipErrorName (code)"),
 * or "" if none; diagnostic text only. */
RS_API const char* rs_last_device_error(void);

/* GF(2^8) multiply (gmu.go:26-28) — for tests. */
RS_API uint8_t rs_gf_mul(uint8_t a, uint8_t b);

#ifdef __cplusplus
}
#endif
#endif /* RS_AMD_H */
