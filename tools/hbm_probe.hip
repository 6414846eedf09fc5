// hbm_probe.hip — HBM calibration kernels (measurement tool, not product).
// Gives the achievable bandwidth of plain access patterns on this MI355X so
// the encode kernel's rate can be read against them.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

__global__ __launch_bounds__(256) void k_copy(const g_u32x4* src, g_u32x4* dst, uint64_t n, int nt) {
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    u32x4 v = src[i];
    if (nt) __builtin_nontemporal_store(v, dst + i); else dst[i] = v;
}

__global__ __launch_bounds__(256) void k_read(const g_u32x4* src, g_u32x4* dst, uint64_t n, int per) {
    uint64_t base = ((uint64_t)blockIdx.x * 256 * per) + threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll 8
    for (int j = 0; j < per; ++j) {
        uint64_t i = base + (uint64_t)j * 256;
        if (i < n) acc ^= src[i];
    }
    if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) dst[0] = acc;  // keeps loads live, never stores
}

__global__ __launch_bounds__(256) void k_write(g_u32x4* dst, uint64_t n, int nt) {
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
    if (nt) __builtin_nontemporal_store(v, dst + i); else dst[i] = v;
}

// The encode access pattern with the math replaced by XOR: stripe s, vectors
// of `vec` bytes, k inputs then m outputs; each workgroup covers `units`
// 16-byte units of every vector (units = 256 * upl, lane-interleaved).
template <int K, int M, int UPL>
__global__ __launch_bounds__(256) void k_pattern(uint8_t* base, uint64_t vec, uint64_t stripe_stride,
                                                 uint64_t chunks_per_stripe, int nstripes, int mapping) {
    uint64_t chunk = blockIdx.x;
    if (mapping == 2) {  // XCD-contiguous: blocks sharing an XCD (b % 8) take one contiguous range
        const uint64_t nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = chunk % 8;
        chunk = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + chunk / 8;
    } else if (mapping == 3) {  // chunk-major across stripes in groups of 8 stripes
        const uint64_t g = chunk / (8 * chunks_per_stripe), w = chunk % (8 * chunks_per_stripe);
        chunk = (g * 8 + w % 8) * chunks_per_stripe + w / 8;
    }
    uint64_t s = chunk / chunks_per_stripe, cb = chunk % chunks_per_stripe;
    if (mapping == 1) { s = chunk % nstripes; cb = chunk / nstripes; }
    const __attribute__((address_space(1))) uint8_t* sp =
        (const __attribute__((address_space(1))) uint8_t*)(base + s * stripe_stride);
    u32x4 x[K][UPL];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int u = 0; u < UPL; ++u)
            x[i][u] = *(const g_u32x4*)(sp + i * vec + (cb * 256 * UPL + u * 256 + threadIdx.x) * 16);
    if (M == 0) {  // read-only variant: keep the loads live without storing
        u32x4 a = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int u = 0; u < UPL; ++u) a ^= x[i][u];
        if (a.x == 0x9e3779b9u && a.y == 0x7f4a7c15u) *(g_u32x4*)(base) = a;
        return;
    }
#pragma unroll
    for (int j = 0; j < M; ++j)
#pragma unroll
        for (int u = 0; u < UPL; ++u) {
            u32x4 a = {(uint32_t)j, 0u, 0u, 0u};
#pragma unroll
            for (int i = 0; i < K; ++i) a ^= x[i][u];
            __builtin_nontemporal_store(a, (g_u32x4*)(sp + (K + j) * vec + (cb * 256 * UPL + u * 256 + threadIdx.x) * 16));
        }
}

// Same pattern with the parity vectors in their own region (pbase).
template <int K, int M>
__global__ __launch_bounds__(256) void k_pattern_sep(uint8_t* base, uint8_t* pbase, uint64_t vec, uint64_t dss,
                                                     uint64_t pss, uint64_t cps) {
    const uint64_t chunk = blockIdx.x;
    const uint64_t s = chunk / cps, cb = chunk % cps;
    const uint64_t off = (cb * 256 + threadIdx.x) * 16;
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = *(const g_u32x4*)(base + s * dss + i * vec + off);
#pragma unroll
    for (int j = 0; j < M; ++j) {
        u32x4 a = {(uint32_t)j, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < K; ++i) a ^= x[i];
        __builtin_nontemporal_store(a, (g_u32x4*)(pbase + s * pss + j * vec + off));
    }
}

// Buffer-instruction (nt) variants of copy / read / write / 10+4 pattern.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t n) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, static_cast<int>(n), 0x00020000);
}
__global__ __launch_bounds__(256) void kb_copy(const uint8_t* src, uint8_t* dst, uint64_t chunk_bytes) {
    const uint64_t base = (uint64_t)blockIdx.x * 4096;
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(src + base, 4096), threadIdx.x * 16, 0, 2);
    __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(dst + base, 4096), threadIdx.x * 16, 0, 2);
}
__global__ __launch_bounds__(256) void kb_read(const uint8_t* src, uint8_t* dst) {
    const uint64_t base = (uint64_t)blockIdx.x * 4096;
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(src + base, 4096), threadIdx.x * 16, 0, 2);
    if (v.x == 0x9e3779b9u && v.y == 0x7f4a7c15u && v.z == 1u) *(u32x4*)dst = v;
}
__global__ __launch_bounds__(256) void kb_write(uint8_t* dst) {
    const uint64_t base = (uint64_t)blockIdx.x * 4096;
    u32x4 v = {blockIdx.x, threadIdx.x, 2u, 3u};
    __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(dst + base, 4096), threadIdx.x * 16, 0, 2);
}
template <int K, int M>
__global__ __launch_bounds__(256) void kb_pattern(const uint8_t* dbase, uint8_t* pbase, uint64_t vec, uint64_t dss,
                                                  uint64_t pss, uint64_t cps) {
    const uint64_t s = blockIdx.x / cps, cb = blockIdx.x % cps;
    const uint32_t off = (uint32_t)(cb * 4096 + threadIdx.x * 16);
    u32x4 x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(dbase + s * dss + i * vec, (uint32_t)vec), off, 0, 2);
#pragma unroll
    for (int j = 0; j < M; ++j) {
        u32x4 a = {(uint32_t)j, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < K; ++i) a ^= x[i];
        __builtin_amdgcn_raw_buffer_store_b128(a, rsrc(pbase + s * pss + j * vec, (uint32_t)vec), off, 0, 2);
    }
}

// 10+4 split pattern with UPL 4 KiB units per vector per workgroup (UPL=2:
// 8 KiB, 4: 16 KiB) and an optional XCD-aware block order (XCD=1: the 8
// round-robin XCDs each walk one contiguous eighth of the chunks).
template <int K, int M, int UPL, int XCD>
__global__ __launch_bounds__(256) void kb_pattern_u(const uint8_t* dbase, uint8_t* pbase, uint64_t vec, uint64_t dss,
                                                    uint64_t pss, uint64_t cps, uint32_t nblocks) {
    uint32_t b = blockIdx.x;
    if (XCD) b = (b % 8) * (nblocks / 8) + b / 8;  // nblocks % 8 == 0 (host checks)
    const uint64_t s = b / cps, cb = b % cps;
    u32x4 x[K][UPL];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int u = 0; u < UPL; ++u)
            x[i][u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(dbase + s * dss + i * vec, (uint32_t)vec),
                                                            (uint32_t)((cb * UPL + u) * 4096 + threadIdx.x * 16), 0, 2);
#pragma unroll
    for (int j = 0; j < M; ++j)
#pragma unroll
        for (int u = 0; u < UPL; ++u) {
            u32x4 a = {(uint32_t)j, 0u, 0u, 0u};
#pragma unroll
            for (int i = 0; i < K; ++i) a ^= x[i][u];
            __builtin_amdgcn_raw_buffer_store_b128(a, rsrc(pbase + s * pss + j * vec, (uint32_t)vec),
                                                   (uint32_t)((cb * UPL + u) * 4096 + threadIdx.x * 16), 0, 2);
        }
}

extern "C" {
// kind: 0 UPL1, 1 UPL2, 2 UPL4, +4 = XCD-aware order.  10+4 split layout.
int probe_buf_u(int kind, void* a, void* b, uint64_t vec, int nstripes, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const int upl = 1 << (kind & 3);
    const uint64_t cps = vec / (4096ull * upl);
    const uint32_t nb = (uint32_t)(cps * nstripes);
    if (nb % 8) return -2;
#define KU(U, X) hipLaunchKernelGGL((kb_pattern_u<10, 4, U, X>), dim3(nb), dim3(256), 0, st, (const uint8_t*)a, \
                                    (uint8_t*)b, vec, 10 * vec, 4 * vec, cps, nb)
    switch (kind) {
        case 0: KU(1, 0); break;
        case 1: KU(2, 0); break;
        case 2: KU(4, 0); break;
        case 4: KU(1, 1); break;
        case 5: KU(2, 1); break;
        case 6: KU(4, 1); break;
        default: return -1;
    }
#undef KU
    return hipGetLastError();
}

int probe_buf(int kind, void* a, void* b, uint64_t bytes, uint64_t vec, int nstripes, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (kind == 0) hipLaunchKernelGGL(kb_copy, dim3(bytes / 4096), dim3(256), 0, st, (const uint8_t*)a, (uint8_t*)b, 4096ull);
    else if (kind == 1) hipLaunchKernelGGL(kb_read, dim3(bytes / 4096), dim3(256), 0, st, (const uint8_t*)a, (uint8_t*)b);
    else if (kind == 2) hipLaunchKernelGGL(kb_write, dim3(bytes / 4096), dim3(256), 0, st, (uint8_t*)b);
    else if (kind == 3) hipLaunchKernelGGL((kb_pattern<10, 4>), dim3(vec / 4096 * nstripes), dim3(256), 0, st,
                                           (const uint8_t*)a, (uint8_t*)b, vec, 10 * vec, 4 * vec, vec / 4096);
    // 10 reads + 1..3 writes: the Reconst mixes (lost vectors written to their own region)
    else if (kind == 4) hipLaunchKernelGGL((kb_pattern<10, 1>), dim3(vec / 4096 * nstripes), dim3(256), 0, st,
                                           (const uint8_t*)a, (uint8_t*)b, vec, 10 * vec, 1 * vec, vec / 4096);
    else if (kind == 5) hipLaunchKernelGGL((kb_pattern<10, 2>), dim3(vec / 4096 * nstripes), dim3(256), 0, st,
                                           (const uint8_t*)a, (uint8_t*)b, vec, 10 * vec, 2 * vec, vec / 4096);
    else if (kind == 6) hipLaunchKernelGGL((kb_pattern<10, 3>), dim3(vec / 4096 * nstripes), dim3(256), 0, st,
                                           (const uint8_t*)a, (uint8_t*)b, vec, 10 * vec, 3 * vec, vec / 4096);
    // in place, Reconst's real layout: stripe = 11 vectors in one region,
    // vectors 1..10 read, vector 0 written (reads and write vec bytes apart)
    else if (kind == 7) hipLaunchKernelGGL((kb_pattern<10, 1>), dim3(vec / 4096 * nstripes), dim3(256), 0, st,
                                           (const uint8_t*)a + vec, (uint8_t*)a, vec, 11 * vec, 11 * vec, vec / 4096);
    // in place, 14-vector stripes, data 4..9 + parity 10..13 read, 0..3 written (lost = 4 data)
    else if (kind == 8) hipLaunchKernelGGL((kb_pattern<10, 4>), dim3(vec / 4096 * nstripes), dim3(256), 0, st,
                                           (const uint8_t*)a + 4 * vec, (uint8_t*)a, vec, 14 * vec, 14 * vec, vec / 4096);
    else return -1;
    return hipGetLastError();
}
int probe_pattern_sep(void* base, void* pbase, uint64_t vec, uint64_t dss, uint64_t pss, int nstripes, void* stream) {
    uint64_t cps = vec / 4096;
    hipLaunchKernelGGL((k_pattern_sep<10, 4>), dim3(cps * nstripes), dim3(256), 0, (hipStream_t)stream,
                       (uint8_t*)base, (uint8_t*)pbase, vec, dss, pss, cps);
    return hipGetLastError();
}

int probe_copy(void* src, void* dst, uint64_t bytes, int nt, void* stream) {
    uint64_t n = bytes / 16;
    hipLaunchKernelGGL(k_copy, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       (const g_u32x4*)src, (g_u32x4*)dst, n, nt);
    return hipGetLastError();
}
int probe_read(void* src, void* dst, uint64_t bytes, int per, void* stream) {
    uint64_t n = bytes / 16;
    uint64_t blocks = (n + 256ull * per - 1) / (256ull * per);
    hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const g_u32x4*)src,
                       (g_u32x4*)dst, n, per);
    return hipGetLastError();
}
int probe_write(void* dst, uint64_t bytes, int nt, void* stream) {
    uint64_t n = bytes / 16;
    hipLaunchKernelGGL(k_write, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, (g_u32x4*)dst, n, nt);
    return hipGetLastError();
}
int probe_pattern(void* base, uint64_t vec, uint64_t pitch, uint64_t stripe_stride, int nstripes, int upl,
                  int mapping, void* stream) {
    uint64_t cps = vec / (256ull * 16 * upl);
    dim3 g(cps * nstripes);
    uint8_t* b = (uint8_t*)base;
    if (upl == 1) hipLaunchKernelGGL((k_pattern<10, 4, 1>), g, dim3(256), 0, (hipStream_t)stream, b, pitch, stripe_stride, cps, nstripes, mapping);
    else if (upl == 2) hipLaunchKernelGGL((k_pattern<10, 4, 2>), g, dim3(256), 0, (hipStream_t)stream, b, pitch, stripe_stride, cps, nstripes, mapping);
    else if (upl == 4) hipLaunchKernelGGL((k_pattern<10, 4, 4>), g, dim3(256), 0, (hipStream_t)stream, b, pitch, stripe_stride, cps, nstripes, mapping);
    else return -1;
    return hipGetLastError();
}
// k/m sweep of the pattern (upl = 1, mapping 0)
int probe_pattern_km(void* base, uint64_t vec, uint64_t pitch, uint64_t stripe_stride, int nstripes, int k, int m,
                     void* stream) {
    uint64_t cps = vec / (256ull * 16);
    dim3 g(cps * nstripes);
    uint8_t* b = (uint8_t*)base;
#define KM(K, M) if (k == K && m == M) { hipLaunchKernelGGL((k_pattern<K, M, 1>), g, dim3(256), 0, (hipStream_t)stream, b, pitch, stripe_stride, cps, nstripes, 0); return hipGetLastError(); }
    KM(1, 1) KM(2, 2) KM(4, 4) KM(7, 7) KM(10, 0) KM(14, 0) KM(4, 0) KM(10, 4) KM(10, 2) KM(12, 4) KM(6, 3) KM(10, 10)
#undef KM
    return -1;
}
}

// Granularity sweep of the 10+4 split pattern: BS lanes per workgroup, BPL
// bytes per lane (16: dwordx4, 8: dwordx2) -> BS*BPL bytes per vector per WG.
template <int K, int M, int BS, int BPL>
__global__ __launch_bounds__(BS) void kb_pattern_g(const uint8_t* dbase, uint8_t* pbase, uint64_t vec, uint64_t dss,
                                                   uint64_t pss, uint64_t cps) {
    const uint64_t s = blockIdx.x / cps, cb = blockIdx.x % cps;
    const uint32_t off = (uint32_t)(cb * (BS * BPL) + threadIdx.x * BPL);
    if constexpr (BPL == 16) {
        u32x4 x[K];
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(dbase + s * dss + i * vec, (uint32_t)vec), off, 0, 2);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            u32x4 a = {(uint32_t)j, 0u, 0u, 0u};
#pragma unroll
            for (int i = 0; i < K; ++i) a ^= x[i];
            __builtin_amdgcn_raw_buffer_store_b128(a, rsrc(pbase + s * pss + j * vec, (uint32_t)vec), off, 0, 2);
        }
    } else {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        u32x2 x[K];
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = __builtin_amdgcn_raw_buffer_load_b64(rsrc(dbase + s * dss + i * vec, (uint32_t)vec), off, 0, 2);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            u32x2 a = {(uint32_t)j, 0u};
#pragma unroll
            for (int i = 0; i < K; ++i) a ^= x[i];
            __builtin_amdgcn_raw_buffer_store_b64(a, rsrc(pbase + s * pss + j * vec, (uint32_t)vec), off, 0, 2);
        }
    }
}

extern "C" int probe_buf_g(int kind, void* a, void* b, uint64_t vec, int nstripes, void* stream) {
    hipStream_t st = (hipStream_t)stream;
#define KG(BS, BPL) do { const uint64_t cps = vec / (BS * BPL); \
    hipLaunchKernelGGL((kb_pattern_g<10, 4, BS, BPL>), dim3(cps * nstripes), dim3(BS), 0, st, (const uint8_t*)a, \
                       (uint8_t*)b, vec, 10 * vec, 4 * vec, cps); } while (0)
    switch (kind) {
        case 0: KG(64, 16); break;
        case 1: KG(128, 16); break;
        case 2: KG(256, 16); break;
        case 3: KG(512, 16); break;
        case 4: KG(1024, 16); break;
        case 5: KG(256, 8); break;
        case 6: KG(128, 8); break;
        case 7: KG(512, 8); break;
        default: return -1;
    }
#undef KG
    return hipGetLastError();
}

// The k+m encode pattern at several geometries (round 4, 16+4 vs 10+4):
// kind 0 = 128 lanes x 8 B, 1 = 256 x 16 B, 2 = 256 x 8 B; data vector i of
// stripe s at a + s*dss + i*vec, output j at b + s*pss + j*vec (split layout:
// b a separate region; interleaved: b = a + k*vec, dss = pss = (k+m)*vec).
extern "C" int probe_km_g(int kind, int k, int m, void* a, void* b, uint64_t vec, uint64_t dss, uint64_t pss,
                          int nstripes, void* stream) {
    hipStream_t st = (hipStream_t)stream;
#define KMG(K, M, BS, BPL) do { const uint64_t cps = vec / (BS * BPL); \
    hipLaunchKernelGGL((kb_pattern_g<K, M, BS, BPL>), dim3(cps * nstripes), dim3(BS), 0, st, (const uint8_t*)a, \
                       (uint8_t*)b, vec, dss, pss, cps); } while (0)
#define KMK(K, M) if (k == K && m == M) { switch (kind) { case 0: KMG(K, M, 128, 8); break; \
    case 1: KMG(K, M, 256, 16); break; case 2: KMG(K, M, 256, 8); break; default: return -1; } \
    return hipGetLastError(); }
    KMK(10, 4) KMK(16, 4) KMK(12, 4) KMK(20, 4)
#undef KMK
#undef KMG
    return -1;
}

// Update / Replace access pattern: K input vectors read, M output vectors read
// and written back in place (XOR for the math), BS lanes x BPL bytes per
// vector per workgroup; stripes interleaved [S][d+p][vec] with inputs at
// base + s*sstride + in_off + i*vec and outputs at base + s*sstride + out_off + j*vec.
template <int K, int M, int BS, int BPL>
__global__ __launch_bounds__(BS) void kb_rmw(uint8_t* base, uint64_t vec, uint64_t sstride, uint64_t in_off,
                                             uint64_t out_off, uint64_t cps) {
    const uint64_t s = blockIdx.x / cps, cb = blockIdx.x % cps;
    const uint32_t off = (uint32_t)(cb * (BS * BPL) + threadIdx.x * BPL);
    uint8_t* st = base + s * sstride;
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    if constexpr (BPL == 16) {
        u32x4 x[K], y[M];
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(st + in_off + i * vec, (uint32_t)vec), off, 0, 2);
#pragma unroll
        for (int j = 0; j < M; ++j) y[j] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(st + out_off + j * vec, (uint32_t)vec), off, 0, 2);
#pragma unroll
        for (int j = 0; j < M; ++j) {
#pragma unroll
            for (int i = 0; i < K; ++i) y[j] ^= x[i];
            __builtin_amdgcn_raw_buffer_store_b128(y[j], rsrc(st + out_off + j * vec, (uint32_t)vec), off, 0, 2);
        }
    } else {
        u32x2 x[K], y[M];
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = __builtin_amdgcn_raw_buffer_load_b64(rsrc(st + in_off + i * vec, (uint32_t)vec), off, 0, 2);
#pragma unroll
        for (int j = 0; j < M; ++j) y[j] = __builtin_amdgcn_raw_buffer_load_b64(rsrc(st + out_off + j * vec, (uint32_t)vec), off, 0, 2);
#pragma unroll
        for (int j = 0; j < M; ++j) {
#pragma unroll
            for (int i = 0; i < K; ++i) y[j] ^= x[i];
            __builtin_amdgcn_raw_buffer_store_b64(y[j], rsrc(st + out_off + j * vec, (uint32_t)vec), off, 0, 2);
        }
    }
}

// kind: 0 = 128 lanes x 8 B, 1 = 256 x 16 B; k = 1 (Replace rn=1) or 2 (Update: old, new), m = 4
extern "C" int probe_rmw(int kind, int k, void* base, uint64_t vec, uint64_t sstride, uint64_t in_off, uint64_t out_off,
                         int nstripes, void* stream) {
    hipStream_t st = (hipStream_t)stream;
#define RMW(K, BS, BPL) do { const uint64_t cps = vec / (BS * BPL); \
    hipLaunchKernelGGL((kb_rmw<K, 4, BS, BPL>), dim3(cps * nstripes), dim3(BS), 0, st, (uint8_t*)base, vec, sstride, \
                       in_off, out_off, cps); } while (0)
    if (k == 1) { if (kind == 0) RMW(1, 128, 8); else RMW(1, 256, 16); }
    else if (k == 2) { if (kind == 0) RMW(2, 128, 8); else RMW(2, 256, 16); }
    else return -1;
#undef RMW
    return hipGetLastError();
}

// Counter calibration (MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are
// calibrated only for 16-B-per-lane streams): one pass over `bytes` with each
// access width, buffer nt like the codec kernels.  Distinct kernel names so
// rocprofv3 attributes the counters per width (tools/fetch_calib.py).
__global__ __launch_bounds__(256) void kc_read16(const uint8_t* src, uint8_t* sink) {
    const uint64_t base = (uint64_t)blockIdx.x * 4096;
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(src + base, 4096), threadIdx.x * 16, 0, 2);
    if (v.x == 0x9e3779b9u && v.y == 0x7f4a7c15u && v.z == 1u) *(u32x4*)sink = v;
}
__global__ __launch_bounds__(256) void kc_read8(const uint8_t* src, uint8_t* sink) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const uint64_t base = (uint64_t)blockIdx.x * 2048;
    u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rsrc(src + base, 2048), threadIdx.x * 8, 0, 2);
    if (v.x == 0x9e3779b9u && v.y == 0x7f4a7c15u) *(u32x2*)sink = v;
}
__global__ __launch_bounds__(256) void kc_write16(uint8_t* dst) {
    const uint64_t base = (uint64_t)blockIdx.x * 4096;
    u32x4 v = {blockIdx.x, threadIdx.x, 2u, 3u};
    __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(dst + base, 4096), threadIdx.x * 16, 0, 2);
}
__global__ __launch_bounds__(256) void kc_write8(uint8_t* dst) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const uint64_t base = (uint64_t)blockIdx.x * 2048;
    u32x2 v = {blockIdx.x, threadIdx.x};
    __builtin_amdgcn_raw_buffer_store_b64(v, rsrc(dst + base, 2048), threadIdx.x * 8, 0, 2);
}
extern "C" int probe_calib(int kind, void* a, uint64_t bytes, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    uint8_t* p = (uint8_t*)a;
    if (bytes % 4096) return -1;
    if (kind == 0) hipLaunchKernelGGL(kc_read16, dim3(bytes / 4096), dim3(256), 0, st, p, p);
    else if (kind == 1) hipLaunchKernelGGL(kc_read8, dim3(bytes / 2048), dim3(256), 0, st, p, p);
    else if (kind == 2) hipLaunchKernelGGL(kc_write16, dim3(bytes / 4096), dim3(256), 0, st, p);
    else if (kind == 3) hipLaunchKernelGGL(kc_write8, dim3(bytes / 2048), dim3(256), 0, st, p);
    else return -1;
    return hipGetLastError();
}

// In-place Reconst access pattern: stripes
// of NV vectors `vec` bytes apart in one buffer (the interleaved
// [S][d+p][len] layout), KR survivors read and KW lost vectors written in
// place; 8-byte lanes, 128-lane workgroups (1 KiB of every vector per chunk),
// buffer nt, XOR instead of the GF math.  DEFER: 0 = read a chunk, write it;
// 1 = each workgroup takes two chunks G/2 apart in the grid (different
// stripes) and stores the first only after the second's loads are issued;
// 2 = the same with adjacent chunks (1 KiB apart).
struct IdxList {
    uint32_t rd[32], wr[32];
};
template <int KR, int KW, int DEFER>
__global__ __launch_bounds__(128) void kin_inplace(uint8_t* base, uint64_t vec, uint64_t sstride, uint32_t cps,
                                                   uint32_t nchunks, IdxList L) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    auto chunk_of = [&](uint32_t c, uint64_t& sb, uint32_t& off) {
        const uint32_t s = c / cps, cb = c % cps;
        sb = (uint64_t)s * sstride;
        off = cb * 1024u + threadIdx.x * 8u;
    };
    auto load = [&](uint64_t sb, uint32_t off, u32x2 (&x)[KR]) {
#pragma unroll
        for (int i = 0; i < KR; ++i)
            x[i] = __builtin_amdgcn_raw_buffer_load_b64(rsrc(base + sb + L.rd[i] * vec, (uint32_t)vec), off, 0, 2);
    };
    auto store = [&](uint64_t sb, uint32_t off, const u32x2 (&x)[KR]) {
#pragma unroll
        for (int j = 0; j < KW; ++j) {
            u32x2 a = {(uint32_t)j, 0u};
#pragma unroll
            for (int i = 0; i < KR; ++i) a ^= x[i];
            __builtin_amdgcn_raw_buffer_store_b64(a, rsrc(base + sb + L.wr[j] * vec, (uint32_t)vec), off, 0, 2);
        }
    };
    if (DEFER == 0) {
        uint64_t sb;
        uint32_t off;
        chunk_of(blockIdx.x, sb, off);
        u32x2 x[KR];
        load(sb, off, x);
        store(sb, off, x);
        return;
    }
    const uint32_t c0 = DEFER == 1 ? blockIdx.x : 2 * blockIdx.x;
    const uint32_t c1 = DEFER == 1 ? blockIdx.x + nchunks / 2 : 2 * blockIdx.x + 1;
    uint64_t sb0, sb1;
    uint32_t off0, off1;
    chunk_of(c0, sb0, off0);
    chunk_of(c1, sb1, off1);
    u32x2 x0[KR], x1[KR];
    load(sb0, off0, x0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    load(sb1, off1, x1);
    store(sb0, off0, x0);
    store(sb1, off1, x1);
}

// Geometry of the run-time assembly kernels (jit_asm.cpp) against the
// perm-table kernels' (in-place Reconst).  GEO (lanes per
// workgroup, bytes a workgroup covers per vector, 8-byte pieces per lane):
//   0: 128 lanes, 1 KiB, 1 piece at 8t          (perm-table kernels)
//   1:  64 lanes, 2 KiB, 4 pieces at 8t + 512k  (assembly kernels, round 3)
//   2: 256 lanes, 2 KiB, 1 piece at 8t
//   3: 128 lanes, 2 KiB, 2 pieces at 8t + 1024k
//   4:  64 lanes, 512 B of 4 stripes: piece k at 8t of stripe 4g + k
//   5: 256 lanes, 8 KiB, 4 pieces at 512w + 8l + 2048k (wave w, lane l)
//   6: 128 lanes, 4 KiB, 4 pieces at 512w + 8l + 1024k
// SPLIT: the lost vectors are written into a separate [S][KW][vec] region
// (`wbase`) instead of in place.  Every load is issued before any store;
// XOR for the math.
template <int GEO>
struct Geo {
    static constexpr int lanes = GEO == 0 ? 128 : GEO == 2 ? 256 : GEO == 3 ? 128 : GEO == 5 ? 256 : GEO == 6 ? 128 : 64;
    static constexpr int P = GEO == 1 || GEO == 4 || GEO >= 5 ? 4 : GEO == 3 ? 2 : 1;
    static constexpr uint32_t chunk = GEO == 0 ? 1024 : GEO == 4 ? 512 : GEO == 5 ? 8192 : GEO == 6 ? 4096 : 2048;
    static constexpr uint32_t step = GEO == 1 ? 512 : GEO == 3 ? 1024 : GEO == 5 ? 2048 : GEO == 6 ? 1024 : 0;
    static constexpr int spp = GEO == 4 ? 4 : 1;                             // stripes per workgroup
};
template <int KR, int KW, int GEO, bool SPLIT>
__global__ __launch_bounds__(Geo<GEO>::lanes) void kin_geo(uint8_t* base, uint8_t* wbase, uint64_t vec,
                                                            uint64_t sstride, uint32_t cps, IdxList L) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    typedef Geo<GEO> G;
    const uint32_t sg = blockIdx.x / cps, cb = blockIdx.x % cps;
    const uint32_t off0 = GEO >= 5 ? cb * G::chunk + (threadIdx.x >> 6) * 512u + (threadIdx.x & 63) * 8u
                                   : cb * G::chunk + threadIdx.x * 8u;
    auto stripe = [&](int k) { return (uint64_t)(sg * G::spp + (G::spp > 1 ? k : 0)); };
    auto offk = [&](int k) { return off0 + (G::spp > 1 ? 0u : G::step * k); };
    u32x2 x[KR][G::P];
#pragma unroll
    for (int i = 0; i < KR; ++i)
#pragma unroll
        for (int k = 0; k < G::P; ++k)
            x[i][k] = __builtin_amdgcn_raw_buffer_load_b64(
                rsrc(base + stripe(k) * sstride + L.rd[i] * vec, (uint32_t)vec), offk(k), 0, 2);
#pragma unroll
    for (int j = 0; j < KW; ++j) {
#pragma unroll
        for (int k = 0; k < G::P; ++k) {
            uint8_t* w = SPLIT ? wbase + (stripe(k) * KW + j) * vec : base + stripe(k) * sstride + L.wr[j] * vec;
            u32x2 a = {(uint32_t)j, 0u};
#pragma unroll
            for (int i = 0; i < KR; ++i) a ^= x[i][k];
            __builtin_amdgcn_raw_buffer_store_b64(a, rsrc(w, (uint32_t)vec), offk(k), 0, 2);
        }
    }
}

// 16-byte pieces, 64 lanes over 2 KiB: GEO 7 = two dwordx4 at 16l + 1024k
// (each wave instruction covers 1 KiB), GEO 8 = two dwordx4 at 32l + 16k
// (a lane's 32 bytes contiguous; each instruction touches every other 16 B)
template <int KR, int KW, int GEO, bool SPLIT>
__global__ __launch_bounds__(64) void kin_geo16(uint8_t* base, uint8_t* wbase, uint64_t vec, uint64_t sstride,
                                                uint32_t cps, IdxList L) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t s = blockIdx.x / cps, cb = blockIdx.x % cps;
    const uint64_t sb = (uint64_t)s * sstride;
    auto offk = [&](int k) {
        return GEO == 7 ? cb * 2048u + threadIdx.x * 16u + 1024u * k : cb * 2048u + threadIdx.x * 32u + 16u * k;
    };
    u32x4 x[KR][2];
#pragma unroll
    for (int i = 0; i < KR; ++i)
#pragma unroll
        for (int k = 0; k < 2; ++k)
            x[i][k] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base + sb + L.rd[i] * vec, (uint32_t)vec), offk(k), 0, 2);
#pragma unroll
    for (int j = 0; j < KW; ++j) {
        uint8_t* w = SPLIT ? wbase + ((uint64_t)s * KW + j) * vec : base + sb + L.wr[j] * vec;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            u32x4 a = {(uint32_t)j, 0u, 0u, 0u};
#pragma unroll
            for (int i = 0; i < KR; ++i) a ^= x[i][k];
            __builtin_amdgcn_raw_buffer_store_b128(a, rsrc(w, (uint32_t)vec), offk(k), 0, 2);
        }
    }
}

// kind = GEO + 16 * SPLIT (GEO 0-8 above); nstripes a multiple of 4
extern "C" int probe_geo(int kind, int shape, void* a, void* w, uint64_t vec, int nstripes, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    IdxList L{};
    const int geo = kind & 15;
    const bool split = kind >= 16;
    if (geo > 8 || nstripes % 4) return -1;
    const uint32_t chunk = geo == 0 ? 1024 : geo == 4 ? 512 : geo == 5 ? 8192 : geo == 6 ? 4096 : 2048;
    const uint32_t cps = static_cast<uint32_t>(vec / chunk);
    const uint32_t groups = geo == 4 ? nstripes / 4 : nstripes;
    const dim3 grid(cps * groups);
#define KG1(KR, KW, G, SP)                                                                                     \
    hipLaunchKernelGGL((kin_geo<KR, KW, G, SP>), grid, dim3(Geo<G>::lanes), 0, st, (uint8_t*)a, (uint8_t*)w, vec, \
                       ss, cps, L)
#define KG16(KR, KW, G, SP)                                                                                    \
    hipLaunchKernelGGL((kin_geo16<KR, KW, G, SP>), grid, dim3(64), 0, st, (uint8_t*)a, (uint8_t*)w, vec, ss, cps, L)
#define KG(KR, KW, NV)                                                          \
    do {                                                                        \
        const uint64_t ss = (uint64_t)(NV) * vec;                               \
        switch (kind) {                                                         \
            case 0: KG1(KR, KW, 0, false); break;                               \
            case 1: KG1(KR, KW, 1, false); break;                               \
            case 2: KG1(KR, KW, 2, false); break;                               \
            case 3: KG1(KR, KW, 3, false); break;                               \
            case 4: KG1(KR, KW, 4, false); break;                               \
            case 5: KG1(KR, KW, 5, false); break;                               \
            case 6: KG1(KR, KW, 6, false); break;                               \
            case 7: KG16(KR, KW, 7, false); break;                              \
            case 8: KG16(KR, KW, 8, false); break;                              \
            case 16: KG1(KR, KW, 0, true); break;                               \
            case 17: KG1(KR, KW, 1, true); break;                               \
            case 18: KG1(KR, KW, 2, true); break;                               \
            case 19: KG1(KR, KW, 3, true); break;                               \
            case 20: KG1(KR, KW, 4, true); break;                               \
            case 21: KG1(KR, KW, 5, true); break;                               \
            case 22: KG1(KR, KW, 6, true); break;                               \
            case 23: KG16(KR, KW, 7, true); break;                              \
            default: KG16(KR, KW, 8, true); break;                              \
        }                                                                       \
    } while (0)
    (void)split;
    if (shape == 0) {
        for (int i = 0; i < 10; ++i) L.rd[i] = 8 + i;
        for (int j = 0; j < 8; ++j) L.wr[j] = j;
        KG(10, 8, 18);
    } else if (shape == 1) {
        const uint32_t wr[5] = {0, 2, 4, 6, 8}, rd[10] = {1, 3, 5, 7, 9, 10, 11, 12, 13, 14};
        for (int i = 0; i < 10; ++i) L.rd[i] = rd[i];
        for (int j = 0; j < 5; ++j) L.wr[j] = wr[j];
        KG(10, 5, 18);
    } else {
        for (int i = 0; i < 10; ++i) L.rd[i] = 4 + i;
        for (int j = 0; j < 4; ++j) L.wr[j] = j;
        KG(10, 4, 14);
    }
#undef KG
#undef KG1
#undef KG16
    return hipGetLastError();
}

// kind: 0/1/2 = DEFER; shape: 0 = 10+8 lost 0-7 (reads 8..17), 1 = 10+8
// lost 0,2,4,6,8 (5 writes), 2 = 10+4 lost 0-3, 3 = 10+8 Encode-like (reads
// 0..9, writes 10..17; the same in-place buffer)
extern "C" int probe_inplace(int kind, int shape, void* a, uint64_t vec, int nstripes, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    IdxList L{};
    const uint32_t cps = static_cast<uint32_t>(vec / 1024);
    const uint32_t nchunks = cps * static_cast<uint32_t>(nstripes);
    const dim3 grid(kind == 0 ? nchunks : nchunks / 2);
#define KIN(KR, KW, NV)                                                                                        \
    do {                                                                                                      \
        const uint64_t ss = (uint64_t)(NV) * vec;                                                              \
        if (kind == 0) hipLaunchKernelGGL((kin_inplace<KR, KW, 0>), grid, dim3(128), 0, st, (uint8_t*)a, vec, ss, cps, nchunks, L); \
        else if (kind == 1) hipLaunchKernelGGL((kin_inplace<KR, KW, 1>), grid, dim3(128), 0, st, (uint8_t*)a, vec, ss, cps, nchunks, L); \
        else hipLaunchKernelGGL((kin_inplace<KR, KW, 2>), grid, dim3(128), 0, st, (uint8_t*)a, vec, ss, cps, nchunks, L); \
    } while (0)
    if (shape == 0) {
        for (int i = 0; i < 10; ++i) L.rd[i] = 8 + i;
        for (int j = 0; j < 8; ++j) L.wr[j] = j;
        KIN(10, 8, 18);
    } else if (shape == 1) {
        const uint32_t w[5] = {0, 2, 4, 6, 8}, r[10] = {1, 3, 5, 7, 9, 10, 11, 12, 13, 14};
        for (int i = 0; i < 10; ++i) L.rd[i] = r[i];
        for (int j = 0; j < 5; ++j) L.wr[j] = w[j];
        KIN(10, 5, 18);
    } else if (shape == 2) {
        for (int i = 0; i < 10; ++i) L.rd[i] = 4 + i;
        for (int j = 0; j < 4; ++j) L.wr[j] = j;
        KIN(10, 4, 14);
    } else {
        for (int i = 0; i < 10; ++i) L.rd[i] = i;
        for (int j = 0; j < 8; ++j) L.wr[j] = 10 + j;
        KIN(10, 8, 18);
    }
#undef KIN
    return hipGetLastError();
}
