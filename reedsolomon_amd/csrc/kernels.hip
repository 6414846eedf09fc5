// kernels.hip — CDNA4 (gfx950) kernels for the GF(2^8) matrix product.
//
// Replaces the reference's hot loops: the chunk loop
// rs.go:146-153, the d x p call loop of encodePart rs.go:181-188 and the
// AVX2 split-nibble kernel gmu_amd64.s:40-329 (mulVectAVX2 / mulVectXORAVX2),
// plus the scalar tail gmu.go:11-23.
//
// Design:
//  * One launch covers every stripe, every row and every column.  A lane
//    owns a 16-byte column slice of every vector of its stripe: it streams
//    the k input slices (global_load_dwordx4, coalesced 1 KiB per wave
//    instruction), keeps the m output slices in VGPRs, and stores each once.
//    HBM traffic is the algorithmic (k+m)*len per stripe.
//  * Multiply-by-constant on four packed bytes = three v_perm_b32 lookups
//    into 8/8/4-entry byte tables (bit groups {0-2},{3-5},{6-7} of x; the
//    map x -> c*x is GF(2)-linear, so the three partial products XOR).  The
//    bit-group extraction is shared by all m rows; per (row, column, dword)
//    the cost is 3 v_perm + ~1.5 XOR (v_bitop3 xor3).  No MFMA: this is
//    byte-table work.
//  * The per-coefficient tables (5 dwords each) are staged once per
//    workgroup into LDS; the inner loop reads one column's tables with
//    wave-uniform ds_read_b128 (broadcast) and keeps them in VGPRs for the
//    lane's 16*VPT bytes.
//  * Rows beyond the launch's row group and columns beyond `cols` (padding
//    up to the batch width KB) use all-zero tables, so every lane runs the
//    same straight-line code: no per-column branches around loads.
//  * Bytes that are not covered by the aligned 16-byte body (len % 16, or
//    vectors whose base/stride is not 16-byte aligned) go to a byte-granular
//    kernel with identical arithmetic.
#include "kernels.hpp"
#include "jit.hpp"
#include "jit_asm.hpp"

#include <cstdlib>
#include <cstring>

namespace rsamd {

constexpr int kBlock = 256;
constexpr int kWideRows = 16;  // output rows per wave of the wide kernels
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) u32x4 g_u32x4;        // global (HBM) 16-byte word
typedef __attribute__((address_space(3))) const u32x4 lds_u32x4;  // LDS 16-byte word

LaunchTuning& tuning() {
    static LaunchTuning t = [] {
        LaunchTuning x{};
        const char* g = std::getenv("RSAMD_MAX_GRID");
        x.max_grid = g ? std::atoi(g) : 0;
        const char* v = std::getenv("RSAMD_VPT");
        x.vpt = v ? std::atoi(v) : 1;
        if (x.vpt != 2) x.vpt = 1;
        const char* n = std::getenv("RSAMD_NT_STORE");
        x.nt_store = n ? std::atoi(n) : 1;
        x.var = -1;
#ifdef RSAMD_EXPERIMENTS  // code-shape experiments exist only in librsamd_exp.so (tools/ab.py)
        const char* e = std::getenv("RSAMD_VAR");
        x.var = e ? std::atoi(e) : -1;
#endif
        const char* l = std::getenv("RSAMD_LDS_PAD");
        x.lds_pad = l ? std::atoi(l) : 0;
        const char* lb = std::getenv("RSAMD_LANE_BYTES");
        x.lane_bytes = (lb && std::atoi(lb) == 16) ? 16 : 8;
        const char* b8 = std::getenv("RSAMD_BLOCK8");
        x.block8 = (b8 && std::atoi(b8) == 256) ? 256 : 128;
        const char* bsl = std::getenv("RSAMD_BITSLICE");
        x.bitslice = (bsl && std::atoi(bsl) == 0) ? 0 : 1;
        x.bs_block = 0;
        x.wide_block = 256;
        x.wide_single_pass = 1;
        // 2 waves per SIMD: fewer 32 * bs-byte chunks in flight per CU; +3-8 %
        // on every generated shape, split and interleaved (10+8 Encode 6.04 ->
        // 6.28 TB/s, 8+5 interleaved 6.06 -> 6.53; profiles/r03/ab_bs_waves.log)
        const char* bw = std::getenv("RSAMD_BS_WAVES");
        x.bs_waves = bw ? std::atoi(bw) : 2;
        x.multi_gpu_plan = -1;
        return x;
    }();
    return t;
}

// c * x for the four bytes of x, given the bit-group indices of x and the
// coefficient's perm table (t[0..4], see gf256.hpp perm_table()).
__device__ __forceinline__ uint32_t gf_mul_packed(uint32_t i0, uint32_t i1, uint32_t i2,
                                                  const uint32_t* t) {
    return __builtin_amdgcn_perm(t[1], t[0], i0) ^ __builtin_amdgcn_perm(t[3], t[2], i1) ^
           __builtin_amdgcn_perm(t[4], t[4], i2);
}

__device__ __forceinline__ void split_groups(uint32_t x, uint32_t& i0, uint32_t& i1, uint32_t& i2) {
    i0 = x & 0x07070707u;
    i1 = (x >> 3) & 0x07070707u;
    i2 = (x >> 6) & 0x03030303u;
}

typedef __attribute__((address_space(1))) uint8_t g_u8;

// Vector addresses live in the kernarg block as integers; casting them to
// address_space(1) pointers makes the compiler emit global_* (not flat_*)
// memory instructions.
__device__ __forceinline__ const g_u8* in_ptr(const MatmulArgs& a, int col, int s) {
    return reinterpret_cast<const g_u8*>(a.ptr[col]) + static_cast<int64_t>(s) * a.ss[a.sid[col] & 3];
}
// `cols` is passed separately so specialised kernels index with a constant.
__device__ __forceinline__ g_u8* out_ptr(const MatmulArgs& a, int cols, int row, int s) {
    const int v = cols + row;
    return reinterpret_cast<g_u8*>(a.ptr[v]) + static_cast<int64_t>(s) * a.ss[a.sid[v] & 3];
}

// ---------------------------------------------------------------------------
// Vector kernel: the aligned 16-byte body of every vector of every stripe.
//   KB   columns per load batch (all KB loads are issued before the math)
//   KFIX cols == KB exactly (fully unrolled single batch)
//   MC   rows per pass (row groups loop when rows > MC)
//   ACC  XOR into the outputs (Update / Replace) instead of overwriting
//   VPT  16-byte units per lane per chunk
//   VAR  code-shape flags (kVar* below); the default is kVarDefault
// ---------------------------------------------------------------------------
// kVarXorOnly is a DIAGNOSTIC (acc ^= x instead of the GF product: the memory
// ceiling of the access pattern).  It exists only in the experiments build
// (-DRSAMD_EXPERIMENTS, librsamd_exp.so); in the product library the flag is 0,
// so no instantiation can compute anything but the GF product.
#ifdef RSAMD_EXPERIMENTS
constexpr int kVarXorOnly = 1;
#else
constexpr int kVarXorOnly = 0;
#endif
enum : int {
    kVarNtLoad = 2,      // non-temporal input loads
    kVarSingleTab = 4,   // no LDS table prefetch across columns (fewer VGPRs)
    kVarBitop3 = 8,      // explicit v_bitop3 (xor3) accumulation
    kVarCarry = 16,      // with kVarBitop3: pair columns through a carried term (1.5 xor3 per product, not 2)
    kVarShift64 = 32,    // bit groups of dword pairs via v_lshrrev_b64 (4 VALU per dword, not 5)
};
// kVarCarry: A/B on MI355X (tools/ab.py, profiles/r01/ab_carry.log): split
// Encode +0.3-2.6 %, interleaved Encode +2 %, Reconst of 4 +2.4 %, 16-pattern
// Reconst +1.6 %, the rest within noise; 8 % fewer VALU instructions.
// kVarShift64: in-process A/B on two boxes (profiles/r01/ab_shift64.log):
// +0.5-1.1 % with 16-byte lane units, +0.5-0.4 % with 8-byte units; VALU per
// wave 959 -> 919 (16 B), 499 -> 479 (8 B).
constexpr int kVarDefault = kVarBitop3 | kVarSingleTab | kVarNtLoad | kVarCarry | kVarShift64;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// 16-byte load / store of vector data.  LAUX / SAUX >= 0 select buffer
// instructions with that cache-policy immediate (bit0 sc0, bit1 nt, bit4 sc1
// on gfx950); -1 keeps global_load/store (nt per VAR / nt_store).  The buffer
// descriptor is built from wave-uniform values (kernarg pointer + stripe
// base), so no waterfall loop is generated (cdna_hip_programming.md T20).
template <int LQ> struct LaneWord;
template <> struct LaneWord<4> { typedef u32x4 type; };
template <> struct LaneWord<2> { typedef u32x2 type; };

// 4*LQ-byte load / store of vector data (LQ = 4: dwordx4, LQ = 2: dwordx2).
// AUX >= 0 selects buffer instructions with that cache-policy immediate (bit0
// sc0, bit1 nt, bit4 sc1 on gfx950); -1 keeps global_load/store (nt per VAR /
// nt_store).  The buffer descriptor is built from wave-uniform values
// (kernarg pointer + stripe base), so no waterfall loop is generated
// (cdna_hip_programming.md T20).
template <int AUX, int LQ = 4>
__device__ __forceinline__ typename LaneWord<LQ>::type load16(const g_u8* base, uint64_t off, uint32_t nbytes,
                                                              bool nt) {
    typedef typename LaneWord<LQ>::type W;
    if constexpr (AUX >= 0) {
        __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc((void*)(base), 0, static_cast<int>(nbytes), 0x00020000);
        if constexpr (LQ == 4) return __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(off), 0, AUX);
        else return __builtin_amdgcn_raw_buffer_load_b64(r, static_cast<int>(off), 0, AUX);
    } else {
        typedef __attribute__((address_space(1))) W gW;
        const gW* src = reinterpret_cast<const gW*>(base + off);
        return nt ? __builtin_nontemporal_load(src) : *src;
    }
}

template <int AUX, int LQ = 4>
__device__ __forceinline__ void store16(g_u8* base, uint64_t off, uint32_t nbytes, typename LaneWord<LQ>::type val,
                                        bool nt) {
    typedef typename LaneWord<LQ>::type W;
    if constexpr (AUX >= 0) {
        __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc((void*)(base), 0, static_cast<int>(nbytes), 0x00020000);
        if constexpr (LQ == 4) __builtin_amdgcn_raw_buffer_store_b128(val, r, static_cast<int>(off), 0, AUX);
        else __builtin_amdgcn_raw_buffer_store_b64(val, r, static_cast<int>(off), 0, AUX);
    } else {
        typedef __attribute__((address_space(1))) W gW;
        gW* o = reinterpret_cast<gW*>(base + off);
        if (nt) __builtin_nontemporal_store(val, o);
        else *o = val;
    }
}

// Default cache policy of the vector kernel: buffer_load/store ... nt (aux 2).
// Measured in-process on MI355X (tools/ab.py): 0.590 ms vs 0.632 ms for
// global_load/store nt on the 10+4 @ 1 MiB x 256 launch.
constexpr int kAuxNt = 2;

// One workgroup-chunk of the product: the lane's 16*VPT-byte slice of every
// input column in, of every output row (up to MC) out.  `in_base(c)` /
// `out_base(r)` give the stripe base address of input column c / output row
// r (wave-uniform); the LDS holds this launch's (or this pattern's) tables.
//   WIN  0: issue all KB column loads up front; >0: rolling window of WIN
//        columns in flight per lane (fewer VGPRs, more resident waves)
struct NoStage {
    __device__ void operator()() const {}
};

// `stage` runs once, after the first column batch's loads are issued and
// before the first LDS table read: a kernel that stages its tables there
// overlaps that global->LDS copy with its data loads.
template <int KB, bool KFIX, int MC, bool ACC, int VPT, int VAR, int LAUX, int SAUX, int WIN, int LQ, int BS, class InBase,
          class OutBase, class Stage = NoStage>
__device__ __forceinline__ void chunk_body(const MatmulArgs& a, const lds_u32x4* lds_tab, int cols, int ncols_pad,
                                           int nrows, int64_t cb, uint64_t nunits, InBase in_base,
                                           OutBase out_base, Stage stage = Stage()) {
    constexpr int COLD = ((MC * 5 + 3) / 4) * 4;  // dwords per column in LDS (16-B multiple)
    constexpr int COLW = COLD / 4;                // 16-byte LDS words per column
    typedef typename LaneWord<LQ>::type W;  // the lane's unit: 4*LQ bytes of one vector
    const int tid = threadIdx.x;
    uint64_t off[VPT];
    bool ok[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        const uint64_t u = static_cast<uint64_t>(cb) * a.units_per_chunk + v * BS + tid;
        ok[v] = u < nunits;
        off[v] = (ok[v] ? u : 0) * (4 * LQ);  // clamp: out-of-range lanes read unit 0, store nothing
    }

    uint32_t acc[MC][VPT][LQ];
#pragma unroll
    for (int r = 0; r < MC; ++r)
#pragma unroll
        for (int v = 0; v < VPT; ++v)
#pragma unroll
            for (int q = 0; q < LQ; ++q) acc[r][v][q] = 0;
    uint32_t carry[MC][VPT][LQ];  // kVarCarry: third partial product of an even column
    if (VAR & kVarCarry) {
#pragma unroll
        for (int r = 0; r < MC; ++r)
#pragma unroll
            for (int v = 0; v < VPT; ++v)
#pragma unroll
                for (int q = 0; q < LQ; ++q) carry[r][v][q] = 0;
    }
    if (ACC) {
#pragma unroll
        for (int r = 0; r < MC; ++r)
            if (r < nrows)
#pragma unroll
                for (int v = 0; v < VPT; ++v) {
                    const W o = load16<LAUX, LQ>(out_base(r), off[v], static_cast<uint32_t>(a.body), false);
#pragma unroll
                    for (int q = 0; q < LQ; ++q) acc[r][v][q] = o[q];
                }
    }

    for (int i0 = 0; i0 < ncols_pad; i0 += KB) {
        // Issue the column loads of this batch first (KB*16*VPT bytes in flight
        // per lane), or the first WIN of them with the rest rolled in below.
        constexpr int kFirst = (WIN > 0 && WIN < KB) ? WIN : KB;
        // Columns of this batch (uniform): a batch past `cols` skips its
        // padding columns' loads and math with a scalar branch.
        const int nb = KFIX ? KB : ((cols - i0) < KB ? (cols - i0) : KB);
        W x[KB][VPT];
        auto load_col = [&](int b) {
            if (!KFIX && b >= nb) return;
            const int c = i0 + b;
            const g_u8* p = in_base(c);
#pragma unroll
            for (int v = 0; v < VPT; ++v)
                x[b][v] = load16<LAUX, LQ>(p, off[v], static_cast<uint32_t>(a.body), (VAR & kVarNtLoad) != 0);
        };
#pragma unroll
        for (int b = 0; b < kFirst; ++b) load_col(b);
        if (i0 == 0) stage();
        // Tables of column b+1 are read from LDS while column b is computed.
        constexpr bool kPrefetchTab = !(VAR & kVarSingleTab);
        u32x4 tv[2][COLW];
        if (kPrefetchTab) {
#pragma unroll
            for (int w = 0; w < COLW; ++w) tv[0][w] = lds_tab[i0 * COLW + w];
        }
#pragma unroll
        for (int b = 0; b < KB; ++b) {
            if (!KFIX && b >= nb) break;
            // Scheduling fence: keeps each column's LDS reads next to its math
            // (hoisted, all k*MC tables would pin ~200 VGPRs: one wave/SIMD).
            __builtin_amdgcn_sched_barrier(0);
            if (kPrefetchTab) {
                if (b + 1 < KB) {
#pragma unroll
                    for (int w = 0; w < COLW; ++w) tv[(b + 1) & 1][w] = lds_tab[(i0 + b + 1) * COLW + w];
                }
            } else {
#pragma unroll
                for (int w = 0; w < COLW; ++w) tv[b & 1][w] = lds_tab[(i0 + b) * COLW + w];
            }
            uint32_t t[COLD];
#pragma unroll
            for (int w = 0; w < COLW; ++w) {
                t[4 * w + 0] = tv[b & 1][w].x; t[4 * w + 1] = tv[b & 1][w].y;
                t[4 * w + 2] = tv[b & 1][w].z; t[4 * w + 3] = tv[b & 1][w].w;
            }
#pragma unroll
            for (int v = 0; v < VPT; ++v) {
                // kVarShift64: bit groups of a dword pair from two 64-bit shifts
                constexpr int QS = ((VAR & kVarShift64) && LQ % 2 == 0) ? 2 : 1;
#pragma unroll
                for (int qp = 0; qp < LQ; qp += QS) {
                uint32_t G0[QS], G1[QS], G2[QS];
                if (!(VAR & kVarXorOnly)) {
                    if constexpr (QS == 2) {
                        const uint64_t X = (static_cast<uint64_t>(x[b][v][qp + 1]) << 32) | x[b][v][qp];
                        uint64_t Y3, Y6;
                        asm volatile("v_lshrrev_b64 %0, 3, %1" : "=v"(Y3) : "v"(X));
                        asm volatile("v_lshrrev_b64 %0, 6, %1" : "=v"(Y6) : "v"(X));
                        G0[0] = x[b][v][qp] & 0x07070707u;
                        G0[1] = x[b][v][qp + 1] & 0x07070707u;
                        G1[0] = static_cast<uint32_t>(Y3) & 0x07070707u;
                        G1[1] = static_cast<uint32_t>(Y3 >> 32) & 0x07070707u;
                        G2[0] = static_cast<uint32_t>(Y6) & 0x03030303u;
                        G2[1] = static_cast<uint32_t>(Y6 >> 32) & 0x03030303u;
                    } else {
                        split_groups(x[b][v][qp], G0[0], G1[0], G2[0]);
                    }
                }
#pragma unroll
                for (int qq = 0; qq < QS; ++qq) {
                    const int q = qp + qq;
                    const uint32_t xq = x[b][v][q];
                    if (VAR & kVarXorOnly) {
#pragma unroll
                        for (int r = 0; r < MC; ++r) acc[r][v][q] ^= xq ^ t[r * 5];
                        continue;
                    }
                    const uint32_t g0 = G0[qq], g1 = G1[qq], g2 = G2[qq];
#pragma unroll
                    for (int r = 0; r < MC; ++r) {
                        const uint32_t* tr = &t[r * 5];
                        if (VAR & kVarBitop3) {
                            const uint32_t p0 = __builtin_amdgcn_perm(tr[1], tr[0], g0);
                            const uint32_t p1 = __builtin_amdgcn_perm(tr[3], tr[2], g1);
                            const uint32_t p2 = __builtin_amdgcn_perm(tr[4], tr[4], g2);
                            if (VAR & kVarCarry) {
                                if ((b & 1) == 0) {
                                    acc[r][v][q] = xor3(acc[r][v][q], p0, p1);
                                    carry[r][v][q] = p2;
                                } else {
                                    acc[r][v][q] = xor3(xor3(acc[r][v][q], carry[r][v][q], p0), p1, p2);
                                }
                            } else {
                                acc[r][v][q] = xor3(xor3(acc[r][v][q], p0, p1), p2, 0);
                            }
                        } else {
                            acc[r][v][q] ^= gf_mul_packed(g0, g1, g2, tr);
                        }
                    }
                }
                }
            }
            // Pin the running sums per column: stops LLVM from reassociating
            // the XOR chains across columns (which keeps every column's
            // partial products live and spills to AGPRs).
#pragma unroll
            for (int r = 0; r < MC; ++r)
#pragma unroll
                for (int v = 0; v < VPT; ++v)
#pragma unroll
                    for (int q = 0; q < LQ; ++q) {
                        asm volatile("" : "+v"(acc[r][v][q]));
                        if ((VAR & kVarCarry) && (b & 1) == 0) asm volatile("" : "+v"(carry[r][v][q]));
                    }
            if (b + kFirst < KB) load_col(b + kFirst);  // rolling window refill
        }
        if ((VAR & kVarCarry) && (nb & 1)) {  // odd column count: fold the last carry
#pragma unroll
            for (int r = 0; r < MC; ++r)
#pragma unroll
                for (int v = 0; v < VPT; ++v)
#pragma unroll
                    for (int q = 0; q < LQ; ++q) acc[r][v][q] ^= carry[r][v][q];
        }
        __builtin_amdgcn_sched_barrier(0);
    }

#pragma unroll
    for (int r = 0; r < MC; ++r) {
        if (r < nrows) {
#pragma unroll
            for (int v = 0; v < VPT; ++v) {
                if (!ok[v]) continue;
                W val;
#pragma unroll
                for (int q = 0; q < LQ; ++q) val[q] = acc[r][v][q];
                store16<SAUX, LQ>(out_base(r), off[v], static_cast<uint32_t>(a.body), val, a.nt_store != 0);
            }
        }
    }
}

template <int KB, bool KFIX, int MC, bool ACC, int VPT, int VAR = kVarDefault, int LAUX = kAuxNt, int SAUX = kAuxNt,
          int WIN = 0>
__global__ __launch_bounds__(kBlock) void gf_matmul_vec(const MatmulArgs a) {
    constexpr int COLD = ((MC * 5 + 3) / 4) * 4;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
    const lds_u32x4* lds_tab = (const lds_u32x4*)(lds32);

    const int cols = KFIX ? KB : a.cols;
    const int ncols_pad = KFIX ? KB : ((cols + KB - 1) / KB) * KB;
    const uint64_t nunits = a.body >> 4;
    const int tid = threadIdx.x;

    for (int rg = 0; rg < a.rows; rg += MC) {
        if (rg) __syncthreads();  // previous group's readers are done with LDS
        // Stage this row group's tables: column i, row rr, entry e -> lds32[i*COLD + rr*5 + e].
        for (int idx = tid; idx < ncols_pad * COLD; idx += kBlock) {
            const int i = idx / COLD;
            const int w = idx - i * COLD;
            const int rr = w / 5;
            uint32_t v = 0;
            if (i < cols && rr < MC && rg + rr < a.rows)
                v = a.tables[(static_cast<int64_t>(i) * a.rows_pad + rg + rr) * 5 + (w - rr * 5)];
            lds32[idx] = v;
        }
        __syncthreads();

        const int nrows = (a.rows - rg) < MC ? (a.rows - rg) : MC;
        for (int64_t chunk = blockIdx.x; chunk < a.total_chunks; chunk += gridDim.x) {
            const int si = static_cast<int>(chunk / a.chunks_per_stripe);
            const int64_t cb = chunk - static_cast<int64_t>(si) * a.chunks_per_stripe;
            const int s = a.stripe_ids ? a.stripe_ids[si] : si;  // uniform: scalar load
            chunk_body<KB, KFIX, MC, ACC, VPT, VAR, LAUX, SAUX, WIN, 4, kBlock>(
                a, lds_tab, cols, ncols_pad, nrows, cb, nunits, [&](int c) { return in_ptr(a, c, s); },
                [&](int r) { return out_ptr(a, cols, rg + r, s); });
        }
    }
}

// One chunk per workgroup, rows <= MC (grid = all chunks): the common case
// without the row-group / grid-stride loops of gf_matmul_vec (less live state).
template <int KB, bool KFIX, int MC, bool ACC, int WIN, bool STAGE_LATE = false, int LQ = 4, int VPT = 1,
          int VAR = kVarDefault, int BS = kBlock, bool XCD = false>
__global__ __launch_bounds__(BS) void gf_matmul_vec1(const MatmulArgs a) {
    constexpr int COLD = ((MC * 5 + 3) / 4) * 4;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
    const lds_u32x4* lds_tab = (const lds_u32x4*)(lds32);
    const int cols = KFIX ? KB : a.cols;
    const int ncols_pad = KFIX ? KB : ((cols + KB - 1) / KB) * KB;
    auto stage = [&]() {
        if (MC == 4 && a.img4) {  // prepared image (get_tables): a plain copy
            for (int idx = threadIdx.x; idx < ncols_pad * COLD; idx += BS) lds32[idx] = a.img4[idx];
        } else {
            for (int idx = threadIdx.x; idx < ncols_pad * COLD; idx += BS) {
                const int i = idx / COLD;
                const int w = idx - i * COLD;
                const int rr = w / 5;
                uint32_t v = 0;
                if (i < cols && rr < MC && rr < a.rows)
                    v = a.tables[(static_cast<int64_t>(i) * a.rows_pad + rr) * 5 + (w - rr * 5)];
                lds32[idx] = v;
            }
        }
        __syncthreads();
    };
    // stripe and chunk of this workgroup: a scalar shift when the chunk count
    // per stripe is a power of two (the grid is < 2^31 chunks).  XCD
    // (experiment, RSAMD_VAR=160): workgroups are dispatched round-robin over
    // the 8 XCDs (b -> XCD b % 8); the remap gives XCD x the contiguous chunks
    // [x * G/8, (x+1) * G/8) (measured slower).
    uint32_t chunk = blockIdx.x;
    if constexpr (XCD) {
        const uint32_t g8 = gridDim.x >> 3;
        if (chunk < (g8 << 3)) chunk = (chunk & 7u) * g8 + (chunk >> 3);
    }
    const uint32_t cps = static_cast<uint32_t>(a.chunks_per_stripe);
    const uint32_t su = a.cps_shift >= 0 ? (chunk >> a.cps_shift) : chunk / cps;
    const int si = static_cast<int>(su);
    const int64_t cb = static_cast<int64_t>(chunk - su * cps);
    const int s = a.stripe_ids ? a.stripe_ids[si] : si;
    if (!STAGE_LATE) stage();
    chunk_body<KB, KFIX, MC, ACC, VPT, VAR, kAuxNt, kAuxNt, WIN, LQ, BS>(
        a, lds_tab, cols, ncols_pad, a.rows, cb, a.body / (4 * LQ), [&](int c) { return in_ptr(a, c, s); },
        [&](int r) { return out_ptr(a, cols, r, s); }, [&]() { if (STAGE_LATE) stage(); });
}

// Multi-pattern mode (rs_reconst_batch_multi): every stripe names a pattern;
// a pattern holds its input / output vector indexes and the offset of its
// prepared LDS table image.  a.ptr / a.sid address ALL d+p vectors of
// stripe 0.  One workgroup = one chunk of one stripe (grid = all chunks).
// The workgroup runs the body built for its own pattern's output count
// (1, 2 or up to MC rows): a uniform branch, so a stripe that lost one vector
// does not pay the VALU work of the batch's widest pattern.
template <int MC, int KB, bool KFIX, int BS, int LQ, int VAR>
__device__ __forceinline__ void multi_chunk(const MatmulArgs& a, const PatternDesc* P, int s, int64_t cb,
                                            uint32_t* lds32) {
    constexpr int COLD = ((MC * 5 + 3) / 4) * 4;
    const lds_u32x4* lds_tab = (const lds_u32x4*)(lds32);
    const int cols = KFIX ? KB : a.cols;
    const int ncols_pad = KFIX ? KB : ((cols + KB - 1) / KB) * KB;
    const uint32_t* img = a.tables + P->tab_off;
    // image columns are CW dwords (4 or 8 rows x 5, a.rows = the batch's most
    // outputs); keep the first COLD of each
    const int CW = multi_image_rows(a.rows) * 5;
    auto stage = [&]() {
        if (COLD == CW) {  // the image is the LDS layout
            for (int idx = threadIdx.x; idx < ncols_pad * COLD; idx += BS) lds32[idx] = img[idx];
        } else {
            for (int idx = threadIdx.x; idx < ncols_pad * COLD; idx += BS) {
                const int c = idx / COLD;
                lds32[idx] = img[c * CW + (idx - c * COLD)];
            }
        }
        __syncthreads();
    };
    stage();
    auto base = [&](uint32_t v) {
        return reinterpret_cast<g_u8*>(a.ptr[v]) + static_cast<int64_t>(s) * a.ss[a.sid[v] & 3];
    };
    chunk_body<KB, KFIX, MC, false, 1, VAR, kAuxNt, kAuxNt, 0, LQ, BS>(
        a, lds_tab, cols, ncols_pad, static_cast<int>(P->nout), cb, a.body / (4 * LQ),
        [&](int c) { return const_cast<const g_u8*>(base(P->in_idx[c])); },
        [&](int r) { return base(P->out_idx[r]); });
}

template <int KB, bool KFIX, int MC, int BS, int LQ, int VAR = kVarDefault>
__global__ __launch_bounds__(BS) void gf_matmul_multi(const MatmulArgs a, const PatternDesc* __restrict__ pats,
                                                          const int32_t* __restrict__ stripe_pat) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
    const uint32_t chunk = blockIdx.x;
    const uint32_t cps = static_cast<uint32_t>(a.chunks_per_stripe);
    const uint32_t su = a.cps_shift >= 0 ? (chunk >> a.cps_shift) : chunk / cps;
    const int s = static_cast<int>(su);
    const int64_t cb = static_cast<int64_t>(chunk - su * cps);
    const int pid = stripe_pat[s];
    if (pid < 0) return;  // stripe not in the batch's work (uniform: whole workgroup)
    const PatternDesc* P = pats + pid;
    const uint32_t nout = P->nout;
    if constexpr (MC > 4) {
        if (nout > 4) return multi_chunk<MC, KB, KFIX, BS, LQ, VAR>(a, P, s, cb, lds32);
    }
    if constexpr (MC > 2) {
        if (nout > 2) return multi_chunk<4, KB, KFIX, BS, LQ, VAR>(a, P, s, cb, lds32);
    }
    if constexpr (MC > 1) {
        if (nout == 2) return multi_chunk<2, KB, KFIX, BS, LQ, VAR>(a, P, s, cb, lds32);
    }
    multi_chunk<1, KB, KFIX, BS, LQ, VAR>(a, P, s, cb, lds32);
}

// ---------------------------------------------------------------------------
// Wide products: more than 8 output rows (Encode of wide codes such as 64+64
// or 200+56, Reconst of 9-128 lost vectors, Update / Replace of wide codes)
// over a run-time matrix, in ONE pass: every input byte is read from HBM once
// whatever the row count (the looped kernel re-reads every input once per
// 8-row group).
//
// A workgroup is NW waves over the same 1 KiB of every vector (lane t owns
// bytes [16t, 16t+16) of the chunk in each); wave w computes up to 16 rows,
// [row0 + 16w, row0 + 16w + 16).  With NW > 1 the waves of a workgroup load
// the same input lines (cached loads: the first fetch goes to HBM, the others
// hit the CU's L1 / the XCD's L2), so HBM still moves each input once.  The
// accumulators of the wave's rows stay in VGPRs (16 B per row and lane).
//
// Coefficient tables come from the `wide` image ([column pair][rows_pad][12]
// dwords, get_tables) through scalar loads: the matrix is the same for every
// lane.  v_perm_b32 may read one SGPR (gfx9 constant-bus limit), so of each
// column's perm pool (T0, T1) / (T2, T3) the dwords T0 and T2 come into VGPRs
// with one v_mov_b64 per (row, column) and T1 / T3 / T4 stay scalar.
// Columns are taken in pairs so the three partial products of two columns
// fold into three xor3 per dword (4.5 VALU per (row, column, dword) without a
// carried term), and the next pair's loads are in flight while this pair is
// computed.  An odd last column is paired with itself against zero tables.
// A wave's rows are computed in groups of 4 whose tables are read together
// (one scalar-load wait per group); the body is specialised for the wave's
// group count, so rows past the matrix cost at most 3 rows of zero tables.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(4))) const uint32_t c_u32;  // constant address space: scalar loads
typedef __attribute__((address_space(4))) const uint64_t c_u64;

template <int R, int LAUX, bool ACC>
__device__ __forceinline__ void wide_body(const MatmulArgs& a, int s, int r0, int nr, uint32_t off) {
    const uint32_t nbytes = static_cast<uint32_t>(a.body);
    const int cols = a.cols;
    uint32_t acc[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (ACC && r < nr) {
            const u32x4 o = load16<0, 4>(out_ptr(a, cols, r0 + r, s), off, nbytes, false);
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] = o[q];
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] = 0;
        }
    }
    auto load_col = [&](int c) { return load16<LAUX, 4>(in_ptr(a, c, s), off, nbytes, false); };
    const int npairs = (cols + 1) >> 1;
    u32x4 xa = load_col(0), xb = load_col(cols > 1 ? 1 : 0);
    c_u32* tab = reinterpret_cast<c_u32*>(reinterpret_cast<uint64_t>(a.wide)) + static_cast<size_t>(r0) * 12;
    for (int p = 0; p < npairs; ++p) {
        // next pair's loads first: in flight while this pair is computed
        const int cn = 2 * p + 2;
        u32x4 na = xa, nb = xb;
        if (cn < cols) {
            na = load_col(cn);
            nb = load_col(cn + 1 < cols ? cn + 1 : cn);
        }
        // bit groups {0-2}, {3-5}, {6-7} of both columns, shared by every row
        uint32_t g[2][3][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const u32x4 x = h ? xb : xa;
#pragma unroll
            for (int q = 0; q < 4; q += 2) {
                const uint64_t X = (static_cast<uint64_t>(x[q + 1]) << 32) | x[q];
                uint64_t Y3, Y6;
                asm("v_lshrrev_b64 %0, 3, %1" : "=v"(Y3) : "v"(X));
                asm("v_lshrrev_b64 %0, 6, %1" : "=v"(Y6) : "v"(X));
                g[h][0][q] = x[q] & 0x07070707u;
                g[h][0][q + 1] = x[q + 1] & 0x07070707u;
                g[h][1][q] = static_cast<uint32_t>(Y3) & 0x07070707u;
                g[h][1][q + 1] = static_cast<uint32_t>(Y3 >> 32) & 0x07070707u;
                g[h][2][q] = static_cast<uint32_t>(Y6) & 0x03030303u;
                g[h][2][q + 1] = static_cast<uint32_t>(Y6 >> 32) & 0x03030303u;
            }
        }
        c_u32* tp = tab + static_cast<size_t>(p) * a.rows_pad * 12;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            c_u32* t = tp + r * 12;
            const uint64_t sa = *reinterpret_cast<c_u64*>(t), sb = *reinterpret_cast<c_u64*>(t + 2);
            uint64_t va, vb;  // (T0, T2) of columns a / b into VGPRs: v_perm reads one SGPR
            asm("v_mov_b64 %0, %1" : "=v"(va) : "s"(sa));
            asm("v_mov_b64 %0, %1" : "=v"(vb) : "s"(sb));
            const uint32_t t0a = static_cast<uint32_t>(va), t2a = static_cast<uint32_t>(va >> 32);
            const uint32_t t0b = static_cast<uint32_t>(vb), t2b = static_cast<uint32_t>(vb >> 32);
            const uint32_t t1a = t[4], t3a = t[5], t1b = t[6], t3b = t[7], t4a = t[8], t4b = t[9];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t p0a = __builtin_amdgcn_perm(t1a, t0a, g[0][0][q]);
                const uint32_t p1a = __builtin_amdgcn_perm(t3a, t2a, g[0][1][q]);
                const uint32_t p2a = __builtin_amdgcn_perm(t4a, t4a, g[0][2][q]);
                const uint32_t p0b = __builtin_amdgcn_perm(t1b, t0b, g[1][0][q]);
                const uint32_t p1b = __builtin_amdgcn_perm(t3b, t2b, g[1][1][q]);
                const uint32_t p2b = __builtin_amdgcn_perm(t4b, t4b, g[1][2][q]);
                acc[r][q] = xor3(xor3(xor3(acc[r][q], p0a, p1a), p2a, p0b), p1b, p2b);
            }
            // a scheduling fence per 4-row group: its tables are loaded
            // together, and the next group's loads can issue under its math
            if ((r & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
        // pin the running sums per pair (no re-association across pairs)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) asm volatile("" : "+v"(acc[r][q]));
        xa = na;
        xb = nb;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r < nr) {
            const u32x4 v = {acc[r][0], acc[r][1], acc[r][2], acc[r][3]};
            store16<kAuxNt, 4>(out_ptr(a, cols, r0 + r, s), off, nbytes, v, true);
        }
    }
}

template <int NW, bool ACC>
__global__ __launch_bounds__(64 * NW) void gf_matmul_wide(const MatmulArgs a, int row0) {
    constexpr int kLoadAux = NW > 1 ? 0 : kAuxNt;  // shared lines stay cached; a lone wave streams
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t chunk = blockIdx.x;
    const uint32_t cps = static_cast<uint32_t>(a.chunks_per_stripe);
    const uint32_t su = a.cps_shift >= 0 ? (chunk >> a.cps_shift) : chunk / cps;
    const int s = a.stripe_ids ? a.stripe_ids[su] : static_cast<int>(su);
    const uint32_t cb = chunk - su * cps;
    const int r0 = row0 + wave * kWideRows;
    const int nr = (a.rows - r0) < kWideRows ? (a.rows - r0) : kWideRows;
    if (nr <= 0) return;  // uniform over the wave (no barrier in this kernel)
    const uint32_t off = cb * 1024u + lane * 16u;
    switch ((nr + 3) >> 2) {  // uniform
        case 1: wide_body<4, kLoadAux, ACC>(a, s, r0, nr, off); break;
        case 2: wide_body<8, kLoadAux, ACC>(a, s, r0, nr, off); break;
        case 3: wide_body<12, kLoadAux, ACC>(a, s, r0, nr, off); break;
        default: wide_body<16, kLoadAux, ACC>(a, s, r0, nr, off); break;
    }
}

// ---------------------------------------------------------------------------
// Byte kernel: any alignment, bytes [start, len) of every vector.  One lane
// per (stripe, 4-byte group); tables are read straight from global memory.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void gf_matmul_bytes(const MatmulArgs a, uint64_t start,
                                                          uint64_t groups_per_stripe) {
    const uint64_t gid = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const uint64_t total = groups_per_stripe * static_cast<uint64_t>(a.nstripes);
    if (gid >= total) return;
    const int si = static_cast<int>(gid / groups_per_stripe);
    const uint64_t pos = start + (gid - static_cast<uint64_t>(si) * groups_per_stripe) * 4;
    const int s = a.stripe_ids ? a.stripe_ids[si] : si;
    const int nb = (a.len - pos) < 4 ? static_cast<int>(a.len - pos) : 4;

    for (int r = 0; r < a.rows; ++r) {
        uint32_t acc = 0;
        g_u8* o = out_ptr(a, a.cols, r, s) + pos;
        if (a.accumulate)
            for (int q = 0; q < nb; ++q) acc |= static_cast<uint32_t>(o[q]) << (8 * q);
        for (int c = 0; c < a.cols; ++c) {
            const g_u8* p = in_ptr(a, c, s) + pos;
            uint32_t x = 0;
            for (int q = 0; q < nb; ++q) x |= static_cast<uint32_t>(p[q]) << (8 * q);
            uint32_t g0, g1, g2;
            split_groups(x, g0, g1, g2);
            uint32_t t[5];
            const uint32_t* tg = a.tables + (static_cast<int64_t>(c) * a.rows_pad + r) * 5;
            for (int e = 0; e < 5; ++e) t[e] = tg[e];
            acc ^= gf_mul_packed(g0, g1, g2, t);
        }
        for (int q = 0; q < nb; ++q) o[q] = static_cast<uint8_t>(acc >> (8 * q));
    }
}

// ---------------------------------------------------------------------------
// Bit-sliced Encode for fixed generator matrices with 5-8 parity rows
// (networks generated by tools/gen_bitslice.py into bitslice_gen.inc).  A lane
// owns 32 bytes of every vector; an 8x8 SWAR bit transpose turns each
// column's 8 dwords into 8 bit-planes (plane b = bit b of the 32 bytes), a
// fixed XOR network over the planes gives every parity plane (multiplying by
// a constant is GF(2)-linear), and the same transpose (an involution) turns
// the parity planes back into bytes.  The networks are column-major: each
// column's planes are combined into the XORs of each 4-plane half's subsets,
// and every parity plane takes one subset of each half per column
// (xor3(acc, lo, hi)).  10+8: ~22 VALU per (column, dword) against ~40 on the
// perm-table path, which is VALU-bound above 4 rows; measured 6.12 vs 5.32
// TB/s (10+8), 6.15 vs 5.05 (10+6), 6.34 vs 4.91 (8+5) on the split layout
// (ab_bitslice*.log, ab_bs_block.log; workgroup size per bs_block_for).
// 4-row shapes stay on the perm-table kernels (6.58 vs 6.01 TB/s at 10+4).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void bs_swap(uint32_t& a, uint32_t& b, int s, uint32_t m) {
    const uint32_t t = ((a >> s) ^ b) & m;
    b ^= t;
    a ^= t << s;
}

__device__ __forceinline__ void bs_transpose8(uint32_t (&w)[8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) bs_swap(w[i], w[i + 4], 4, 0x0F0F0F0Fu);
    bs_swap(w[0], w[2], 2, 0x33333333u);
    bs_swap(w[1], w[3], 2, 0x33333333u);
    bs_swap(w[4], w[6], 2, 0x33333333u);
    bs_swap(w[5], w[7], 2, 0x33333333u);
#pragma unroll
    for (int i = 0; i < 8; i += 2) bs_swap(w[i], w[i + 1], 1, 0x55555555u);
}

__device__ __forceinline__ uint32_t bs_x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

template <int D, int P>
struct BsNet;
#include "bitslice_gen.inc"

template <int D, int P, int BS, int Q = 8>
__global__ __launch_bounds__(BS) void gf_bitslice(const MatmulArgs a) {
    // A workgroup covers 32*BS bytes of every vector.  Lane t's 32-byte unit
    // is 32/Q pieces of Q bytes, piece k at Q*t + k*Q*BS of the chunk, so each
    // wave instruction reads / writes 64*Q bytes contiguously (Q = 8: the
    // dwordx2 pattern of the perm-table kernels).  Pieces past `body` read 0
    // and are not written (buffer range checks), so no lane masks.
    static_assert(Q == 8 || Q == 16, "piece size");
    constexpr int NP = 32 / Q;   // pieces per lane unit
    constexpr int DW = Q / 4;    // dwords per piece
    typedef typename LaneWord<DW>::type W;
    const uint32_t chunk = blockIdx.x;
    const uint32_t cps = static_cast<uint32_t>(a.chunks_per_stripe);
    const uint32_t su = a.cps_shift >= 0 ? (chunk >> a.cps_shift) : chunk / cps;
    // grouped launches (multi-pattern Reconst fallback) name their stripes
    const int s = a.stripe_ids ? a.stripe_ids[su] : static_cast<int>(su);
    const uint32_t cb = chunk - su * cps;
    const uint32_t off = cb * (32u * BS) + static_cast<uint32_t>(Q) * threadIdx.x;
    const uint32_t nbytes = static_cast<uint32_t>(a.body);
    auto fetch = [&](int c, uint32_t (&w)[8]) {  // issue the loads of column c's 32 bytes
        const g_u8* p = in_ptr(a, c, s);
        // the offset passes through a volatile asm, which stays after the
        // previous column's pins: the loads are issued here, a few columns
        // ahead, not all hoisted to the top (VGPRs, occupancy)
        uint32_t o32 = off;
        asm volatile("" : "+v"(o32));
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            const W v = load16<kAuxNt, DW>(p, o32 + static_cast<uint32_t>(k * Q * BS), nbytes, true);
#pragma unroll
            for (int q = 0; q < DW; ++q) w[k * DW + q] = v[q];
        }
    };
    BsNet<D, P>::run(fetch, [&](int r, uint32_t (&o)[8]) {
        bs_transpose8(o);
        g_u8* q = out_ptr(a, D, r, s);
#pragma unroll
        for (int k = 0; k < NP; ++k) {
            W v;
#pragma unroll
            for (int e = 0; e < DW; ++e) v[e] = o[k * DW + e];
            store16<kAuxNt, DW>(q, off + static_cast<uint32_t>(k * Q * BS), nbytes, v, true);
        }
    });
}

// The bit-sliced kernel for this launch, or null: Encode (overwrite) of a
// generated shape whose matrix equals the generated one byte for byte.
// `bs` receives the workgroup size: rs_tune("bs_block", 64 | 128 | 256), or
// 0 (default) for the per-layout rule of bs_block_for().
typedef void (*BsKernel)(const MatmulArgs);
static int bs_block_for(const MatmulArgs& a) {
    const int b = tuning().bs_block;
    if (b) return b;
    // Same-process A/B on two boxes (tools/ab_bs_block.sh,
    // profiles/r01/ab_bs_block.log, Encode @ 1 MiB): with parity in a
    // separate region 64 lanes win or tie every shape (10+8 6.12-6.20 vs
    // 5.86-6.14 TB/s at 128, 10+6 6.16-6.28 vs 5.95-6.09, 8+8 6.18-6.29 vs
    // 5.48-5.97 at 256).  With parity inside the data's stripes (interleaved
    // [S][d+p][len]) the best size follows the stripe pitch: 10+8 runs 5.78 at
    // 256 vs 5.28 at 128 and 5.04 at 64, 12+8 5.75 / 5.79 / 5.50, while 10+6,
    // 8+5 and 8+8 are best at 64 (5.90, 6.10, 6.00).
    const int64_t stride = a.ss[a.sid[0] & 3];
    const int64_t gap = static_cast<int64_t>(a.ptr[a.cols] - a.ptr[0]);
    const bool interleaved = a.nstripes > 1 && a.ss[a.sid[a.cols] & 3] == stride && gap > 0 && gap < stride;
    return interleaved && a.cols + a.rows >= 18 ? 256 : 64;
}
static BsKernel bs_kernel_for(const MatmulArgs& a, int* bs) {
    const LaunchTuning& tu = tuning();
    if (!tu.bitslice || a.accumulate || !a.host_mat) return nullptr;
    *bs = bs_block_for(a);
    for (const BsShape& sh : kBsShapes)
        if (sh.d == a.cols && sh.p == a.rows &&
            std::memcmp(sh.gen, a.host_mat, static_cast<size_t>(sh.d) * sh.p) == 0) {
#define RSAMD_BS_CASE(D, P)                                                              \
    if (sh.d == D && sh.p == P)                                                          \
        return *bs == 64 ? gf_bitslice<D, P, 64, 8> : *bs == 256 ? gf_bitslice<D, P, 256, 8> \
                                                                 : gf_bitslice<D, P, 128, 8>;
            RSAMD_BS_SHAPES(RSAMD_BS_CASE)
#undef RSAMD_BS_CASE
        }
    return nullptr;
}

// ---------------------------------------------------------------------------
// Host-call engine (engine.cpp): one resident kernel serves the small
// synchronous host calls.  Each workgroup (one wave) polls the doorbell line
// of the ring in host memory; a new value in both seq words (written last by
// the host) means the line's fields are the new call's.  The workgroup then
// computes its share of the units straight out of / into the caller's pinned
// staging buffer over PCIe, and reports the doorbell value in its done word.
// Exit conditions every wave reaches: the stop word, or `idle_ticks` of the
// 100 MHz realtime counter without a doorbell.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t sys_load64(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, int lane) {
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), lane);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), lane);
    return (static_cast<uint64_t>(hi) << 32) | lo;
}
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {  // every lane holds the same value
    const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
    const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

constexpr int kEngineColBatch = 16;  // column loads in flight per lane (one PCIe round trip per batch)
// slot headers read ahead by each poll (8 words each: one 64-lane load)
constexpr int kEngineLook = kEngineSlots - 1 < 7 ? kEngineSlots - 1 : 7;

struct EngineCall {
    const uint64_t* vaddr;  // LDS: device address of vector i of stripe 0
    uint64_t stride;
    uint32_t units, total;
    int cols;
    bool accumulate;
    uint32_t local, nwg;    // this workgroup's index among the call's nwg workgroups
};

// This workgroup's units of one call: 16 bytes of every vector of one stripe
// per lane and unit, all column loads of a batch in flight together (host
// memory: one PCIe round trip per batch), ROWS output rows.
template <int ROWS>
__device__ __forceinline__ void engine_units(const EngineCall& e, const uint32_t* tab) {
    typedef __attribute__((address_space(1))) u32x4 gq;
    // lanes enumerated wave-major: a call of up to nwg * 64 units runs on
    // the first wave of each of its workgroups, larger ones spread over them all
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t step = e.nwg * blockDim.x;
    for (uint32_t u = (wave * e.nwg + e.local) * 64u + lane; u < e.total; u += step) {
        const uint32_t si = u / e.units, k = u - si * e.units;
        const uint64_t sb = static_cast<uint64_t>(si) * e.stride + static_cast<uint64_t>(k) * 16;
        u32x4 acc[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r)
            acc[r] = e.accumulate ? __builtin_nontemporal_load(reinterpret_cast<const gq*>(e.vaddr[e.cols + r] + sb))
                                  : u32x4{0, 0, 0, 0};
        for (int c0 = 0; c0 < e.cols; c0 += kEngineColBatch) {
            const int nb = (e.cols - c0) < kEngineColBatch ? (e.cols - c0) : kEngineColBatch;
            u32x4 x[kEngineColBatch];
#pragma unroll
            for (int b = 0; b < kEngineColBatch; ++b)
                if (b < nb) x[b] = __builtin_nontemporal_load(reinterpret_cast<const gq*>(e.vaddr[c0 + b] + sb));
#pragma unroll
            for (int b = 0; b < kEngineColBatch; ++b) {
                if (b < nb) {
                    __builtin_amdgcn_sched_barrier(0);
                    uint32_t t[ROWS * 5];
#pragma unroll
                    for (int i = 0; i < ROWS * 5; ++i) t[i] = tab[((c0 + b) * kEngineMaxRows) * 5 + i];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        uint32_t g0, g1, g2;
                        split_groups(x[b][q], g0, g1, g2);
#pragma unroll
                        for (int r = 0; r < ROWS; ++r) acc[r][q] ^= gf_mul_packed(g0, g1, g2, &t[r * 5]);
                    }
#pragma unroll
                    for (int r = 0; r < ROWS; ++r) asm volatile("" : "+v"(acc[r]));
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int r = 0; r < ROWS; ++r)
            __builtin_nontemporal_store(acc[r], reinterpret_cast<gq*>(e.vaddr[e.cols + r] + sb));
    }
}

// A lone call's rows spread over the waves of each workgroup: wave `row`
// computes that one row over the workgroup's units (every wave loads the same
// input lines; one row is ~1/ROWS of the VALU work, which bounds a lone call
// at one wave per workgroup: ~720 dependent VALU for 10 x 4 at ~4-5 cycles).
__device__ __forceinline__ void engine_units_row(const EngineCall& e, const uint32_t* tab, int row) {
    typedef __attribute__((address_space(1))) u32x4 gq;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t step = e.nwg * 64u;
    for (uint32_t u = e.local * 64u + lane; u < e.total; u += step) {
        const uint32_t si = u / e.units, k = u - si * e.units;
        const uint64_t sb = static_cast<uint64_t>(si) * e.stride + static_cast<uint64_t>(k) * 16;
        u32x4 acc = e.accumulate ? __builtin_nontemporal_load(reinterpret_cast<const gq*>(e.vaddr[e.cols + row] + sb))
                                 : u32x4{0, 0, 0, 0};
        for (int c0 = 0; c0 < e.cols; c0 += kEngineColBatch) {
            const int nb = (e.cols - c0) < kEngineColBatch ? (e.cols - c0) : kEngineColBatch;
            u32x4 x[kEngineColBatch];
#pragma unroll
            for (int b = 0; b < kEngineColBatch; ++b)
                if (b < nb) x[b] = __builtin_nontemporal_load(reinterpret_cast<const gq*>(e.vaddr[c0 + b] + sb));
#pragma unroll
            for (int b = 0; b < kEngineColBatch; ++b) {
                if (b < nb) {
                    uint32_t t[5];
#pragma unroll
                    for (int i = 0; i < 5; ++i) t[i] = tab[((c0 + b) * kEngineMaxRows + row) * 5 + i];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        uint32_t g0, g1, g2;
                        split_groups(x[b][q], g0, g1, g2);
                        acc[q] ^= gf_mul_packed(g0, g1, g2, t);
                    }
                }
            }
        }
        __builtin_nontemporal_store(acc, reinterpret_cast<gq*>(e.vaddr[e.cols + row] + sb));
    }
}

// A lone call's rows over the waves of each workgroup with the inputs read
// once (host_engine_split_rows 2): wave w loads columns w, w + nw, ... of the
// workgroup's 64 units into LDS (the loads of all waves in flight together),
// and after a barrier wave r < rows combines every column from LDS into row r.
// The row-per-wave variant above read every input over PCIe once per wave.
constexpr int kEngineShareCols = 8;  // columns per wave (nw >= 4 for 32 columns)
__device__ __forceinline__ void engine_units_shared(const EngineCall& e, const uint32_t* tab, int rows,
                                                    u32x4 (*sh)[64]) {
    typedef __attribute__((address_space(1))) u32x4 gq;
    const int wave = static_cast<int>(threadIdx.x >> 6), lane = static_cast<int>(threadIdx.x & 63);
    const int nw = static_cast<int>(blockDim.x >> 6);
    for (uint32_t u0 = e.local * 64u; u0 < e.total; u0 += e.nwg * 64u) {  // (uniform over the workgroup)
        const uint32_t u = u0 + static_cast<uint32_t>(lane);
        const bool valid = u < e.total;
        const uint32_t si = valid ? u / e.units : 0, k = valid ? u - si * e.units : 0;
        const uint64_t sb = static_cast<uint64_t>(si) * e.stride + static_cast<uint64_t>(k) * 16;
        u32x4 x[kEngineShareCols];
#pragma unroll
        for (int j = 0; j < kEngineShareCols; ++j) {
            const int c = wave + j * nw;
            if (c < e.cols)
                x[j] = valid ? __builtin_nontemporal_load(reinterpret_cast<const gq*>(e.vaddr[c] + sb)) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int j = 0; j < kEngineShareCols; ++j) {
            const int c = wave + j * nw;
            if (c < e.cols) sh[c][lane] = x[j];
        }
        __syncthreads();
        if (wave < rows) {
            u32x4 acc = e.accumulate && valid
                            ? __builtin_nontemporal_load(reinterpret_cast<const gq*>(e.vaddr[e.cols + wave] + sb))
                            : u32x4{0, 0, 0, 0};
            for (int c = 0; c < e.cols; ++c) {
                const u32x4 v = sh[c][lane];
                uint32_t t[5];
#pragma unroll
                for (int i = 0; i < 5; ++i) t[i] = tab[(c * kEngineMaxRows + wave) * 5 + i];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t g0, g1, g2;
                    split_groups(v[q], g0, g1, g2);
                    acc[q] ^= gf_mul_packed(g0, g1, g2, t);
                }
            }
            if (valid) __builtin_nontemporal_store(acc, reinterpret_cast<gq*>(e.vaddr[e.cols + wave] + sb));
        }
        __syncthreads();  // (the next group's loads overwrite sh)
    }
}

__global__ __launch_bounds__(512) void gf_engine(EngineRing* ring, const EngineSlot* vslots, uint64_t start,
                                                 uint64_t epoch, uint64_t idle_ticks, uint64_t life_ticks,
                                                 uint32_t poll_gap) {
    // the call slots: in device memory the host writes through the BAR
    // (vslots: polls and table loads stay in local HBM) or in the ring
    const EngineSlot* const slots = vslots ? vslots : ring->slot;
    constexpr int kPollWords = 8 * (1 + kEnginePtrLines);  // a slot's header + address lines
    __shared__ __attribute__((aligned(16))) uint32_t tab[kEngineMaxCols * kEngineMaxRows * 5];
    __shared__ uint64_t s_raw[kPollWords];  // the lines wave 0 saw (s_raw[0] = 0: leave)
    __shared__ uint64_t s_vaddr[kEngineMaxCols + kEngineMaxRows];
    __shared__ u32x4 s_in[kEngineMaxCols][64];  // host_engine_split_rows 2: a group's inputs
    const int lane = threadIdx.x & 63;
    const bool poller = threadIdx.x < 64;  // wave 0 polls and signals; the others wait at the barrier
    // a relaunch resumes after the last call this workgroup completed
    uint64_t last = uniform_u64(sys_load64(&ring->done[blockIdx.x]));
    last = last > start ? last : start;
    // bounded lifetime: a device-wide synchronisation (hipDeviceSynchronize,
    // hipFree, torch.cuda.synchronize) waits for a running instance, so no
    // instance outlives life_ticks even while calls keep arriving; the host
    // sees the gone word and relaunches on the next call
    const uint64_t t_birth = __builtin_amdgcn_s_memrealtime();
    uint32_t tab_have = 0xffffffffu;
    for (;;) {
        uint64_t t_seen = 0;
        const EngineSlot* slot = &slots[(last + 1) % kEngineSlots];
        if (poller) {
            const uint64_t* lines = reinterpret_cast<const uint64_t*>(slot);
            uint64_t w = 0, seq = 0;
            uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            auto issue = [&]() -> uint64_t { return lane < kPollWords ? sys_load64(&lines[lane]) : 0; };
            // does the call whose header word 5 is w5 name this workgroup?
            auto concerns = [&](uint64_t w5) {
                const uint32_t g0 = static_cast<uint32_t>(w5 >> 8) & 0xff, ng = static_cast<uint32_t>(w5 >> 16) & 0xff;
                return (blockIdx.x + gridDim.x - g0) % gridDim.x < ng;
            };
            // the call number if the read shows call `want` complete, else 0
            auto probe_at = [&](uint64_t x, uint64_t want) -> uint64_t {
                const uint64_t s0 = lane_u64(x, 0), s1 = lane_u64(x, 7);
                if (s0 != s1 || s0 != want) return 0;
                // address mode: the lines holding this call's addresses carry its tag
                const uint64_t w4 = lane_u64(x, 4), w5 = lane_u64(x, 5);
                const int nv = static_cast<int>((w4 >> 32) & 0xffff) + static_cast<int>(w4 >> 48);
                bool tagged = true;
                if (w5 & 8)
                    for (int l = 1; l <= (nv + 6) / 7 && l <= kEnginePtrLines; ++l)
                        tagged = tagged && lane_u64(x, 8 * l + 7) == s0;
                return tagged ? s0 : 0;
            };
            auto probe = [&](uint64_t x) -> uint64_t { return probe_at(x, last + 1); };
            // stop word, or no call for idle_ticks: seq stays 0 and every wave leaves
            auto leave = [&](uint64_t x, uint32_t n) {
                if (lane_u64(x, 6) >= epoch) return true;
                if ((n & 31) != 0) return false;
                const uint64_t now = __builtin_amdgcn_s_memrealtime();
                return now - t0 > idle_ticks || now - t_birth > life_ticks;
            };
            if (poll_gap == 0) {  // one read per round trip
                // With the slot's lines the same round trip brings the headers
                // of the next kEngineLook slots: rung calls that name other
                // workgroups are passed without another read (each used to cost
                // this workgroup a PCIe round trip, which bounded concurrent
                // callers' throughput), and the done word records them.
                uint64_t cur = last + 1;
                for (uint32_t n = 1;; ++n) {
                    const uint64_t* ln = reinterpret_cast<const uint64_t*>(&slots[cur % kEngineSlots]);
                    const uint64_t* nh = reinterpret_cast<const uint64_t*>(&slots[(cur + 1 + lane / 8) % kEngineSlots]);
                    w = lane < kPollWords ? sys_load64(&ln[lane]) : 0;
                    const uint64_t hn = lane < 8 * kEngineLook ? sys_load64(&nh[lane % 8]) : 0;
                    if ((seq = probe_at(w, cur)) == 0) {
                        if (leave(w, n)) break;
                        __builtin_amdgcn_s_sleep(2);
                        continue;
                    }
                    if (concerns(lane_u64(w, 5))) break;  // call cur is this workgroup's: w holds its lines
                    uint64_t passed = cur;
#pragma unroll
                    for (int k = 0; k < kEngineLook; ++k) {
                        const uint64_t s0 = lane_u64(hn, 8 * k), s1 = lane_u64(hn, 8 * k + 7);
                        if (s0 != s1 || s0 != passed + 1 || lane_u64(hn, 8 * k + 6) >= epoch ||
                            concerns(lane_u64(hn, 8 * k + 5)))
                            break;
                        ++passed;
                    }
                    if (lane == 0)
                        __hip_atomic_store(&ring->done[blockIdx.x], passed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    cur = passed + 1;
                    seq = 0;
                    n = 0;  // (progress: the idle window starts again)
                    t0 = __builtin_amdgcn_s_memrealtime();
                }
            } else {  // two reads in flight, poll_gap ticks apart; the older is checked first
                uint64_t wa = issue();
                while (__builtin_amdgcn_s_memrealtime() - t0 < poll_gap) __builtin_amdgcn_s_sleep(1);
                uint64_t wb = issue();
                for (uint32_t n = 1;; ++n) {
                    if ((seq = probe(wa)) != 0 || leave(wa, n)) {
                        w = wa;
                        break;
                    }
                    wa = issue();
                    if ((seq = probe(wb)) != 0 || leave(wb, n)) {
                        w = wb;
                        break;
                    }
                    wb = issue();
                }
            }
            t_seen = __builtin_amdgcn_s_memrealtime();
            if (lane < kPollWords) s_raw[lane] = lane == 0 ? seq : w;
            if (seq == 0 && lane == 0)  // (release: after this workgroup's last done word)
                __hip_atomic_store(&ring->gone[blockIdx.x], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        const uint64_t seq = s_raw[0];
        if (seq == 0) return;  // uniform over the workgroup (doorbell values start at 1)
        slot = &slots[seq % kEngineSlots];  // (the poller may have passed calls that name other workgroups)
        const uint64_t base = s_raw[1], stride = s_raw[2];
        const uint64_t w3 = s_raw[3], w4 = s_raw[4], w5 = s_raw[5];
        const uint32_t pitch = static_cast<uint32_t>(w3), units = static_cast<uint32_t>(w3 >> 32);
        const uint32_t nstripes = static_cast<uint32_t>(w4);
        const int rows = static_cast<int>((w4 >> 32) & 0xffff), cols = static_cast<int>(w4 >> 48);
        const bool accumulate = (w5 & 1) != 0;
        const bool coherent = (w5 & 2) != 0;  // fine-grained buffer: stores need no L2 write-back
        const bool addressed = (w5 & 8) != 0;
        // the call's workgroups: nwg of them from wg0 on (wrapping); the others only pass it
        const uint32_t wg0 = static_cast<uint32_t>(w5 >> 8) & 0xff, nwg = static_cast<uint32_t>(w5 >> 16) & 0xff;
        const uint32_t local = (blockIdx.x + gridDim.x - wg0) % gridDim.x;
        const bool works = local < nwg;
        const bool stamps = (w5 & 4) != 0 && local == 0;
        if (works && static_cast<int>(threadIdx.x) < rows + cols) {
            const int i = threadIdx.x;
            s_vaddr[i] = addressed ? s_raw[8 * (1 + i / 7) + i % 7] : base + static_cast<uint64_t>(i) * pitch;
        }
        // system-scope acquire, always: without it the first call on a fresh
        // coherent block read zeros (lines the runtime's clear left in L2).
        // The polling wave's covers its own table loads; the other waves that
        // load call data acquire after the barrier below
        if (works && poller) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const uint32_t tab_id = static_cast<uint32_t>(w5 >> 32);
        if (works && tab_id != tab_have) {  // [col][kEngineMaxRows][5] dwords, every load in flight at once (one PCIe trip)
            if (poller) {
                constexpr int kTabPerLane = kEngineMaxCols * kEngineMaxRows * 5 / 64;
                const int n = cols * kEngineMaxRows * 5;
                uint32_t t[kTabPerLane];
#pragma unroll
                for (int k = 0; k < kTabPerLane; ++k)
                    if (lane + 64 * k < n) t[k] = __builtin_nontemporal_load(&slot->tables[lane + 64 * k]);
#pragma unroll
                for (int k = 0; k < kTabPerLane; ++k)
                    if (lane + 64 * k < n) tab[lane + 64 * k] = t[k];
            }
            tab_have = tab_id;
        }
        __syncthreads();  // tables and addresses ready; s_raw read by every wave
        // Every other wave that loads this call's data acquires too.  The
        // polling wave's invalidate already covers its workgroup's caches on
        // this build (no threadgroup-split mode: a workgroup's waves share the
        // CU's L1 and the XCD's L2), but the memory model does not promise
        // that, and a lone call (the latency case) loads on the first wave
        // only, so only overlapping calls pay for it.  With shared rows a wave
        // loads an input column (wave < cols) and, for XOR-accumulate calls,
        // the old output of its own row (wave < rows).
        const int nwaves = static_cast<int>(blockDim.x >> 6), my_wave = static_cast<int>(threadIdx.x >> 6);
        const bool split_rows = (w5 & 16) != 0 && rows <= nwaves;
        const bool shared_rows = (w5 & 32) != 0 && rows <= nwaves && nwaves * kEngineShareCols >= cols;
        if (works && !poller &&
            ((shared_rows && (my_wave < cols || (accumulate && my_wave < rows))) || (split_rows && my_wave < rows) ||
             ((threadIdx.x >> 6) * nwg + local) * 64u < nstripes * units))
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const uint64_t t_tab = __builtin_amdgcn_s_memrealtime();
        const EngineCall call{s_vaddr, stride, units, works ? nstripes * units : 0u, cols, accumulate, local, nwg};
        if (works && shared_rows) {
            engine_units_shared(call, tab, rows, s_in);
        } else if (works && split_rows) {
            const int wave = static_cast<int>(threadIdx.x >> 6);
            if (wave < rows) engine_units_row(call, tab, wave);
        } else if (works) switch (rows) {
            case 1: engine_units<1>(call, tab); break;
            case 2: engine_units<2>(call, tab); break;
            case 3: engine_units<3>(call, tab); break;
            case 4: engine_units<4>(call, tab); break;
            case 5: engine_units<5>(call, tab); break;
            case 6: engine_units<6>(call, tab); break;
            case 7: engine_units<7>(call, tab); break;
            default: engine_units<8>(call, tab); break;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store of this wave acknowledged
        __syncthreads();                                   // ... and of every wave
        if (poller) {
            const uint64_t t_stored = __builtin_amdgcn_s_memrealtime();
            if (works && !coherent) {  // write back the L2 (every wave's stores are in it)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            if (lane == 0) __hip_atomic_store(&ring->done[blockIdx.x], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (stamps && lane < 5) {  // after the done word: diagnostics never delay the call
                const uint64_t t_rel = __builtin_amdgcn_s_memrealtime();
                const uint64_t v =
                    lane == 0 ? t_seen : lane == 1 ? t_tab : lane == 2 ? t_stored : lane == 3 ? t_rel : seq;
                __hip_atomic_store(&ring->stamp[lane], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        last = seq;
    }
}

hipError_t launch_engine(EngineRing* ring_dev, const EngineSlot* vslots, int groups, int waves_per_group,
                         uint64_t start, uint64_t epoch, uint64_t idle_ticks, uint64_t life_ticks,
                         uint32_t poll_gap_ticks, hipStream_t stream) {
    if (groups < 1 || groups > kEngineMaxGroups || waves_per_group < 1 || waves_per_group > kEngineMaxGroupWaves)
        return hipErrorInvalidValue;
    (void)hipGetLastError();
    hipLaunchKernelGGL(gf_engine, dim3(groups), dim3(64 * waves_per_group), 0, stream, ring_dev, vslots, start, epoch,
                       idle_ticks, life_ticks, poll_gap_ticks);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Host-side dispatch.
// ---------------------------------------------------------------------------
using VecKernel = void (*)(const MatmulArgs);

struct Variant {
    VecKernel fn;
    int kb, mc, vpt;
    bool kfix;
    const char* name;
    bool one_chunk = false;  // gf_matmul_vec1: needs grid == total chunks and rows <= mc
    int lq = 4;              // dwords per lane unit (4: 16-byte units, 2: 8-byte units)
    int bs = kBlock;         // lanes per workgroup
};

#define RSAMD_VARIANT(KB, KFIX, MC, ACC, VPT) \
    Variant { gf_matmul_vec<KB, KFIX, MC, ACC, VPT>, KB, MC, VPT, KFIX, \
              "gf_matmul_vec<" #KB "," #KFIX "," #MC "," #ACC "," #VPT ">" }
#define RSAMD_VARIANT_V(KB, KFIX, MC, ACC, VPT, VAR) \
    Variant { gf_matmul_vec<KB, KFIX, MC, ACC, VPT, VAR>, KB, MC, VPT, KFIX, \
              "gf_matmul_vec<" #KB "," #KFIX "," #MC "," #ACC "," #VPT "," #VAR ">" }
#define RSAMD_VARIANT_G(KB, KFIX, MC, ACC) \
    Variant { gf_matmul_vec<KB, KFIX, MC, ACC, 1, kVarDefault, -1, -1>, KB, MC, 1, KFIX, \
              "gf_matmul_vec<" #KB "," #KFIX "," #MC "," #ACC ",1,global>" }
// Specialised encode kernels: rolling 5-column load window (73 VGPRs, 6 waves/SIMD).
#define RSAMD_VARIANT_W5(K) \
    Variant { gf_matmul_vec<K, true, 4, false, 1, kVarDefault, kAuxNt, kAuxNt, 5>, K, 4, 1, true, \
              "gf_matmul_vec<" #K ",true,4,false,1,win5>" }
#define RSAMD_VARIANT_WIN(W) \
    Variant { gf_matmul_vec<10, true, 4, false, 1, kVarDefault, kAuxNt, kAuxNt, W>, 10, 4, 1, true, \
              "gf_matmul_vec<10,true,4,false,1,win" #W ">" }
#define RSAMD_VARIANT_AUX(VAR, LAUX, SAUX) \
    Variant { gf_matmul_vec<10, true, 4, false, 1, VAR, LAUX, SAUX>, 10, 4, 1, true, \
              "gf_matmul_vec<10,true,4,false,1," #VAR "," #LAUX "," #SAUX ">" }

// Experimental code shapes of the 10+4 encode kernel (RSAMD_VAR=<flags> /
// rs_tune("var")), used by tools/ab.py and tools/sweep.sh to A/B variants.
// Compiled only into the experiments build (librsamd_exp.so,
// -DRSAMD_EXPERIMENTS): some of them are XOR-only diagnostics whose output is
// not the GF product, so the product library has no switch that reaches them.
#ifndef RSAMD_EXPERIMENTS
static bool pick_experimental(int, int, bool, int, Variant*) { return false; }
static int exp_var() { return -1; }
#else
static int exp_var() { return tuning().var; }
static bool pick_experimental(int rows, int cols, bool acc, int vpt, Variant* out) {
    const int var = tuning().var;
    if (var < 0 || acc || cols != 10 || rows <= 2 || rows > 4) return false;
#define RSAMD_CASE(V)                                                                                  \
    case V:                                                                                           \
        *out = vpt == 2 ? RSAMD_VARIANT_V(10, true, 4, false, 2, V) : RSAMD_VARIANT_V(10, true, 4, false, 1, V); \
        return true;
    // var >= 100: buffer-instruction cache-policy experiments (body < 2 GiB)
    switch (var) {
        case 100: *out = RSAMD_VARIANT_AUX(12, 2, 2); return true;     // nt / nt
        case 101: *out = RSAMD_VARIANT_AUX(12, 18, 2); return true;    // nt sc1 / nt
        case 102: *out = RSAMD_VARIANT_AUX(12, 3, 2); return true;     // sc0 nt / nt
        case 103: *out = RSAMD_VARIANT_AUX(12, 2, 3); return true;     // nt / sc0 nt
        case 104: *out = RSAMD_VARIANT_AUX(12, 2, 18); return true;    // nt / sc1 nt
        case 105: *out = RSAMD_VARIANT_AUX(12, 2, 0); return true;     // nt / default
        case 106: *out = RSAMD_VARIANT_AUX(12, 19, 19); return true;   // sc0 sc1 nt both
        case 107: *out = RSAMD_VARIANT_AUX(12, 16, 2); return true;    // sc1 / nt
        case 108: *out = RSAMD_VARIANT_AUX(14, -1, -1); return true;   // global nt loads / global nt stores
        case 109: *out = RSAMD_VARIANT_AUX(8, 2, 2); return true;      // buffer nt, double-buffered tables
        case 110: *out = RSAMD_VARIANT_AUX(13, 2, 2); return true;     // DIAGNOSTIC xor-only, buffer nt
        case 123: *out = RSAMD_VARIANT_WIN(3); return true;
        case 124: *out = RSAMD_VARIANT_WIN(4); return true;
        case 125: *out = RSAMD_VARIANT_WIN(5); return true;
        case 126: *out = RSAMD_VARIANT_WIN(6); return true;
        case 128: *out = RSAMD_VARIANT_WIN(8); return true;
        case 130: *out = Variant{gf_matmul_vec1<10, true, 4, false, 5>, 10, 4, 1, true, "vec1<10,w5>", true}; return true;
        case 131: *out = Variant{gf_matmul_vec1<10, true, 4, false, 3>, 10, 4, 1, true, "vec1<10,w3>", true}; return true;
        case 132: *out = Variant{gf_matmul_vec1<10, true, 4, false, 0>, 10, 4, 1, true, "vec1<10,w0>", true}; return true;
        case 133: *out = Variant{gf_matmul_vec1<10, true, 4, false, 4>, 10, 4, 1, true, "vec1<10,w4>", true}; return true;
        // DIAGNOSTIC xor-only one-chunk kernels (the memory ceiling of each lane width)
        case 140: *out = Variant{gf_matmul_vec1<10, true, 4, false, 0, false, 4, 1, kVarDefault | kVarXorOnly>, 10, 4, 1,
                                 true, "vec1<10,16B,xor>", true, 4}; return true;
        case 141: *out = Variant{gf_matmul_vec1<10, true, 4, false, 0, false, 2, 1, kVarDefault | kVarXorOnly>, 10, 4, 1,
                                 true, "vec1<10,8B,xor>", true, 2}; return true;
        case 142: *out = Variant{gf_matmul_vec1<10, true, 4, false, 0, true, 2, 1, kVarDefault | kVarXorOnly>, 10, 4, 1,
                                 true, "vec1<10,8B,late,xor>", true, 2}; return true;
        // without the paired-column XOR accumulation (kVarCarry)
        case 143: *out = Variant{gf_matmul_vec1<10, true, 4, false, 0, false, 2, 1, kVarDefault & ~kVarCarry>, 10, 4, 1,
                                 true, "vec1<10,8B,nocarry>", true, 2}; return true;
        case 144: *out = Variant{gf_matmul_vec1<10, true, 4, false, 0, false, 4, 1, kVarDefault & ~kVarCarry>, 10, 4, 1,
                                 true, "vec1<10,16B,nocarry>", true, 4}; return true;
        // without the 64-bit-shift bit-group split (kVarShift64)
        case 146: *out = Variant{gf_matmul_vec1<10, true, 4, false, 0, false, 4, 1, kVarDefault & ~kVarShift64>, 10, 4,
                                 1, true, "vec1<10,16B,noshift64>", true, 4}; return true;
        case 147: *out = Variant{gf_matmul_vec1<10, true, 4, false, 0, false, 2, 1, kVarDefault & ~kVarShift64>, 10, 4,
                                 1, true, "vec1<10,8B,noshift64>", true, 2}; return true;
        // workgroup size: 64 / 128 lanes (one / two waves), 16- or 8-byte units, tables staged early / late
#define RSAMD_BSV(LATE, LQ, BS, TAG) \
    Variant{gf_matmul_vec1<10, true, 4, false, 0, LATE, LQ, 1, kVarDefault, BS>, 10, 4, 1, true, TAG, true, LQ, BS}
        case 150: *out = RSAMD_BSV(false, 4, 64, "vec1<10,16B,bs64>"); return true;
        case 151: *out = RSAMD_BSV(false, 4, 128, "vec1<10,16B,bs128>"); return true;
        case 152: *out = RSAMD_BSV(false, 2, 64, "vec1<10,8B,bs64>"); return true;
        case 153: *out = RSAMD_BSV(false, 2, 128, "vec1<10,8B,bs128>"); return true;
        case 154: *out = RSAMD_BSV(true, 4, 64, "vec1<10,16B,bs64,late>"); return true;
        case 155: *out = RSAMD_BSV(true, 4, 128, "vec1<10,16B,bs128,late>"); return true;
        case 156: *out = RSAMD_BSV(true, 2, 128, "vec1<10,8B,bs128,late>"); return true;
        case 157: *out = RSAMD_BSV(false, 2, 512, "vec1<10,8B,bs512>"); return true;
        case 159: *out = Variant{gf_matmul_vec1<10, true, 4, false, 0, false, 2, 1, kVarDefault | kVarXorOnly, 128>, 10,
                                 4, 1, true, "vec1<10,8B,bs128,xor>", true, 2, 128}; return true;
        case 158: *out = RSAMD_BSV(false, 2, 1024, "vec1<10,8B,bs1024>"); return true;
        // XCD-contiguous chunk order (each XCD streams its own eighth of the chunks)
        case 160: *out = Variant{gf_matmul_vec1<10, true, 4, false, 0, false, 2, 1, kVarDefault, 128, true>, 10, 4, 1,
                                 true, "vec1<10,8B,bs128,xcd>", true, 2, 128}; return true;
#undef RSAMD_BSV
        default: break;
    }
    switch (var) {
        RSAMD_CASE(0)
        RSAMD_CASE(1)
        RSAMD_CASE(2)
        RSAMD_CASE(4)
        RSAMD_CASE(6)
        RSAMD_CASE(8)
        RSAMD_CASE(10)
        RSAMD_CASE(12)
        RSAMD_CASE(14)
        default: return false;
    }
#undef RSAMD_CASE
}
#endif  // RSAMD_EXPERIMENTS

static Variant pick_global(int rows, bool acc) {  // global_* ops: vectors >= 2 GiB
    if (!acc) {
        if (rows == 1) return RSAMD_VARIANT_G(4, false, 1, false);
        if (rows == 2) return RSAMD_VARIANT_G(4, false, 2, false);
        if (rows <= 4) return RSAMD_VARIANT_G(4, false, 4, false);
        return RSAMD_VARIANT_G(4, false, 8, false);
    }
    if (rows == 1) return RSAMD_VARIANT_G(4, false, 1, true);
    if (rows == 2) return RSAMD_VARIANT_G(4, false, 2, true);
    if (rows <= 4) return RSAMD_VARIANT_G(4, false, 4, true);
    return RSAMD_VARIANT_G(4, false, 8, true);
}

// One-chunk kernels come in three builds: 16-byte lane units on 256-lane
// workgroups, and 8-byte units on 128-lane (default) or 256-lane workgroups
// (rs_tune("block8", 128 | 256)).  A/B (tools/ab.py, same process,
// profiles/r01/ab_block8.log): 128 lanes (1 KiB per vector per workgroup)
// win or tie at 8 KiB-1 MiB: 1 MiB split Encode 6.59-6.64 vs 6.56-6.57 TB/s,
// 128 KiB Update 6.16 vs 5.62, Reconst of 4 6.53 vs 6.20.  (Staging the
// tables after the data loads and two 8-byte units per lane were measured
// and dropped: both slower.)
#define RSAMD_V1(KB, KFIX, MC, ACC, WIN, LQ, BS, TAG)                                                  \
    Variant{gf_matmul_vec1<KB, KFIX, MC, ACC, WIN, false, LQ, 1, kVarDefault, BS>, KB, MC, 1, KFIX,       \
            "gf_matmul_vec1<" #KB "," #KFIX "," #MC "," #ACC "," #WIN "," TAG ">", true, LQ, BS}
#define RSAMD_VARIANT1(KB, KFIX, MC, ACC, WIN)                                                         \
    (lane16                      ? RSAMD_V1(KB, KFIX, MC, ACC, WIN, 4, 256, "16B")                      \
     : tuning().block8 == 128 ? RSAMD_V1(KB, KFIX, MC, ACC, WIN, 2, 128, "8B,128 lanes")             \
                                 : RSAMD_V1(KB, KFIX, MC, ACC, WIN, 2, 256, "8B"))

// 5-8 output rows: VALU-bound, and 16-byte lane units amortise each column's
// 40-dword LDS table over twice the data of 8-byte units (10+8 Encode @ 1 MiB:
// 5.29 TB/s vs 4.60 with 8-byte units and 4.43 with the looped kernel,
// profiles/r01/ab_rows8.log).  rs_tune("lane_bytes", 8) does not apply here.
#define RSAMD_VARIANT1_WIDE(KB, KFIX, MC, ACC, WIN)                                                    \
    (tuning().wide_block == 128 ? RSAMD_V1(KB, KFIX, MC, ACC, WIN, 4, 128, "16B,128 lanes")               \
                                : RSAMD_V1(KB, KFIX, MC, ACC, WIN, 4, 256, "16B"))

// Loop-free one-chunk-per-workgroup kernels (the default launch: grid = all
// chunks, rows <= MC).  A/B on MI355X, 10+4 @ 1 MiB x 256 (tools/ab.py, 2 x 30
// interleaved rounds): vec1 all-loads-up-front 0.589 ms, vec1 5-column window
// 0.600, looped kernel with window 0.602, looped without 0.611; XOR-only
// diagnostic 0.591 (the memory pattern's own ceiling).
static bool pick_one_chunk(int rows, int cols, bool acc, bool lane16, Variant* out) {
    if (!acc) {
        if (cols == 10 && rows > 2 && rows <= 4) { *out = RSAMD_VARIANT1(10, true, 4, false, 0); return true; }
        if (cols == 12 && rows > 2 && rows <= 4) { *out = RSAMD_VARIANT1(12, true, 4, false, 0); return true; }
        if (cols == 10 && rows == 1) { *out = RSAMD_VARIANT1(10, true, 1, false, 0); return true; }
        if (cols == 10 && rows == 2) { *out = RSAMD_VARIANT1(10, true, 2, false, 0); return true; }
        // 5-8 columns: one 8-column batch instead of two of 4 (all loads in
        // flight at once; 8+4 Encode +6.6 %, 6+3 +7 %, 8+6 +11 %, Reconst
        // +1.5-9.5 %, profiles/r01/ab_cols8.log).  var=200: also above 8.
        // 3-4 rows over more than 4 runtime columns: 16-byte units (8+3
        // Encode +6 %, 6+3 +7 %, 16+3 +7.7 %, 16+4 +8 %, 20+4 +5.6 %, 8+4 +3 %;
        // the fixed-column 10 / 12 kernels, 1-2 rows and accumulate launches
        // stay on 8-byte units, profiles/r01/ab_lane_generic*.log).  var=201
        // keeps 8-byte units (A/B).
        const bool wide34 = rows > 2 && rows <= 4 && cols > 4 && exp_var() != 201;
        if (cols > 4 && (cols <= 8 || exp_var() == 200)) {
            if (rows == 1) { *out = RSAMD_VARIANT1(8, false, 1, false, 0); return true; }
            if (rows == 2) { *out = RSAMD_VARIANT1(8, false, 2, false, 0); return true; }
            if (wide34) { *out = RSAMD_VARIANT1_WIDE(8, false, 4, false, 0); return true; }
            if (rows <= 4) { *out = RSAMD_VARIANT1(8, false, 4, false, 0); return true; }
        }
        if (rows == 1) { *out = RSAMD_VARIANT1(4, false, 1, false, 0); return true; }
        if (rows == 2) { *out = RSAMD_VARIANT1(4, false, 2, false, 0); return true; }
        if (wide34) { *out = RSAMD_VARIANT1_WIDE(4, false, 4, false, 0); return true; }
        if (rows <= 4) { *out = RSAMD_VARIANT1(4, false, 4, false, 0); return true; }
        if (cols == 10 && rows <= 8) { *out = RSAMD_VARIANT1_WIDE(10, true, 8, false, 0); return true; }
        if (cols == 12 && rows <= 8) { *out = RSAMD_VARIANT1_WIDE(12, true, 8, false, 0); return true; }
        if (rows <= 8 && cols > 4 && (cols <= 8 || exp_var() == 200)) {
            *out = RSAMD_VARIANT1_WIDE(8, false, 8, false, 0);
            return true;
        }
        if (rows <= 8) { *out = RSAMD_VARIANT1_WIDE(4, false, 8, false, 0); return true; }
        return false;
    }
    if (cols == 2 && rows > 2 && rows <= 4) { *out = RSAMD_VARIANT1(2, true, 4, true, 0); return true; }
    if (rows == 1) { *out = RSAMD_VARIANT1(4, false, 1, true, 0); return true; }
    if (rows == 2) { *out = RSAMD_VARIANT1(4, false, 2, true, 0); return true; }
    if (rows <= 4) { *out = RSAMD_VARIANT1(4, false, 4, true, 0); return true; }
    if (rows <= 8) { *out = RSAMD_VARIANT1_WIDE(4, false, 8, true, 0); return true; }
    return false;
}

static Variant pick(int rows, int cols, bool acc, int vpt, uint64_t body, bool lane16) {
    if (body >= (uint64_t{1} << 31)) return pick_global(rows, acc);
    Variant ex;
    if (pick_experimental(rows, cols, acc, vpt, &ex)) return ex;
    if (vpt == 1 && tuning().max_grid <= 0 && pick_one_chunk(rows, cols, acc, lane16, &ex)) return ex;
    // Looped kernels: row groups (rows > 4), grid caps, or VPT experiments.
    if (!acc) {
        if (cols == 10 && rows > 2 && rows <= 4)
            return vpt == 2 ? RSAMD_VARIANT(10, true, 4, false, 2) : RSAMD_VARIANT_W5(10);
        if (cols == 12 && rows > 2 && rows <= 4)
            return vpt == 2 ? RSAMD_VARIANT(12, true, 4, false, 2) : RSAMD_VARIANT_W5(12);
        if (rows == 1) return RSAMD_VARIANT(4, false, 1, false, 1);
        if (rows == 2) return RSAMD_VARIANT(4, false, 2, false, 1);
        if (rows <= 4) return RSAMD_VARIANT(4, false, 4, false, 1);
        return RSAMD_VARIANT(4, false, 8, false, 1);
    }
    if (rows == 1) return RSAMD_VARIANT(4, false, 1, true, 1);
    if (rows == 2) return RSAMD_VARIANT(4, false, 2, true, 1);
    if (rows <= 4) return RSAMD_VARIANT(4, false, 4, true, 1);
    return RSAMD_VARIANT(4, false, 8, true, 1);
}

// Lane width of the one-chunk kernels: 8-byte units (dwordx2, 512 B per wave
// instruction) on 128-lane workgroups, unless rs_tune("lane_bytes", 16)
// forces 16-byte units (dwordx4, 1 KiB) on 256-lane workgroups.  Same-process
// A/B on MI355X (tools/ab.py AB_VEC=..., profiles/r01/ab_lane_size_sweep.log):
// with 256-lane workgroups the 16-byte build won 3-4-output launches on
// vectors <= 32 KiB and interleaved Encode up to 256 KiB; with the 8-byte
// build on 128-lane workgroups, 8-byte units win every size and shape of the
// 10-column kernels (8 KiB split Encode 6.65 vs 6.30 TB/s, interleaved 6.42
// vs 5.78, Reconst of 4 6.46 vs 6.05; 32 KiB-1 MiB: +0-8 %).  Runtime-column
// launches with 3-8 rows pick 16-byte units themselves (pick_one_chunk).
static bool lane16_for(const MatmulArgs&) { return tuning().lane_bytes == 16; }

const char* vector_kernel_name(int rows, int cols, int accumulate) {
    return pick(rows, cols, accumulate != 0, tuning().vpt, 0, tuning().lane_bytes == 16).name;
}

static bool aligned16(uint64_t v) { return (v & 15u) == 0; }

// The wide kernel for `rows` (> 8) output rows: 16 rows per wave, NW waves
// per workgroup; rows beyond 16*NW take further passes (> 128 rows only).
using VecKernelRow = void (*)(const MatmulArgs, int);
static VecKernelRow wide_kernel_for(int rows, bool acc, int* rw, int* nw) {
#define RSAMD_WIDE(NW)                                                     \
    do {                                                                   \
        *rw = kWideRows;                                                   \
        *nw = NW;                                                          \
        return acc ? gf_matmul_wide<NW, true> : gf_matmul_wide<NW, false>; \
    } while (0)
    if (rows <= 16) RSAMD_WIDE(1);
    if (rows <= 32) RSAMD_WIDE(2);
    if (rows <= 64) RSAMD_WIDE(4);
    RSAMD_WIDE(8);
#undef RSAMD_WIDE
}

hipError_t launch_gf_multi(MatmulArgs& a, const PatternDesc* pats, const int32_t* stripe_pat, hipStream_t stream) {
    if (a.len == 0 || a.nstripes <= 0) return hipSuccess;
    a.body = a.len;  // caller guarantees len % 16 == 0, aligned vectors, len < 2 GiB
    a.tail_start = a.len;
    a.nt_store = 1;
    // the one-chunk kernels' shapes: 8-byte lanes on block8-lane workgroups
    // (128 by default) or 16-byte lanes on 256
    const int lq = tuning().lane_bytes == 16 ? 4 : 2;
    const int bs = lq == 4 ? kBlock : tuning().block8;
    a.units_per_chunk = bs;
    const uint64_t nunits = a.body / (4 * lq);
    a.chunks_per_stripe = static_cast<int64_t>((nunits + bs - 1) / bs);
    a.total_chunks = a.chunks_per_stripe * a.nstripes;
    a.cps_shift = -1;
    for (int sh = 0; sh < 31; ++sh)
        if ((int64_t{1} << sh) == a.chunks_per_stripe) a.cps_shift = sh;
    // a.rows = the largest output count over the batch's patterns (<= 8)
    const bool k10 = a.cols == 10;
    const int mc = a.rows <= 1 ? 1 : a.rows == 2 ? 2 : a.rows <= 4 ? 4 : 8;
    const int ncols_pad = k10 ? 10 : ((a.cols + 3) / 4) * 4;
    const size_t lds = static_cast<size_t>(ncols_pad) * (((mc * 5 + 3) / 4) * 4) * 4;
    const dim3 grid(static_cast<unsigned>(a.total_chunks));
    // HIP keeps the last failing call's status until read: clear anything an
    // unrelated earlier call (ours, the caller's, a framework's) left there,
    // so the hipGetLastError below reports this launch only
    (void)hipGetLastError();
#define RSAMD_MULTI(KB, KFIX, MC)                                                                          \
    do {                                                                                                  \
        if (lq == 4)                                                                                      \
            hipLaunchKernelGGL((gf_matmul_multi<KB, KFIX, MC, kBlock, 4>), grid, dim3(kBlock), lds, stream, a, \
                               pats, stripe_pat);                                                         \
        else if (bs == 128)                                                                               \
            hipLaunchKernelGGL((gf_matmul_multi<KB, KFIX, MC, 128, 2>), grid, dim3(128), lds, stream, a, pats, \
                               stripe_pat);                                                               \
        else                                                                                              \
            hipLaunchKernelGGL((gf_matmul_multi<KB, KFIX, MC, kBlock, 2>), grid, dim3(kBlock), lds, stream, a, \
                               pats, stripe_pat);                                                         \
    } while (0)
    if (k10) {
        if (mc == 1) RSAMD_MULTI(10, true, 1);
        else if (mc == 2) RSAMD_MULTI(10, true, 2);
        else if (mc == 4) RSAMD_MULTI(10, true, 4);
        else RSAMD_MULTI(10, true, 8);
    } else {
        if (mc == 1) RSAMD_MULTI(4, false, 1);
        else if (mc == 2) RSAMD_MULTI(4, false, 2);
        else if (mc == 4) RSAMD_MULTI(4, false, 4);
        else RSAMD_MULTI(4, false, 8);
    }
#undef RSAMD_MULTI
    return hipGetLastError();
}

int multi_table_dwords(int cols, int max_out) {
    return (cols == 10 ? 10 : ((cols + 3) / 4) * 4) * multi_image_rows(max_out) * 5;
}

// ---------------------------------------------------------------------------
// GPU planner of rs_reconst_batch_multi: one wave per
// distinct erasure pattern writes the table image and descriptor that
// reconst_multi (batches.cpp) would otherwise build on the host (plan_reconst,
// the inverse, combined_matrix, perm_table), so a batch whose stripes carry
// hundreds of patterns does not wait for the host.
//
// With no survivor list the survivors are every vector not needed, vs[0..d)
// the first d in index order (checkReconst rs.go:264-325): the d - dn
// surviving data vectors K, then the first dn surviving parity vectors P.
// The dn lost data vectors L satisfy enc[P][L] D_L = P ^ enc[P][K] D_K, so
// with Minv = (enc[P][L])^-1 (dn x dn, dn <= nn <= 8):
//   lost data L_l : coef(q) = Minv[l][j]                       (vs[q] = P_j)
//                             ^_j Minv[l][j] * enc[P_j][vs[q]]  (vs[q] in K)
//   lost parity v : coef(q) = enc[v][vs[q]] (vs[q] < d) ^ ^_l enc[v][L_l] * coef_l(q)
// A vector's coefficients over d independent survivors are unique, so these
// are the rows of the host's combined matrix (rows of the inverse of the
// d x d survivor submatrix, codec.cpp) byte for byte.
//
// The parity rows are Cauchy (matrix.go:37-54, codec.cpp make_encode_matrix):
// enc[i][j] = 1 / (i ^ j) for a parity row i and a data column j, so every
// entry the planner needs is an inverse from the field tables, and
// enc[P][L] is the Cauchy matrix of x_j = P_j, y_l = L_l, whose inverse has a
// closed form (in characteristic 2, where minus is plus):
//   Minv[l][j] = prod_k (x_j + y_k) * prod_k (x_k + y_l)
//              / ((x_j + y_l) * prod_{k != j} (x_j + x_k) * prod_{k != l} (y_l + y_k))
// (every factor is non-zero: the x are distinct parity indexes, the y
// distinct data indexes).  A lane per entry sums the factors' logarithms: no
// Gauss-Jordan chain, no encoding-matrix reads.  tests/test_gpu_parity.py
// compares every planned row with the oracle's inverse.
// ---------------------------------------------------------------------------
constexpr int kPlanWaves = 4;

// The field's log / exp tables as device constants (gf256.hpp's GfTables:
// 0x11d, exp doubled), so a launch uploads nothing for them
struct GfLogExp {
    uint8_t log[256];
    uint8_t exp[512];
};
constexpr GfLogExp make_gf_log_exp() {
    GfLogExp t{};
    unsigned v = 1;
    for (int i = 0; i < 255; ++i) {
        t.exp[i] = static_cast<uint8_t>(v);
        t.log[v] = static_cast<uint8_t>(i);
        v <<= 1;
        if (v & 0x100) v ^= 0x11d;
    }
    for (int i = 255; i < 512; ++i) t.exp[i] = t.exp[i - 255];
    return t;
}
__constant__ GfLogExp kGfLogExp = make_gf_log_exp();

// c * 2^b for b = 0..7 (multiplication by x, reduced by 0x11d): the columns
// of multiplication by c as a GF(2)-linear map, from which c * e for any e is
// the XOR of the entries of e's bits (no table lookups)
__device__ __forceinline__ void gf_basis(uint32_t c, uint32_t (&cb)[8]) {
    cb[0] = c;
#pragma unroll
    for (int b = 1; b < 8; ++b) cb[b] = ((cb[b - 1] << 1) ^ ((cb[b - 1] & 0x80u) ? 0x11du : 0u)) & 0xffu;
}

// N: the most outputs a pattern of the launch has, rounded to 4 or 8 (the
// image rows; a batch of 1-4-loss patterns keeps the small instance)
template <int N>
__global__ __launch_bounds__(64 * kPlanWaves) void gf_plan_multi(const PlanArgs a) {
    __shared__ uint8_t lg[256], ex[512];
    __shared__ uint16_t s_vs[kPlanWaves][256];
    __shared__ int s_nr[kPlanWaves][N];
    __shared__ uint8_t s_minv[kPlanWaves][N][N];
    __shared__ uint8_t s_coef[kPlanWaves][N][256];  // the lost data rows' coefficients per survivor column
    for (int i = threadIdx.x; i < 256; i += blockDim.x) lg[i] = kGfLogExp.log[i];
    for (int i = threadIdx.x; i < 512; i += blockDim.x) ex[i] = kGfLogExp.exp[i];
    // the stripe -> pattern map into device memory for the multi kernel
    // (grid-stride over every thread of the launch)
    for (int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x); i < a.nstripes;
         i += static_cast<int>(gridDim.x * blockDim.x))
        a.pat_dst[i] = a.pat_src[i];
    const int w = static_cast<int>(threadIdx.x >> 6), lane = static_cast<int>(threadIdx.x & 63);
    const int gi = static_cast<int>(blockIdx.x) * kPlanWaves + w;
    const bool live = gi < a.npat;  // (every wave reaches the barrier)
    const int d = a.d, n = a.d + a.p;
    // 1. survivors vs[0, d) and needed vectors nr[0, nn) in index order
    //    (loops unrolled over the 4 mask words: constant indexes, no scratch)
    int nn = 0, dn = 0;
    if (live) {
        const uint64_t* mk = a.masks + static_cast<size_t>(gi) * a.words;
        int ns = 0;
        const uint64_t lt = __lanemask_lt();
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int v0 = 64 * k;
            if (v0 >= n) break;
            const uint64_t mwk = mk[k];
            const int v = v0 + lane;
            const bool in = v < n;
            const bool need = in && ((mwk >> lane) & 1u);
            const uint64_t bs = __ballot(in && !need), bn = __ballot(need), bd = __ballot(need && v < d);
            if (in && !need) {
                const int rk = ns + __popcll(bs & lt);
                if (rk < d) s_vs[w][rk] = static_cast<uint16_t>(v);
            }
            if (need) {
                const int rk = nn + __popcll(bn & lt);
                if (rk < N) s_nr[w][rk] = v;
            }
            ns += __popcll(bs);
            nn += __popcll(bn);
            dn += __popcll(bd);
        }
    }
    __syncthreads();  // (the field tables)
    if (!live) return;  // (no barrier below: the rest is the wave's own)
    // the wave's LDS writes land before its later reads (program order, waited)
    auto wave_fence = [] { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); };
    // log / exp lookups: the products and inverses below are independent of
    // one another, so their LDS latencies overlap
    auto tmul = [&](uint32_t x, uint32_t y) -> uint32_t { return (x && y) ? ex[lg[x] + lg[y]] : 0u; };
    auto cinv = [&](uint32_t z) -> uint32_t { return ex[255 - lg[z]]; };  // z != 0
    // 2. Minv by the closed form, a lane per entry (x_k = P_k = vs[d - dn + k],
    //    y_k = L_k = nr[k]: the lost data come first in nr)
    for (int e = lane; e < N * N; e += 64) {
        const int l = e / N, j = e % N;
        if (l >= dn || j >= dn) continue;
        const uint32_t xj = s_vs[w][d - dn + j], yl = static_cast<uint32_t>(s_nr[w][l]);
        int num = 0, den = lg[xj ^ yl];
#pragma unroll
        for (int k = 0; k < N; ++k) {
            if (k >= dn) break;
            const uint32_t xk = s_vs[w][d - dn + k], yk = static_cast<uint32_t>(s_nr[w][k]);
            num += lg[xj ^ yk] + lg[xk ^ yl];
            if (k != j) den += lg[xj ^ xk];
            if (k != l) den += lg[yl ^ yk];
        }
        s_minv[w][l][j] = ex[(num + 255 * 4 * N - den) % 255];
    }
    wave_fence();
    // 3. the lost data rows' coefficients, a lane per (column, row) pair so a
    //    short code (10 columns) still keeps the wave busy
    for (int e = lane; e < d * N; e += 64) {
        const int q = e / N, l = e % N;
        if (l >= dn) continue;
        const uint32_t u = s_vs[w][q];
        uint32_t c = 0;
        if (static_cast<int>(u) >= d) {
            c = s_minv[w][l][q - (d - dn)];
        } else {
#pragma unroll
            for (int j = 0; j < N; ++j)
                if (j < dn) c ^= tmul(s_minv[w][l][j], cinv(static_cast<uint32_t>(s_vs[w][d - dn + j]) ^ u));
        }
        s_coef[w][l][q] = static_cast<uint8_t>(c);
    }
    wave_fence();
    // 4. every row's coefficient (the lost parity rows from the lost data
    //    ones), its column's table image ([column][img_rows x 5 dwords],
    //    perm_table in gf256.hpp; zero past the rows and columns) and the
    //    descriptor
    uint32_t* img = a.tabs + static_cast<size_t>(gi) * a.tdw;
    const int cw = a.img_rows * 5;  // dwords per image column (img_rows == N)
    const int ncol = a.tdw / cw;
    for (int e = lane; e < ncol * N; e += 64) {
        const int q = e / N, r = e % N;
        uint32_t coef = 0;
        if (q < d && r < nn) {
            if (r < dn) {
                coef = s_coef[w][r][q];
            } else {
                const uint32_t u = s_vs[w][q], v = static_cast<uint32_t>(s_nr[w][r]);
                coef = static_cast<int>(u) < d ? cinv(v ^ u) : 0u;
#pragma unroll
                for (int l = 0; l < N; ++l)
                    if (l < dn) coef ^= tmul(cinv(v ^ static_cast<uint32_t>(s_nr[w][l])), s_coef[w][l][q]);
            }
        }
        uint32_t cb[8];
        gf_basis(coef, cb);
        // c * e for the 3-bit groups as XORs of the basis (e's bits)
        const uint32_t a3 = cb[0] ^ cb[1];
        uint32_t t[5];
        t[0] = (cb[0] << 8) | (cb[1] << 16) | (a3 << 24);
        t[1] = cb[2] | (cb[2] ^ cb[0]) << 8 | (cb[2] ^ cb[1]) << 16 | (cb[2] ^ a3) << 24;
        const uint32_t b3 = cb[3] ^ cb[4];
        t[2] = (cb[3] << 8) | (cb[4] << 16) | (b3 << 24);
        t[3] = cb[5] | (cb[5] ^ cb[3]) << 8 | (cb[5] ^ cb[4]) << 16 | (cb[5] ^ b3) << 24;
        t[4] = (cb[6] << 8) | (cb[7] << 16) | ((cb[6] ^ cb[7]) << 24);
#pragma unroll
        for (int k = 0; k < 5; ++k) img[q * cw + r * 5 + k] = t[k];
    }
    PatternDesc* P = a.descs + gi;
    for (int i = lane; i < 256; i += 64) P->in_idx[i] = i < d ? s_vs[w][i] : 0;
    if (lane < N) P->out_idx[lane] = lane < nn ? static_cast<uint32_t>(s_nr[w][lane]) : 0u;
    if (lane == 0) {
        P->tab_off = static_cast<uint32_t>(gi) * static_cast<uint32_t>(a.tdw);
        P->nout = static_cast<uint32_t>(nn);
    }
}

// 16 bytes per lane, grid-stride (kernels.hpp launch_copy_in)
__global__ __launch_bounds__(256) void copy_in(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n) {
    for (size_t i = blockIdx.x * size_t{256} + threadIdx.x; i < n; i += size_t{gridDim.x} * 256) dst[i] = src[i];
}

hipError_t launch_copy_in(uint8_t* dst, const uint8_t* src_host_dev, size_t bytes, hipStream_t stream) {
    if (bytes == 0) return hipSuccess;
    if ((bytes & 15) || (reinterpret_cast<uintptr_t>(dst) & 15) || (reinterpret_cast<uintptr_t>(src_host_dev) & 15))
        return hipErrorInvalidValue;
    (void)hipGetLastError();  // report this launch only (see launch_gf_multi)
    const size_t n = bytes / 16;
    const size_t want = (n + 255) / 256;
    const unsigned grid = static_cast<unsigned>(want < 1024 ? want : 1024);
    hipLaunchKernelGGL(copy_in, dim3(grid), dim3(256), 0, stream, reinterpret_cast<uint4*>(dst),
                       reinterpret_cast<const uint4*>(src_host_dev), n);
    return hipGetLastError();
}

hipError_t launch_gf_plan_multi(const PlanArgs& a, hipStream_t stream) {
    if (a.npat <= 0) return hipSuccess;
    if (a.img_rows != 4 && a.img_rows != 8) return hipErrorInvalidValue;  // the instance's N is its image rows
    (void)hipGetLastError();  // report this launch only (see launch_gf_multi)
    const unsigned grid = static_cast<unsigned>((a.npat + kPlanWaves - 1) / kPlanWaves);
    if (a.img_rows > 4)
        hipLaunchKernelGGL(gf_plan_multi<8>, dim3(grid), dim3(64 * kPlanWaves), 0, stream, a);
    else
        hipLaunchKernelGGL(gf_plan_multi<4>, dim3(grid), dim3(64 * kPlanWaves), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_gf_matmul(MatmulArgs& a, hipStream_t stream) {
    if (a.len == 0 || a.nstripes <= 0 || a.rows <= 0 || a.cols <= 0) return hipSuccess;
    // Vector body only when every base pointer and both stripe strides are
    // 16-byte aligned (global_load/store_dwordx4 on naturally aligned data).
    bool aligned = true;
    for (int v = 0; v < a.cols + a.rows && aligned; ++v)
        aligned = aligned16(a.ptr[v]) && (a.nstripes == 1 || aligned16(static_cast<uint64_t>(a.ss[a.sid[v] & 3])));
    a.body = aligned ? (a.len & ~static_cast<uint64_t>(15)) : 0;
    a.tail_start = a.body;

    int bs = 128;
    if (BsKernel bk = a.body ? bs_kernel_for(a, &bs) : nullptr) {
        // bit-sliced Encode: 32-byte lane units (four 8-byte pieces) on
        // bs-lane workgroups, 32 * bs bytes of every vector per workgroup
        a.units_per_chunk = bs;
        a.nt_store = 1;
        a.chunks_per_stripe = static_cast<int64_t>((a.body + 32 * bs - 1) / (32 * bs));
        a.total_chunks = a.chunks_per_stripe * a.nstripes;
        a.cps_shift = -1;
        for (int sh = 0; sh < 31; ++sh)
            if ((int64_t{1} << sh) == a.chunks_per_stripe) a.cps_shift = sh;
        if (a.total_chunks <= 0x7fffffff && a.body < (uint64_t{1} << 31)) {
            // occupancy cap (rs_tune("bs_waves", n)): dynamic LDS the kernel
            // does not use, so at most n waves per SIMD share a CU's 160 KiB
            size_t lds = 0;
            const int bw = tuning().bs_waves;
            if (bw > 0 && bw < 8) {
                const int wgs = std::max(1, bw * 4 / (bs / 64));
                lds = std::min<size_t>(65536, 163840 / wgs);
            }
            (void)hipGetLastError();  // report this launch only (see launch_gf_multi)
            hipLaunchKernelGGL(bk, dim3(static_cast<unsigned>(a.total_chunks)), dim3(bs), lds, stream, a);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        } else {  // too large for one grid / 31-bit buffer offsets: the perm-table kernels
            bk = nullptr;
        }
        if (bk) a.body = 0;  // the vector path below is done; only the tail remains
    }
    // 5-128 output rows over a run-time matrix: the bit-sliced network
    // generated for this matrix (jit.cpp / jit_asm.cpp), once it is ready
    // (XOR-accumulate launches from jit_min_acc_cols columns on: jit.hpp)
    if (a.body && a.body < (uint64_t{1} << 31) && a.rows >= g_jit_min_rows && a.rows <= jit_max_rows() &&
        a.cols <= jit_max_cols() && (!a.accumulate || a.cols >= g_jit_min_acc_cols)) {
        // hiprtc kernels: 256-lane workgroups from 24 columns on whatever the
        // layout (40+8 Reconst of 8: 5.56-5.61 vs 4.98 TB/s, 24+8: 5.68 vs
        // 5.29; 20+12 Reconst of 12 5.83 vs 5.92 and 16+8 Encode 5.70-5.99 vs
        // 5.90-6.02 stay better at 64; profiles/r02/ab_jit_wide2.log,
        // ab_jit_ao.log, ab_jit_pf.log), else the build-time kernels' per-layout rule
        const int jbs = (bs_block_for(a) == 256 || (tuning().bs_block == 0 && a.cols >= 24)) ? 256 : 64;
        const uint64_t bytes = a.body * static_cast<uint64_t>(a.nstripes) * static_cast<uint64_t>(a.rows + a.cols);
        const auto hold = jit_launch_guard();  // (the kernel stays loaded until it is enqueued)
        const JitKernel k = jit_kernel_for(a, jbs, bytes);
        if (k.fn && k.is_asm) {
            // assembly kernel: grid (2 KiB chunks, stripes), nw waves per
            // workgroup; vector v of stripe s at ptr[v] + s * 16 * stride16[v]
            AsmArgs x;
            std::memset(&x, 0, sizeof x);
            x.body = static_cast<uint32_t>(a.body);
            x.stripe_ids = reinterpret_cast<uint64_t>(a.stripe_ids);
            bool ok = true;
            for (int v = 0; v < a.cols + a.rows && ok; ++v) {
                const int64_t ss = (a.nstripes > 1 || a.stripe_ids) ? a.ss[a.sid[v] & 3] : 0;  // (a listed stripe may be > 0)
                ok = ss >= 0 && ss % 16 == 0 && (ss >> 4) <= 0xffffffffll;
                x.ptr[v] = a.ptr[v];
                x.stride16[v] = static_cast<uint32_t>(ss >> 4);
            }
            if (ok) {
                // layout 0: one workgroup per 2 KiB chunk; layout 1: chunk
                // groups of nw chunks, G row groups each, in blocks of 8
                // chunk groups (the kernel maps x back, jit_asm.cpp)
                const uint64_t chunks = (a.body + kAsmChunk - 1) / kAsmChunk;
                // (layout 2: chunk groups of one chunk, G row groups each)
                const uint64_t cgs = k.layout == 2 ? chunks : (chunks + k.nw - 1) / k.nw;
                const unsigned gx = static_cast<unsigned>(k.layout >= 1 ? (cgs + 7) / 8 * 8 * k.groups : chunks);
                for (int y0 = 0; y0 < a.nstripes; y0 += 65535) {
                    x.stripe0 = static_cast<uint32_t>(y0);
                    const unsigned gy = static_cast<unsigned>(a.nstripes - y0 < 65535 ? a.nstripes - y0 : 65535);
                    size_t sz = sizeof x;
                    void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &x, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                                     HIP_LAUNCH_PARAM_END};
                    (void)hipGetLastError();
                    const hipError_t e = hipModuleLaunchKernel(k.fn, gx, gy, 1, 64 * k.nw, 1, 1, 0, stream, nullptr,
                                                               extra);
                    if (e != hipSuccess) return e;
                }
                jit_count_launch();
                a.body = 0;
            }
        } else if (k.fn) {
            a.units_per_chunk = jbs;
            a.nt_store = 1;
            a.chunks_per_stripe = static_cast<int64_t>((a.body + 32 * jbs - 1) / (32 * jbs));
            a.total_chunks = a.chunks_per_stripe * a.nstripes;
            a.cps_shift = -1;
            for (int sh = 0; sh < 31; ++sh)
                if ((int64_t{1} << sh) == a.chunks_per_stripe) a.cps_shift = sh;
            if (a.total_chunks <= 0x7fffffff) {
                void* params[] = {&a};
                (void)hipGetLastError();
                const hipError_t e = hipModuleLaunchKernel(k.fn, static_cast<unsigned>(a.total_chunks), 1, 1, jbs, 1,
                                                           1, 0, stream, params, nullptr);
                if (e != hipSuccess) return e;
                jit_count_launch();
                a.body = 0;
            }
        }
    }

    // More than 8 output rows and no compiled network: the single-pass wide
    // kernels (every input read once), in passes of NW*RW rows
    if (a.body && a.body < (uint64_t{1} << 31) && a.rows > 8 && a.wide && tuning().wide_single_pass) {
        int rw = 16, nw = 1;
        VecKernelRow fn = wide_kernel_for(a.rows, a.accumulate != 0, &rw, &nw);
        a.units_per_chunk = 64;  // 16-byte units: 1 KiB of every vector per workgroup
        a.nt_store = 1;
        a.chunks_per_stripe = static_cast<int64_t>((a.body + 1023) / 1024);
        a.total_chunks = a.chunks_per_stripe * a.nstripes;
        a.cps_shift = -1;
        for (int sh = 0; sh < 31; ++sh)
            if ((int64_t{1} << sh) == a.chunks_per_stripe) a.cps_shift = sh;
        if (a.total_chunks <= 0x7fffffff) {
            for (int row0 = 0; row0 < a.rows; row0 += rw * nw) {
                (void)hipGetLastError();
                hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(a.total_chunks)), dim3(64 * nw), 0, stream, a, row0);
                const hipError_t e = hipGetLastError();
                if (e != hipSuccess) return e;
            }
            a.body = 0;
        }
    }

    if (a.body) {
        const LaunchTuning& tu = tuning();
        Variant var = pick(a.rows, a.cols, a.accumulate != 0, tu.vpt, a.body, lane16_for(a));
        if (var.one_chunk) {  // one workgroup per chunk: the grid must fit a 31-bit dimension
            const uint64_t chunks = (a.body / (4 * var.lq) + var.bs - 1) / var.bs * static_cast<uint64_t>(a.nstripes);
            if (chunks > 0x7fffffffull)
                var = a.accumulate ? RSAMD_VARIANT(4, false, 4, true, 1) : RSAMD_VARIANT(4, false, 4, false, 1);
        }
        a.units_per_chunk = var.bs * var.vpt;
        a.nt_store = tu.nt_store;
        const uint64_t nunits = a.body / (4 * var.lq);
        a.chunks_per_stripe = static_cast<int64_t>((nunits + a.units_per_chunk - 1) / a.units_per_chunk);
        a.total_chunks = a.chunks_per_stripe * a.nstripes;
        a.cps_shift = -1;
        for (int sh = 0; sh < 31; ++sh)
            if ((int64_t{1} << sh) == a.chunks_per_stripe) a.cps_shift = sh;
        int64_t grid = a.total_chunks;
        if (!var.one_chunk) {
            if (tu.max_grid > 0 && grid > tu.max_grid) grid = tu.max_grid;
            if (grid > 0x7fffffff) grid = 65536 * 8;  // looped kernels stride over the rest
        }
        const int ncols_pad = var.kfix ? var.kb : ((a.cols + var.kb - 1) / var.kb) * var.kb;
        const int cold = ((var.mc * 5 + 3) / 4) * 4;
        size_t lds = static_cast<size_t>(ncols_pad) * cold * 4;
        if (tu.lds_pad > 0 && static_cast<size_t>(tu.lds_pad) > lds) lds = tu.lds_pad;  // occupancy experiments

        (void)hipGetLastError();  // report this launch only (see launch_gf_multi)
        hipLaunchKernelGGL(var.fn, dim3(static_cast<unsigned>(grid)), dim3(var.bs), lds, stream, a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (a.tail_start < a.len) {
        const uint64_t groups = (a.len - a.tail_start + 3) / 4;
        const uint64_t total = groups * static_cast<uint64_t>(a.nstripes);
        const uint64_t grid = (total + kBlock - 1) / kBlock;
        (void)hipGetLastError();
        hipLaunchKernelGGL(gf_matmul_bytes, dim3(static_cast<unsigned>(grid)), dim3(kBlock), 0, stream, a,
                           a.tail_start, groups);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace rsamd
