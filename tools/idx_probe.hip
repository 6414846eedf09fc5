// idx_probe.hip — cost and semantics of relative VGPR addressing
// (s_set_gpr_idx_on / s_set_gpr_idx_idx) on gfx950, for a matrix-generic
// bit-sliced GF(2^8) kernel: output plane i of row r of column c is
// acc ^= LO[m & 15] ^ HI[m >> 4] with m a run-time mask, LO / HI the 16
// subset XORs of each half of the column's 8 bit-planes held in VGPRs.
//
// Per plane the probe runs one of:
//   idx2   s_set_gpr_idx_idx a; v_mov_b32 t, v[LO]; s_set_gpr_idx_idx b;
//          v_bitop3_b32 acc, v[HI], acc, t      (2 SALU + 2 VALU, SRC0 relative)
//   plain  v_bitop3_b32 acc, v[LO+a], acc, v[HI+b]   (the compiled network: 1 VALU)
// with W waves per SIMD, and checks idx2's result against the host.
//
//   hipcc --offload-arch=gfx950 -O3 tools/idx_probe.hip -o tools/_build/idx_probe && tools/_build/idx_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
            return 1;                                                         \
        }                                                                     \
    } while (0)

// table v[100:131] = (seed + k) ^ k; 8 accumulators v[140:147]
#define INIT                                                            \
    "v_mov_b32 v140, 0\n v_mov_b32 v141, 0\n v_mov_b32 v142, 0\n"       \
    "v_mov_b32 v143, 0\n v_mov_b32 v144, 0\n v_mov_b32 v145, 0\n"       \
    "v_mov_b32 v146, 0\n v_mov_b32 v147, 0\n"
#define CLOB                                                                                                         \
    "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113",  \
        "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126",      \
        "v127", "v128", "v129", "v130", "v131", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147",      \
        "v150", "v151", "s40", "s41", "s42", "s44", "s45", "s46", "scc"

__device__ __forceinline__ void fill_table(uint32_t seed) {
#define T(k) asm volatile("v_add_u32 v" #k ", " #k ", %0\n v_xor_b32 v" #k ", " #k ", v" #k : : "v"(seed) : "v" #k);
    T(100) T(101) T(102) T(103) T(104) T(105) T(106) T(107) T(108) T(109) T(110) T(111) T(112) T(113) T(114)
    T(115) T(116) T(117) T(118) T(119) T(120) T(121) T(122) T(123) T(124) T(125) T(126) T(127) T(128) T(129)
    T(130) T(131)
#undef T
}

// one plane, relative: a = LO index, b = HI index (SGPR values 0..15)
#define IDX2(ACC, A, B)                                            \
    "s_set_gpr_idx_idx " A "\n"                                    \
    "v_mov_b32 v150, v100\n"                                       \
    "s_set_gpr_idx_idx " B "\n"                                    \
    "v_bitop3_b32 " ACC ", v116, " ACC ", v150 bitop3:0x96\n"
// m0 written directly: S holds (a | 0x1000) | (b | 0x1000) << 16 (index in
// [7:0], SRC0-relative mode bit in [15:12] of each half)
#define IDX2M(ACC, S)                                              \
    "s_mov_b32 m0, " S "\n"                                        \
    "v_mov_b32 v150, v100\n"                                       \
    "s_lshr_b32 m0, " S ", 16\n"                                   \
    "v_bitop3_b32 " ACC ", v116, " ACC ", v150 bitop3:0x96\n"
// two planes interleaved: both lookups of LO, then both of HI
#define IDX2I(ACC1, ACC2, S1, S2)                                  \
    "s_mov_b32 m0, " S1 "\n"                                       \
    "v_mov_b32 v150, v100\n"                                       \
    "s_mov_b32 m0, " S2 "\n"                                       \
    "v_mov_b32 v151, v100\n"                                       \
    "s_lshr_b32 m0, " S1 ", 16\n"                                  \
    "v_bitop3_b32 " ACC1 ", v116, " ACC1 ", v150 bitop3:0x96\n"    \
    "s_lshr_b32 m0, " S2 ", 16\n"                                  \
    "v_bitop3_b32 " ACC2 ", v116, " ACC2 ", v151 bitop3:0x96\n"
#define PLAIN(ACC, A, B) "v_bitop3_b32 " ACC ", v" A ", " ACC ", v" B " bitop3:0x96\n"

// 8 planes per step; indices per plane (a, b) = (s40, s41), (s41, s42), ...
#define BODY_IDX                                                                                      \
    IDX2("v140", "s40", "s41") IDX2("v141", "s41", "s42") IDX2("v142", "s42", "s40")                  \
    IDX2("v143", "s40", "s42") IDX2("v144", "s41", "s40") IDX2("v145", "s42", "s41")                  \
    IDX2("v146", "s40", "s40") IDX2("v147", "s42", "s42")
// s44..s46 = packed (s40, s41), (s41, s42), (s42, s40) index pairs
#define BODY_M                                                                                        \
    IDX2M("v140", "s44") IDX2M("v141", "s45") IDX2M("v142", "s46") IDX2M("v143", "s44")               \
    IDX2M("v144", "s45") IDX2M("v145", "s46") IDX2M("v146", "s44") IDX2M("v147", "s45")
#define BODY_I                                                                                        \
    IDX2I("v140", "v141", "s44", "s45") IDX2I("v142", "v143", "s46", "s44")                          \
    IDX2I("v144", "v145", "s45", "s46") IDX2I("v146", "v147", "s44", "s45")
#define BODY_PLAIN                                                                                    \
    PLAIN("v140", "103", "121") PLAIN("v141", "105", "117") PLAIN("v142", "101", "127")               \
    PLAIN("v143", "111", "119") PLAIN("v144", "108", "116") PLAIN("v145", "100", "131")               \
    PLAIN("v146", "114", "123") PLAIN("v147", "107", "125")

__global__ __launch_bounds__(256) void k_idx(uint64_t* cyc, uint32_t* out, int iters, int a0, int a1, int a2) {
    fill_table(threadIdx.x + 1);
    uint32_t r[8];
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    asm volatile(INIT
                 "s_mov_b32 s40, %8\n s_mov_b32 s41, %9\n s_mov_b32 s42, %10\n"
                 "s_set_gpr_idx_on s40, gpr_idx(SRC0)\n"
                 "s_mov_b32 s43, %11\n"
                 "1:\n" BODY_IDX BODY_IDX BODY_IDX BODY_IDX
                 "s_sub_u32 s43, s43, 1\n s_cmp_lg_u32 s43, 0\n s_cbranch_scc1 1b\n"
                 "s_set_gpr_idx_off\n"
                 "v_mov_b32 %0, v140\n v_mov_b32 %1, v141\n v_mov_b32 %2, v142\n v_mov_b32 %3, v143\n"
                 "v_mov_b32 %4, v144\n v_mov_b32 %5, v145\n v_mov_b32 %6, v146\n v_mov_b32 %7, v147\n"
                 : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7])
                 : "s"(a0), "s"(a1), "s"(a2), "s"(iters)
                 : CLOB, "s43");
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
    for (int i = 0; i < 8; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 8 + i] = r[i];
}

#define KM(NAME, BODY)                                                                                       \
    __global__ __launch_bounds__(256) void NAME(uint64_t* cyc, uint32_t* out, int iters, int a0, int a1, int a2) { \
        fill_table(threadIdx.x + 1);                                                                         \
        uint32_t r[8];                                                                                       \
        const int p0 = (a0 | 0x1000) | ((a1 | 0x1000) << 16), p1 = (a1 | 0x1000) | ((a2 | 0x1000) << 16),     \
                  p2 = (a2 | 0x1000) | ((a0 | 0x1000) << 16);                                                 \
        __syncthreads();                                                                                     \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                                    \
        asm volatile(INIT "s_mov_b32 s44, %8\n s_mov_b32 s45, %9\n s_mov_b32 s46, %10\n"                     \
                     "s_set_gpr_idx_on s44, gpr_idx(SRC0)\n"                                                 \
                     "s_mov_b32 s43, %11\n"                                                                  \
                     "1:\n" BODY BODY BODY BODY "s_sub_u32 s43, s43, 1\n s_cmp_lg_u32 s43, 0\n s_cbranch_scc1 1b\n" \
                     "s_set_gpr_idx_off\n"                                                                   \
                     "v_mov_b32 %0, v140\n v_mov_b32 %1, v141\n v_mov_b32 %2, v142\n v_mov_b32 %3, v143\n"        \
                     "v_mov_b32 %4, v144\n v_mov_b32 %5, v145\n v_mov_b32 %6, v146\n v_mov_b32 %7, v147\n"        \
                     : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]),      \
                       "=v"(r[7])                                                                             \
                     : "s"(p0), "s"(p1), "s"(p2), "s"(iters)                                                  \
                     : CLOB, "s43");                                                                          \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                                    \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;        \
        for (int i = 0; i < 8; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 8 + i] = r[i];            \
    }
KM(k_idx2m, BODY_M)
KM(k_idx2i, BODY_I)

__global__ __launch_bounds__(256) void k_plain(uint64_t* cyc, uint32_t* out, int iters, int, int, int) {
    fill_table(threadIdx.x + 1);
    uint32_t r[8];
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    asm volatile(INIT "s_mov_b32 s43, %8\n"
                 "1:\n" BODY_PLAIN BODY_PLAIN BODY_PLAIN BODY_PLAIN
                 "s_sub_u32 s43, s43, 1\n s_cmp_lg_u32 s43, 0\n s_cbranch_scc1 1b\n"
                 "v_mov_b32 %0, v140\n v_mov_b32 %1, v141\n v_mov_b32 %2, v142\n v_mov_b32 %3, v143\n"
                 "v_mov_b32 %4, v144\n v_mov_b32 %5, v145\n v_mov_b32 %6, v146\n v_mov_b32 %7, v147\n"
                 : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7])
                 : "s"(iters)
                 : CLOB, "s43");
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
    for (int i = 0; i < 8; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 8 + i] = r[i];
}

typedef void (*Kern)(uint64_t*, uint32_t*, int, int, int, int);

static uint32_t tab(uint32_t lane_seed, int k) { return (lane_seed + static_cast<uint32_t>(k)) ^ static_cast<uint32_t>(k); }

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int maxw = cus * 4 * 8;
    uint64_t* cyc;
    uint32_t* out;
    CHECK(hipMalloc(&cyc, sizeof(uint64_t) * maxw));
    CHECK(hipMalloc(&out, 4ull * 8 * maxw * 64));
    const int a[3] = {3, 11, 6};
    // ---- semantics: each variant for 1 and 5 iterations on one workgroup
    int bad = 0;
    const int pl_idx[8][2] = {{0, 1}, {1, 2}, {2, 0}, {0, 2}, {1, 0}, {2, 1}, {0, 0}, {2, 2}};
    const int pl_m[8][2] = {{0, 1}, {1, 2}, {2, 0}, {0, 1}, {1, 2}, {2, 0}, {0, 1}, {1, 2}};
    struct V {
        Kern fn;
        const int (*pl)[2];
    } vs[] = {{(Kern)k_idx, pl_idx}, {(Kern)k_idx2m, pl_m}, {(Kern)k_idx2i, pl_m}};
    for (const V& v : vs)
        for (int iters : {1, 5}) {
            hipLaunchKernelGGL(v.fn, dim3(1), dim3(256), 0, 0, cyc, out, iters, a[0], a[1], a[2]);
            CHECK(hipDeviceSynchronize());
            std::vector<uint32_t> h(256 * 8);
            CHECK(hipMemcpy(h.data(), out, 4 * h.size(), hipMemcpyDeviceToHost));
            for (int t = 0; t < 256; ++t)
                for (int p = 0; p < 8; ++p) {
                    uint32_t acc = 0;
                    const uint32_t seed = static_cast<uint32_t>(t) + 1;
                    for (int s = 0; s < 4 * iters; ++s)
                        acc ^= tab(seed, 100 + a[v.pl[p][0]]) ^ tab(seed, 116 + a[v.pl[p][1]]);
                    if (h[t * 8 + p] != acc && bad++ < 5)
                        std::printf("MISMATCH variant %d iters %d lane %d plane %d: got %08x want %08x\n",
                                    static_cast<int>(&v - vs), iters, t, p, h[t * 8 + p], acc);
                }
        }
    std::printf("relative addressing (SRC0 of v_mov_b32 and of VOP3 v_bitop3_b32; s_set_gpr_idx_idx and m0 writes): %s\n", bad ? "WRONG" : "results ok");
    // ---- cost
    const int kIters = 2048;
    std::printf("cycles per plane per SIMD (median over waves), by waves per SIMD\n%-8s %8s %8s %8s %8s\n", "variant", "W=1",
                "W=2", "W=4", "W=8");
    struct P {
        const char* name;
        Kern fn;
    } ps[] = {{"idx2", (Kern)k_idx}, {"idx2m", (Kern)k_idx2m}, {"idx2i", (Kern)k_idx2i}, {"plain", (Kern)k_plain}};
    for (const P& p : ps) {
        std::printf("%-8s", p.name);
        for (int w : {1, 2, 4, 8}) {
            const int waves = cus * 4 * w;
            hipLaunchKernelGGL(p.fn, dim3(cus * w), dim3(256), 0, 0, cyc, out, 16, a[0], a[1], a[2]);
            CHECK(hipDeviceSynchronize());
            hipLaunchKernelGGL(p.fn, dim3(cus * w), dim3(256), 0, 0, cyc, out, kIters, a[0], a[1], a[2]);
            CHECK(hipDeviceSynchronize());
            std::vector<uint64_t> h(waves);
            CHECK(hipMemcpy(h.data(), cyc, sizeof(uint64_t) * waves, hipMemcpyDeviceToHost));
            std::sort(h.begin(), h.end());
            std::printf(" %8.2f", static_cast<double>(h[waves / 2]) / (32.0 * kIters * w));
        }
        std::printf("\n");
    }
    return bad ? 1 : 0;
}
