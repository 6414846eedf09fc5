// valu_probe.hip — issue cost of the VALU instructions the GF(2^8) kernels
// are made of, on gfx950 (cycles per wave-instruction per SIMD).
//
// Each kernel runs a loop of 32 independent instructions of one kind (8
// independent chains of 4, so no dependency stalls) with W waves per SIMD
// (1 / 2 / 4 / 8 resident: 256 CUs x 4 SIMDs x W waves), stamps
// s_memtime around the loop, and reports shader cycles per instruction per
// SIMD = cycles * 1 / (W * instructions per wave) (median over waves).
//
//   hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o /tmp/valu_probe && /tmp/valu_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
            return 1;                                                              \
        }                                                                          \
    } while (0)

constexpr int kIters = 2048;

#define OP8(ASM)                                                                         \
    asm volatile(ASM : "+v"(a0) : "v"(b), "v"(c));                                       \
    asm volatile(ASM : "+v"(a1) : "v"(b), "v"(c));                                       \
    asm volatile(ASM : "+v"(a2) : "v"(b), "v"(c));                                       \
    asm volatile(ASM : "+v"(a3) : "v"(b), "v"(c));                                       \
    asm volatile(ASM : "+v"(a4) : "v"(b), "v"(c));                                       \
    asm volatile(ASM : "+v"(a5) : "v"(b), "v"(c));                                       \
    asm volatile(ASM : "+v"(a6) : "v"(b), "v"(c));                                       \
    asm volatile(ASM : "+v"(a7) : "v"(b), "v"(c));

#define PROBE(NAME, ASM, T)                                                                                    \
    __global__ __launch_bounds__(256) void NAME(uint64_t* cyc, T* sink, int iters) {                           \
        T a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,   \
          a7 = a0 + 7;                                                                                         \
        T b = blockIdx.x * 3 + 1, c = threadIdx.x * 5 + 7;                                                     \
        __syncthreads();                                                                                       \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                                      \
        for (int i = 0; i < iters; ++i) {                                                                      \
            OP8(ASM) OP8(ASM) OP8(ASM) OP8(ASM)                                                                \
        }                                                                                                      \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                                      \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;        \
        sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;                    \
    }

PROBE(p_xor, "v_xor_b32 %0, %0, %1", uint32_t)
PROBE(p_and, "v_and_b32 %0, %0, %1", uint32_t)
PROBE(p_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96", uint32_t)
PROBE(p_perm, "v_perm_b32 %0, %1, %2, %0", uint32_t)
PROBE(p_lshr, "v_lshrrev_b32 %0, 3, %0", uint32_t)
PROBE(p_lshr64, "v_lshrrev_b64 %0, 3, %0", uint64_t)
PROBE(p_and_or, "v_and_or_b32 %0, %0, %1, %2", uint32_t)
PROBE(p_mov64, "v_mov_b64 %0, %1", uint64_t)
PROBE(p_pk_mov, "v_pk_mov_b32 %0, %1, %1 op_sel:[0,1]", uint64_t)
PROBE(p_fma, "v_fma_f32 %0, %0, %1, %2", float)

typedef void (*Probe)(uint64_t*, void*, int);  // (the kernels' sink pointer type differs; same ABI)

int main() {
    struct P {
        const char* name;
        const void* fn;
        int bytes;
    } probes[] = {{"v_xor_b32", (const void*)p_xor, 4},           {"v_and_b32", (const void*)p_and, 4},
                  {"v_bitop3_b32", (const void*)p_bitop3, 4},     {"v_perm_b32", (const void*)p_perm, 4},
                  {"v_lshrrev_b32", (const void*)p_lshr, 4},      {"v_lshrrev_b64", (const void*)p_lshr64, 8},
                  {"v_and_or_b32", (const void*)p_and_or, 4},     {"v_mov_b64", (const void*)p_mov64, 8},
                  {"v_pk_mov_b32", (const void*)p_pk_mov, 8},     {"v_fma_f32", (const void*)p_fma, 4}};
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint64_t* cyc;
    void* sink;
    const int maxw = cus * 4 * 8;
    CHECK(hipMalloc(&cyc, sizeof(uint64_t) * maxw));
    CHECK(hipMalloc(&sink, 8ull * maxw * 64));
    std::printf("CUs %d; cycles per wave-instruction per SIMD (median over waves), by waves per SIMD\n", cus);
    std::printf("%-16s %8s %8s %8s %8s\n", "instruction", "W=1", "W=2", "W=4", "W=8");
    for (const P& p : probes) {
        std::printf("%-16s", p.name);
        for (int w : {1, 2, 4, 8}) {
            // w workgroups of 4 waves per CU (w waves on each SIMD)
            const int waves = cus * 4 * w;
            hipLaunchKernelGGL((Probe)p.fn, dim3(cus * w), dim3(256), 0, 0, cyc, (void*)sink, 16);  // warm
            CHECK(hipDeviceSynchronize());
            hipLaunchKernelGGL((Probe)p.fn, dim3(cus * w), dim3(256), 0, 0, cyc, (void*)sink, kIters);
            CHECK(hipDeviceSynchronize());
            std::vector<uint64_t> h(waves);
            CHECK(hipMemcpy(h.data(), cyc, sizeof(uint64_t) * waves, hipMemcpyDeviceToHost));
            std::sort(h.begin(), h.end());
            const double instr = 32.0 * kIters;
            std::printf(" %8.2f", static_cast<double>(h[waves / 2]) / (instr * w));
        }
        std::printf("\n");
    }
    return 0;
}
