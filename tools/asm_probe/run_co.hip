// Diagnostics: run hand-assembled code objects (tools/asm_probe) on the GPU.
//   run_co wave_id.co               -> v0 / wave id / branch per lane of a 128-lane workgroup
//   run_co bs.co bs.mat rows cols nw -> one 2 KiB chunk of one stripe through a generated
//                                       bit-sliced kernel, every output row checked (GF(2^8)/0x11d)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::printf("%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);  \
            return 1;                                                                       \
        }                                                                                   \
    } while (0)

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) p ^= a;
        const bool hi = a & 0x80;
        a <<= 1;
        if (hi) a ^= 0x1d;
        b >>= 1;
    }
    return p;
}

struct AsmArgs {  // jit_asm.hpp layout
    uint32_t body, stripe0;
    uint64_t stripe_ids;
    uint64_t ptr[260];
    uint32_t stride16[260];
};

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    hipModule_t m;
    CHECK(hipModuleLoad(&m, argv[1]));
    if (argc == 2) {
        hipFunction_t f;
        CHECK(hipModuleGetFunction(&f, m, "rs_dbg"));
        void* d;
        CHECK(hipMalloc(&d, 4096));
        CHECK(hipMemset(d, 0xff, 4096));
        struct { void* p; } arg{d};
        size_t sz = sizeof arg;
        void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &arg, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
        CHECK(hipModuleLaunchKernel(f, 1, 1, 1, 128, 1, 1, 0, nullptr, nullptr, extra));
        CHECK(hipDeviceSynchronize());
        uint32_t h[1024];
        CHECK(hipMemcpy(h, d, 4096, hipMemcpyDeviceToHost));
        for (int l = 0; l < 128; l += 16)
            std::printf("lane %3d: v0=0x%08x wave=%u branch=0x%x wgx=%u\n", l, h[l], h[128 + l], h[256 + l],
                        h[384 + l]);
        return 0;
    }
    const int rows = std::atoi(argv[3]), cols = std::atoi(argv[4]), nw = std::atoi(argv[5]);
    std::vector<uint8_t> mat(rows * cols);
    FILE* fm = std::fopen(argv[2], "rb");
    if (!fm || std::fread(mat.data(), 1, mat.size(), fm) != mat.size()) return 3;
    std::fclose(fm);
    hipFunction_t f;
    CHECK(hipModuleGetFunction(&f, m, "rs_bs_asm"));
    const int n = 2048, nv = rows + cols;
    std::vector<uint8_t> h(nv * n);
    for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint8_t>(std::rand());
    uint8_t* d;
    CHECK(hipMalloc(&d, h.size()));
    CHECK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
    AsmArgs a;
    std::memset(&a, 0, sizeof a);
    a.body = n;
    for (int v = 0; v < nv; ++v) a.ptr[v] = reinterpret_cast<uint64_t>(d + v * n);
    size_t sz = sizeof a;
    void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    CHECK(hipModuleLaunchKernel(f, 1, 1, 1, 64 * nw, 1, 1, 0, nullptr, nullptr, extra));
    CHECK(hipDeviceSynchronize());
    std::vector<uint8_t> g(h.size());
    CHECK(hipMemcpy(g.data(), d, g.size(), hipMemcpyDeviceToHost));
    for (int r = 0; r < rows; ++r) {
        int bad = 0, untouched = 0;
        for (int i = 0; i < n; ++i) {
            uint8_t e = 0;
            for (int c = 0; c < cols; ++c) e ^= gmul(mat[r * cols + c], h[c * n + i]);
            bad += g[(cols + r) * n + i] != e;
            untouched += g[(cols + r) * n + i] == h[(cols + r) * n + i];
        }
        std::printf("row %2d: %4d bytes wrong, %4d untouched\n", r, bad, untouched);
    }
    return 0;
}
