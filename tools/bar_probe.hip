// Diagnostics (round 3): can the host write a call's
// inputs and doorbell straight into device memory (posted PCIe writes through
// the BAR), so that the resident engine polls and reads local HBM instead of
// paying PCIe read round trips?
//
//   1. which VRAM pools the CPU agent may access (HSA pool info), and whether
//      fine-grained / uncached hipExtMallocWithFlags memory is CPU-writable
//      (guarded by a SIGSEGV handler, so a refusal is reported, not fatal);
//   2. doorbell ping-pong: host bell -> GPU poll -> done word in host memory,
//      bell in host memory (today's engine) vs bell in device memory;
//   3. a whole 10+4 @ 8 KiB call: copy 80 KiB in, ring, 8 workgroups compute
//      (XOR stand-in), write 32 KiB + done words to host memory, copy out;
//      inputs in pinned host memory (today) vs device memory written by the CPU.
//
// Every kernel bounds each poll in time and returns at its first time-out, and
// the host never makes a runtime call while a kernel runs.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>
#include <setjmp.h>
#include <signal.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                               \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::printf("%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);     \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
constexpr int kIn = 10, kOut = 4, kLen = 8192, kGroups = 8;
constexpr uint64_t kPollLimit = 50'000'000;  // 0.5 s at the 100 MHz s_memrealtime clock

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------- HSA report
static hsa_agent_t g_cpu{}, g_gpu{};
static hsa_status_t find_agents(hsa_agent_t a, void*) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
    if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t report_pool(hsa_amd_memory_pool_t p, void*) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    size_t size = 0;
    bool all = false, alloc = false;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SIZE, &size);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_ACCESSIBLE_BY_ALL, &all);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
    hsa_amd_memory_pool_access_t acc = HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED;
    hsa_amd_agent_memory_pool_get_info(g_cpu, p, HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &acc);
    std::printf("  gpu pool: flags=0x%x (%s%s%s) size=%.1f GiB alloc=%d accessible_by_all=%d cpu_access=%s\n", flags,
                flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED ? "fine " : "",
                flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED ? "coarse " : "",
                flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT ? "kernarg" : "", size / 1073741824.0, alloc, all,
                acc == HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED          ? "never"
                : acc == HSA_AMD_MEMORY_POOL_ACCESS_ALLOWED_BY_DEFAULT   ? "allowed-by-default"
                                                                          : "disallowed-by-default");
    return HSA_STATUS_SUCCESS;
}

// ---------------------------------------------------------------- guarded CPU access
static sigjmp_buf g_jmp;
static void on_segv(int) { siglongjmp(g_jmp, 1); }
static bool cpu_rw_ok(void* p) {
    struct sigaction sa{}, old_segv{}, old_bus{};
    sa.sa_handler = on_segv;
    sigaction(SIGSEGV, &sa, &old_segv);
    sigaction(SIGBUS, &sa, &old_bus);
    bool ok = false;
    if (sigsetjmp(g_jmp, 1) == 0) {
        volatile uint64_t* q = static_cast<volatile uint64_t*>(p);
        q[0] = 0x1234567890abcdefull;
        _mm_sfence();
        ok = q[0] == 0x1234567890abcdefull;
    }
    sigaction(SIGSEGV, &old_segv, nullptr);
    sigaction(SIGBUS, &old_bus, nullptr);
    return ok;
}

// ---------------------------------------------------------------- kernels
__device__ __forceinline__ uint64_t sys_load(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// wave 0 of workgroup 0 answers bell value i with done = i, n times
__global__ void pingpong(const uint64_t* bell, uint64_t* done, int n) {
    if (threadIdx.x != 0) return;
    for (int i = 1; i <= n; ++i) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (sys_load(bell) != static_cast<uint64_t>(i))
            if (__builtin_amdgcn_s_memrealtime() - t0 > kPollLimit) {
                sys_store(done, ~0ull);
                return;
            }
        sys_store(done, i);
    }
}

// a stand-in for one GF(2^8) coefficient product of a dword (~5 VALU, the
// cost of the perm-table product) when HEAVY, else a shift
template <bool HEAVY>
__device__ __forceinline__ u4 coef(u4 x, int c, int r) {
    if (!HEAVY) return (c + r) & 1 ? x : (x << 1);
    const uint32_t k = 0x9E3779B9u * (c * 8 + r + 1);
    u4 t = x ^ (x << 3);
    t &= u4{k, k, k, k};
    t ^= x >> 5;
    return t ^ (u4{k, k, k, k} >> 7);
}

// n calls: wait for bell == i, every workgroup computes its 1/8 of the
// stripe (16 B per lane); WAVES == 1: each lane all 4 rows, WAVES == 4: wave
// w row w (the same input lines loaded by each wave); stores to host memory,
// then its done word
template <int WAVES, bool HEAVY, bool RELEASE>
__global__ __launch_bounds__(64 * WAVES) void call_sim(const uint64_t* bell, const u4* in, u4* out, uint64_t* done,
                                                        int n) {
    __shared__ int s_ok;
    const int units = kLen / 16, u = blockIdx.x * 64 + (threadIdx.x & 63), wave = threadIdx.x >> 6;
    for (int i = 1; i <= n; ++i) {
        if (threadIdx.x == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            int ok = 1;
            while (sys_load(bell) != static_cast<uint64_t>(i))
                if (__builtin_amdgcn_s_memrealtime() - t0 > kPollLimit) {
                    ok = 0;
                    break;
                }
            s_ok = ok;
        }
        __syncthreads();
        if (!s_ok) {
            if (threadIdx.x == 0) sys_store(&done[16 * blockIdx.x], ~0ull);
            return;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        u4 x[kIn];
#pragma unroll
        for (int c = 0; c < kIn; ++c) x[c] = __builtin_nontemporal_load(&in[c * units + u]);
#pragma unroll
        for (int r = 0; r < kOut; ++r) {
            if (WAVES == 1 || r == wave) {
                u4 a = u4{0, 0, 0, 0};
#pragma unroll
                for (int c = 0; c < kIn; ++c) a ^= coef<HEAVY>(x[c], c, r);
                __builtin_nontemporal_store(a, &out[r * units + u]);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            if (RELEASE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // write back the L2 before the done word
            sys_store(&done[16 * blockIdx.x], i);
        }
        __syncthreads();
    }
}

static u4 coef_host(u4 x, int c, int r, bool heavy) {
    if (!heavy) return (c + r) & 1 ? x : (x << 1);
    const uint32_t k = 0x9E3779B9u * (c * 8 + r + 1);
    u4 t = x ^ (x << 3);
    t &= u4{k, k, k, k};
    t ^= x >> 5;
    return t ^ (u4{k, k, k, k} >> 7);
}

static void expected(const uint8_t* in, uint8_t* out, bool heavy) {
    const u4* x = reinterpret_cast<const u4*>(in);
    u4* o = reinterpret_cast<u4*>(out);
    const int units = kLen / 16;
    for (int r = 0; r < kOut; ++r)
        for (int k = 0; k < units; ++k) {
            u4 a = u4{0, 0, 0, 0};
            for (int c = 0; c < kIn; ++c) a ^= coef_host(x[c * units + k], c, r, heavy);
            o[r * units + k] = a;
        }
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0 : v[v.size() / 2];
}

// bell_dev: bell word in device memory (else host); in_dev: inputs in device memory
static void run_pingpong(const char* name, uint64_t* bell, uint64_t* done, int n) {
    *reinterpret_cast<volatile uint64_t*>(bell) = 0;
    *reinterpret_cast<volatile uint64_t*>(done) = 0;
    _mm_sfence();
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(pingpong, dim3(1), dim3(64), 0, 0, bell, done, n);
    std::vector<double> t;
    volatile uint64_t* d = done;
    volatile uint64_t* b = bell;
    const double start = now_us();
    while (now_us() - start < 20000) {}  // let the kernel start
    bool failed = false;
    for (int i = 1; i <= n && !failed; ++i) {
        const double t0 = now_us();
        *b = i;
        _mm_sfence();
        while (*d != static_cast<uint64_t>(i))
            if (now_us() - t0 > 200000) {
                failed = true;
                break;
            }
        t.push_back(now_us() - t0);
    }
    CHECK(hipDeviceSynchronize());
    std::printf("pingpong %-28s median %.2f us  p10 %.2f  p90 %.2f  %s\n", name, median(t),
                [&] { auto v = t; std::sort(v.begin(), v.end()); return v[v.size() / 10]; }(),
                [&] { auto v = t; std::sort(v.begin(), v.end()); return v[v.size() * 9 / 10]; }(),
                failed ? "FAILED (time-out)" : "ok");
}

template <int WAVES, bool HEAVY, bool RELEASE = true>
static void run_call(const char* name, uint64_t* bell, uint8_t* in, uint8_t* out, uint64_t* done, int n) {
    std::vector<uint8_t> src(kIn * kLen), dst(kOut * kLen), want(kOut * kLen);
    for (size_t i = 0; i < src.size(); ++i) src[i] = static_cast<uint8_t>(i * 131 + 7);
    *reinterpret_cast<volatile uint64_t*>(bell) = 0;
    for (int g = 0; g < kGroups; ++g) reinterpret_cast<volatile uint64_t*>(done)[16 * g] = 0;
    _mm_sfence();
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL((call_sim<WAVES, HEAVY, RELEASE>), dim3(kGroups), dim3(64 * WAVES), 0, 0, bell, reinterpret_cast<const u4*>(in),
                       reinterpret_cast<u4*>(out), done, n);
    const double start = now_us();
    while (now_us() - start < 20000) {}
    std::vector<double> t, tin, tout;
    bool failed = false, wrong = false;
    volatile uint64_t* b = bell;
    for (int i = 1; i <= n && !failed; ++i) {
        std::memcpy(src.data(), &i, sizeof i);  // every call's inputs differ
        const double t0 = now_us();
        std::memcpy(in, src.data(), src.size());
        _mm_sfence();
        const double t1 = now_us();
        *b = i;
        _mm_sfence();
        for (int g = 0; g < kGroups && !failed; ++g)
            while (reinterpret_cast<volatile uint64_t*>(done)[16 * g] != static_cast<uint64_t>(i))
                if (now_us() - t0 > 200000) {
                    failed = true;
                    break;
                }
        const double t2 = now_us();
        std::memcpy(dst.data(), out, dst.size());
        const double t3 = now_us();
        t.push_back(t3 - t0);
        tin.push_back(t1 - t0);
        tout.push_back(t3 - t2);
        if ((i == n || i == 1) && !wrong) {
            expected(src.data(), want.data(), HEAVY);
            if (std::memcmp(dst.data(), want.data(), dst.size()) != 0) {
                wrong = true;
                size_t k = 0, nbad = 0;
                while (dst[k] == want[k]) ++k;
                for (size_t q = 0; q < dst.size(); ++q) nbad += dst[q] != want[q];
                size_t zeros = 0;
                for (size_t q = 0; q < dst.size(); ++q) zeros += dst[q] == 0;
                std::printf("  call %d: %zu of %zu bytes differ, first at %zu (got %02x want %02x), %zu zero bytes\n",
                            i, nbad, dst.size(), k, dst[k], want[k], zeros);
            }
        }
    }
    CHECK(hipDeviceSynchronize());
    std::printf("call %d wave%s %s  %-34s median %.2f us (copy in %.2f, copy out %.2f)  %s%s\n", WAVES,
                WAVES > 1 ? "s" : " ", HEAVY ? "gf-cost" : "xor    ", name, median(t), median(tin), median(tout),
                failed ? "FAILED (time-out) " : "", wrong ? "WRONG RESULT" : "results ok");
}

int main() {
    CHECK(hipSetDevice(0));
    CHECK(hipFree(nullptr));
    hsa_init();
    hsa_iterate_agents(find_agents, nullptr);
    std::printf("HSA pools of the GPU agent, as seen by the CPU agent:\n");
    hsa_amd_agent_iterate_memory_pools(g_gpu, report_pool, nullptr);

    uint64_t *hbell = nullptr, *hdone = nullptr;
    uint8_t *hin = nullptr, *hout = nullptr;
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&hbell), 4096, hipHostMallocCoherent | hipHostMallocMapped));
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&hdone), 8192, hipHostMallocCoherent | hipHostMallocMapped));
    // fine-grained (coherent) pinned blocks, as the engine's staging blocks:
    // the GPU's stores bypass its L2 and its loads see the CPU's latest bytes
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&hin), kIn * kLen, hipHostMallocCoherent | hipHostMallocMapped));
    CHECK(hipHostMalloc(reinterpret_cast<void**>(&hout), kOut * kLen, hipHostMallocCoherent | hipHostMallocMapped));

    const int n = 400;
    run_pingpong("bell in host memory", hbell, hdone, n);
    run_call<1, false, false>("inputs+bell in host memory (no release)", hbell, hin, hout, hdone, n);
    run_call<1, false>("inputs+bell in host memory", hbell, hin, hout, hdone, n);
    run_call<1, true>("inputs+bell in host memory", hbell, hin, hout, hdone, n);
    run_call<4, true>("inputs+bell in host memory", hbell, hin, hout, hdone, n);

    struct Kind {
        const char* name;
        unsigned flags;
    } kinds[] = {{"fine-grained VRAM", hipDeviceMallocFinegrained}, {"uncached VRAM", hipDeviceMallocUncached}};
    for (const Kind& k : kinds) {
        void* d = nullptr;
        hipError_t e = hipExtMallocWithFlags(&d, 1 << 20, k.flags);
        if (e != hipSuccess) {
            std::printf("%s: hipExtMallocWithFlags failed: %s\n", k.name, hipGetErrorString(e));
            continue;
        }
        hipPointerAttribute_t attr{};
        CHECK(hipPointerGetAttributes(&attr, d));
        std::printf("%s: device ptr %p host ptr %p\n", k.name, attr.devicePointer, attr.hostPointer);
        bool ok = cpu_rw_ok(d);
        std::printf("  CPU write/read before allow_access: %s\n", ok ? "ok" : "refused");
        if (!ok) {
            const hsa_status_t s = hsa_amd_agents_allow_access(1, &g_cpu, nullptr, d);
            ok = s == HSA_STATUS_SUCCESS && cpu_rw_ok(d);
            std::printf("  hsa_amd_agents_allow_access(cpu): status %d, CPU write/read %s\n", static_cast<int>(s),
                        ok ? "ok" : "refused");
        }
        if (ok) {
            uint8_t* base = static_cast<uint8_t*>(d);
            uint64_t* dbell = reinterpret_cast<uint64_t*>(base);
            uint8_t* din = base + 65536;
            std::vector<uint8_t> src(kIn * kLen, 1);
            std::vector<double> tc;
            for (int i = 0; i < 200; ++i) {
                const double t0 = now_us();
                std::memcpy(din, src.data(), src.size());
                _mm_sfence();
                tc.push_back(now_us() - t0);
            }
            std::printf("  CPU memcpy of 80 KiB into it: median %.2f us\n", median(tc));
            char nm[96];
            std::snprintf(nm, sizeof nm, "bell in %s", k.name);
            run_pingpong(nm, dbell, hdone, n);
            std::snprintf(nm, sizeof nm, "inputs+bell in %s", k.name);
            run_call<1, false>(nm, dbell, din, hout, hdone, n);
            run_call<1, true>(nm, dbell, din, hout, hdone, n);
            run_call<4, true>(nm, dbell, din, hout, hdone, n);
            std::snprintf(nm, sizeof nm, "bell only in %s", k.name);
            run_call<1, true>(nm, dbell, hin, hout, hdone, n);
            run_call<4, true>(nm, dbell, hin, hout, hdone, n);
        }
        CHECK(hipFree(d));
    }
    return 0;
}
