// Diagnostics: which part of the resident doorbell loop stalls?  Variants of
// a 256-lane resident kernel (lane 0 polls, the workgroup waits at a
// barrier), each with a hard bound on the poll count so it always exits.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

struct Ring {
    uint64_t seq;
    uint64_t stop;
    uint64_t pad[14];
    uint64_t done[64 * 16];  // workgroup b: done[16 * b]
    uint64_t polls[16];
};

constexpr int kIn = 10, kOut = 4, kLen = 8192;
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

// 10 inputs of 8 KiB in, 4 outputs out (XOR stand-in for the GF product);
// workgroup b covers a 1/nwg slice of the columns
__device__ __forceinline__ void payload(const u4* in, u4* out) {
    const int units = kLen / 16;
    const int per = units / gridDim.x;
    for (int u = blockIdx.x * per + threadIdx.x; u < (blockIdx.x + 1) * per; u += blockDim.x) {
        u4 acc[kOut];
        for (int j = 0; j < kOut; ++j) acc[j] = u4{0, 0, 0, 0};
        for (int i = 0; i < kIn; ++i) {
            const u4 x = __builtin_nontemporal_load(&in[i * units + u]);
            for (int j = 0; j < kOut; ++j) acc[j] ^= x + u4{uint32_t(j), 0, 0, 0};
        }
        for (int j = 0; j < kOut; ++j) __builtin_nontemporal_store(acc[j], &out[j * units + u]);
    }
}

// F bit0: s_sleep between polls, bit1: realtime idle check, bit2: fences around the work
template <int F>
__global__ void resident(Ring* r, uint64_t start, uint64_t max_polls, const u4* in, u4* out, int with_payload) {
    __shared__ uint64_t s_seq;
    uint64_t last = start, n = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            const uint64_t t0 = (F & 2) ? __builtin_amdgcn_s_memrealtime() : 0;
            uint64_t v;
            for (;;) {
                v = __hip_atomic_load(&r->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                ++n;
                if (v != last) break;
                if (__hip_atomic_load(&r->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) || n >= max_polls ||
                    ((F & 2) && __builtin_amdgcn_s_memrealtime() - t0 > 20000000)) {
                    v = ~uint64_t{0};
                    break;
                }
                if (F & 1) __builtin_amdgcn_s_sleep(1);
            }
            s_seq = v;
        }
        __syncthreads();
        const uint64_t v = s_seq;
        __syncthreads();
        if (v == ~uint64_t{0}) break;
        if (F & 4) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        if (with_payload) payload(in, out);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            if (F & 4) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&r->done[16 * blockIdx.x], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        last = v;
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(&r->polls[0], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void once(Ring* r, uint64_t seq, const u4* in, u4* out, int with_payload) {
    if (with_payload) payload(in, out);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&r->done[16 * blockIdx.x], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

#include <algorithm>
#include <vector>

static double pct(std::vector<double> v, double q) {
    if (v.empty()) return -1;
    std::sort(v.begin(), v.end());
    return v[static_cast<size_t>(q * (v.size() - 1))];
}

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    Ring* ring = nullptr;
    uint8_t *hin = nullptr, *hout = nullptr;
    if (hipHostMalloc(reinterpret_cast<void**>(&ring), sizeof(Ring), hipHostMallocMapped | hipHostMallocCoherent) ||
        hipHostMalloc(reinterpret_cast<void**>(&hin), kIn * kLen, hipHostMallocMapped | hipHostMallocCoherent) ||
        hipHostMalloc(reinterpret_cast<void**>(&hout), kOut * kLen, hipHostMallocMapped | hipHostMallocCoherent))
        return 1;
    std::memset(ring, 0, sizeof(Ring));
    Ring* dr = nullptr;
    void *din = nullptr, *dout = nullptr;
    (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&dr), ring, 0);
    (void)hipHostGetDevicePointer(&din, hin, 0);
    (void)hipHostGetDevicePointer(&dout, hout, 0);
    std::vector<uint8_t> user_in(kIn * kLen, 7), user_out(kOut * kLen);
    uint64_t seq = 0;
    auto wait_all = [&](int nwg, uint64_t want) {
        auto a = std::chrono::steady_clock::now();
        for (int b = 0; b < nwg; ++b)
            while (__atomic_load_n(&ring->done[16 * b], __ATOMIC_ACQUIRE) != want)
                if (std::chrono::steady_clock::now() - a > std::chrono::milliseconds(5)) return false;
        return true;
    };
    for (int with_payload = 0; with_payload < 2; ++with_payload)
        for (int nwg : {1, 4, 8, 16})
            for (int copies = 0; copies < 1 + with_payload; ++copies) {
                // launch per call, host spins on the completion words
                std::vector<double> tl;
                for (int i = 0; i < 1500; ++i) {
                    ++seq;
                    auto a = std::chrono::steady_clock::now();
                    if (copies) std::memcpy(hin, user_in.data(), user_in.size());
                    hipLaunchKernelGGL(once, dim3(nwg), dim3(256), 0, s, dr, seq, (const u4*)din, (u4*)dout, with_payload);
                    const bool ok = wait_all(nwg, seq);
                    if (copies) std::memcpy(user_out.data(), hout, user_out.size());
                    if (ok && i >= 100)
                        tl.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
                }
                (void)hipStreamSynchronize(s);
                // resident kernel, doorbell
                ring->stop = 0;
                hipLaunchKernelGGL(resident<7>, dim3(nwg), dim3(256), 0, s, dr, seq, uint64_t{3000000}, (const u4*)din,
                                   (u4*)dout, with_payload);
                std::vector<double> td;
                int missed = 0;
                for (int i = 0; i < 1500; ++i) {
                    ++seq;
                    auto a = std::chrono::steady_clock::now();
                    if (copies) std::memcpy(hin, user_in.data(), user_in.size());
                    __atomic_store_n(&ring->seq, seq, __ATOMIC_RELEASE);
                    const bool ok = wait_all(nwg, seq);
                    if (copies) std::memcpy(user_out.data(), hout, user_out.size());
                    missed += !ok;
                    if (ok && i >= 100)
                        td.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
                }
                __atomic_store_n(&ring->stop, 1, __ATOMIC_RELEASE);
                (void)hipStreamSynchronize(s);
                printf("{\"payload\": %d, \"workgroups\": %d, \"host_copies\": %d, \"launch_flag_median_us\": %.2f, "
                       "\"launch_flag_p90_us\": %.2f, \"doorbell_median_us\": %.2f, \"doorbell_p90_us\": %.2f, "
                       "\"doorbell_p99_us\": %.2f, \"doorbell_missed\": %d}\n",
                       with_payload, nwg, copies, pct(tl, 0.5), pct(tl, 0.9), pct(td, 0.5), pct(td, 0.9), pct(td, 0.99),
                       missed);
                fflush(stdout);
            }
    std::vector<double> tc;
    for (int i = 0; i < 1500; ++i) {
        auto a = std::chrono::steady_clock::now();
        std::memcpy(hin, user_in.data(), user_in.size());
        std::memcpy(user_out.data(), hout, user_out.size());
        tc.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
    }
    printf("{\"host_memcpy_80K_in_32K_out_median_us\": %.2f}\n", pct(tc, 0.5));
    return 0;
}
