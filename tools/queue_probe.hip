// Does a resident kernel on one stream block kernels on other streams?
// (HIP maps streams onto a few hardware queues; a kernel that stays resident
// holds its queue.)  A resident kernel (spins on a host flag, leaves on it or
// after 0.3 s) runs on stream R; then a short kernel is launched on each of 8
// other streams and we time how long each takes to complete (polling with
// hipStreamQuery, never a blocking wait).  R is a plain stream, a high-
// priority stream, or a CU-masked stream (hipExtStreamCreateWithCUMask).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <vector>

__global__ void resident(volatile uint64_t* flag, uint64_t max_ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(const_cast<uint64_t*>(flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
           __builtin_amdgcn_s_memrealtime() - t0 < max_ticks)
        __builtin_amdgcn_s_sleep(10);
}
__global__ void tiny(int* p) {
    if (threadIdx.x == 0) p[blockIdx.x] += 1;
}

int main() {
    uint64_t* flag = nullptr;
    (void)hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocCoherent | hipHostMallocMapped);
    uint64_t* dflag = nullptr;
    (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), flag, 0);
    int* d = nullptr;
    (void)hipMalloc(&d, 4096);
    std::vector<hipStream_t> others(8);
    for (auto& s : others) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int mode = 0; mode < 3; ++mode) {
        hipStream_t r = nullptr;
        if (mode == 0) (void)hipStreamCreateWithFlags(&r, hipStreamNonBlocking);
        if (mode == 1) {
            int lo = 0, hi = 0;
            (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
            (void)hipStreamCreateWithPriority(&r, hipStreamNonBlocking, hi);
        }
        if (mode == 2) {
            std::vector<uint32_t> mask(8, 0xffffffffu);  // every CU
            if (hipExtStreamCreateWithCUMask(&r, static_cast<uint32_t>(mask.size()), mask.data()) != hipSuccess) {
                printf("{\"mode\": \"cu_mask\", \"error\": \"create\"}\n");
                continue;
            }
        }
        *flag = 0;
        hipLaunchKernelGGL(resident, dim3(1), dim3(64), 0, r, dflag, uint64_t{30000000});  // 0.3 s cap
        auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(20)) {
        }
        int blocked = 0;
        double worst = 0;
        for (auto& s : others) {
            auto a = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, s, d);
            while (hipStreamQuery(s) == hipErrorNotReady &&
                   std::chrono::steady_clock::now() - a < std::chrono::milliseconds(50)) {
            }
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
            if (us > 20000) ++blocked;
            worst = us > worst ? us : worst;
        }
        __atomic_store_n(flag, 1, __ATOMIC_RELEASE);
        (void)hipDeviceSynchronize();
        printf("{\"mode\": \"%s\", \"other_streams\": 8, \"blocked_over_20ms\": %d, \"worst_us\": %.1f}\n",
               mode == 0 ? "plain" : mode == 1 ? "high_priority" : "cu_mask", blocked, worst);
        fflush(stdout);
        (void)hipStreamDestroy(r);
    }
    return 0;
}
