// Frequency of the s_memrealtime counter (the engine's idle clock): a kernel
// stamps the counter when the host raises a flag and again at a second flag
// ~100 ms (host clock) later.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

__global__ void stamp(uint64_t* w) {  // w[0], w[1]: flags (host); w[2], w[3]: stamps (device)
    while (__hip_atomic_load(&w[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) __builtin_amdgcn_s_sleep(1);
    const uint64_t a = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(&w[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) __builtin_amdgcn_s_sleep(1);
    const uint64_t b = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_store(&w[2], a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&w[3], b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
    uint64_t* w = nullptr;
    (void)hipHostMalloc(reinterpret_cast<void**>(&w), 64, hipHostMallocCoherent | hipHostMallocMapped);
    w[0] = w[1] = w[2] = w[3] = 0;
    uint64_t* dw = nullptr;
    (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&dw), w, 0);
    hipLaunchKernelGGL(stamp, dim3(1), dim3(64), 0, 0, dw);
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(&w[0], 1, __ATOMIC_RELEASE);
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    auto t1 = std::chrono::steady_clock::now();
    __atomic_store_n(&w[1], 1, __ATOMIC_RELEASE);
    (void)hipDeviceSynchronize();
    const double s = std::chrono::duration<double>(t1 - t0).count();
    printf("{\"ticks\": %llu, \"host_s\": %.6f, \"MHz\": %.2f}\n", (unsigned long long)(w[3] - w[2]), s,
           (w[3] - w[2]) / s / 1e6);
    return 0;
}
