// Round-trip floor of a synchronous GPU call on this box (measurement tool):
// empty kernel launch + stream sync, with blocking and spin waits.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void empty_kernel(int* p) {
    if (threadIdx.x == 0 && p) p[0] = 1;
}

static double med(std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    int* d = nullptr;
    (void)hipMalloc(&d, 4);
    for (int mode = 0; mode < 3; ++mode) {
        std::vector<double> t;
        for (int i = 0; i < 2000; ++i) {
            auto a = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, d);
            if (mode == 0) (void)hipStreamSynchronize(s);
            else if (mode == 1) {
                (void)hipEventRecord(ev, s);
                (void)hipEventSynchronize(ev);
            } else {
                while (hipStreamQuery(s) == hipErrorNotReady) {
                }
            }
            auto b = std::chrono::steady_clock::now();
            if (i >= 100) t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
        }
        printf("{\"wait\": \"%s\", \"median_us\": %.2f}\n",
               mode == 0 ? "hipStreamSynchronize" : mode == 1 ? "event record + sync" : "hipStreamQuery spin", med(t));
    }
    return 0;
}
