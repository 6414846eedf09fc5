// Diagnostics for tools/doorbell_probe.hip: can a kernel read a host word the
// host keeps changing?  (a) one launch per read, each load form; (b) a
// resident poller with a bounded poll count (it always exits).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

struct Ring {
    uint64_t seq;
    uint64_t stop;
    uint64_t pad[14];
    uint64_t done[16];
    uint64_t polls[16];
};

template <int FORM>
__device__ __forceinline__ uint64_t rd(uint64_t* p) {
    if (FORM == 0) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (FORM == 1) return *reinterpret_cast<volatile uint64_t*>(p);
    if (FORM == 2) return __builtin_nontemporal_load(p);
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int FORM>
__global__ void read_once(Ring* r) {
    if (threadIdx.x == 0) {
        const uint64_t v = rd<FORM>(&r->seq);
        __hip_atomic_store(&r->done[0], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <int FORM>
__global__ void poller(Ring* r, uint64_t start, uint64_t max_polls) {
    if (threadIdx.x != 0) return;
    uint64_t last = start, n = 0;
    while (n < max_polls) {
        const uint64_t v = rd<FORM>(&r->seq);
        ++n;
        if (v != last) {
            __hip_atomic_store(&r->done[0], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            last = v;
        }
        if (rd<FORM>(&r->stop)) break;
    }
    __hip_atomic_store(&r->polls[0], n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int coherent = 1; coherent >= 0; --coherent) {
        Ring* ring = nullptr;
        const unsigned fl = hipHostMallocMapped | (coherent ? hipHostMallocCoherent : hipHostMallocNonCoherent);
        if (hipHostMalloc(reinterpret_cast<void**>(&ring), sizeof(Ring), fl) != hipSuccess) {
            printf("{\"error\": \"hipHostMalloc\", \"coherent\": %d}\n", coherent);
            continue;
        }
        std::memset(ring, 0, sizeof(Ring));
        Ring* dr = nullptr;
        (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&dr), ring, 0);
        void (*once[4])(Ring*) = {read_once<0>, read_once<1>, read_once<2>, read_once<3>};
        for (int form = 0; form < 4; ++form) {
            int good = 0;
            for (int i = 0; i < 20; ++i) {
                __atomic_store_n(&ring->seq, 1000 + 100 * form + i, __ATOMIC_RELEASE);
                hipLaunchKernelGGL(once[form], dim3(1), dim3(64), 0, s, dr);
                (void)hipStreamSynchronize(s);
                good += __atomic_load_n(&ring->done[0], __ATOMIC_ACQUIRE) == uint64_t(1000 + 100 * form + i);
            }
            printf("{\"test\": \"read_once\", \"coherent\": %d, \"form\": %d, \"correct_of_20\": %d}\n", coherent, form, good);
            fflush(stdout);
        }
        void (*pol[4])(Ring*, uint64_t, uint64_t) = {poller<0>, poller<1>, poller<2>, poller<3>};
        for (int form = 0; form < 4; ++form) {
            ring->stop = 0;
            ring->polls[0] = 0;
            uint64_t seq = __atomic_load_n(&ring->seq, __ATOMIC_ACQUIRE);
            hipLaunchKernelGGL(pol[form], dim3(1), dim3(64), 0, s, dr, seq, uint64_t{2000000});
            int seen = 0;
            double lat_sum = 0;
            for (int i = 0; i < 200; ++i) {
                ++seq;
                auto a = std::chrono::steady_clock::now();
                __atomic_store_n(&ring->seq, seq, __ATOMIC_RELEASE);
                bool ok = false;
                while (std::chrono::steady_clock::now() - a < std::chrono::milliseconds(5))
                    if (__atomic_load_n(&ring->done[0], __ATOMIC_ACQUIRE) == seq) {
                        ok = true;
                        break;
                    }
                auto b = std::chrono::steady_clock::now();
                if (ok) {
                    ++seen;
                    lat_sum += std::chrono::duration<double, std::micro>(b - a).count();
                }
            }
            __atomic_store_n(&ring->stop, 1, __ATOMIC_RELEASE);
            (void)hipStreamSynchronize(s);
            printf("{\"test\": \"poller\", \"coherent\": %d, \"form\": %d, \"seen_of_200\": %d, \"mean_rtt_us\": %.2f, "
                   "\"polls\": %llu}\n", coherent, form, seen, seen ? lat_sum / seen : -1.0,
                   (unsigned long long)ring->polls[0]);
            fflush(stdout);
        }
        (void)hipHostFree(ring);
    }
    return 0;
}
