// engine.cpp — the host-call engine: small synchronous host calls (the Go
// API's one-stripe Encode / Reconst / Update / Replace on 8 KiB vectors, and
// the coalesced batches of concurrent ones) are served by a resident kernel
// (gf_engine, kernels.hip) through a doorbell in host memory, instead of a
// kernel launch plus a stream synchronisation per call.
//
// Measured on MI355X (tools/doorbell_probe3.hip, profiles/r02/doorbell_probe.log):
// an empty call's round trip is 11.8 us with launch + hipStreamSynchronize,
// 5.9 us with launch + a host-memory completion flag, 4.3 us through a
// doorbell; with a 10+4 @ 8 KiB stripe read and written over PCIe 12.4 / 7.1 us
// (launch + flag / doorbell, 4 workgroups).
//
// Protocol (one call at a time per handle; eng_mu):
//   host: tables (when the matrix changed) -> header fields -> seq0 -> seq1
//         (x86 stores become visible in program order, so a kernel that reads
//         both seq words new also reads the fields new), then spin until every
//         workgroup's done word holds the new value.
//   kernel: each workgroup polls the header line, computes its share straight
//         over the caller's pinned staging buffer, writes its done word.
// The kernel leaves on the stop word or after host_engine_idle_us without a
// doorbell (so it never outlives its callers, and never holds a hardware
// queue that other streams share for long).  The host rings a running engine
// only within half that window of its last call; otherwise it stops the old
// instance and launches a new one.  If an instance is found gone while a call
// is pending, a new one resumes it: workgroups that already finished the call
// (done word) skip it, so no unit is computed twice (Update / Replace XOR
// into their outputs).
#include <immintrin.h>

#include <cstdio>
#include <cstdlib>

#include <hip/hip_ext.h>

#include "codec_internal.hpp"

namespace rsamd {
namespace detail {

int g_engine = [] {                     // rs_tune("host_engine", 0 | 1); env RSAMD_HOST_ENGINE
    const char* e = std::getenv("RSAMD_HOST_ENGINE");
    return e ? (std::atoi(e) ? 1 : 0) : 1;
}();
int g_engine_waves = 8;                 // rs_tune("host_engine_waves", 1..16): workgroups of one wave
int g_engine_idle_us = 200;             // rs_tune("host_engine_idle_us")
// Batches up to this many bytes go to the engine, larger ones launch: its
// few workgroups lose to a full-GPU launch past about one 10+4 @ 8 KiB stripe
// (8 threads of 8 KiB calls: 15.2 GiB/s at 128 KiB, 11.0 at 1 MiB,
// profiles/r02/host_concurrency_engine.log).
size_t g_engine_max_bytes = 128u << 10;  // rs_tune("host_engine_max_bytes")
static const bool g_engine_trace = std::getenv("RSAMD_ENGINE_TRACE") != nullptr;

// Doorbell rings are fine-grained (coherent) pinned memory: allocated once
// per process and device and recycled across handles, never freed (no
// allocate / free churn of coherent mappings while other work runs).
namespace {
std::mutex g_ring_mu;
std::vector<std::pair<int, EngineRing*>> g_ring_pool;  // (device, host address) of idle rings
}  // namespace

static EngineRing* ring_get(int device) {
    {
        std::lock_guard<std::mutex> lk(g_ring_mu);
        for (size_t i = 0; i < g_ring_pool.size(); ++i)
            if (g_ring_pool[i].first == device) {
                EngineRing* r = g_ring_pool[i].second;
                g_ring_pool.erase(g_ring_pool.begin() + static_cast<long>(i));
                return r;
            }
    }
    void* h = nullptr;
    if (hipHostMalloc(&h, sizeof(EngineRing), hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable) !=
        hipSuccess)
        return nullptr;
    return static_cast<EngineRing*>(h);
}

static void ring_put(int device, EngineRing* r) {
    std::lock_guard<std::mutex> lk(g_ring_mu);
    g_ring_pool.emplace_back(device, r);
}

void engine_stop(rs_t* rs) {
    if (!rs->eng_running) return;
    __atomic_store_n(&rs->eng_ring->stop, 1, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(rs->eng_stream);  // every wave checks the stop word while polling
    __atomic_store_n(&rs->eng_ring->stop, 0, __ATOMIC_RELEASE);
    rs->eng_running = false;
}

void engine_shutdown(rs_t* rs) {
    std::lock_guard<std::mutex> lk(rs->eng_mu);
    if (!rs->eng_ring) return;
    DeviceGuard g(rs->device);
    engine_stop(rs);
    if (rs->eng_stream) (void)hipStreamDestroy(rs->eng_stream);
    if (!rs->eng_running) ring_put(rs->device, rs->eng_ring);  // (a ring an instance may still read is dropped)
    rs->eng_stream = nullptr;
    rs->eng_ring = rs->eng_dring = nullptr;
}

// The engine's stream must own its hardware queue: HIP maps streams onto a
// few hardware queues, and a resident kernel holds its queue, so kernels of
// any stream sharing it would wait until the engine leaves
// (tools/queue_probe.hip, profiles/r02/queue_probe.log: with the resident
// kernel on a plain stream 2 of 8 other streams stalled for the whole 50 ms
// window; on a CU-masked or a high-priority stream none did).  A CU-masked
// stream (every CU enabled) gets a queue of its own.
static hipStream_t engine_stream() {
    hipStream_t st = nullptr;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                 hipSuccess && cus > 0) {
        std::vector<uint32_t> mask(static_cast<size_t>((cus + 31) / 32), 0);
        for (int c = 0; c < cus; ++c) mask[static_cast<size_t>(c / 32)] |= 1u << (c % 32);
        if (hipExtStreamCreateWithCUMask(&st, static_cast<uint32_t>(mask.size()), mask.data()) == hipSuccess) return st;
    }
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess &&
        hipStreamCreateWithPriority(&st, hipStreamNonBlocking, hi) == hipSuccess)
        return st;
    return nullptr;
}

static int engine_launch(rs_t* rs, int waves, uint64_t start) {
    const uint64_t idle_ticks = static_cast<uint64_t>(g_engine_idle_us) * 100;  // 100 MHz realtime counter
    RS_TRY(hip_ok(launch_engine(rs->eng_dring, waves, start, idle_ticks, rs->eng_stream), "engine launch"));
    rs->eng_running = true;
    rs->eng_waves = waves;
    rs->eng_idle_us = g_engine_idle_us;
    rs->eng_launches.fetch_add(1, std::memory_order_relaxed);
    return RS_OK;
}

int engine_call(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* dev_base, size_t pitch,
                size_t stride, int nstripes, bool accumulate, bool coherent) {
    if (!g_engine || rows < 1 || rows > kEngineMaxRows || cols < 1 || cols > kEngineMaxCols || nstripes < 1 ||
        pitch % 16 || stride % 16 || (reinterpret_cast<uintptr_t>(dev_base) & 15))
        return RS_ERR_INVAL;
    if (stride * static_cast<size_t>(nstripes) > g_engine_max_bytes) return RS_ERR_INVAL;
    const uint64_t units = pitch / 16;
    if (units * static_cast<uint64_t>(nstripes) >= (uint64_t{1} << 31) || pitch >= (size_t{1} << 32))
        return RS_ERR_INVAL;
    const auto t_call = std::chrono::steady_clock::now();
    std::lock_guard<std::mutex> lk(rs->eng_mu);
    if (!rs->eng_ring) {
        EngineRing* h = ring_get(rs->device);
        if (!h) return RS_ERR_NOMEM;
        std::memset(h, 0, sizeof(EngineRing));
        void* d = nullptr;
        const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
        if (e != hipSuccess || !d) {
            ring_put(rs->device, h);
            return dev_fail(e != hipSuccess ? e : hipErrorInvalidValue, "engine ring device pointer");
        }
        hipStream_t st = engine_stream();
        if (!st) {
            ring_put(rs->device, h);
            return dev_fail(hipErrorInvalidValue, "engine stream");
        }
        rs->eng_ring = h;
        rs->eng_dring = static_cast<EngineRing*>(d);
        rs->eng_stream = st;
        rs->eng_seq = 0;
        rs->eng_tab_key.clear();
    }
    EngineRing* ring = rs->eng_ring;
    const int waves = g_engine_waves < 1 ? 1 : g_engine_waves > kEngineMaxWaves ? kEngineMaxWaves : g_engine_waves;
    auto now = std::chrono::steady_clock::now();
    // ring a running instance only well inside ITS idle window (it may have
    // been launched with another host_engine_idle_us)
    if (rs->eng_running && (now - rs->eng_last > std::chrono::microseconds(rs->eng_idle_us) / 2 ||
                            rs->eng_waves != waves || rs->eng_idle_us != g_engine_idle_us))
        engine_stop(rs);
    if (!rs->eng_running) RS_TRY(engine_launch(rs, waves, rs->eng_seq));
    const auto idle = std::chrono::microseconds(rs->eng_idle_us);

    // coefficient tables, [col][kEngineMaxRows][5] (kernel reloads them when tab_id changes)
    const size_t mbytes = static_cast<size_t>(rows) * cols;
    const bool same = rs->eng_tab_key.size() == mbytes + 2 && rs->eng_tab_key[0] == rows &&
                      rs->eng_tab_key[1] == cols && std::memcmp(rs->eng_tab_key.data() + 2, mat, mbytes) == 0;
    if (!same) {
        uint32_t tmp[kEngineMaxCols * kEngineMaxRows * 5] = {};
        for (int c = 0; c < cols; ++c)
            for (int r = 0; r < rows; ++r)
                perm_table(mat[static_cast<size_t>(r) * cols + c], &tmp[(c * kEngineMaxRows + r) * 5]);
        std::memcpy(ring->tables, tmp, static_cast<size_t>(cols) * kEngineMaxRows * 5 * 4);
        rs->eng_tab_key.assign(2, 0);
        rs->eng_tab_key[0] = static_cast<uint8_t>(rows);
        rs->eng_tab_key[1] = static_cast<uint8_t>(cols);
        rs->eng_tab_key.insert(rs->eng_tab_key.end(), mat, mat + mbytes);
        ++rs->eng_tab_id;
    }
    volatile EngineHeader* h = &ring->hdr;
    h->base = reinterpret_cast<uint64_t>(dev_base);
    h->stride = stride;
    h->pitch = static_cast<uint32_t>(pitch);
    h->units = static_cast<uint32_t>(units);
    h->nstripes = static_cast<uint32_t>(nstripes);
    h->rows = static_cast<uint16_t>(rows);
    h->cols = static_cast<uint16_t>(cols);
    h->flags = (accumulate ? 1u : 0u) | (coherent ? 2u : 0u);
    h->tab_id = rs->eng_tab_id;
    const uint64_t seq = ++rs->eng_seq;
    std::atomic_thread_fence(std::memory_order_release);
    __atomic_store_n(&ring->hdr.seq0, seq, __ATOMIC_RELEASE);
    __atomic_store_n(&ring->hdr.seq1, seq, __ATOMIC_RELEASE);

    auto t_ring = std::chrono::steady_clock::now();
    for (int w = 0; w < rs->eng_waves; ++w) {
        uint32_t spins = 0;
        while (__atomic_load_n(&ring->done[w], __ATOMIC_ACQUIRE) != seq) {
            _mm_pause();
            if ((++spins & 4095) != 0) continue;
            now = std::chrono::steady_clock::now();
            if (now - t_ring < idle + std::chrono::milliseconds(1)) continue;
            // the instance may have left before this doorbell (host thread
            // descheduled past the idle window): resume the call in a new one
            const hipError_t q = hipStreamQuery(rs->eng_stream);
            if (q == hipSuccess) {
                rs->eng_running = false;
                RS_TRY(engine_launch(rs, rs->eng_waves, seq - 1));
                t_ring = std::chrono::steady_clock::now();
            } else if (q != hipErrorNotReady) {
                rs->eng_running = false;
                return dev_fail(q, "engine call");
            } else if (now - t_ring > std::chrono::seconds(10)) {
                return dev_fail(hipErrorLaunchTimeOut, "engine call (no completion in 10 s)");
            }
        }
    }
    rs->eng_last = std::chrono::steady_clock::now();
    rs->eng_calls.fetch_add(1, std::memory_order_relaxed);
    if (g_engine_trace) {  // diagnostics: calls slower than 100 us, with where the time went
        const double us = std::chrono::duration<double, std::micro>(rs->eng_last - t_call).count();
        if (us > 100)
            std::fprintf(stderr, "engine slow call: %.1f us total, %.1f us before the doorbell, seq %llu, n %d\n", us,
                         std::chrono::duration<double, std::micro>(t_ring - t_call).count(),
                         static_cast<unsigned long long>(seq), nstripes);
    }
    return RS_OK;
}

}  // namespace detail
}  // namespace rsamd
