// engine.cpp — the host-call engine: small synchronous host calls (the Go
// API's one-stripe Encode / Reconst / Update / Replace on 8 KiB vectors, and
// the coalesced batches of concurrent ones) are served by a resident kernel
// (gf_engine, kernels.hip) through a doorbell in host memory, instead of a
// kernel launch plus a stream synchronisation per call.
//
// Measured on MI355X (round 2's doorbell probe, profiles/r02/doorbell_probe.log):
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
// The kernel leaves on the stop word, after host_engine_idle_us without a
// doorbell (so it never outlives its callers, and never holds a hardware
// queue that other streams share for long), or once it has run
// host_engine_life_us even while calls keep coming (a device-wide
// synchronisation - hipDeviceSynchronize, hipFree, torch.cuda.synchronize -
// waits for a running instance, so that wait is bounded).  The host does not
// predict either exit: it rings the running instance, and a workgroup that
// left before seeing the call shows up in its gone word; the host (at the
// next call, or a waiter) then stops what is left of the instance and
// launches a new one, which resumes the pending calls: workgroups that
// already finished a call (done word) skip it, so no unit is computed twice
// (Update / Replace XOR into their outputs).
#include <immintrin.h>
#include <pthread.h>
#include <unistd.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <map>
#include <condition_variable>
#include <deque>
#include <thread>

#include <hip/hip_ext.h>

#include "codec_internal.hpp"

namespace rsamd {
namespace detail {

int g_engine = [] {                     // rs_tune("host_engine", 0 | 1); env RSAMD_HOST_ENGINE
    const char* e = std::getenv("RSAMD_HOST_ENGINE");
    return e ? (std::atoi(e) ? 1 : 0) : 1;
}();
int g_engine_waves = 8;                 // rs_tune("host_engine_waves", 1..64): workgroups (one polling wave each)
int g_engine_group_waves = 8;           // rs_tune("host_engine_group_waves", 1..8): waves per workgroup
// Idle exit (rs_tune("host_engine_idle_us")).  A call that finds the engine
// gone pays a relaunch (10+4 @ 8 KiB: ~39 us instead of ~11), so the engine
// stays through the gaps of a steadily calling thread: at 200 us a caller
// that checked each result between calls relaunched it on every 16-64 KiB
// call (registered 16 / 32 / 64 KiB Encode 35 / 41 / 49 us against 10.7 /
// 15.3 / 23.0 us at 2 ms; profiles/r04/engine_idle.log).  Device-wide
// synchronisations wait at most host_engine_life_us anyway.
int g_engine_idle_us = 2000;
// Longest life of one instance (rs_tune("host_engine_life_us")): a relaunch
// costs a stream sync and a launch (~20-30 us of stalled calls), so 4 ms
// keeps that under 1 % of a busy engine's time.
int g_engine_life_us = 4000;
// Doorbell polls: 0 = one read per PCIe round trip; n = a second read in
// flight, issued n ticks (10 ns) after the first; rs_tune("host_engine_poll_gap")
int g_engine_poll_gap = [] {  // (env RSAMD_ENGINE_POLL_GAP)
    const char* e = std::getenv("RSAMD_ENGINE_POLL_GAP");
    return e ? std::atoi(e) : 0;
}();
// Call slots (and the pageable calls' input staging, host_calls.cpp) in
// device memory the host writes through the BAR, so that the engine polls and
// reads local memory instead of host memory over PCIe.  Off by default:
// measured slower on MI355X (profiles/r03/host_latency_vram.log, 10+4 @ 8 KiB
// Encode 13.8 us against 11.0 pageable, 9.7 against 9.2 registered): an
// uncached device-memory read round trip is ~2.1 us against ~2.4 us for host
// memory over PCIe (tools/bar_probe.hip, profiles/r03/bar_probe.log), while
// the host's copy of 80 KiB of inputs through the BAR takes 1.5 us against
// 0.55 us into pinned host memory.  Taken by handles whose engine starts after
// the change; rs_tune("host_engine_vram", 0 | 1), env RSAMD_ENGINE_VRAM.
// Platforms that map no device memory for the CPU keep host memory.
int g_engine_vram = [] {
    const char* e = std::getenv("RSAMD_ENGINE_VRAM");
    return e ? (std::atoi(e) ? 1 : 0) : 0;
}();
// Batches up to this many bytes go to the engine, larger ones launch.
size_t g_engine_max_bytes = 1u << 20;  // rs_tune("host_engine_max_bytes")
// 16-byte units per workgroup a call is spread over (0: one per lane of a
// workgroup); rs_tune("host_engine_wg_units")
int g_engine_wg_units = 0;
// A lone call's output rows computed by separate waves of each workgroup
// (1: each wave reads every input; 2: the waves load the inputs once into
// LDS, default, for calls of >= 3 rows and >= 4 columns that one 64-unit group
// per workgroup covers) or all by its first wave (0); rs_tune("host_engine_split_rows").
// 1 measured slower: each wave reads every input over PCIe again (host memory
// is not cached), 10+4 @ 8 KiB Encode 10.8 -> 20.5 us, Reconst of 4 10.9 -> 20.4
// (profiles/r03/host_latency_split_rows.log)
int g_engine_split_rows = 2;
// A call that finds the engine gone (idle exit) and no call pending is served
// by the launch path, and the engine is relaunched while that call's kernel
// runs (engine_warm), instead of the call waiting for the relaunch: ~39 us ->
// the launch path's ~20-25 us for the first call after a quiet period;
// rs_tune("host_engine_cold_launch", 1 default | 0).
int g_engine_cold_launch = 1;
// Waiters spin this long, then yield the core between polls; rs_tune("host_engine_yield_us"), 0 = never
// (default): 8-64 threads on the box measured the same either way and a lone
// caller ~1 us slower with it (profiles/r02/engine_yield.log)
int g_engine_yield_us = 0;
static const bool g_engine_trace = std::getenv("RSAMD_ENGINE_TRACE") != nullptr;
const bool g_phase_trace = g_engine_trace;

namespace {
std::atomic<uint64_t> g_phase_ns[kPhCount];
std::atomic<uint64_t> g_phase_n[kPhCount];
const char* const kPhaseName[kPhCount] = {"join",     "copy_in", "wait_run", "pre_bell", "bell",
                                          "wake",     "copy_out", "gpu_tab", "gpu_work", "gpu_release"};
void phase_report() {
    std::fprintf(stderr, "{\"host_call_phases_mean_us\": {");
    for (int p = 0; p < kPhCount; ++p) {
        const uint64_t n = g_phase_n[p].load();
        std::fprintf(stderr, "%s\"%s\": %.3f", p ? ", " : "", kPhaseName[p], n ? g_phase_ns[p].load() / 1e3 / n : 0.0);
    }
    std::fprintf(stderr, "}, \"calls\": %llu}\n", static_cast<unsigned long long>(g_phase_n[kPhCopyIn].load()));
}
}  // namespace

void phase_add_ns(HostPhase p, uint64_t ns) {
    static const bool registered = [] { return std::atexit(phase_report) == 0; }();
    (void)registered;
    g_phase_ns[p].fetch_add(ns, std::memory_order_relaxed);
    g_phase_n[p].fetch_add(1, std::memory_order_relaxed);
}

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

// ---- coherent pinned blocks, recycled (codec_internal.hpp)
namespace {
std::mutex g_coh_mu;
std::multimap<size_t, std::pair<uint8_t*, void*>> g_coh_free;  // size class -> (host, device) of idle blocks
}  // namespace

uint8_t* coherent_get(size_t bytes, size_t* cap, void** dev) {
    size_t cls = 4096;
    while (cls < bytes) cls <<= 1;
    {
        std::lock_guard<std::mutex> lk(g_coh_mu);
        auto it = g_coh_free.find(cls);
        if (it != g_coh_free.end()) {
            uint8_t* p = it->second.first;
            *dev = it->second.second;
            g_coh_free.erase(it);
            *cap = cls;
            return p;
        }
    }
    void* h = nullptr;
    if (hipHostMalloc(&h, cls, hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
        (void)hipGetLastError();
        d = nullptr;
    }
    *dev = d;
    *cap = cls;
    return static_cast<uint8_t*>(h);
}

void coherent_put(uint8_t* p, size_t cap) {
    if (!p) return;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
        (void)hipGetLastError();
        d = nullptr;
    }
    std::lock_guard<std::mutex> lk(g_coh_mu);
    g_coh_free.emplace(cap, std::make_pair(p, d));
}

// ---- device memory the host writes through the BAR
namespace {
std::mutex g_vram_mu;
std::multimap<std::pair<int, size_t>, uint8_t*> g_vram_free;  // (device, size class) -> idle blocks
std::vector<int> g_vram_state;                                // per device: 0 unknown, 1 usable, 2 not mapped for the CPU
}  // namespace

// Can this process read and write [p, p + 8) from the CPU?  Asked of the
// kernel through a pipe (EFAULT instead of a signal when it is not mapped).
static bool cpu_can_access(void* p) {
    int fd[2];
    if (pipe(fd) != 0) return false;
    const uint64_t probe = 0x5253414d44564d31ull;
    uint64_t back = 0;
    bool ok = write(fd[1], &probe, 8) == 8 && read(fd[0], p, 8) == 8;  // the kernel stores into p
    ok = ok && write(fd[1], p, 8) == 8 && read(fd[0], &back, 8) == 8 && back == probe;  // ... and loads from it
    close(fd[0]);
    close(fd[1]);
    return ok;
}

uint8_t* host_writable_vram_get(int device, size_t bytes, size_t* cap) {
    size_t cls = size_t{64} << 10;
    while (cls < bytes) cls <<= 1;
    std::lock_guard<std::mutex> lk(g_vram_mu);
    if (device < 0) return nullptr;
    if (g_vram_state.size() <= static_cast<size_t>(device)) g_vram_state.resize(static_cast<size_t>(device) + 1, 0);
    if (g_vram_state[static_cast<size_t>(device)] == 2) return nullptr;
    auto it = g_vram_free.find({device, cls});
    if (it != g_vram_free.end()) {
        uint8_t* p = it->second;
        g_vram_free.erase(it);
        *cap = cls;
        return p;
    }
    void* d = nullptr;
    Region region("hipExtMallocWithFlags (host-writable device block)");
    if (hipExtMallocWithFlags(&d, cls, hipDeviceMallocUncached) != hipSuccess || !d) {
        (void)hipGetLastError();
        return nullptr;
    }
    uint8_t* p = static_cast<uint8_t*>(d);
    if (g_vram_state[static_cast<size_t>(device)] == 0) {
        const bool ok = cpu_can_access(p) && cpu_can_access(p + cls - 8);
        g_vram_state[static_cast<size_t>(device)] = ok ? 1 : 2;
        if (!ok) {
            (void)hipFree(d);
            return nullptr;
        }
    }
    *cap = cls;
    return p;
}

void host_writable_vram_put(int device, uint8_t* p, size_t cap) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_vram_mu);
    g_vram_free.emplace(std::make_pair(device, cap), p);
}

static EngineSlot* slots_of(rs_t* rs) { return rs->eng_vslots ? rs->eng_vslots : rs->eng_ring->slot; }
static size_t vslots_cap() {
    size_t cls = size_t{64} << 10;
    while (cls < sizeof(EngineSlot) * kEngineSlots) cls <<= 1;
    return cls;
}

static void engine_dump(const rs_t* rs, const char* what) {  // diagnostics
    const EngineRing* r = rs->eng_ring;
    std::fprintf(stderr, "engine %s: epoch %llu seq %llu running %d waves %d | done/gone:", what,
                 static_cast<unsigned long long>(rs->eng_epoch), static_cast<unsigned long long>(rs->eng_seq),
                 rs->eng_running ? 1 : 0, rs->eng_waves);
    for (int w = 0; w < rs->eng_waves; ++w)
        std::fprintf(stderr, " %llu/%llu", static_cast<unsigned long long>(r->done[w]),
                     static_cast<unsigned long long>(r->gone[w]));
    std::fprintf(stderr, "\n");
}

static void signal_stop(EngineSlot* slots, uint64_t epoch) {  // every slot: a wave polls whichever holds its next call
    for (int i = 0; i < kEngineSlots; ++i) __atomic_store_n(&slots[i].hdr.stop, epoch, __ATOMIC_RELEASE);
    _mm_sfence();  // (device-memory slots: write-combined stores leave now)
}

static void engine_signal_stop(rs_t* rs) { signal_stop(slots_of(rs), rs->eng_epoch); }

// Running instances of every handle (slots, epoch), so that the library's own
// device-wide drains (rs_host_unregister, the table registry's recycle, JIT
// eviction) can ask them to leave first instead of waiting out their idle
// window (up to host_engine_idle_us, 2 ms).  Taken after eng_mu, never
// before it.  A stop word written this way is an ordinary early exit for the
// handle: calls already rung are served first, and the next call finds the
// instance gone and relaunches it (engine_relaunch_if_gone).  Slots are never
// freed (rings and device slot blocks are pooled), so a stale entry can only
// cost another instance an early exit, never a stray write.
namespace {
std::mutex g_active_mu;
std::map<EngineSlot*, uint64_t> g_active;  // running instance's slots -> its epoch
}  // namespace

static void active_set(rs_t* rs, bool running) {
    std::lock_guard<std::mutex> lk(g_active_mu);
    if (running) g_active[slots_of(rs)] = rs->eng_epoch;
    else g_active.erase(slots_of(rs));
}

void engines_quiesce() {
    std::lock_guard<std::mutex> lk(g_active_mu);
    for (auto& kv : g_active) signal_stop(kv.first, kv.second);
}

// Caller holds eng_mu.  Calls already rung are served first (a wave checks
// its slot's call number before the stop word).
void engine_stop(rs_t* rs) {
    if (!rs->eng_running) return;
    engine_signal_stop(rs);
    Region region("engine stop (instance leaving)");
    // Watch the gone words (host memory, no runtime calls) until every
    // workgroup of the latest instance has left, then one stream sync.
    // (A busy loop of hipStreamQuery here left the process hanging in the
    // runtime's teardown at exit, 1 run in 8: profiles/r02/exit_hang.log.)
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spins = 0;; ++spins) {
        bool all = true;
        for (int w = 0; w < rs->eng_waves && all; ++w)
            all = __atomic_load_n(&rs->eng_ring->gone[w], __ATOMIC_ACQUIRE) == rs->eng_epoch;
        if (all) break;
        _mm_pause();
        if ((spins & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
            engine_dump(rs, "stop: workgroups still running after 1 s; waiting on the stream");
            break;
        }
    }
    (void)hipStreamSynchronize(rs->eng_stream);
    rs->eng_running = false;
    active_set(rs, false);
}

// ---- the warmer: relaunches engines that a cold call declined, off the
// caller's thread (engine_warm_async).  One thread per process, started at
// the first request and joined by an exit handler registered then (after the
// HIP runtime was loaded, so it runs before the runtime's own teardown).
namespace {
struct Warmer {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<rs_t*> q;
    rs_t* cur = nullptr;  // the handle being warmed (engine_shutdown waits for it)
    bool stop = false;
    std::thread th;
    pid_t owner = 0;
};
// Never destroyed (see jit.cpp's Jit).  A forked child inherits the object
// but not the thread, possibly with `mu` held by it at the fork, and a queue
// of the parent's handles: its pthread_atfork handler gives the child a fresh
// Warmer (the inherited one is left alone; advisor r05).
Warmer* g_warmer = nullptr;
void warmer_fork_child() { g_warmer = new Warmer; }
Warmer& warmer() {
    static const bool init = [] {
        g_warmer = new Warmer;
        return pthread_atfork(nullptr, nullptr, warmer_fork_child) == 0;
    }();
    (void)init;
    return *g_warmer;
}
void warmer_atexit() {
    Warmer& w = warmer();
    {
        std::lock_guard<std::mutex> lk(w.mu);
        if (!w.th.joinable() || w.owner != getpid()) return;
        w.stop = true;
    }
    w.cv.notify_all();
    w.th.join();
}
void warmer_loop() {
    Warmer& w = warmer();
    std::unique_lock<std::mutex> lk(w.mu);
    for (;;) {
        w.cv.wait(lk, [&] { return w.stop || !w.q.empty(); });
        if (w.stop) return;
        rs_t* rs = w.q.front();
        w.q.pop_front();
        w.cur = rs;
        lk.unlock();
        {
            DeviceGuard g(rs->device);
            engine_warm(rs, true);
        }
        lk.lock();
        w.cur = nullptr;
        w.cv.notify_all();
    }
}
}  // namespace

void engine_warm_async(rs_t* rs) {
    if (!rs->eng_warm_wanted.load(std::memory_order_acquire)) return;
    Warmer& w = warmer();
    std::lock_guard<std::mutex> lk(w.mu);
    if (w.stop) return;
    if (w.cur != rs && std::find(w.q.begin(), w.q.end(), rs) == w.q.end()) w.q.push_back(rs);
    if (!w.th.joinable()) {  // (a forked child's fresh Warmer starts its own)
        static const bool registered = std::atexit(warmer_atexit) == 0;
        (void)registered;
        w.owner = getpid();
        w.th = std::thread(warmer_loop);
    }
    w.cv.notify_one();
}

void engine_shutdown(rs_t* rs) {
    {  // no warm of this handle queued or running past this point
        Warmer& w = warmer();
        std::unique_lock<std::mutex> wl(w.mu);
        w.q.erase(std::remove(w.q.begin(), w.q.end(), rs), w.q.end());
        w.cv.wait(wl, [&] { return w.cur != rs; });
    }
    std::lock_guard<std::mutex> lk(rs->eng_mu);
    if (!rs->eng_ring) return;
    DeviceGuard g(rs->device);
    engine_stop(rs);
    if (rs->eng_stream) (void)hipStreamDestroy(rs->eng_stream);
    if (!rs->eng_running) {  // (a ring an instance may still read is dropped)
        ring_put(rs->device, rs->eng_ring);
        if (rs->eng_vslots) host_writable_vram_put(rs->device, reinterpret_cast<uint8_t*>(rs->eng_vslots), vslots_cap());
    }
    rs->eng_stream = nullptr;
    rs->eng_ring = rs->eng_dring = nullptr;
    rs->eng_vslots = nullptr;
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

// Oldest call some workgroup of the latest instance's shape has not completed
// yet, minus one (= eng_seq when every rung call is complete).
static uint64_t engine_low_done(const rs_t* rs) {
    uint64_t lo = rs->eng_seq;
    for (int w = 0; w < rs->eng_waves; ++w)
        lo = std::min<uint64_t>(lo, __atomic_load_n(&rs->eng_ring->done[w], __ATOMIC_ACQUIRE));
    return lo;
}

// Caller holds eng_mu; no instance is running.  `start` <= every done word of
// the workgroups [0, rs->eng_waves) of the previous shape (a relaunch passes
// their minimum; a new shape is launched only after engine_drain, when all of
// them equal eng_seq).
static int engine_launch(rs_t* rs, int waves, int group_waves, uint64_t start) {
    const uint64_t idle_ticks = static_cast<uint64_t>(g_engine_idle_us) * 100;  // 100 MHz realtime counter
    const uint64_t life_ticks = static_cast<uint64_t>(g_engine_life_us) * 100;
    const uint64_t epoch = rs->eng_epoch + 1;
    Region region("engine launch");
    // Every workgroup of the new instance starts after max(call `start`, its
    // own done word).  A workgroup the previous shape did not have
    // (host_engine_waves raised) may hold a stale done word from an older
    // instance: every call rung since was served by the previous shape's
    // workgroups alone (calls name workgroups of their own instance's grid),
    // so bring it to `start` here, so the slot-reuse wait and a later relaunch
    // (min over done words) never wait on a call that workgroup will never
    // see.  Workgroups of the previous shape keep their done words: one that
    // left before a call reached it resumes at that call (raising its word
    // would report the call complete with its units never written).  No
    // instance runs: the host is the only writer.
    const int prev = rs->eng_ring ? rs->eng_waves : 0;
    for (int w = prev; w < waves; ++w)
        if (__atomic_load_n(&rs->eng_ring->done[w], __ATOMIC_ACQUIRE) < start)
            __atomic_store_n(&rs->eng_ring->done[w], start, __ATOMIC_RELEASE);
    RS_TRY(hip_ok(launch_engine(rs->eng_dring, rs->eng_vslots, waves, group_waves, start, epoch, idle_ticks,
                                life_ticks, static_cast<uint32_t>(g_engine_poll_gap), rs->eng_stream),
                  "engine launch"));
    if (g_engine_trace) std::fprintf(stderr, "engine launch: epoch %llu start %llu\n",
                                     static_cast<unsigned long long>(epoch), static_cast<unsigned long long>(start));
    __atomic_store_n(&rs->eng_epoch, epoch, __ATOMIC_RELEASE);  // (waiters read it without eng_mu)
    rs->eng_running = true;
    rs->eng_waves = waves;
    rs->eng_group_waves = group_waves;
    rs->eng_idle_us = g_engine_idle_us;
    rs->eng_life_us = g_engine_life_us;
    rs->eng_poll_gap = g_engine_poll_gap;
    rs->eng_launches.fetch_add(1, std::memory_order_relaxed);
    active_set(rs, true);
    return RS_OK;
}

// Some workgroup of the running instance left (idle window): the rest leave
// too (stop word), and once the instance is off the stream a new one starts;
// each of its workgroups resumes after its own done word.  Never launch
// behind a running instance: with kernels queued that way (or a
// hipStreamQuery while one runs) the runtime's teardown deadlocked at
// process exit, 1 run in 3 (profiles/r02/exit_hang.log).  Caller holds eng_mu.
static int engine_relaunch_if_gone(rs_t* rs) {
    if (!rs->eng_running) return RS_OK;
    bool gone = false;
    for (int w = 0; w < rs->eng_waves && !gone; ++w)
        gone = __atomic_load_n(&rs->eng_ring->gone[w], __ATOMIC_ACQUIRE) == rs->eng_epoch;
    if (!gone) return RS_OK;
    if (g_engine_trace) engine_dump(rs, "gone");
    engine_stop(rs);
    uint64_t start = ~uint64_t{0};
    for (int w = 0; w < rs->eng_waves; ++w) start = std::min<uint64_t>(start, rs->eng_ring->done[w]);
    return engine_launch(rs, rs->eng_waves, rs->eng_group_waves, start);
}

namespace {
struct EngineWork {
    const uint8_t* mat;
    int rows, cols;
    const uint8_t* base;           // batch mode: vector i of stripe s at base + s * stride + i * pitch
    size_t pitch, stride;
    int nstripes;
    const uint8_t* const* addr;    // address mode (one stripe): vector i at addr[i] (cols inputs, rows outputs)
    size_t units;                  // 16-byte units per vector
    bool accumulate, coherent;
};
}  // namespace

// Workgroups [w0, w0 + n) (mod waves) all past call `seq`.
static bool all_done(const EngineRing* r, int waves, int w0, int n, uint64_t seq) {
    for (int i = 0; i < n; ++i)
        if (__atomic_load_n(&r->done[(w0 + i) % waves], __ATOMIC_ACQUIRE) < seq) return false;
    return true;
}

// A call not complete after 10 s.  The instance is stopped before the error
// is returned (workgroups serve the calls already rung before they read the
// stop word, and the stream is synchronised), so once the caller has the
// error the GPU can no longer write into the buffers it hands back (pinned
// pool blocks, registered caller memory).  The handle's engine is then
// retired: its later calls take the launch paths.
static int engine_timeout(rs_t* rs, bool locked) {
    std::unique_lock<std::mutex> lk(rs->eng_mu, std::defer_lock);
    if (!locked) lk.lock();
    engine_dump(rs, "no completion in 10 s; stopping the instance and retiring the handle's engine");
    engine_stop(rs);
    rs->eng_failed = true;
    return dev_fail(hipErrorLaunchTimeOut, "engine call (no completion in 10 s)");
}

// Wait until workgroups [w0, w0 + n) completed call `seq`: spin (calls take
// ~10 us), relaunching the engine if a workgroup left before the call reached
// it.  `locked`: the caller holds eng_mu (slot reuse wait); otherwise it is
// taken only for a relaunch.
static int engine_wait(rs_t* rs, uint64_t seq, int waves, int w0, int n, bool locked) {
    Region region(locked ? "engine wait (slot reuse)" : "engine wait (call)");
    const EngineRing* r = rs->eng_ring;
    auto t0 = std::chrono::steady_clock::now();
    bool yielding = false;
    for (uint32_t spins = 1; !all_done(r, waves, w0, n, seq); ++spins) {
        // A call waited on this long (an 8 KiB call takes ~10 us) is queued
        // behind others: give the core to threads that copy (with more callers
        // than cores, spinning waiters starved the copiers).
        if (yielding) std::this_thread::yield();
        else _mm_pause();
        if ((spins & 63) != 0) continue;
        if (!yielding && g_engine_yield_us > 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(g_engine_yield_us))
            yielding = true;
        bool gone = false;
        for (int w = 0; w < waves && !gone; ++w)
            gone = __atomic_load_n(&r->done[w], __ATOMIC_ACQUIRE) < seq &&
                   __atomic_load_n(&r->gone[w], __ATOMIC_ACQUIRE) == __atomic_load_n(&rs->eng_epoch, __ATOMIC_ACQUIRE);
        if (gone) {
            std::unique_lock<std::mutex> lk(rs->eng_mu, std::defer_lock);
            if (!locked) lk.lock();
            RS_TRY(engine_relaunch_if_gone(rs));  // (no-op when another waiter already relaunched)
        }
        if ((spins & 4095) != 0) continue;
        // (no runtime calls while an instance runs: a hipStreamQuery here
        // left the runtime's teardown deadlocked at process exit; a faulting
        // instance ends the process through the runtime's fault handler)
        const auto now = std::chrono::steady_clock::now();
        if (now - t0 > std::chrono::seconds(10)) return engine_timeout(rs, locked);
    }
    return RS_OK;
}

// Caller holds eng_mu.  Every call rung so far completed by every workgroup,
// on the shape it was rung for (calls name workgroups of their instance's
// grid, so another shape cannot serve them): the instance is relaunched with
// the same shape if it is gone or stopped while calls are pending.  Needed
// before any engine_stop that is not followed by a relaunch of the same shape
// (a new shape, the table registry's recycle): without it a workgroup that
// left before a pending call reached it would never serve that call.
int engine_drain(rs_t* rs) {
    if (!rs->eng_ring || rs->eng_waves <= 0 || engine_low_done(rs) >= rs->eng_seq) return RS_OK;
    if (!rs->eng_running) RS_TRY(engine_launch(rs, rs->eng_waves, rs->eng_group_waves, engine_low_done(rs)));
    return engine_wait(rs, rs->eng_seq, rs->eng_waves, 0, rs->eng_waves, true);
}

static void engine_shape(int* waves, int* gwaves) {
    *waves = g_engine_waves < 1 ? 1 : g_engine_waves > kEngineMaxGroups ? kEngineMaxGroups : g_engine_waves;
    *gwaves = g_engine_group_waves < 1                      ? 1
              : g_engine_group_waves > kEngineMaxGroupWaves ? kEngineMaxGroupWaves
                                                            : g_engine_group_waves;
}

// The knobs changed since the latest instance started (caller holds eng_mu).
static bool engine_reshape(const rs_t* rs, int waves, int gwaves) {
    return rs->eng_waves > 0 &&
           (rs->eng_waves != waves || rs->eng_group_waves != gwaves || rs->eng_idle_us != g_engine_idle_us ||
            rs->eng_life_us != g_engine_life_us || rs->eng_poll_gap != g_engine_poll_gap);
}

static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Caller holds eng_mu.  An instance ran before, none is serving now, every
// call rung so far is complete, and the handle has been quiet for at least
// the idle window: a sporadic caller, whose call would wait for a relaunch.
// (An instance that left at the end of its life while calls keep coming is
// relaunched by the next call as before: that caller pays ~the launch path's
// time anyway, and the calls behind it find the engine.)
static bool engine_cold(const rs_t* rs) {
    if (rs->eng_waves <= 0 || engine_low_done(rs) < rs->eng_seq) return false;
    if (now_ns() - rs->eng_last_ns.load(std::memory_order_relaxed) < int64_t{1000} * rs->eng_idle_us) return false;
    if (!rs->eng_running) return true;
    for (int w = 0; w < rs->eng_waves; ++w)
        if (__atomic_load_n(&rs->eng_ring->gone[w], __ATOMIC_ACQUIRE) == rs->eng_epoch) return true;
    return false;
}

bool engine_cold_now(rs_t* rs) {
    if (!g_engine_cold_launch || !g_engine) return false;
    // (a busy handle answers without the lock: its last call is recent)
    if (now_ns() - rs->eng_last_ns.load(std::memory_order_relaxed) < int64_t{1000} * g_engine_idle_us) return false;
    std::lock_guard<std::mutex> lk(rs->eng_mu);
    int waves, gwaves;
    engine_shape(&waves, &gwaves);
    return !rs->eng_failed && rs->eng_ring && !engine_reshape(rs, waves, gwaves) && engine_cold(rs);
}

void engine_warm(rs_t* rs, bool wait_lock) {
    if (!rs->eng_warm_wanted.load(std::memory_order_acquire)) return;
    std::unique_lock<std::mutex> lk(rs->eng_mu, std::defer_lock);
    if (wait_lock) lk.lock();
    else if (!lk.try_lock()) return;  // a call holds it: that call (re)launches the engine itself
    if (!rs->eng_warm_wanted.exchange(false, std::memory_order_acq_rel)) return;
    if (rs->eng_failed || !rs->eng_ring) return;
    Region region("engine warm (relaunch behind a launch-path call)");
    int waves, gwaves;
    engine_shape(&waves, &gwaves);
    if (engine_reshape(rs, waves, gwaves)) return;  // the next engine call reshapes it
    if (engine_relaunch_if_gone(rs) != RS_OK) return;
    if (!rs->eng_running && engine_drain(rs) == RS_OK && !rs->eng_running)
        (void)engine_launch(rs, waves, gwaves, rs->eng_seq);
}

static int engine_run(rs_t* rs, const EngineWork& wk) {
    const int rows = wk.rows, cols = wk.cols;
    const auto t_call = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(rs->eng_mu, std::defer_lock);
    {
        Region region("engine submit lock");
        lk.lock();
    }
    if (rs->eng_failed) return RS_ERR_INVAL;  // retired after a timeout: the caller launches instead
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
        rs->eng_vslots = nullptr;
        if (g_engine_vram) {
            size_t cap = 0;
            if (uint8_t* v = host_writable_vram_get(rs->device, sizeof(EngineSlot) * kEngineSlots, &cap)) {
                std::memset(v, 0, sizeof(EngineSlot) * kEngineSlots);
                _mm_sfence();
                rs->eng_vslots = reinterpret_cast<EngineSlot*>(v);
            }
        }
        rs->eng_seq = 0;
        rs->eng_epoch = 0;
        rs->eng_tab_key.clear();
        for (uint32_t& t : rs->eng_slot_tab) t = 0;
    }
    EngineRing* ring = rs->eng_ring;
    int waves, gwaves;
    engine_shape(&waves, &gwaves);
    const bool reshape = engine_reshape(rs, waves, gwaves);
    if (g_engine_cold_launch && !reshape && engine_cold(rs)) {
        // idle exit with nothing pending: this call takes the launch path and
        // the engine restarts behind it (engine_warm), for the calls that follow
        rs->eng_warm_wanted.store(true, std::memory_order_release);
        return RS_ERR_INVAL;
    }
    if (reshape) {
        // new shape: the calls in flight finish on the old one, and the old
        // instance is gone before the next one reads done words
        RS_TRY(engine_drain(rs));
        engine_stop(rs);
    }
    RS_TRY(engine_relaunch_if_gone(rs));
    if (!rs->eng_running) {
        RS_TRY(engine_drain(rs));  // (a stopped instance with calls pending relaunches on its own shape)
        if (!rs->eng_running) RS_TRY(engine_launch(rs, waves, gwaves, rs->eng_seq));
    }
    const int inst_waves = rs->eng_waves;

    const uint64_t seq = rs->eng_seq + 1;
    EngineSlot* slot = &slots_of(rs)[seq % kEngineSlots];
    if (seq > static_cast<uint64_t>(kEngineSlots))  // the slot's previous call must be past every workgroup
        RS_TRY(engine_wait(rs, seq - kEngineSlots, inst_waves, 0, inst_waves, true));
    rs->eng_seq = seq;
    // The call's workgroups, rotating.  A lone call (none other in flight)
    // spreads over every workgroup's first wave: more loads over PCIe in
    // flight at once (10+4 @ 8 KiB Encode 16.0 -> 11.0 us pageable, 14.0 ->
    // 9.5 us registered, profiles/r02/engine_s.log).  Calls that overlap
    // others take one unit per lane of one workgroup, so concurrent calls run
    // on different workgroups (8 threads: 29 GiB/s against 14 when every call
    // spreads).  rs_tune("host_engine_wg_units", n) fixes n units per workgroup.
    const bool lone = rs->eng_inflight.load(std::memory_order_acquire) == 0;
    const uint64_t per_wg = g_engine_wg_units > 0 ? static_cast<uint64_t>(g_engine_wg_units)
                            : lone                ? uint64_t{64}
                                                  : static_cast<uint64_t>(64 * rs->eng_group_waves);
    const uint64_t total = wk.units * static_cast<uint64_t>(wk.nstripes);
    const int nwg = static_cast<int>(std::min<uint64_t>(inst_waves, (total + per_wg - 1) / per_wg));
    const int wg0 = rs->eng_next_wg % inst_waves;
    rs->eng_next_wg = (wg0 + nwg) % inst_waves;

    // coefficient tables, [col][kEngineMaxRows][5]; tab_id names the matrix
    const size_t mbytes = static_cast<size_t>(rows) * cols;
    const bool same = rs->eng_tab_key.size() == mbytes + 2 && rs->eng_tab_key[0] == rows &&
                      rs->eng_tab_key[1] == cols && std::memcmp(rs->eng_tab_key.data() + 2, wk.mat, mbytes) == 0;
    if (!same) {
        rs->eng_tab_key.assign(2, 0);
        rs->eng_tab_key[0] = static_cast<uint8_t>(rows);
        rs->eng_tab_key[1] = static_cast<uint8_t>(cols);
        rs->eng_tab_key.insert(rs->eng_tab_key.end(), wk.mat, wk.mat + mbytes);
        ++rs->eng_tab_id;
    }
    uint32_t& slot_tab = rs->eng_slot_tab[seq % kEngineSlots];
    if (slot_tab != rs->eng_tab_id) {
        uint32_t tmp[kEngineMaxCols * kEngineMaxRows * 5] = {};
        for (int c = 0; c < cols; ++c)
            for (int r = 0; r < rows; ++r)
                perm_table(wk.mat[static_cast<size_t>(r) * cols + c], &tmp[(c * kEngineMaxRows + r) * 5]);
        std::memcpy(slot->tables, tmp, static_cast<size_t>(cols) * kEngineMaxRows * 5 * 4);
        slot_tab = rs->eng_tab_id;
    }
    if (wk.addr) {  // address lines, each tagged with this call's number
        const int nv = rows + cols;
        for (int l = 0; l < (nv + 6) / 7; ++l) {
            volatile uint64_t* line = slot->ptr[l];
            for (int j = 0; j < 7 && 7 * l + j < nv; ++j) line[j] = reinterpret_cast<uint64_t>(wk.addr[7 * l + j]);
            line[7] = seq;
        }
    }
    volatile EngineHeader* h = &slot->hdr;
    h->base = reinterpret_cast<uint64_t>(wk.base);
    h->stride = wk.stride;
    h->pitch = static_cast<uint32_t>(wk.pitch);
    h->units = static_cast<uint32_t>(wk.units);
    h->nstripes = static_cast<uint32_t>(wk.nstripes);
    h->rows = static_cast<uint16_t>(rows);
    h->cols = static_cast<uint16_t>(cols);
    // a lone call with all its units on the workgroups' first waves also
    // spreads its rows over their waves (host_engine_split_rows)
    // (mode 2, the inputs read once into LDS: only where one group of 64 units
    // per workgroup covers the call and there are enough rows and columns to
    // share - 10+4 @ 8 KiB Encode 11.1 -> 10.5 us pageable, 9.7 -> 8.8
    // registered; 64 KiB calls and 1-2-column Update / Replace were slower,
    // profiles/r04/engine_shared_rows.log)
    const bool split = g_engine_split_rows && lone && per_wg == 64 && rows > 1 && rows <= rs->eng_group_waves &&
                       (g_engine_split_rows != 2 ||
                        (rows >= 3 && cols >= 4 && total <= uint64_t{64} * static_cast<uint64_t>(inst_waves)));
    h->flags = (wk.accumulate ? 1u : 0u) | (wk.coherent ? 2u : 0u) | (g_engine_trace ? 4u : 0u) | (wk.addr ? 8u : 0u) |
               (split ? (g_engine_split_rows == 2 ? 32u : 16u) : 0u) | (static_cast<uint32_t>(wg0) << 8) |
               (static_cast<uint32_t>(nwg) << 16);
    h->tab_id = rs->eng_tab_id;
    // (write-combined device-memory slots and staging blocks: sfence makes
    // every store before it visible first, tables, addresses and inputs
    // included; for host memory it costs nothing measurable)
    _mm_sfence();
    __atomic_store_n(&slot->hdr.seq0, seq, __ATOMIC_RELEASE);
    __atomic_store_n(&slot->hdr.seq1, seq, __ATOMIC_RELEASE);
    _mm_sfence();
    rs->eng_inflight.fetch_add(1, std::memory_order_acq_rel);
    lk.unlock();

    const auto t_ring = std::chrono::steady_clock::now();
    const int wrc = engine_wait(rs, seq, inst_waves, wg0, nwg, false);
    rs->eng_inflight.fetch_sub(1, std::memory_order_acq_rel);
    rs->eng_last_ns.store(now_ns(), std::memory_order_relaxed);
    RS_TRY(wrc);
    const auto t_done = std::chrono::steady_clock::now();
    rs->eng_calls.fetch_add(1, std::memory_order_relaxed);
    if (g_engine_trace) {  // diagnostics: calls slower than 100 us, with where the time went
        phase_add(kPhPreBell, t_call, t_ring);
        phase_add(kPhBell, t_ring, t_done);
        // workgroup 0's stamps land just after its done word (bounded wait; other calls may overwrite them)
        for (int i = 0; i < 100000 && __atomic_load_n(&ring->stamp[4], __ATOMIC_ACQUIRE) != seq; ++i) _mm_pause();
        if (__atomic_load_n(&ring->stamp[4], __ATOMIC_ACQUIRE) == seq) {
            uint64_t st[4];
            for (int i = 0; i < 4; ++i) st[i] = __atomic_load_n(&ring->stamp[i], __ATOMIC_ACQUIRE);
            if (__atomic_load_n(&ring->stamp[4], __ATOMIC_ACQUIRE) == seq) {
                phase_add_ns(kPhGpuTab, (st[1] - st[0]) * 10);
                phase_add_ns(kPhGpuWork, (st[2] - st[1]) * 10);
                phase_add_ns(kPhGpuRel, (st[3] - st[2]) * 10);
            }
        }
        const double us = std::chrono::duration<double, std::micro>(t_done - t_call).count();
        if (us > 100)
            std::fprintf(stderr, "engine slow call: %.1f us total, %.1f us before the doorbell, seq %llu, n %d\n", us,
                         std::chrono::duration<double, std::micro>(t_ring - t_call).count(),
                         static_cast<unsigned long long>(seq), wk.nstripes);
    }
    return RS_OK;
}

static bool engine_shape_ok(int rows, int cols) {
    return g_engine && rows >= 1 && rows <= kEngineMaxRows && cols >= 1 && cols <= kEngineMaxCols;
}

bool engine_accepts(int rows, int cols, size_t bytes) {
    return engine_shape_ok(rows, cols) && bytes <= g_engine_max_bytes;
}

int engine_call(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* dev_base, size_t pitch,
                size_t stride, int nstripes, bool accumulate, bool coherent) {
    if (!engine_shape_ok(rows, cols) || nstripes < 1 || pitch % 16 || stride % 16 ||
        (reinterpret_cast<uintptr_t>(dev_base) & 15))
        return RS_ERR_INVAL;
    if (stride * static_cast<size_t>(nstripes) > g_engine_max_bytes) return RS_ERR_INVAL;
    const uint64_t units = pitch / 16;
    if (units * static_cast<uint64_t>(nstripes) >= (uint64_t{1} << 31) || pitch >= (size_t{1} << 32))
        return RS_ERR_INVAL;
    EngineWork wk{mat, rows, cols, dev_base, pitch, stride, nstripes, nullptr, units, accumulate, coherent};
    return engine_run(rs, wk);
}

int engine_call_addr(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* in, uint8_t* const* out,
                     size_t size, bool accumulate) {
    if (!engine_shape_ok(rows, cols) || size == 0 || size % 16 ||
        size * static_cast<size_t>(rows + cols) > g_engine_max_bytes)
        return RS_ERR_INVAL;
    const uint8_t* addr[kEngineMaxCols + kEngineMaxRows];
    for (int i = 0; i < cols + rows; ++i) {
        addr[i] = i < cols ? in[i] : out[i - cols];
        if (reinterpret_cast<uintptr_t>(addr[i]) & 15) return RS_ERR_INVAL;
    }
    EngineWork wk{mat, rows, cols, nullptr, 0, 0, 1, addr, size / 16, accumulate, false};
    return engine_run(rs, wk);
}

}  // namespace detail
}  // namespace rsamd
