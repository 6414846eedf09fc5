// codec_internal.hpp — internals shared by librsamd's host-side sources:
//   codec.cpp         handle, matrices, inverse cache, checks, planning, small ABI
//   host_calls.cpp    the synchronous host-memory calls (rs_encode ... rs_replace)
//   batches.cpp       device-resident single-stripe and batched calls
//   host_batches.cpp  host-resident batches, zero-copy, device groups
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/rs_amd.h"
#include "gf256.hpp"
#include "kernels.hpp"
#include "watchdog.hpp"

#define RS_TRY(x)                 \
    do {                          \
        int rc_ = (x);            \
        if (rc_) return rc_;      \
    } while (0)

namespace rsamd {
namespace detail {

constexpr int kMaxVects = 256;                              // rs.go:47
constexpr uint64_t kMaxInverseCacheBytes = 16ull << 20;     // rs.go:50
extern size_t g_registry_max;  // coefficient-table registry cap (distinct matrices per handle)
extern size_t g_tab_inplace_max;  // launches up to this many input bytes read a new matrix's tables in place
extern int g_tab_stage_vram;      // table staging slots in host-writable device memory when the platform maps it

// Record which HIP call failed (thread-local, read by rs_last_device_error)
// and return RS_ERR_DEVICE.
int dev_fail(hipError_t e, const char* where);
// RS_OK, or dev_fail(e, where) when the HIP call failed.
inline int hip_ok(hipError_t e, const char* where) { return e == hipSuccess ? RS_OK : dev_fail(e, where); }

// ---------------------------------------------------------------- device helpers

struct DeviceGuard {  // switch to the handle's device, restore the caller's on exit
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) return;
        ok = (prev == dev) || hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (ok && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

inline uint64_t rup(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// Process-wide pool of pinned host blocks, mapped for every device
// (host_calls.cpp).  Blocks are recycled across handles and never freed, so
// pinned mappings are not created and torn down while other work runs;
// sizes are rounded up to a power of two (>= 64 KiB).
struct PinnedBlock {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;   // device address (same for every device with unified addressing)
    size_t bytes = 0;
};
int pinned_get(size_t bytes, PinnedBlock* out);
void pinned_put(PinnedBlock& b);


}  // namespace detail
}  // namespace rsamd

// ---------------------------------------------------------------- the handle

struct rs_codec {
    int d = 0, p = 0;
    std::vector<uint8_t> enc;  // (d+p) x d; GenMatrix = enc[d*d:]   rs.go:30-31,65-68

    // inverse cache rs.go:33-39,70-74
    bool cache_enabled = false;
    uint64_t cache_max = 0;
    std::atomic<uint64_t> cache_n{0};
    std::mutex cache_mu;
    std::unordered_map<uint64_t, std::vector<uint8_t>> cache;
    // codes beyond 64 vectors (no reference cache, rs.go:70-74): the combined
    // Reconst matrices of recent patterns, keyed by the survivor and need
    // bitmaps (codec.cpp combined_matrix; bounded, cleared when full)
    std::mutex wide_mu;
    std::unordered_map<std::string, std::vector<uint8_t>> wide_cache;

    // device state (created lazily; the handle works on a GPU-less host)
    std::mutex dev_mu;
    int device = -1;
    bool device_ready = false;

    std::mutex tab_mu;  // coefficient-table registry: matrix bytes -> device perm tables
    struct TableEntry {
        uint32_t* dev = nullptr;
        hipEvent_t ready = nullptr;      // its upload's completion (nullptr once seen complete)
        hipStream_t stream = nullptr;    // ... enqueued on this stream
        bool arena = false;              // written by the host into the first-sight arena (uncached VRAM)
        size_t bytes = 0;
    };
    std::map<std::string, TableEntry> tables;
    // Pinned staging of table uploads (async on the launching stream, so a new
    // matrix does not wait for the kernels already queued): a slot is reused
    // once the copy enqueued from it kRing uploads earlier has finished.
    struct TabStage {
        uint8_t* host = nullptr;
        const uint8_t* dev_host = nullptr;  // its device address (a first-sight launch reads it in place)
        bool vram = false;                  // host-writable device memory (else coherent pinned host memory)
        size_t cap = 0;
        hipEvent_t done = nullptr;
        bool pending = false;
    };
    static constexpr int kTabStages = 4;
    TabStage tab_stage[kTabStages];
    int tab_stage_next = 0;
    // Matrices a small launch has used once with its tables read in place
    // from a staging slot (get_tables), by a 64-bit hash of the registry key
    // (a collision only makes a first sight upload): the second sight
    // uploads them.  Bounded (cleared when full).
    std::unordered_set<uint64_t> tab_seen;
    // First-sight arena (get_tables): host-writable device memory the host
    // writes new matrices' tables into for small launches; registry entries
    // point into it until the matrix's next use moves them to ordinary
    // device memory.  Space is reclaimed only with the registry (after a
    // device drain).
    uint8_t* tab_arena = nullptr;
    size_t tab_arena_cap = 0, tab_arena_off = 0;
    uint64_t tab_uploads = 0, tab_inplace = 0;  // (rs_coef_table_stats)

    std::mutex stage_mu;  // staging for the host-memory entry points
    uint8_t* stage = nullptr;
    size_t stage_bytes = 0;
    uint8_t* hstage = nullptr;  // pinned host mirror of `stage` (small-vector fast path)
    size_t hstage_bytes = 0;
    uint8_t* bounce = nullptr;  // pinned bounce buffer of the staged path's pageable copies (two halves)
    hipEvent_t bounce_ev[2] = {nullptr, nullptr};
    uint8_t* slots = nullptr;   // device staging slots of the staged (non-zero-copy) host path
    bool zc_pending = false;    // a zero-copy kernel may still be using hstage
    hipEvent_t chunk_ev[3] = {nullptr, nullptr, nullptr};  // host-call chunk pipeline slots
    hipStream_t stream = nullptr;

    // Host-call coalescing: concurrent small host calls of one shape (matrix,
    // size, mode) join a shared batch in a pinned buffer, each caller copying
    // its own vectors in and out on its own thread; the batch runs as ONE
    // multi-stripe zero-copy launch.  Two batches: one fills while the other
    // runs (host_calls.cpp host_call).
    struct CoBatch {
        enum State { kIdle, kFilling, kRunning, kDone } state = kIdle;
        std::vector<uint8_t> mat;  // the shape: matrix bytes, rows, cols, size, mode
        int rows = 0, cols = 0;
        size_t size = 0;
        bool accumulate = false;
        size_t pitch = 0, stride = 0;
        int cap = 0;               // stripes this batch may take
        uint8_t* host = nullptr;   // pinned [cap][cols + rows][pitch] (a pool block)
        uint8_t* dev = nullptr;    // its device-mapped address
        size_t host_bytes = 0;
        rsamd::detail::PinnedBlock blk;
        int joined = 0, ready = 0, released = 0;
        int rc = 0;
        bool launchable = false;   // linger window started (host_coalesce_linger_us)
        std::chrono::steady_clock::time_point deadline;
    };
    std::mutex co_mu;
    std::condition_variable co_cv;
    static constexpr int kCoBatches = 3;
    CoBatch co[kCoBatches];
    int co_running = 0;
    std::mutex co_launch_mu;       // the launch fallback: one batch at a time on co_stream
    int co_active = 0;             // callers inside host_call
    std::atomic<uint64_t> co_gen{0};  // bumped at every batch state change (spinning waiters watch it)
    std::atomic<uint64_t> co_launches{0}, co_calls{0};

    // DMA pipeline of rs_encode_host_batch (host_batches.cpp): device ring,
    // copy-in / compute / copy-out streams and per-slot events, kept across
    // calls (a per-call hipMalloc / hipFree of the ring cost ~25 % of a
    // 128-stripe call).  Guarded by stage_mu.
    uint8_t* dma_ring = nullptr;
    size_t dma_ring_bytes = 0;
    hipStream_t dma_stream[3] = {nullptr, nullptr, nullptr};
    hipEvent_t dma_ev[3][8] = {};
    hipStream_t co_stream = nullptr;

    // Completion flags of the launch-path host calls (flag_sync,
    // host_calls.cpp): pinned words the stream writes after the call's
    // kernel, one per stream (stream under stage_mu, co_stream under
    // co_launch_mu).
    struct DoneFlag {
        uint32_t* host = nullptr;
        void* dev = nullptr;
        uint32_t seq = 0;
    };
    DoneFlag stream_flag, co_flag;

    // Upload ring for per-call device descriptors (multi-pattern Reconst):
    // pinned host slot -> device slot on a private copy stream, so the copy
    // for call n+1 overlaps call n's kernel instead of stalling the stream.
    static constexpr int kUploadSlots = 4;
    struct UploadSlot {
        uint8_t* host = nullptr;
        const uint8_t* host_dev = nullptr;  // the host buffer's device address (mapped pinned memory)
        uint8_t* dev = nullptr;
        size_t cap = 0, dcap = 0;  // host / device bytes
        hipEvent_t copied = nullptr, done = nullptr;
        bool in_flight = false;
    };
    std::mutex up_mu;
    UploadSlot up[kUploadSlots];
    int up_next = 0;
    hipStream_t up_stream = nullptr;

    // Host-call engine (engine.cpp): resident kernel + doorbell ring serving
    // the small host calls.  eng_mu guards submission and the instance; a
    // caller waits for its call's completion without it.
    std::mutex eng_mu;
    rsamd::EngineRing* eng_ring = nullptr;   // host address (fine-grained pinned)
    rsamd::EngineRing* eng_dring = nullptr;  // its device address
    // the call slots in device memory the host writes through the BAR (the
    // engine polls local HBM), or nullptr: the slots of eng_ring
    rsamd::EngineSlot* eng_vslots = nullptr;
    hipStream_t eng_stream = nullptr;
    bool eng_running = false;
    int eng_waves = 0;       // the latest instance's workgroups (kept once it stops: calls still
                             // pending resume on this shape, engine_drain)
    int eng_group_waves = 0; // ... and waves per workgroup
    int eng_idle_us = 0;     // the running instance's idle window
    int eng_life_us = 0;     // ... and its maximum life
    bool eng_failed = false; // retired after a call timed out (calls take the launch paths)
    int eng_poll_gap = 0;    // ... and its doorbell poll gap
    uint64_t eng_seq = 0;
    int eng_next_wg = 0;     // first workgroup of the next call
    uint64_t eng_epoch = 0;  // the latest instance launched (its gone words / stop word carry it)
    uint32_t eng_tab_id = 0;                          // the latest matrix's table id
    uint32_t eng_slot_tab[rsamd::kEngineSlots] = {};  // table id each slot holds
    std::vector<uint8_t> eng_tab_key;
    std::atomic<uint64_t> eng_calls{0}, eng_launches{0};
    std::atomic<int> eng_inflight{0};  // calls rung and not yet seen complete by their callers
    std::atomic<bool> eng_warm_wanted{false};  // a call declined a cold engine: relaunch it (engine_warm)
    std::atomic<int64_t> eng_last_ns{0};       // steady-clock time of the latest engine call's completion

    // Reference-compat Update / Replace (rs_set_ref_l1d): the L1D bytes of the
    // host whose rs.go bytes to reproduce, 0 = the re-encode definition.
    std::atomic<int> ref_l1d{0};

    const uint8_t* gen() const { return enc.data() + static_cast<size_t>(d) * d; }

    ~rs_codec();
    void release_device();
};

inline rs_codec::~rs_codec() { release_device(); }

namespace rsamd {
namespace detail {
// Host-call engine (engine.cpp).  engine_call: RS_ERR_INVAL when the call
// does not fit the engine (the caller launches instead).
int engine_call(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* dev_base, size_t pitch,
                size_t stride, int nstripes, bool accumulate, bool coherent);
// Address mode: one stripe whose vectors (cols inputs, rows outputs; device
// addresses, 16-byte aligned, size a multiple of 16) lie anywhere, e.g. in
// memory the caller registered.
int engine_call_addr(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* in, uint8_t* const* out,
                     size_t size, bool accumulate);
// Would the engine take a call of this shape moving `bytes` in all?
bool engine_accepts(int rows, int cols, size_t bytes);
void engine_stop(rs_t* rs);  // caller holds eng_mu
// Every call rung so far complete (relaunching the latest shape if needed);
// caller holds eng_mu.  Precedes an engine_stop that no same-shape relaunch
// follows.
int engine_drain(rs_t* rs);
void engine_shutdown(rs_t* rs);
// After a call that the engine declined because it was cold (idle exit) has
// enqueued its kernel on the launch path: relaunch the engine now, while that
// kernel runs, so the next call finds it (no-op unless a call declined).
void engine_warm(rs_t* rs, bool wait_lock = false);
// The same on the library's warmer thread: the caller only queues the request
// (a cold call's latency stays the launch path's).
void engine_warm_async(rs_t* rs);
// Would an engine call now be declined as cold (see engine_warm)?  Lets a
// caller skip staging meant for the engine.
bool engine_cold_now(rs_t* rs);
// Ask every handle's running engine instance to leave (its pending calls are
// served first), ahead of a device-wide synchronisation by the library.
void engines_quiesce();
extern int g_engine, g_engine_waves, g_engine_group_waves, g_engine_idle_us, g_engine_life_us, g_engine_wg_units,
    g_engine_yield_us, g_engine_poll_gap, g_engine_vram, g_engine_split_rows, g_engine_cold_launch;
// Device memory the host can write through the BAR (uncached for the GPU:
// its loads always see the host's latest bytes), or nullptr when the
// platform maps no such memory for the CPU (engine.cpp).  Blocks are pooled
// per device and never freed while the process runs.
uint8_t* host_writable_vram_get(int device, size_t bytes, size_t* cap);
// Coherent, mapped pinned host blocks (table staging slots, completion
// flags) recycled process-wide instead of freed with their handle, as the
// engine's rings are: no allocate / free churn of coherent mappings while
// other work runs.  Size classes: powers of two from 4 KiB.
// *dev receives the block's device address.  nullptr when out of memory.
uint8_t* coherent_get(size_t bytes, size_t* cap, void** dev);
void coherent_put(uint8_t* p, size_t cap);
void host_writable_vram_put(int device, uint8_t* p, size_t cap);
extern size_t g_engine_max_bytes;

// Diagnostics (env RSAMD_ENGINE_TRACE): where the time of the synchronous
// host calls goes, as mean us per call and phase, printed at process exit.
enum HostPhase {
    kPhJoin,      // enter -> own stripe slot in a batch
    kPhCopyIn,    // caller vectors -> pinned slot
    kPhWaitRun,   // ready -> this batch starts running (or is done, for non-runners)
    kPhPreBell,   // engine_call entry -> doorbell rung (lock, relaunch, tables, header)
    kPhBell,      // doorbell rung -> every done word seen
    kPhWake,      // batch done -> caller resumes
    kPhCopyOut,   // pinned slot -> caller vectors
    kPhGpuTab,    // engine workgroup 0: doorbell seen -> acquire done, tables in LDS
    kPhGpuWork,   //   -> its stores acknowledged
    kPhGpuRel,    //   -> release write-back done, done word written
    kPhCount
};
extern const bool g_phase_trace;
void phase_add_ns(HostPhase p, uint64_t ns);
inline void phase_add(HostPhase p, std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    phase_add_ns(p, static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count()));
}
}  // namespace detail
}  // namespace rsamd

inline void rs_codec::release_device() {
    {
        if (!device_ready) return;
        static const bool trace = std::getenv("RSAMD_TEARDOWN_TRACE") != nullptr;  // diagnostics
        auto step = [](const char* what) {
            if (trace) std::fprintf(stderr, "rs_free: %s\n", what);
        };
        rsamd::detail::Region region("rs_free teardown");
        step("engine shutdown");
        rsamd::detail::engine_shutdown(this);
        rsamd::detail::DeviceGuard g(device);
        step("stream sync");
        if (stream) (void)hipStreamSynchronize(stream);
        step("device sync");
        (void)hipDeviceSynchronize();
        step("frees");
        for (auto& kv : tables) {
            if (!kv.second.arena) (void)hipFree(kv.second.dev);
            if (kv.second.ready) (void)hipEventDestroy(kv.second.ready);
        }
        if (tab_arena) rsamd::detail::host_writable_vram_put(device, tab_arena, tab_arena_cap);
        for (TabStage& t : tab_stage) {
            if (t.host && t.vram) rsamd::detail::host_writable_vram_put(device, t.host, t.cap);
            else if (t.host) rsamd::detail::coherent_put(t.host, t.cap);
            if (t.done) (void)hipEventDestroy(t.done);
        }
        for (UploadSlot& u : up) {
            if (u.host) rsamd::detail::coherent_put(u.host, u.cap);
            if (u.dev) (void)hipFree(u.dev);
            if (u.copied) (void)hipEventDestroy(u.copied);
            if (u.done) (void)hipEventDestroy(u.done);
        }
        if (up_stream) (void)hipStreamDestroy(up_stream);
        if (stage) (void)hipFree(stage);
        if (hstage) (void)hipHostFree(hstage);
        if (bounce) (void)hipHostFree(bounce);
        for (hipEvent_t e : bounce_ev)
            if (e) (void)hipEventDestroy(e);
        for (CoBatch& b : co)
            if (b.blk.host) rsamd::detail::pinned_put(b.blk);
        for (hipStream_t s : dma_stream)
            if (s) (void)hipStreamSynchronize(s);
        if (dma_ring) (void)hipFree(dma_ring);
        for (auto& row : dma_ev)
            for (hipEvent_t e : row)
                if (e) (void)hipEventDestroy(e);
        for (hipStream_t s : dma_stream)
            if (s) (void)hipStreamDestroy(s);
        if (co_stream) (void)hipStreamDestroy(co_stream);
        for (DoneFlag* f : {&stream_flag, &co_flag})
            if (f->host) rsamd::detail::coherent_put(reinterpret_cast<uint8_t*>(f->host), 4096);
        for (hipEvent_t e : chunk_ev)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
        step("done");
    }
}

namespace rsamd {
namespace detail {

// ---------------------------------------------------------------- matrix.go (codec.cpp)
std::vector<uint8_t> make_encode_matrix(int d, int p);              // matrix.go:37-54
int invert(const uint8_t* src, size_t len, int n, uint8_t* out);    // matrix.go:85-147
uint64_t cache_key(const int* survived, int ns);                    // rs.go:414-420

// ---------------------------------------------------------------- device product (codec.cpp)
int ensure_device(rs_t* rs);
int get_tables(rs_t* rs, const uint8_t* mat, int rows, int cols, hipStream_t stream, const uint32_t** out,
               int* rows_pad_out, uint64_t launch_in_bytes = ~uint64_t{0}, int* inplace_slot = nullptr);
int matmul_ex(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* in_ptrs,
              const uint8_t* in_sid, uint8_t* const* out_ptrs, const uint8_t* out_sid, const int64_t ss[4],
              int nstripes, uint64_t len, bool accumulate, hipStream_t stream, const int32_t* stripe_ids = nullptr);
int matmul(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* in_ptrs, int64_t in_ss,
           uint8_t* const* out_ptrs, int64_t out_ss, int nstripes, uint64_t len, bool accumulate,
           hipStream_t stream);

// One leased upload slot (see rs_codec::up).  Holds the ring lock from
// acquire() until the consumer's kernels are enqueued; the destructor records
// the slot's `done` event on the consumer stream.
class UploadLease {
public:
    explicit UploadLease(rs_t* rs) : rs_(rs), lk_(rs->up_mu) {}
    ~UploadLease() {
        if (slot_ && st_) {
            (void)hipEventRecord(slot_->done, st_);
            slot_->in_flight = true;
        }
    }
    // A pinned host buffer of `bytes` to fill (slot free for reuse on return),
    // whose device copy has room for `dev_bytes` (at least `bytes`): the part
    // past `bytes` is the consumer kernels' to write (the GPU planner).
    int acquire(size_t bytes, uint8_t** host, size_t dev_bytes = 0) {
        rs_codec::UploadSlot& u = rs_->up[rs_->up_next];
        rs_->up_next = (rs_->up_next + 1) % rs_codec::kUploadSlots;
        if (!rs_->up_stream) {
            const hipError_t e = hipStreamCreateWithFlags(&rs_->up_stream, hipStreamNonBlocking);
            if (e != hipSuccess) {
                rs_->up_stream = nullptr;
                return dev_fail(e, "upload stream create");
            }
        }
        if (u.in_flight) {  // the kernel that read this slot's device copy has finished
            RS_TRY(hip_ok(hipEventSynchronize(u.done), "upload slot event sync"));
            u.in_flight = false;
        }
        for (hipEvent_t* ev : {&u.copied, &u.done})
            if (!*ev && hip_ok(hipEventCreateWithFlags(ev, hipEventDisableTiming), "upload event create")) {
                *ev = nullptr;
                return RS_ERR_DEVICE;
            }
        auto round = [](size_t b) { return (b + (size_t{64} << 10) - 1) & ~((size_t{64} << 10) - 1); };
        if (u.cap < bytes) {
            if (u.host) rsamd::detail::coherent_put(u.host, u.cap);
            u.host = nullptr;
            u.host_dev = nullptr;
            u.cap = 0;
            // coherent and mapped (a recycled block): a kernel may read it in place (map() below)
            size_t cap = 0;
            void* hd = nullptr;
            u.host = rsamd::detail::coherent_get(round(bytes), &cap, &hd);
            if (!u.host) return RS_ERR_NOMEM;
            u.host_dev = static_cast<const uint8_t*>(hd);
            u.cap = cap;
        }
        const size_t dneed = dev_bytes > bytes ? dev_bytes : bytes;
        if (u.dcap < dneed) {
            if (u.dev) (void)hipFree(u.dev);
            u.dev = nullptr;
            u.dcap = 0;
            const size_t cap = round(dneed);
            if (hipMalloc(reinterpret_cast<void**>(&u.dev), cap) != hipSuccess) {
                u.dev = nullptr;
                return RS_ERR_NOMEM;
            }
            u.dcap = cap;
        }
        slot_ = &u;
        bytes_ = bytes;
        *host = u.host;
        return RS_OK;
    }
    // Copy the filled host buffer to the device ahead of the consumer's work
    // on `st`: a copy kernel on `st` reading the mapped buffer (the DMA copy
    // on the upload stream plus the cross-stream event cost 5.8 + 17-19 us of
    // GPU time per call, profiles/r05/planner_keyw/timeline_before/), or,
    // without a device address for the buffer, that DMA copy.
    int upload(hipStream_t st, uint8_t** dev) {
        st_ = st;
        const size_t b16 = (bytes_ + 15) & ~size_t{15};  // (slots are 64 KiB multiples)
        if (slot_->host_dev) {
            RS_TRY(hip_ok(launch_copy_in(slot_->dev, slot_->host_dev, b16, st), "upload copy kernel"));
        } else {
            RS_TRY(hip_ok(hipMemcpyAsync(slot_->dev, slot_->host, bytes_, hipMemcpyHostToDevice, rs_->up_stream),
                          "upload copy"));
            RS_TRY(hip_ok(hipEventRecord(slot_->copied, rs_->up_stream), "upload event record"));
            RS_TRY(hip_ok(hipStreamWaitEvent(st, slot_->copied, 0), "upload stream wait"));
        }
        *dev = slot_->dev;
        return RS_OK;
    }

    // No copy: the consumer kernels on `st` read the filled host buffer in
    // place through its device address (and may write the device slot); the
    // slot is reused only after they finish (the destructor's `done` event).
    // Does the acquired slot have a device address for map()?
    bool mappable() const { return slot_ && slot_->host_dev; }
    int map(hipStream_t st, const uint8_t** host_dev, uint8_t** dev) {
        if (!slot_->host_dev) return dev_fail(hipErrorInvalidValue, "upload slot device address");
        st_ = st;
        *host_dev = slot_->host_dev;
        *dev = slot_->dev;
        return RS_OK;
    }

private:
    rs_t* rs_;
    std::lock_guard<std::mutex> lk_;
    rs_codec::UploadSlot* slot_ = nullptr;
    hipStream_t st_ = nullptr;
    size_t bytes_ = 0;
};

// Address of vector v (0..d+p) of stripe 0 and its stride selector under a layout.
struct LayoutAddr {
    const rs_layout_t* L;
    int d;
    uint8_t* ptr(int v) const {
        return v < d ? L->data_base + v * L->data_vect_stride : L->parity_base + (v - d) * L->parity_vect_stride;
    }
    uint8_t sid(int v) const { return v < d ? 0 : 1; }
};

// ---------------------------------------------------------------- reference checks (codec.cpp)
int check_encode(const rs_t* rs, const size_t* lens, int n);
int check_encode_idx(const size_t* lens, const int* idx, int cnt);
int check_vect_idx(const int* idx, int cnt, int n);
int plan_reconst(const rs_t* rs, const int* survived, int ns, const int* need, int nn, int* vs, int* nvs,
                 int* nr, int* nnr, int* dn);
int get_inverse(rs_t* rs, const int* survived_d, std::vector<uint8_t>& inv);
int reconst_matrix(rs_t* rs, const int* survived_d, const int* need, int nn, uint8_t* out);
int combined_matrix(rs_t* rs, const int* vs, const int* nr, int nnr, int dn, std::vector<uint8_t>& m);
int check_update(const rs_t* rs, size_t old_len, size_t new_len, int row, const size_t* plens, int np);
int check_replace(const rs_t* rs, const size_t* dlens, int nd, const int* rows, int nr, const size_t* plens,
                  int np);
std::vector<uint8_t> update_matrix(const rs_t* rs, int row);
std::vector<uint8_t> replace_matrix(const rs_t* rs, const int* rows, int nr);

// Reference-compat mode for Update / Replace (rs_set_ref_l1d(rs,
// l1d_bytes), per handle; 0 = off, the default).  The reference's encodePart
// (rs.go:175-203) runs its sub-16-byte tail pass over the WHOLE last chunk
// [start, end) of getSplitSize (rs.go:158-173: L1D/2 bytes), so under
// updateOnly (Update rs.go:447, Replace rs.go:527) that chunk's 16-byte body
// is XORed twice and keeps its old parity.  With the mode on, the product
// skips exactly that byte range [lo, hi) for the given L1D size, so the
// parity bytes equal the reference's on a host with that L1D.  Returns false
// when the size has no such range (or the mode is off).
// Per-stripe erasure masks of the multi-pattern Reconst entry points:
// `words` uint64 words per stripe (1: the d+p <= 64 API, 4: the *_multi256
// API), vector v at bit v % 64 of word v / 64.
struct MaskView {
    const uint64_t* m;
    int words;
    const uint64_t* row(int s) const { return m + static_cast<size_t>(s) * words; }
    bool bit(int s, int v) const { return (v >> 6) < words && (row(s)[v >> 6] >> (v & 63) & 1); }
    bool any(int s) const {
        for (int w = 0; w < words; ++w)
            if (row(s)[w]) return true;
        return false;
    }
    int count(int s) const {
        int c = 0;
        for (int w = 0; w < words; ++w) c += __builtin_popcountll(row(s)[w]);
        return c;
    }
    // any bit at or above nvec (a vector the stripe does not have)
    bool beyond(int s, int nvec) const {
        for (int w = 0; w < words; ++w) {
            const int lo = w * 64;
            const uint64_t valid = nvec >= lo + 64 ? ~uint64_t{0} : nvec <= lo ? 0 : ((uint64_t{1} << (nvec - lo)) - 1);
            if (row(s)[w] & ~valid) return true;
        }
        return false;
    }
    MaskView from(int first) const { return MaskView{row(first), words}; }
};
int reconst_multi(rs_t* rs, const rs_layout_t* L, int nstripes, size_t len, MaskView masks, void* stream);
int check_masks(int d, int p, MaskView masks, int nstripes);

bool ref_update_skip(int l1d, uint64_t size, uint64_t* lo, uint64_t* hi);
// Run op(offset, length) over [0, size) minus the range the handle's
// reference-compat setting skips (read once per call).
template <class Op>
int update_ranges(const rs_t* rs, uint64_t size, Op op) {
    uint64_t lo = 0, hi = 0;
    if (!ref_update_skip(rs->ref_l1d.load(std::memory_order_relaxed), size, &lo, &hi)) return op(uint64_t{0}, size);
    if (lo > 0) RS_TRY(op(uint64_t{0}, lo));
    if (hi < size) RS_TRY(op(hi, size - hi));
    return RS_OK;
}

// Reconst on one stripe whose vectors are addressed by `ptr` (host staging
// slots or caller device pointers).  Shared by rs_reconst / rs_reconst_dev /
// rs_reconst_batch.  `before_parity` lets the host path copy the rebuilt data
// back before the parity check runs (the reference returns the parity-pass
// error with the data already rebuilt).
struct ReconstPlan {
    int vs[kMaxVects], nr[kMaxVects];
    int nvs = 0, nnr = 0, dn = 0;
};

int check_reconst_passes(const rs_t* rs, const ReconstPlan& pl, const size_t* lens, int n, int* parity_rc);

// ---------------------------------------------------------------- host calls (host_calls.cpp)
extern size_t g_pinned_max, g_zc_max, g_chunk, g_chunk_split, g_coalesce_max;
extern int g_coalesce_linger_us, g_co_running, g_engine_direct;
int host_product(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* src, uint8_t* const* dst,
                 size_t size, bool accumulate);
// host_product for a synchronous host call, coalesced with concurrent calls
// of the same shape (takes stage_mu itself).
int host_call(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* src, uint8_t* const* dst,
              size_t size, bool accumulate);
// Wait for everything queued on `st` so far (see host_calls.cpp).
int flag_sync(hipStream_t st, rs_codec::DoneFlag& f, const char* where);
extern int g_host_flag_sync;

// ---------------------------------------------------------------- host batches (host_batches.cpp)
extern int g_host_batch_zc, g_host_dma_1d, g_bind_numa, g_host_pageable_stage, g_copy_nt, g_copy_coalesce;
extern size_t g_pageable_slot;  // pageable host batches: stripe bytes per chunk (host_batches.cpp)
extern int g_unregister_revoke;  // rs_host_unregister returns the caller's pages to no GPU access (host_batches.cpp)
// dst[i] <- src[i] (n vectors, len bytes each) on the host copy pool (host_calls.cpp).
void parallel_copy(uint8_t* const* dst, const uint8_t* const* src, int n, size_t len);
int bind_thread_to_device(int device);
int host_device_range(const void* p, size_t bytes, uint8_t** dev);
// Device address of [p, p+bytes) inside a range registered with
// rs_host_register, or nullptr.
uint8_t* registered_device_ptr(const void* p, size_t bytes);
extern std::atomic<int> g_reg_count;
// Devices some handle of this process has launched on (bit per ordinal < 64):
// rs_host_unregister drains them before a range leaves the runtime.
extern std::atomic<uint64_t> g_devices_used;
size_t batch_extent(int64_t ss, int64_t vs, int nstripes, int nvec, size_t len);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Every int-returning C ABI entry point runs its body through this guard, so
// no C++ exception (an allocation failure in a std:: container, a thread
// that cannot start) ever unwinds into a C or cgo caller.
template <class F>
int abi_guard(F&& body) noexcept {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        return RS_ERR_NOMEM;
    } catch (...) {
        return dev_fail(hipErrorUnknown, "unexpected C++ exception");
    }
}

}  // namespace detail
}  // namespace rsamd
