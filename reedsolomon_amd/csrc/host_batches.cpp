// host_batches.cpp — host-resident batches of stripes: zero-copy kernels
// over pinned / registered memory, the H2D / kernel / D2H pipeline for
// pageable memory, and device groups (one process, several GPUs).
#include <dlfcn.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <thread>

#include "codec_internal.hpp"

using namespace rsamd;
using namespace rsamd::detail;

namespace rsamd {
namespace detail {

// Device address of the host range [p, p+bytes) when all of it lies in one
// pinned / registered, device-mapped allocation (both ends translate by the
// same offset); RS_ERR_INVAL otherwise (pageable memory: never give a kernel
// such an address).
int host_device_range(const void* p, size_t bytes, uint8_t** dev) {
    *dev = nullptr;
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return RS_ERR_INVAL;
    }
    if (at.type != hipMemoryTypeHost) return RS_ERR_INVAL;
    void* d0 = nullptr;
    void* d1 = nullptr;
    const uint8_t* last = static_cast<const uint8_t*>(p) + bytes - 1;
    if (hipHostGetDevicePointer(&d0, const_cast<void*>(p), 0) != hipSuccess || !d0 ||
        hipHostGetDevicePointer(&d1, const_cast<uint8_t*>(last), 0) != hipSuccess || !d1) {
        (void)hipGetLastError();
        return RS_ERR_INVAL;
    }
    if (static_cast<uint8_t*>(d1) - static_cast<uint8_t*>(d0) != static_cast<ptrdiff_t>(bytes - 1))
        return RS_ERR_INVAL;
    *dev = static_cast<uint8_t*>(d0);
    return RS_OK;
}

// Host memory registered with the HIP runtime, as disjoint page spans.
// rs_host_register rounds the caller's range out to whole pages and takes a
// reference on every span that covers part of it, registering only the pages
// no span covers yet, so two caller ranges that share a page (heap buffers
// side by side) never register that page twice and neither unregister pulls
// it from under the other.  A partial first or last page of a range is
// registered as a span of its own, so the page a neighbour shares is the only
// one that outlives the range's unregister (a span shared whole would keep the
// range's own pages registered after the caller freed them, and a later
// buffer at those addresses would get the runtime's stale pinning).  A span
// leaves the runtime when its last reference goes, after every device this
// process launched on has been drained (a kernel the caller queued over the
// range may still be reading it); the drain runs without g_reg_mu, the spans
// waiting for it are "dying": not found by lookups, and a registration that
// touches one waits until it is gone.  The
// library-owned pool (rs_host_alloc) holds a permanent reference on its
// blocks: they are registered once and stay registered and mapped while the
// process runs, however often they are handed out again.  Host calls look
// their vectors up here (registered_device_ptr) and, when every vector lies
// inside one span, run the kernel straight over the caller's memory.
namespace {
struct Span {
    uintptr_t hi;   // [key, hi): whole pages
    uint8_t* dev;   // device address of the span's first byte
    int refs;
};
struct PoolBlock {
    size_t bytes;
    bool free;
};
std::mutex g_reg_mu;
std::condition_variable g_reg_cv;                       // a dying span left the runtime
std::map<uintptr_t, Span> g_spans;                      // disjoint page spans, by first address
std::map<uintptr_t, uintptr_t> g_dying;                 // [lo, hi) spans unregistered, waiting for the drain
struct UserReg {
    size_t bytes;
    std::vector<uintptr_t> spans;  // the spans it holds a reference on
};
std::map<uintptr_t, UserReg> g_user;                    // rs_host_register'ed ranges, by address
std::map<uintptr_t, PoolBlock> g_pool;                  // every pool block ever handed out
std::multimap<size_t, uintptr_t> g_pool_free;           // size class -> free pool block
size_t g_pool_mapped = 0, g_pool_in_use = 0;
// Pool memory comes in slabs the pool owns whole: 2 MiB-aligned runs of whole
// 2 MiB granules (KFD's SVM granularity here, amdgpu svm_default_granularity
// 9), registered once, never sharing a granule with another mapping (a
// caller's buffer mapped next to a 128 KiB block used to share one; DESIGN.md
// §5.8), never backed by transparent huge pages (no collapse or split
// invalidates them).  Classes below 2 MiB are carved from a slab of their own
// class as blocks are first handed out.
constexpr size_t kPoolGranule = size_t{2} << 20;
struct Slab {
    uintptr_t next = 0, end = 0;
};
std::map<size_t, Slab> g_slab;  // size class -> the slab its next new block comes from

uintptr_t page_bytes() {
    static const uintptr_t ps = [] {
        const long v = sysconf(_SC_PAGESIZE);
        return v > 0 ? static_cast<uintptr_t>(v) : uintptr_t{4096};
    }();
    return ps;
}

// Caller holds g_reg_mu.  Registers [lo, hi) with the runtime as a new span
// holding one reference.
int span_register(uintptr_t lo, uintptr_t hi) {
    void* p = reinterpret_cast<void*>(lo);
    {
        Region region("hipHostRegister");
        RS_TRY(hip_ok(hipHostRegister(p, hi - lo, hipHostRegisterMapped | hipHostRegisterPortable), "hipHostRegister"));
    }
    void* dev = nullptr;
    if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess || !dev) {
        (void)hipGetLastError();
        (void)hipHostUnregister(p);
        return dev_fail(hipErrorInvalidValue, "hipHostGetDevicePointer (registered span)");
    }
    g_spans.emplace(lo, Span{hi, static_cast<uint8_t*>(dev), 1});
    return RS_OK;
}

// Every device this process launched on has finished its queued work.
// Resident host-call engines are asked to leave first (they would hold the
// sync for their idle window).
void drain_used_devices() {
    engines_quiesce();
    const uint64_t used = g_devices_used.load(std::memory_order_acquire);
    for (int dv = 0; dv < 64; ++dv)
        if (used & (uint64_t{1} << dv)) {
            DeviceGuard g(dv);
            (void)hipDeviceSynchronize();
        }
}

// Drops one reference on each span in `spans` (caller holds g_reg_mu);
// spans whose last reference went are removed from the lookup and returned
// as [lo, hi).
std::vector<std::pair<uintptr_t, uintptr_t>> spans_release(const std::vector<uintptr_t>& spans) {
    std::vector<std::pair<uintptr_t, uintptr_t>> dead;
    for (uintptr_t lo : spans) {
        auto it = g_spans.find(lo);
        if (it != g_spans.end() && --it->second.refs == 0) {
            dead.emplace_back(lo, it->second.hi);
            g_spans.erase(it);
        }
    }
    g_reg_count.store(static_cast<int>(g_spans.size()));
    return dead;
}

// hipHostRegister on this system grants the GPUs in-place access to the
// range through KFD's shared-virtual-memory ranges, and hipHostUnregister
// does not take it back: HIP forgets the registration, but the pages stay
// GPU-mapped (HSA_AMD_SVM_ATTRIB_ACCESS_QUERY reports AGENT_ACCESSIBLE_IN_PLACE)
// until they leave the process (tools/ptr_state_probe.py,
// profiles/r06/ptr_state_probe_svm.log).  The caller then frees the memory;
// every later trim or discard of those pages by the allocator (Go's
// scavenger, glibc's trim) has the kernel tear down a GPU mapping nobody
// uses, which with XNACK off means evicting and restoring the process's GPU
// queues.  So after the runtime's unregister the library returns the pages
// that belonged to the caller's range alone (whole pages inside
// [ptr, ptr + bytes); a partial edge page may hold a neighbour the runtime
// is copying) to their never-registered state: AGENT_NO_ACCESS for every GPU.
// rs_tune("host_unregister_revoke", 1 default | 0); best effort (no ROCr
// SVM API: nothing is done).
struct SvmApi {
    typedef struct { uint64_t attribute, value; } Pair;
    int (*set)(void*, size_t, Pair*, size_t) = nullptr;
    std::vector<uint64_t> gpus;  // agent handles
    SvmApi() {
        void* h = dlopen("libhsa-runtime64.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) return;
        auto iterate = reinterpret_cast<int (*)(int (*)(uint64_t, void*), void*)>(dlsym(h, "hsa_iterate_agents"));
        auto info = reinterpret_cast<int (*)(uint64_t, int, void*)>(dlsym(h, "hsa_agent_get_info"));
        set = reinterpret_cast<int (*)(void*, size_t, Pair*, size_t)>(dlsym(h, "hsa_amd_svm_attributes_set"));
        if (!iterate || !info || !set) {
            set = nullptr;
            return;
        }
        struct Ctx {
            decltype(info) get;
            std::vector<uint64_t>* out;
        } ctx{info, &gpus};
        iterate(
            [](uint64_t agent, void* c) -> int {
                Ctx* x = static_cast<Ctx*>(c);
                uint32_t kind = 0;
                if (x->get(agent, 17 /* HSA_AGENT_INFO_DEVICE */, &kind) == 0 && kind == 1 /* GPU */)
                    x->out->push_back(agent);
                return 0;
            },
            &ctx);
        if (gpus.empty()) set = nullptr;
    }
};
const SvmApi& svm_api() {
    static const SvmApi a;
    return a;
}

// [lo, hi): whole pages of one caller's range, just unregistered (see above).
void svm_revoke(uintptr_t lo, uintptr_t hi) {
    if (!g_unregister_revoke || lo >= hi) return;
    const SvmApi& a = svm_api();
    if (!a.set) return;
    std::vector<SvmApi::Pair> attrs;
    for (uint64_t g : a.gpus) attrs.push_back({0x202 /* HSA_AMD_SVM_ATTRIB_AGENT_NO_ACCESS */, g});
    (void)a.set(reinterpret_cast<void*>(lo), hi - lo, attrs.data(), attrs.size());
}

bool overlaps_dying(uintptr_t lo, uintptr_t hi) {  // caller holds g_reg_mu
    auto it = g_dying.upper_bound(lo);
    if (it != g_dying.begin() && std::prev(it)->second > lo) return true;
    return it != g_dying.end() && it->first < hi;
}
}  // namespace
std::atomic<int> g_reg_count{0};
int g_unregister_revoke = [] {  // (svm_revoke above)
    const char* e = std::getenv("RSAMD_UNREGISTER_REVOKE");
    return e ? (std::atoi(e) ? 1 : 0) : 1;
}();

// [p, p + bytes) inside one span AND inside a live registration or a pool
// block: pages a span keeps for another registration (a shared page's whole
// span) do not make a range the caller unregistered zero-copy again.  The
// registration is searched among the 8 nearest starting at or below p (a
// range under a registration that starts further back takes the staged path:
// same bytes).
uint8_t* registered_device_ptr(const void* p, size_t bytes) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_spans.upper_bound(a);
    if (it == g_spans.begin()) return nullptr;
    --it;
    if (a >= it->second.hi) return nullptr;
    // the range may run over adjacent spans (a registration's own edge pages):
    // zero-copy only when the runtime mapped them contiguously for the device
    for (auto cur = it; a + bytes > cur->second.hi;) {
        auto next = std::next(cur);
        if (next == g_spans.end() || next->first != cur->second.hi ||
            next->second.dev != cur->second.dev + (cur->second.hi - cur->first))
            return nullptr;
        cur = next;
    }
    bool live = false;
    auto pb = g_pool.upper_bound(a);
    if (pb != g_pool.begin()) {
        --pb;
        live = a + bytes <= pb->first + pb->second.bytes;
    }
    auto ur = g_user.upper_bound(a);
    for (int k = 0; k < 8 && !live && ur != g_user.begin(); ++k) {
        --ur;
        live = a + bytes <= ur->first + ur->second.bytes;
    }
    return live ? it->second.dev + (a - it->first) : nullptr;
}

// Bind the calling thread to the CPUs local to `device` (its PCI function's
// sysfs local_cpulist), within the process's current affinity.  Host-side
// staging copies and page-locked buffers then stay on the GPU's NUMA node.
// Best effort: returns RS_ERR_INVAL when the topology cannot be read.
int bind_thread_to_device(int device) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) return RS_ERR_INVAL;
    for (char* c = bus; *c; ++c) *c = static_cast<char>(std::tolower(static_cast<unsigned char>(*c)));
    std::FILE* f = std::fopen((std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist").c_str(), "r");
    if (!f) return RS_ERR_INVAL;
    char list[4096] = {0};
    const bool got = std::fgets(list, sizeof list, f) != nullptr;
    std::fclose(f);
    if (!got) return RS_ERR_INVAL;
    cpu_set_t allowed, want;
    CPU_ZERO(&want);
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return RS_ERR_INVAL;
    for (char* tok = std::strtok(list, ",\n"); tok; tok = std::strtok(nullptr, ",\n")) {
        int a = -1, b = -1;
        if (std::sscanf(tok, "%d-%d", &a, &b) < 1) continue;
        if (b < a) b = a;
        for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (c >= 0 && CPU_ISSET(c, &allowed)) CPU_SET(c, &want);
    }
    if (CPU_COUNT(&want) == 0) return RS_ERR_INVAL;
    return pthread_setaffinity_np(pthread_self(), sizeof want, &want) == 0 ? RS_OK : RS_ERR_INVAL;
}

// Bytes spanned by a [S][nvec][len] batch with non-negative strides.
size_t batch_extent(int64_t ss, int64_t vs, int nstripes, int nvec, size_t len) {
    return static_cast<size_t>(nstripes - 1) * static_cast<size_t>(ss) +
           static_cast<size_t>(nvec - 1) * static_cast<size_t>(vs) + len;
}

// Zero-copy host batches (on by default): kernels read and write pinned host
// memory over PCIe directly.  Measured on MI355X: 72 GiB/s of (k+m)*vec for
// 10+4 encode at 8 KiB-1 MiB vectors vs 13-57 GiB/s for the DMA pipeline.
int g_host_batch_zc = 1;
// DMA pipeline copies of a dense layout: 0 = one 2-D copy per chunk (default:
// 70.4-70.7 GiB/s for 10+4 @ 1 MiB x 128 vs 66.8-67.1 with 1-D copies,
// tools/dma_ab.py), 1 = one 1-D hipMemcpyAsync per stripe.
int g_host_dma_1d = 0;
// Group worker threads bind to their GPU's local CPUs (bind_thread_to_device).
int g_bind_numa = 1;
// Pageable host batches are staged through the pinned mirror (stripes above
// kPageableStripeMax in byte windows: encode_pageable_batch,
// reconst_pageable_batch); 0 = Encode takes the DMA pipeline's 1-D runtime
// copies and a pageable multi-pattern Reconst is refused (RS_ERR_INVAL).
int g_host_pageable_stage = 1;

}  // namespace detail
}  // namespace rsamd

// Pageable caller memory, stripes up to kPageableStripeMax bytes: staged
// through the handle's pinned mirror (rs->hstage).  Chunks of stripes are
// copied in by the host copy pool, processed by one zero-copy launch straight
// out of the mirror, and their outputs copied back, with 3 chunks in flight
// (the copy-in of chunk c+1 overlaps chunk c's kernel).  The runtime's
// pageable hipMemcpyAsync costs a staging round trip per copy (10+4 @ 8 KiB:
// 4.2 GiB/s with one 1-D copy per stripe).  A mirror stripe is [d+p][pitch].
// rows_in(s, add) / rows_out(s, add) name the vectors of stripe s to copy in
// / out (add(v) per vector index); launch(first, count, dev_slot, stripe
// bytes, pitch) enqueues the kernel on rs->stream.  Caller holds stage_mu.
constexpr size_t kPageableStripeMax = size_t{16} << 20;
// Bytes of stripes per chunk (at least one stripe); rs_tune("host_pageable_slot").
size_t rsamd::detail::g_pageable_slot = size_t{8} << 20;
// Larger pageable stripes go through the same mirror in byte windows of
// every vector (Encode and Reconst are byte-wise: a window of all d+p
// vectors is a stripe of its own), so no pageable byte is handed to the
// runtime's pageable copies, which leave the caller's pages GPU-mapped in
// place after the copy (~200 us of driver work when that memory is freed,
// DESIGN.md §5.8).  Window: the largest 256-byte multiple that keeps a
// stripe within kPageableStripeMax.
static size_t pageable_window(int nvec) {
    return std::max<size_t>(256, (kPageableStripeMax / static_cast<size_t>(nvec)) & ~size_t{255});
}

template <class RowsIn, class RowsOut, class Launch>
static int pageable_pipeline(rs_t* rs, uint8_t* base, int64_t ss, int64_t vs, int nstripes, size_t len,
                             RowsIn rows_in, RowsOut rows_out, Launch launch) {
    const int nvec = rs->d + rs->p;
    if (!rs->stream) RS_TRY(hip_ok(hipStreamCreateWithFlags(&rs->stream, hipStreamNonBlocking), "stream create"));
    if (rs->zc_pending) RS_TRY(hip_ok(hipStreamSynchronize(rs->stream), "host-call stream sync"));
    const size_t pitch = rup(len, 256);
    const size_t sbytes = pitch * static_cast<size_t>(nvec);
    const int cs = static_cast<int>(std::max<size_t>(1, std::min<size_t>(nstripes, g_pageable_slot / sbytes)));
    const int nch = (nstripes + cs - 1) / cs;
    const int ns = nch > 1 ? 3 : 1;
    const size_t slot = sbytes * static_cast<size_t>(cs);
    if (slot * ns > rs->hstage_bytes) {
        if (rs->hstage) (void)hipHostFree(rs->hstage);
        rs->hstage = nullptr;
        rs->hstage_bytes = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&rs->hstage), slot * ns, hipHostMallocDefault) != hipSuccess) {
            rs->hstage = nullptr;
            return RS_ERR_NOMEM;
        }
        rs->hstage_bytes = slot * ns;
    }
    void* dbase = nullptr;
    RS_TRY(hip_ok(hipHostGetDevicePointer(&dbase, rs->hstage, 0), "mirror device pointer"));
    if (!dbase) return dev_fail(hipErrorInvalidValue, "mirror device pointer");
    for (int i = 0; i < ns; ++i)
        if (!rs->chunk_ev[i] && hip_ok(hipEventCreateWithFlags(&rs->chunk_ev[i], hipEventDisableTiming), "event create")) {
            rs->chunk_ev[i] = nullptr;
            return RS_ERR_DEVICE;
        }
    std::vector<uint8_t*> cd(static_cast<size_t>(cs) * nvec);
    std::vector<const uint8_t*> csrc(cd.size());
    auto count = [&](int c) { return std::min(cs, nstripes - c * cs); };
    auto hslot = [&](int c) { return rs->hstage + static_cast<size_t>(c % ns) * slot; };
    auto finish = [&](int c) -> int {  // wait for chunk c, copy its outputs back
        RS_TRY(hip_ok(hipEventSynchronize(rs->chunk_ev[c % ns]), "pageable batch chunk sync"));
        int n = 0;
        for (int t = 0; t < count(c); ++t) {
            uint8_t* st = base + static_cast<int64_t>(c * cs + t) * ss;
            const uint8_t* h = hslot(c) + static_cast<size_t>(t) * sbytes;
            rows_out(c * cs + t, [&](int v) {
                cd[n] = st + v * vs;
                csrc[n++] = h + static_cast<size_t>(v) * pitch;
            });
        }
        parallel_copy(cd.data(), csrc.data(), n, len);
        return RS_OK;
    };
    int rc = RS_OK;
    int done = 0;
    rs->zc_pending = true;
    for (int c = 0; c < nch && rc == RS_OK; ++c) {
        if (c >= ns) {
            rc = finish(done++);
            if (rc) break;
        }
        int n = 0;
        for (int t = 0; t < count(c); ++t) {
            const uint8_t* st = base + static_cast<int64_t>(c * cs + t) * ss;
            uint8_t* h = hslot(c) + static_cast<size_t>(t) * sbytes;
            rows_in(c * cs + t, [&](int v) {
                cd[n] = h + static_cast<size_t>(v) * pitch;
                csrc[n++] = st + v * vs;
            });
        }
        parallel_copy(cd.data(), csrc.data(), n, len);
        rc = launch(c * cs, count(c), static_cast<uint8_t*>(dbase) + static_cast<size_t>(c % ns) * slot, sbytes,
                    pitch);
        if (rc == RS_OK) rc = hip_ok(hipEventRecord(rs->chunk_ev[c % ns], rs->stream), "pageable batch chunk record");
    }
    while (rc == RS_OK && done < nch) rc = finish(done++);
    if (rc) (void)hipStreamSynchronize(rs->stream);  // never leave a kernel on the mirror
    rs->zc_pending = false;
    return rc;
}

// Encode of a pageable batch: data vectors in, parity out.
static int encode_pageable_batch(rs_t* rs, uint8_t* base, int64_t ss, int64_t vs, int nstripes, size_t len) {
    const int d = rs->d, p = rs->p;
    return pageable_pipeline(
        rs, base, ss, vs, nstripes, len,
        [&](int, auto add) { for (int i = 0; i < d; ++i) add(i); },
        [&](int, auto add) { for (int j = 0; j < p; ++j) add(d + j); },
        [&](int, int n, uint8_t* dslot, size_t sbytes, size_t pitch) {
            const uint8_t* in[kMaxVects];
            uint8_t* out[kMaxVects];
            for (int i = 0; i < d; ++i) in[i] = dslot + static_cast<size_t>(i) * pitch;
            for (int j = 0; j < p; ++j) out[j] = dslot + static_cast<size_t>(d + j) * pitch;
            return matmul(rs, rs->gen(), p, d, in, static_cast<int64_t>(sbytes), out, static_cast<int64_t>(sbytes), n,
                          len, false, rs->stream);
        });
}

// The errors rs_reconst_batch_multi would return for these masks, before
// anything is copied or launched.
int rsamd::detail::check_masks(int d, int p, MaskView masks, int nstripes) {
    const int nvec = d + p;
    if (nvec > 64 * masks.words) return RS_ERR_INVAL;
    for (int s = 0; s < nstripes; ++s) {
        if (masks.beyond(s, nvec)) return RS_ERR_ILLEGAL_VECTS;
        if (masks.count(s) > p) return RS_ERR_TOO_MANY_LOST;
    }
    return RS_OK;
}

// Multi-pattern Reconst of a pageable batch: the first d survivors of every
// stripe with work in, the lost vectors (rebuilt in the mirror) out.  Masks
// are validated before any copy or launch.
static int reconst_pageable_batch(rs_t* rs, uint8_t* base, int64_t ss, int64_t vs, int nstripes, size_t len,
                                  MaskView masks) {
    const int d = rs->d, p = rs->p, nvec = d + p;
    RS_TRY(check_masks(d, p, masks, nstripes));
    return pageable_pipeline(
        rs, base, ss, vs, nstripes, len,
        [&](int s, auto add) {  // the first d survivors: all the kernel reads (rs.go's choice)
            if (!masks.any(s)) return;
            for (int v = 0, n = 0; v < nvec && n < d; ++v)
                if (!masks.bit(s, v)) {
                    add(v);
                    ++n;
                }
        },
        [&](int s, auto add) {
            for (int v = 0; v < nvec; ++v)
                if (masks.bit(s, v)) add(v);
        },
        [&](int first, int n, uint8_t* dslot, size_t sbytes, size_t pitch) {
            const rs_layout_t L{dslot, static_cast<int64_t>(sbytes), static_cast<int64_t>(pitch),
                                dslot + static_cast<size_t>(d) * pitch, static_cast<int64_t>(sbytes),
                                static_cast<int64_t>(pitch)};
            return reconst_multi(rs, &L, n, len, masks.from(first), rs->stream);
        });
}

extern "C" {

int rs_host_register(void* ptr, size_t bytes) {
    return abi_guard([&]() -> int {
        if (!ptr || !bytes) return RS_ERR_INVAL;
        const uintptr_t a = reinterpret_cast<uintptr_t>(ptr), ps = page_bytes();
        if (a + bytes < a) return RS_ERR_INVAL;
        const uintptr_t lo = a & ~(ps - 1), hi = (a + bytes + ps - 1) & ~(ps - 1);
        std::unique_lock<std::mutex> lk(g_reg_mu);
        if (g_user.count(a)) return RS_ERR_INVAL;  // already registered at this address
        // pages of an unregister still draining: wait until they left the runtime
        g_reg_cv.wait(lk, [&] { return !overlaps_dying(lo, hi); });
        if (g_user.count(a)) return RS_ERR_INVAL;
        // piece boundaries: a partial first / last page is a span of its own
        uintptr_t cuts[3];
        int ncut = 0;
        if (a != lo && lo + ps < hi) cuts[ncut++] = lo + ps;
        if (a + bytes != hi && hi - ps > lo && (ncut == 0 || hi - ps > cuts[0])) cuts[ncut++] = hi - ps;
        cuts[ncut++] = hi;
        std::vector<uintptr_t> held;
        uintptr_t cur = lo;
        int rc = RS_OK;
        for (int c = 0; c < ncut && rc == RS_OK; ++c) {
            const uintptr_t piece_hi = cuts[c];
            while (cur < piece_hi && rc == RS_OK) {
                auto it = g_spans.upper_bound(cur);  // the span covering cur, if any, precedes it
                if (it != g_spans.begin() && std::prev(it)->second.hi > cur) {
                    Span& sp = std::prev(it)->second;
                    ++sp.refs;
                    held.push_back(std::prev(it)->first);
                    cur = sp.hi;
                    continue;
                }
                // the gap up to the next span, within this piece
                const uintptr_t end = it != g_spans.end() && it->first < piece_hi ? it->first : piece_hi;
                rc = span_register(cur, end);
                if (rc == RS_OK) {
                    held.push_back(cur);
                    cur = end;
                }
            }
        }
        if (rc != RS_OK) {  // roll back: nothing used the new spans yet
            for (auto& d : spans_release(held)) (void)hipHostUnregister(reinterpret_cast<void*>(d.first));
            return rc;
        }
        g_user.emplace(a, UserReg{bytes, std::move(held)});
        g_reg_count.store(static_cast<int>(g_spans.size()));
        return RS_OK;
    });
}

int rs_host_device_pointer(const void* host_ptr, size_t bytes, void** dev_ptr) {
    return abi_guard([&]() -> int {
        if (!host_ptr || !bytes || !dev_ptr) return RS_ERR_INVAL;
        *dev_ptr = nullptr;
        uint8_t* d = nullptr;
        RS_TRY(host_device_range(host_ptr, bytes, &d));
        *dev_ptr = d;
        return RS_OK;
    });
}

int rs_bind_thread_to_device(int device) {
    return abi_guard([&]() -> int { return bind_thread_to_device(device); });
}

int rs_host_unregister(void* ptr) {
    return abi_guard([&]() -> int {
        if (!ptr) return RS_ERR_INVAL;
        std::unique_lock<std::mutex> lk(g_reg_mu);
        auto it = g_user.find(reinterpret_cast<uintptr_t>(ptr));
        if (it == g_user.end()) return RS_ERR_INVAL;
        const std::vector<std::pair<uintptr_t, uintptr_t>> dead = spans_release(it->second.spans);
        const uintptr_t ps = page_bytes(), ua = it->first;
        const uintptr_t in_lo = (ua + ps - 1) & ~(ps - 1), in_hi = (ua + it->second.bytes) & ~(ps - 1);
        g_user.erase(it);
        if (dead.empty()) return RS_OK;  // every page still held by another registration or the pool
        // No longer found by the lookup; whatever the caller queued over the
        // range finishes before the pages leave the runtime.  The drain runs
        // without g_reg_mu (host calls on other registered memory go on); a
        // registration of these pages from another thread waits for it, so
        // the runtime is never asked to register pages it still holds.
        for (auto& d : dead) g_dying.emplace(d.first, d.second);
        lk.unlock();
        drain_used_devices();
        int rc = RS_OK;
        for (auto& d : dead) {
            const int r = hip_ok(hipHostUnregister(reinterpret_cast<void*>(d.first)), "hipHostUnregister");
            if (rc == RS_OK) rc = r;
            // the caller's own whole pages of this span: GPU access revoked (above)
            if (r == RS_OK) svm_revoke(std::max(d.first, in_lo), std::min(d.second, in_hi));
        }
        lk.lock();
        for (auto& d : dead) g_dying.erase(d.first);
        lk.unlock();
        g_reg_cv.notify_all();
        return rc;
    });
}

int rs_host_alloc(size_t bytes, void** out) {
    return abi_guard([&]() -> int {
        if (!out) return RS_ERR_INVAL;
        *out = nullptr;
        if (bytes == 0 || bytes > (size_t{1} << 40)) return RS_ERR_INVAL;
        size_t cls = size_t{64} << 10;
        while (cls < bytes) cls <<= 1;
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto f = g_pool_free.find(cls);
        if (f != g_pool_free.end()) {
            const uintptr_t b = f->second;
            g_pool_free.erase(f);
            g_pool[b].free = false;
            g_pool_in_use += cls;
            *out = reinterpret_cast<void*>(b);
            return RS_OK;
        }
        Slab& sl = g_slab[cls];
        if (sl.end - sl.next < cls) {  // a new slab: whole granules, 2 MiB-aligned
            const size_t sb = std::max(cls, kPoolGranule);
            void* m = mmap(nullptr, sb + kPoolGranule, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (m == MAP_FAILED) return RS_ERR_NOMEM;
            const uintptr_t a = reinterpret_cast<uintptr_t>(m), lo = (a + kPoolGranule - 1) & ~(kPoolGranule - 1);
            if (lo > a) munmap(m, lo - a);
            if (a + kPoolGranule > lo) munmap(reinterpret_cast<void*>(lo + sb), a + kPoolGranule - lo);
            (void)madvise(reinterpret_cast<void*>(lo), sb, MADV_NOHUGEPAGE);
            const int rc = span_register(lo, lo + sb);  // the pool's own reference: never released
            if (rc != RS_OK) {
                munmap(reinterpret_cast<void*>(lo), sb);
                return rc;
            }
            g_reg_count.store(static_cast<int>(g_spans.size()));
            g_pool_mapped += sb;
            sl.next = lo;
            sl.end = lo + sb;
        }
        const uintptr_t b = sl.next;
        sl.next += cls;
        g_pool.emplace(b, PoolBlock{cls, false});
        g_pool_in_use += cls;
        *out = reinterpret_cast<void*>(b);
        return RS_OK;
    });
}

int rs_host_free(void* ptr) {
    return abi_guard([&]() -> int {
        if (!ptr) return RS_OK;
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_pool.find(reinterpret_cast<uintptr_t>(ptr));
        if (it == g_pool.end() || it->second.free) return RS_ERR_INVAL;  // not a pool block, or freed twice
        it->second.free = true;
        g_pool_in_use -= it->second.bytes;
        g_pool_free.emplace(it->second.bytes, it->first);
        return RS_OK;
    });
}

int rs_host_pool_stats(size_t* mapped, size_t* in_use, size_t* blocks, size_t* spans) {
    return abi_guard([&]() -> int {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        if (mapped) *mapped = g_pool_mapped;
        if (in_use) *in_use = g_pool_in_use;
        if (blocks) *blocks = g_pool.size();
        if (spans) *spans = g_spans.size();
        return RS_OK;
    });
}

// Host-resident encode, three paths: pinned / registered memory -> one
// zero-copy launch over it; pageable memory with stripes <= 16 MiB ->
// encode_pageable_batch (pinned mirror); otherwise a three-stage DMA pipeline
// over a ring of `streams` device slots.  H2D copies run on one stream,
// kernels on a second, D2H on a third, linked by events, so the copy engines
// of both PCIe directions and the CUs work on different chunks at once:
//     h2d:  [wait slot free] copy data(c)  -> ev_in[slot]
//     comp: [wait ev_in]     encode(c)     -> ev_enc[slot]
//     d2h:  [wait ev_enc]    copy parity(c)-> ev_free[slot]
int rs_encode_host_batch(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride, int nstripes,
                         size_t len, int stripes_per_chunk, int streams) {
    return abi_guard([&]() -> int {
        if (!rs || nstripes < 0 || (nstripes > 0 && !base)) return RS_ERR_INVAL;
        if (stripe_stride < 0 || vect_stride < 0) return RS_ERR_INVAL;  // host extents are [base, base+extent)
        if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
        if (nstripes == 0) return RS_OK;
        if (stripes_per_chunk <= 0) stripes_per_chunk = 8;
        int slots = streams <= 0 ? 3 : std::min(streams, 8);
        RS_TRY(ensure_device(rs));
        DeviceGuard g(rs->device);
        const int d = rs->d, p = rs->p;
        uint8_t* zc = nullptr;
        const bool pinned =
            host_device_range(base, batch_extent(stripe_stride, vect_stride, nstripes, d + p, len), &zc) == RS_OK;
        if (g_host_batch_zc && pinned) {
            // pinned / registered caller memory: one launch straight over it
            std::lock_guard<std::mutex> lk(rs->stage_mu);
            if (!rs->stream)
                RS_TRY(hip_ok(hipStreamCreateWithFlags(&rs->stream, hipStreamNonBlocking), "stream create"));
            const uint8_t* in[kMaxVects];
            uint8_t* out[kMaxVects];
            for (int i = 0; i < d; ++i) in[i] = zc + i * vect_stride;
            for (int j = 0; j < p; ++j) out[j] = zc + (d + j) * vect_stride;
            int rc = matmul(rs, rs->gen(), p, d, in, stripe_stride, out, stripe_stride, nstripes, len, false,
                            rs->stream);
            const int sync_rc = hip_ok(hipStreamSynchronize(rs->stream), "host-batch sync");
            return rc ? rc : sync_rc;
        }
        if (!pinned && g_host_pageable_stage) {
            std::lock_guard<std::mutex> lk(rs->stage_mu);
            if (rup(len, 256) * static_cast<size_t>(d + p) <= kPageableStripeMax)
                return encode_pageable_batch(rs, base, stripe_stride, vect_stride, nstripes, len);
            const size_t w = pageable_window(d + p);  // large stripes: byte windows of every vector
            for (size_t off = 0; off < len; off += w)
                RS_TRY(encode_pageable_batch(rs, base + off, stripe_stride, vect_stride, nstripes,
                                             std::min(w, len - off)));
            return RS_OK;
        }
        // [S][d+p][len] with 256-B-multiple len: data and parity of a stripe are contiguous rows
        const bool dense = vect_stride == static_cast<int64_t>(len) && len % 256 == 0;
        // Pageable memory takes 1-D copies only: a 2-D (rectangle) copy from
        // pageable memory with unaligned widths / pitches (8,195-byte vectors)
        // faulted inside the runtime's copy (hipErrorIllegalAddress at the
        // stream sync, intermittently, tests/test_gpu_parity.py
        // test_encode_host_batch_pipeline); pinned memory keeps the 2-D
        // copies (70.4-70.7 vs 66.8-67.1 GiB/s, tools/dma_ab.py).
        const bool rect = pinned && !g_host_dma_1d;
        const size_t pitch = dense ? len : rup(len, 256);
        const int64_t dstripe = static_cast<int64_t>(pitch) * (d + p);
        const size_t slot_bytes = static_cast<size_t>(dstripe) * stripes_per_chunk;
        std::lock_guard<std::mutex> lk(rs->stage_mu);
        int rc = RS_OK;
        if (slot_bytes * slots > rs->dma_ring_bytes) {
            if (rs->dma_ring) {
                for (hipStream_t s : rs->dma_stream)
                    if (s) (void)hipStreamSynchronize(s);
                (void)hipFree(rs->dma_ring);
            }
            rs->dma_ring = nullptr;
            rs->dma_ring_bytes = 0;
            if (hipMalloc(&rs->dma_ring, slot_bytes * slots) != hipSuccess) {
                rs->dma_ring = nullptr;
                return RS_ERR_NOMEM;
            }
            rs->dma_ring_bytes = slot_bytes * slots;
        }
        uint8_t* ring = rs->dma_ring;
        for (hipStream_t& s : rs->dma_stream)
            if (!s && hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "stream create")) {
                s = nullptr;
                return RS_ERR_DEVICE;
            }
        for (auto& row : rs->dma_ev)
            for (int i = 0; i < slots; ++i)
                if (!row[i] && hip_ok(hipEventCreateWithFlags(&row[i], hipEventDisableTiming), "event create")) {
                    row[i] = nullptr;
                    return RS_ERR_DEVICE;
                }
        hipStream_t sh = rs->dma_stream[0], sc = rs->dma_stream[1], sd = rs->dma_stream[2];
        hipEvent_t* ev_in = rs->dma_ev[0];
        hipEvent_t* ev_enc = rs->dma_ev[1];
        hipEvent_t* ev_free = rs->dma_ev[2];
        auto ok = [&](hipError_t e) {
            if (e != hipSuccess && rc == RS_OK) rc = dev_fail(e, "host-batch DMA pipeline");
            return rc == RS_OK;
        };
        const uint8_t* in[kMaxVects];
        uint8_t* out[kMaxVects];
        int chunk = 0;
        for (int c0 = 0; c0 < nstripes && rc == RS_OK; c0 += stripes_per_chunk, ++chunk) {
            const int cn = std::min(stripes_per_chunk, nstripes - c0);
            const int slot = chunk % slots;
            uint8_t* dev = ring + static_cast<size_t>(slot) * slot_bytes;
            uint8_t* hb = base + static_cast<int64_t>(c0) * stripe_stride;
            if (chunk >= slots && !ok(hipStreamWaitEvent(sh, ev_free[slot], 0))) break;
            if (dense && !rect) {  // cn 1-D copies of d*len bytes
                bool good = true;
                for (int s = 0; s < cn && good; ++s)
                    good = ok(hipMemcpyAsync(dev + static_cast<int64_t>(s) * dstripe, hb + s * stripe_stride,
                                             static_cast<size_t>(d) * len, hipMemcpyHostToDevice, sh));
                if (!good) break;
            } else if (dense) {  // one 2-D copy: cn rows of d*len bytes
                if (!ok(hipMemcpy2DAsync(dev, dstripe, hb, stripe_stride, static_cast<size_t>(d) * len, cn,
                                         hipMemcpyHostToDevice, sh)))
                    break;
            } else if (!rect) {  // cn * d 1-D copies of len bytes
                bool good = true;
                for (int s = 0; s < cn && good; ++s)
                    for (int i = 0; i < d && good; ++i)
                        good = ok(hipMemcpyAsync(dev + static_cast<int64_t>(s) * dstripe + i * pitch,
                                                 hb + s * stripe_stride + i * vect_stride, len, hipMemcpyHostToDevice,
                                                 sh));
                if (!good) break;
            } else {
                bool good = true;
                for (int i = 0; i < d && good; ++i)
                    good = ok(hipMemcpy2DAsync(dev + i * pitch, dstripe, hb + i * vect_stride, stripe_stride, len,
                                               cn, hipMemcpyHostToDevice, sh));
                if (!good) break;
            }
            if (!ok(hipEventRecord(ev_in[slot], sh)) || !ok(hipStreamWaitEvent(sc, ev_in[slot], 0))) break;
            for (int i = 0; i < d; ++i) in[i] = dev + i * pitch;
            for (int j = 0; j < p; ++j) out[j] = dev + (d + j) * pitch;
            rc = matmul(rs, rs->gen(), p, d, in, dstripe, out, dstripe, cn, len, false, sc);
            if (rc) break;
            if (!ok(hipEventRecord(ev_enc[slot], sc)) || !ok(hipStreamWaitEvent(sd, ev_enc[slot], 0))) break;
            if (dense && !rect) {
                bool good = true;
                for (int s = 0; s < cn && good; ++s)
                    good = ok(hipMemcpyAsync(hb + s * stripe_stride + d * vect_stride,
                                             dev + static_cast<int64_t>(s) * dstripe + d * pitch,
                                             static_cast<size_t>(p) * len, hipMemcpyDeviceToHost, sd));
                if (!good) break;
            } else if (dense) {
                if (!ok(hipMemcpy2DAsync(hb + d * vect_stride, stripe_stride, dev + d * pitch, dstripe,
                                         static_cast<size_t>(p) * len, cn, hipMemcpyDeviceToHost, sd)))
                    break;
            } else if (!rect) {
                bool good = true;
                for (int s = 0; s < cn && good; ++s)
                    for (int j = 0; j < p && good; ++j)
                        good = ok(hipMemcpyAsync(hb + s * stripe_stride + (d + j) * vect_stride,
                                                 dev + static_cast<int64_t>(s) * dstripe + (d + j) * pitch, len,
                                                 hipMemcpyDeviceToHost, sd));
                if (!good) break;
            } else {
                bool good = true;
                for (int j = 0; j < p && good; ++j)
                    good = ok(hipMemcpy2DAsync(hb + (d + j) * vect_stride, stripe_stride, dev + (d + j) * pitch,
                                               dstripe, len, cn, hipMemcpyDeviceToHost, sd));
                if (!good) break;
            }
            if (!ok(hipEventRecord(ev_free[slot], sd))) break;
        }
        for (hipStream_t s : {sh, sc, sd}) {
            const hipError_t e = hipStreamSynchronize(s);
            if (e != hipSuccess) rc = dev_fail(e, "host-batch DMA pipeline sync");
        }
        return rc;
    });
}

// ---------------------------------------------------------------- device groups

struct rs_group {
    std::vector<rs_t*> members;
};

int rs_group_new(int data_num, int parity_num, const int* devices, int ndev, rs_group_t** out) {
    return abi_guard([&]() -> int {
        if (!out) return RS_ERR_INVAL;
        *out = nullptr;
        if (ndev <= 0 || ndev > 1024 || !devices) return RS_ERR_INVAL;
        rs_group_t* g = new (std::nothrow) rs_group();
        if (!g) return RS_ERR_NOMEM;
        for (int i = 0; i < ndev; ++i) {
            rs_t* r = nullptr;
            int rc = devices[i] < 0 ? RS_ERR_INVAL : rs_new(data_num, parity_num, devices[i], &r);
            if (rc) {
                rs_group_free(g);
                return rc;
            }
            g->members.push_back(r);
        }
        *out = g;
        return RS_OK;
    });
}

void rs_group_free(rs_group_t* g) {
    if (!g) return;
    for (rs_t* r : g->members) rs_free(r);
    delete g;
}

int rs_group_size(const rs_group_t* g) { return g ? static_cast<int>(g->members.size()) : 0; }

// Member i's contiguous slice of a batch (every group entry point splits this way).
static void group_slice(int nstripes, int n, int i, int* lo, int* hi) {
    *lo = static_cast<int>(static_cast<int64_t>(nstripes) * i / n);
    *hi = static_cast<int>(static_cast<int64_t>(nstripes) * (i + 1) / n);
}

int rs_group_slice(const rs_group_t* g, int nstripes, int i, int* lo, int* hi) {
    if (!g || !lo || !hi || nstripes < 0 || i < 0 || i >= static_cast<int>(g->members.size())) return RS_ERR_INVAL;
    group_slice(nstripes, static_cast<int>(g->members.size()), i, lo, hi);
    return RS_OK;
}

rs_t* rs_group_codec(rs_group_t* g, int i) {
    return g && i >= 0 && i < static_cast<int>(g->members.size()) ? g->members[i] : nullptr;
}

int rs_group_encode_host_batch(rs_group_t* g, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                               int nstripes, size_t len, int stripes_per_chunk, int streams) {
    return abi_guard([&]() -> int {
        if (!g || g->members.empty() || nstripes < 0 || (nstripes > 0 && !base)) return RS_ERR_INVAL;
        if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
        const int n = static_cast<int>(g->members.size());
        std::vector<int> rc(n, RS_OK);
        std::vector<std::thread> th;
        for (int i = 0; i < n; ++i) {
            int lo = 0, hi = 0;
            group_slice(nstripes, n, i, &lo, &hi);
            if (hi <= lo) continue;
            auto job = [&, i, lo, hi] {
                rc[i] = rs_encode_host_batch(g->members[i], base + static_cast<int64_t>(lo) * stripe_stride,
                                             stripe_stride, vect_stride, hi - lo, len, stripes_per_chunk, streams);
            };
            try {
                const int dev = g->members[i]->device;
                th.emplace_back([job, dev] {  // a worker of its own: bind it to the GPU's NUMA node
                    if (g_bind_numa) (void)bind_thread_to_device(dev);
                    job();
                });
            } catch (...) {
                job();  // no thread available: run this slice here
            }
        }
        for (std::thread& t : th) t.join();
        for (int r : rc)
            if (r) return r;
        return RS_OK;
    });
}

static int reconst_host_multi(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride, int nstripes,
                              size_t len, MaskView masks) {
    if (!rs || nstripes < 0 || (nstripes > 0 && (!base || !masks.m))) return RS_ERR_INVAL;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    if (nstripes == 0) return RS_OK;
    if (stripe_stride < 0 || vect_stride < 0) return RS_ERR_INVAL;
    const int d = rs->d, p = rs->p;
    RS_TRY(check_masks(d, p, masks, nstripes));  // before any device work, copy or launch
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    uint8_t* zc = nullptr;
    if (host_device_range(base, batch_extent(stripe_stride, vect_stride, nstripes, d + p, len), &zc) != RS_OK) {
        // pageable memory: staged through the pinned mirror (large stripes in
        // byte windows of every vector)
        if (!g_host_pageable_stage) return RS_ERR_INVAL;
        std::lock_guard<std::mutex> lk(rs->stage_mu);
        if (rup(len, 256) * static_cast<size_t>(d + p) <= kPageableStripeMax)
            return reconst_pageable_batch(rs, base, stripe_stride, vect_stride, nstripes, len, masks);
        const size_t w = pageable_window(d + p);
        for (size_t off = 0; off < len; off += w)
            RS_TRY(reconst_pageable_batch(rs, base + off, stripe_stride, vect_stride, nstripes, std::min(w, len - off),
                                          masks));
        return RS_OK;
    }
    rs_layout_t L{zc, stripe_stride, vect_stride, zc + static_cast<int64_t>(d) * vect_stride, stripe_stride,
                  vect_stride};
    std::lock_guard<std::mutex> lk(rs->stage_mu);
    if (!rs->stream) RS_TRY(hip_ok(hipStreamCreateWithFlags(&rs->stream, hipStreamNonBlocking), "stream create"));
    int rc = reconst_multi(rs, &L, nstripes, len, masks, rs->stream);
    const int sync_rc = hip_ok(hipStreamSynchronize(rs->stream), "host-batch sync");
    return rc ? rc : sync_rc;
}

static int group_reconst_host_multi(rs_group_t* g, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                                    int nstripes, size_t len, MaskView masks) {
    if (!g || g->members.empty() || nstripes < 0 || (nstripes > 0 && (!base || !masks.m))) return RS_ERR_INVAL;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    // every slice's masks checked before any member starts (no partial batch)
    RS_TRY(check_masks(g->members[0]->d, g->members[0]->p, masks, nstripes));
    const int n = static_cast<int>(g->members.size());
    std::vector<int> rc(n, RS_OK);
    std::vector<std::thread> th;
    for (int i = 0; i < n; ++i) {
        int lo = 0, hi = 0;
        group_slice(nstripes, n, i, &lo, &hi);
        if (hi <= lo) continue;
        auto job = [&, i, lo, hi] {
            rc[i] = reconst_host_multi(g->members[i], base + static_cast<int64_t>(lo) * stripe_stride, stripe_stride,
                                       vect_stride, hi - lo, len, masks.from(lo));
        };
        try {
            const int dev = g->members[i]->device;
            th.emplace_back([job, dev] {  // a worker of its own: bind it to the GPU's NUMA node
                if (g_bind_numa) (void)bind_thread_to_device(dev);
                job();
            });
        } catch (...) {
            job();  // no thread available: run this slice here
        }
    }
    for (std::thread& t : th) t.join();
    for (int r : rc)
        if (r) return r;
    return RS_OK;
}

int rs_reconst_host_batch_multi(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride, int nstripes,
                                size_t len, const uint64_t* need_masks) {
    return abi_guard([&]() -> int {
        return reconst_host_multi(rs, base, stripe_stride, vect_stride, nstripes, len, MaskView{need_masks, 1});
    });
}

int rs_reconst_host_batch_multi256(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride, int nstripes,
                                   size_t len, const uint64_t* need_masks) {
    return abi_guard([&]() -> int {
        return reconst_host_multi(rs, base, stripe_stride, vect_stride, nstripes, len, MaskView{need_masks, 4});
    });
}

int rs_group_reconst_host_batch_multi(rs_group_t* g, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                                      int nstripes, size_t len, const uint64_t* need_masks) {
    return abi_guard([&]() -> int {
        return group_reconst_host_multi(g, base, stripe_stride, vect_stride, nstripes, len, MaskView{need_masks, 1});
    });
}

int rs_group_reconst_host_batch_multi256(rs_group_t* g, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                                         int nstripes, size_t len, const uint64_t* need_masks) {
    return abi_guard([&]() -> int {
        return group_reconst_host_multi(g, base, stripe_stride, vect_stride, nstripes, len, MaskView{need_masks, 4});
    });
}

}  // extern "C"
