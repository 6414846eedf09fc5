// host_calls.cpp — the synchronous host-memory entry points (the Go API's
// shape: rs_encode / rs_reconst / rs_update / rs_replace on caller vectors
// in pageable host memory): column-chunked zero-copy staging through a
// pinned mirror, or the staged DMA paths for large vectors.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <chrono>

#include "host_pool.hpp"
#include "codec_internal.hpp"

#include <immintrin.h>

using namespace rsamd;
using namespace rsamd::detail;

namespace rsamd {
namespace detail {

// ---------------------------------------------------------------- host staging

// Vectors up to this size go through the pinned host mirror: the caller's
// bytes are memcpy'd into pinned memory and each direction is ONE DMA over
// contiguous slots, instead of one pageable copy (staged by the runtime) per
// vector.  Larger vectors use the runtime's pipelined pageable copies.
size_t g_pinned_max = 256 * 1024;
// Host calls on vectors up to this size take the chunked zero-copy pipeline
// (host_matmul: the kernel reads and writes the pinned mirror over PCIe, no
// DMA set-up either way); larger ones the staged path (device staging slots,
// DMA through the pinned bounce buffer).  Round 1 measured the runtime's
// pageable copies 7 % faster than the pipeline at 4 MiB and set 2 MiB here;
// since the bounce buffer replaced those copies (round 3) the staged path is
// the slower one at every size (4 MiB Encode 2,267-2,448 vs 1,592-1,939 us,
// profiles/r04/host_zc_threshold.log), so there is no limit by default.
size_t g_zc_max = SIZE_MAX;

bool use_pinned(rs_t* rs, int slots, size_t pitch) {
    if (pitch > g_pinned_max) return false;
    const size_t need = pitch * static_cast<size_t>(slots);
    if (need <= rs->hstage_bytes) return true;
    if (rs->hstage) {
        (void)hipStreamSynchronize(rs->stream);
        (void)hipHostFree(rs->hstage);
        rs->hstage = nullptr;
        rs->hstage_bytes = 0;
        rs->zc_pending = false;
    }
    if (hipHostMalloc(reinterpret_cast<void**>(&rs->hstage), need, hipHostMallocDefault) != hipSuccess) return false;
    rs->hstage_bytes = need;
    return true;
}

// Device staging area of the staged host path: `slots` vectors of `pitch`
// bytes (pitch 256-aligned so every slot takes the vector kernel), at
// rs->slots.  Caller holds stage_mu.
int ensure_stage(rs_t* rs, int slots, size_t size, size_t* pitch) {
    *pitch = rup(size, 256);
    const size_t need = *pitch * static_cast<size_t>(slots);
    if (!rs->stream) RS_TRY(hip_ok(hipStreamCreateWithFlags(&rs->stream, hipStreamNonBlocking), "stream create"));
    if (need > rs->stage_bytes) {
        if (rs->stage) {
            (void)hipStreamSynchronize(rs->stream);
            (void)hipFree(rs->stage);
            rs->stage = nullptr;
            rs->stage_bytes = 0;
        }
        if (hipMalloc(&rs->stage, need) != hipSuccess) {
            rs->stage = nullptr;
            return RS_ERR_NOMEM;
        }
        rs->stage_bytes = need;
    }
    rs->slots = rs->stage;
    return RS_OK;
}

// Host vectors src[0..n) (size bytes each) -> device staging slots
// [first, first+n).  Caller holds stage_mu and called ensure_stage.
int stage_in(rs_t* rs, const uint8_t* const* src, int n, size_t size, size_t pitch, int first, int total_slots);
int stage_out(rs_t* rs, uint8_t* const* dst, int n, size_t size, size_t pitch, int first, int total_slots);

int h2d(rs_t* rs, uint8_t* dst, const uint8_t* src, size_t n) {
    return hip_ok(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, rs->stream), "host-call H2D copy");
}
int d2h(rs_t* rs, uint8_t* dst, const uint8_t* src, size_t n) {
    return hip_ok(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, rs->stream), "host-call D2H copy");
}
int sync(rs_t* rs) {
    return hip_ok(hipStreamSynchronize(rs->stream), "host-call stream sync");
}

// A launch-path host call waits for its kernel through a flag instead of
// hipStreamSynchronize: the stream writes a sequence number into a pinned
// word after the kernel (hipStreamWriteValue32, ordered behind it, so the
// kernel's stores to host memory are complete) and the caller spins on the
// word.  A launch + stream sync has a ~12 us floor on MI355X against ~6 us for
// a launch + host flag (profiles/r02/doorbell_probe.log).  Falls back to the
// stream sync when the write cannot be queued, or after 10 s without the
// flag.  rs_tune("host_flag_sync", 1 default | 0).
int g_host_flag_sync = 1;

int flag_sync(hipStream_t st, rs_codec::DoneFlag& f, const char* where) {
    if (g_host_flag_sync && !f.host) {  // (a recycled coherent block: its word starts at this handle's seq)
        size_t cap = 0;
        void* d = nullptr;
        if (uint8_t* h = coherent_get(64, &cap, &d)) {
            if (d) {
                f.host = reinterpret_cast<uint32_t*>(h);
                f.dev = d;
                __atomic_store_n(f.host, f.seq, __ATOMIC_RELEASE);
            } else {
                coherent_put(h, cap);
            }
        }
    }
    if (!g_host_flag_sync || !f.host) return hip_ok(hipStreamSynchronize(st), where);
    const uint32_t v = ++f.seq;
    if (hipStreamWriteValue32(st, f.dev, v, 0) != hipSuccess) {
        (void)hipGetLastError();
        return hip_ok(hipStreamSynchronize(st), where);
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spins = 1; __atomic_load_n(f.host, __ATOMIC_ACQUIRE) != v; ++spins) {
        _mm_pause();
        if ((spins & 4095) != 0) continue;
        const auto waited = std::chrono::steady_clock::now() - t0;
        if (waited < std::chrono::microseconds(200)) continue;  // (a call's kernel is done within ~30 us)
        // A faulted kernel or queue never writes the flag: the stream's error
        // comes back now instead of after the 10 s bound (advisor r05).
        // (This stream holds no resident kernel.)
        const hipError_t q = hipStreamQuery(st);
        if (q != hipSuccess && q != hipErrorNotReady) return hip_ok(q, where);
        if (q == hipErrorNotReady) (void)hipGetLastError();
        if (waited > std::chrono::seconds(10)) return hip_ok(hipStreamSynchronize(st), where);
    }
    return RS_OK;
}

// Pageable vectors never go to the runtime's pageable copies (which pin the
// caller's pages behind the scenes): they pass through a pinned bounce buffer
// of the handle, two halves of kBounceHalf, so the host copy of one piece
// overlaps the DMA of the other.  (Round 3: the full GPU suite failed 2 runs
// in 3 with hipErrorIllegalAddress at the first runtime pageable H2D copy of
// a staged call, always in the one test that forces that path; every other
// copy of the library reads or writes pinned memory.)
constexpr size_t kBounceHalf = size_t{2} << 20;

static int ensure_bounce(rs_t* rs) {
    if (rs->bounce) return RS_OK;
    for (hipEvent_t& e : rs->bounce_ev)
        if (!e) RS_TRY(hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "bounce event"));
    void* h = nullptr;
    if (hipHostMalloc(&h, 2 * kBounceHalf, hipHostMallocDefault) != hipSuccess) return RS_ERR_NOMEM;
    rs->bounce = static_cast<uint8_t*>(h);
    return RS_OK;
}

static int bounce_h2d(rs_t* rs, uint8_t* dev, const uint8_t* src, size_t n, size_t* piece) {
    RS_TRY(ensure_bounce(rs));
    for (size_t off = 0; off < n; off += kBounceHalf, ++*piece) {
        const int h = static_cast<int>(*piece & 1);
        const size_t b = std::min(kBounceHalf, n - off);
        uint8_t* buf = rs->bounce + h * kBounceHalf;
        if (*piece >= 2) RS_TRY(hip_ok(hipEventSynchronize(rs->bounce_ev[h]), "bounce wait"));  // its last copy read it
        std::memcpy(buf, src + off, b);
        RS_TRY(h2d(rs, dev + off, buf, b));
        RS_TRY(hip_ok(hipEventRecord(rs->bounce_ev[h], rs->stream), "bounce record"));
    }
    return RS_OK;
}

static int bounce_d2h(rs_t* rs, uint8_t* dst, const uint8_t* dev, size_t n) {
    RS_TRY(ensure_bounce(rs));
    const size_t pieces = (n + kBounceHalf - 1) / kBounceHalf;
    auto issue = [&](size_t k) {
        const size_t off = k * kBounceHalf, b = std::min(kBounceHalf, n - off);
        const int h = static_cast<int>(k & 1);
        RS_TRY(d2h(rs, rs->bounce + h * kBounceHalf, dev + off, b));
        return hip_ok(hipEventRecord(rs->bounce_ev[h], rs->stream), "bounce record");
    };
    if (pieces) RS_TRY(issue(0));
    for (size_t k = 0; k < pieces; ++k) {
        if (k + 1 < pieces) RS_TRY(issue(k + 1));  // (the half piece k + 1 uses was emptied at k - 1)
        const int h = static_cast<int>(k & 1);
        RS_TRY(hip_ok(hipEventSynchronize(rs->bounce_ev[h]), "bounce wait"));
        const size_t off = k * kBounceHalf;
        std::memcpy(dst + off, rs->bounce + h * kBounceHalf, std::min(kBounceHalf, n - off));
    }
    return RS_OK;
}

int stage_in(rs_t* rs, const uint8_t* const* src, int n, size_t size, size_t pitch, int first, int total_slots) {
    if (n <= 0) return RS_OK;
    uint8_t* dev = rs->stage + static_cast<size_t>(first) * pitch;
    if (use_pinned(rs, total_slots, pitch)) {
        uint8_t* h = rs->hstage + static_cast<size_t>(first) * pitch;
        for (int i = 0; i < n; ++i) std::memcpy(h + static_cast<size_t>(i) * pitch, src[i], size);
        return h2d(rs, dev, h, static_cast<size_t>(n - 1) * pitch + size);
    }
    size_t piece = 0;
    for (int i = 0; i < n; ++i) RS_TRY(bounce_h2d(rs, dev + static_cast<size_t>(i) * pitch, src[i], size, &piece));
    return RS_OK;
}

// Device staging slots [first, first+n) -> host vectors dst[0..n); synchronous.
int stage_out(rs_t* rs, uint8_t* const* dst, int n, size_t size, size_t pitch, int first, int total_slots) {
    if (n <= 0) return sync(rs);
    const uint8_t* dev = rs->stage + static_cast<size_t>(first) * pitch;
    if (use_pinned(rs, total_slots, pitch)) {
        uint8_t* h = rs->hstage + static_cast<size_t>(first) * pitch;
        RS_TRY(d2h(rs, h, dev, static_cast<size_t>(n - 1) * pitch + size));
        RS_TRY(sync(rs));
        for (int i = 0; i < n; ++i) std::memcpy(dst[i], h + static_cast<size_t>(i) * pitch, size);
        return RS_OK;
    }
    for (int i = 0; i < n; ++i) RS_TRY(bounce_d2h(rs, dst[i], dev + static_cast<size_t>(i) * pitch, size));
    return sync(rs);
}


// Column-chunk size of the host-call pipeline (bytes per vector per chunk):
// at least g_chunk, and at least 1/g_chunk_split of the vectors (0 = g_chunk
// alone), within 8 MiB per slot.  Each chunk costs a launch, an event wait
// and two pool dispatches (~20 us), so large vectors take a few large chunks:
// 10+4 pageable Encode at 1 / 2 MiB 397-408 / 780-881 us with 128 KiB
// chunks, 337-353 / 601-666 with host_chunk_split 4 (alternating in one
// process, profiles/r06/host_chunk_split_ab_1m.log); 4 / 16 MiB 1.6-2.4 /
// 6.6-6.8 ms -> 1.1-1.4 / 4.1-4.4 ms (host_chunk_split_sweep.log).
size_t g_chunk = 128 * 1024;
size_t g_chunk_split = 4;
// Total copy bytes of one chunk above which the staging copies are split
// over the host copy pool.
constexpr size_t kParallelCopyMin = 512 * 1024;

// Staging copies of large batches store with non-temporal stores
// (rs_tune("host_copy_nt"), default 1): the pinned mirror is read by the GPU
// over PCIe and the caller's outputs are not read back at once, so the
// copies skip the read-for-ownership of every destination line and leave the
// caches to the source.  Pieces below 4 KiB, and CPUs without AVX2, use memcpy.
int g_copy_nt = 1;
static const bool g_copy_avx2 = __builtin_cpu_supports("avx2");

__attribute__((target("avx2"))) static void copy_nt(uint8_t* dst, const uint8_t* src, size_t b) {
    const size_t head = (32 - (reinterpret_cast<uintptr_t>(dst) & 31)) & 31;
    std::memcpy(dst, src, head);
    size_t i = head;
    for (; i + 128 <= b; i += 128) {
        const __m256i a0 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
        const __m256i a1 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
        const __m256i a2 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
        const __m256i a3 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), a0);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 32), a1);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 64), a2);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 96), a3);
    }
    std::memcpy(dst + i, src + i, b - i);
    _mm_sfence();  // the streamed lines are globally visible before the copier reports the piece done
}

static void copy_piece(uint8_t* dst, const uint8_t* src, size_t b) {
    if (g_copy_nt && g_copy_avx2 && b >= 4096) copy_nt(dst, src, b);
    else std::memcpy(dst, src, b);
}

// Vectors that lie back to back in both source and destination (the data
// rows of a dense [S][d+p][len] batch and its mirror stripe) are copied as
// one run, in 64 KiB pieces, instead of one piece per vector: 8 KiB vectors
// otherwise cost a pool hand-out per 8 KiB.  rs_tune("host_copy_coalesce").
int g_copy_coalesce = 1;

// dst[i] <- src[i] (n vectors, len bytes each) on the copy pool, in
// 64 KiB pieces so every thread gets work; on the calling thread alone when
// the pool is busy with another caller's copies.
void parallel_copy(uint8_t* const* dst, const uint8_t* const* src, int n, size_t len) {
    const size_t piece = 64 * 1024;
    if (len * static_cast<size_t>(n) < kParallelCopyMin || (n <= 1 && len <= piece)) {
        for (int i = 0; i < n; ++i) std::memcpy(dst[i], src[i], len);
        return;
    }
    struct Run {
        uint8_t* d;
        const uint8_t* s;
        size_t bytes;
    };
    std::vector<Run> runs;
    runs.reserve(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i) {
        if (g_copy_coalesce && !runs.empty() && runs.back().d + runs.back().bytes == dst[i] &&
            runs.back().s + runs.back().bytes == src[i])
            runs.back().bytes += len;
        else
            runs.push_back(Run{dst[i], src[i], len});
    }
    std::vector<Run> pieces;
    for (const Run& r : runs)
        for (size_t off = 0; off < r.bytes; off += piece)
            pieces.push_back(Run{r.d + off, r.s + off, std::min(piece, r.bytes - off)});
    CopyPool::get().run_or_inline(pieces.size(), [&](size_t k) { copy_piece(pieces[k].d, pieces[k].s, pieces[k].bytes); });
}

// The synchronous host-memory product behind rs_encode / rs_reconst /
// rs_update / rs_replace: dst[r] (=|^=) sum_c mat[r][c] x src[c], all host
// pointers, `size` bytes each.  The vectors are cut into column chunks;
// each chunk is copied into a slot of the pinned mirror (several host
// threads), processed by the kernel straight out of the mirror over PCIe
// (zero-copy: no DMA set-up), and copied back, with up to 3 chunks in
// flight so copies overlap the GPU.  Caller holds stage_mu.
int host_matmul(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* src, uint8_t* const* dst,
                size_t size, bool accumulate) {
    const int nvec = rows + cols;
    if (!rs->stream) RS_TRY(hip_ok(hipStreamCreateWithFlags(&rs->stream, hipStreamNonBlocking), "stream create"));
    // chunk: max(g_chunk, size / g_chunk_split) per vector, <= 8 MiB per slot, 4 KiB multiple
    size_t C = rup(size, 256);
    const size_t want = g_chunk_split ? std::max(g_chunk, rup(size / g_chunk_split, 4096)) : g_chunk;
    const size_t cap = std::max<size_t>(4096, std::min(want, (size_t{8} << 20) / nvec) & ~size_t{4095});
    if (C > cap) C = cap;
    const size_t nch = (size + C - 1) / C;
    const int ns = nch > 1 ? 3 : 1;
    const size_t slot = C * static_cast<size_t>(nvec);
    if (rs->zc_pending) RS_TRY(sync(rs));
    if (slot * ns > rs->hstage_bytes) {
        if (rs->hstage) {
            (void)hipHostFree(rs->hstage);
            rs->hstage = nullptr;
            rs->hstage_bytes = 0;
        }
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
    auto hslot = [&](size_t c, int v) { return rs->hstage + (c % ns) * slot + static_cast<size_t>(v) * C; };
    auto dslot = [&](size_t c, int v) {
        return static_cast<uint8_t*>(dbase) + (c % ns) * slot + static_cast<size_t>(v) * C;
    };
    auto clen = [&](size_t c) { return std::min(C, size - c * C); };
    auto finish = [&](size_t c) -> int {  // wait for chunk c, copy its outputs back
        RS_TRY(hip_ok(hipEventSynchronize(rs->chunk_ev[c % ns]), "host-call chunk sync"));
        uint8_t* d[kMaxVects];
        const uint8_t* h[kMaxVects];
        for (int r = 0; r < rows; ++r) {
            d[r] = dst[r] + c * C;
            h[r] = hslot(c, cols + r);
        }
        parallel_copy(d, h, rows, clen(c));
        return RS_OK;
    };
    int rc = RS_OK;
    size_t done = 0;
    for (size_t c = 0; c < nch && rc == RS_OK; ++c) {
        if (c >= static_cast<size_t>(ns)) {
            rc = finish(done++);
            if (rc) break;
        }
        const size_t len = clen(c);
        uint8_t* h[2 * kMaxVects];
        const uint8_t* s_[2 * kMaxVects];
        int n = 0;
        for (int i = 0; i < cols; ++i, ++n) {
            h[n] = hslot(c, i);
            s_[n] = src[i] + c * C;
        }
        if (accumulate)
            for (int r = 0; r < rows; ++r, ++n) {
                h[n] = hslot(c, cols + r);
                s_[n] = dst[r] + c * C;
            }
        parallel_copy(h, s_, n, len);
        const uint8_t* in[kMaxVects];
        uint8_t* out[kMaxVects];
        for (int i = 0; i < cols; ++i) in[i] = dslot(c, i);
        for (int r = 0; r < rows; ++r) out[r] = dslot(c, cols + r);
        rs->zc_pending = true;
        rc = matmul(rs, mat, rows, cols, in, 0, out, 0, 1, len, accumulate, rs->stream);
        if (rc == RS_OK) rc = hip_ok(hipEventRecord(rs->chunk_ev[c % ns], rs->stream), "host-call chunk record");
    }
    while (rc == RS_OK && done < nch) rc = finish(done++);
    if (rc) (void)hipStreamSynchronize(rs->stream);  // never leave a kernel on the mirror
    rs->zc_pending = false;
    return rc;
}

// Host-call dispatcher: the chunked zero-copy pipeline (default), or the
// older staged paths (device staging + pinned DMA or pageable copies) for
// vectors above host_zc_max (kept for A/B).
int host_product(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* src, uint8_t* const* dst,
                 size_t size, bool accumulate) {
    if (size <= g_zc_max) return host_matmul(rs, mat, rows, cols, src, dst, size, accumulate);
    size_t pitch = 0;
    RS_TRY(ensure_stage(rs, cols + rows, size, &pitch));
    const uint8_t* in[kMaxVects];
    uint8_t* out[kMaxVects];
    const uint8_t* s_[2 * kMaxVects];
    for (int i = 0; i < cols; ++i) {
        in[i] = rs->slots + static_cast<size_t>(i) * pitch;
        s_[i] = src[i];
    }
    for (int r = 0; r < rows; ++r) {
        out[r] = rs->slots + static_cast<size_t>(cols + r) * pitch;
        s_[cols + r] = dst[r];
    }
    RS_TRY(stage_in(rs, s_, accumulate ? cols + rows : cols, size, pitch, 0, cols + rows));
    RS_TRY(matmul(rs, mat, rows, cols, in, 0, out, 0, 1, size, accumulate, rs->stream));
    return stage_out(rs, dst, rows, size, pitch, cols, cols + rows);
}

// ---------------------------------------------------------------- pinned pool

namespace {
std::mutex g_pinned_mu;
std::multimap<size_t, PinnedBlock> g_pinned_free;
}  // namespace

int pinned_get(size_t bytes, PinnedBlock* out) {
    size_t cls = size_t{64} << 10;
    while (cls < bytes) cls <<= 1;
    {
        std::lock_guard<std::mutex> lk(g_pinned_mu);
        auto it = g_pinned_free.find(cls);
        if (it != g_pinned_free.end()) {
            *out = it->second;
            g_pinned_free.erase(it);
            return RS_OK;
        }
    }
    void* h = nullptr;
    Region region("hipHostMalloc (pinned pool block)");
    // default (coarse-grained) pinned memory: the zero-copy kernels and the
    // engine (system-scope acquire / release fences) read it faster than
    // coherent memory (10+4 @ 8 KiB host Encode 10.1 vs 11.1 us)
    if (hipHostMalloc(&h, cls, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) return RS_ERR_NOMEM;
    void* d = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess || !d) {
        std::lock_guard<std::mutex> lk(g_pinned_mu);
        g_pinned_free.emplace(cls, PinnedBlock{static_cast<uint8_t*>(h), nullptr, cls});  // kept, never handed out
        return dev_fail(e != hipSuccess ? e : hipErrorInvalidValue, "pinned block device pointer");
    }
    *out = PinnedBlock{static_cast<uint8_t*>(h), static_cast<uint8_t*>(d), cls};
    return RS_OK;
}

void pinned_put(PinnedBlock& b) {
    if (b.host && b.dev) {
        std::lock_guard<std::mutex> lk(g_pinned_mu);
        g_pinned_free.emplace(b.bytes, b);
    }
    b = PinnedBlock{};
}

// ---------------------------------------------------------------- coalescing

// Vectors up to this size take part in host-call coalescing (0 = off).
size_t g_coalesce_max = 128 * 1024;
// Group-commit window: a ready batch waits up to this long for more callers
// before it launches (0 = launch as soon as the GPU is free; the default).
int g_coalesce_linger_us = 0;
// Waiters spin this long on a batch state change before blocking, and only
// while at most this many callers are inside host_call.
int g_co_spin_us = 30;
int g_co_spin_callers = 8;
// Coalesced batches in flight at once (the engine overlaps their round trips).
int g_co_running = 2;
// Small calls the engine takes skip coalescing: each caller stages its own
// stripe in a pinned pool block and rings the engine itself; calls of
// several threads are in flight at once on different engine workgroups.
int g_engine_direct = 1;
static const bool g_host_trace = std::getenv("RSAMD_ENGINE_TRACE") != nullptr;
// Upper bound on one coalesced batch's pinned bytes and stripe count.
constexpr size_t kCoalesceBytes = size_t{32} << 20;
constexpr int kCoalesceStripes = 256;

using CoBatch = rs_codec::CoBatch;

static bool same_shape(const CoBatch& b, const uint8_t* mat, int rows, int cols, size_t size, bool acc) {
    return b.rows == rows && b.cols == cols && b.size == size && b.accumulate == acc &&
           std::memcmp(b.mat.data(), mat, static_cast<size_t>(rows) * cols) == 0;
}

// (Re)shape an idle batch for calls of this shape.  Caller holds co_mu.
static int init_batch(CoBatch& b, const uint8_t* mat, int rows, int cols, size_t size, bool acc) {
    b.mat.assign(mat, mat + static_cast<size_t>(rows) * cols);
    b.rows = rows;
    b.cols = cols;
    b.size = size;
    b.accumulate = acc;
    b.pitch = rup(size, 256);
    b.stride = b.pitch * static_cast<size_t>(rows + cols);
    b.cap = static_cast<int>(std::max<size_t>(1, std::min<size_t>(kCoalesceStripes, kCoalesceBytes / b.stride)));
    const size_t need = b.stride * static_cast<size_t>(b.cap);
    if (need > b.host_bytes) {
        pinned_put(b.blk);
        b.host = b.dev = nullptr;
        b.host_bytes = 0;
        RS_TRY(pinned_get(need, &b.blk));
        b.host = b.blk.host;
        b.dev = b.blk.dev;
        b.host_bytes = b.blk.bytes;
    }
    b.joined = b.ready = b.released = 0;
    b.launchable = false;
    b.rc = RS_OK;
    b.state = CoBatch::kFilling;
    return RS_OK;
}

// One launch over the batch's n stripes, straight out of the pinned buffer
// (zero-copy), then wait for it.
static int run_batch(rs_t* rs, const CoBatch& b, int n) {
    // small batches: the resident engine (engine.cpp), no launch and no stream sync
    const int erc = engine_call(rs, b.mat.data(), b.rows, b.cols, b.dev, b.pitch, b.stride, n, b.accumulate,
                                /*coherent*/ false);  // measured: outputs stale without the release write-back
    if (erc != RS_ERR_INVAL) return erc;
    const uint8_t* in[kMaxVects];
    uint8_t* out[kMaxVects];
    for (int i = 0; i < b.cols; ++i) in[i] = b.dev + static_cast<size_t>(i) * b.pitch;
    for (int r = 0; r < b.rows; ++r) out[r] = b.dev + static_cast<size_t>(b.cols + r) * b.pitch;
    Region region("coalesced batch launch + sync");
    std::lock_guard<std::mutex> lk(rs->co_launch_mu);
    const int rc = matmul(rs, b.mat.data(), b.rows, b.cols, in, static_cast<int64_t>(b.stride), out,
                          static_cast<int64_t>(b.stride), n, b.size, b.accumulate, rs->co_stream);
    engine_warm_async(rs);  // (a cold engine declined this batch: it restarts behind it, on the warmer thread)
    const int src = flag_sync(rs->co_stream, rs->co_flag, "coalesced batch sync");  // never leave a kernel on the buffer
    return rc ? rc : src;
}

// Wait for the next batch state change: spin briefly on co_gen (a futex
// wake costs several us, as much as a whole engine call), then block.
static void co_wait(rs_t* rs, std::unique_lock<std::mutex>& lk) {
    Region region("coalesce wait");
    const uint64_t g = rs->co_gen.load(std::memory_order_acquire);
    if (rs->co_active > g_co_spin_callers) {  // oversubscribed: spinners would take the copiers' CPUs
        rs->co_cv.wait(lk);
        return;
    }
    lk.unlock();
    const auto t0 = std::chrono::steady_clock::now();
    bool changed = false;
    for (uint32_t i = 0; !changed; ++i) {
        changed = rs->co_gen.load(std::memory_order_acquire) != g;
        if ((i & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(g_co_spin_us)) break;
    }
    lk.lock();
    if (!changed && rs->co_gen.load(std::memory_order_acquire) == g) rs->co_cv.wait(lk);
}

static void co_changed(rs_t* rs) {  // caller holds co_mu
    rs->co_gen.fetch_add(1, std::memory_order_acq_rel);
    rs->co_cv.notify_all();
}

// The synchronous host calls' entry (rs_encode / rs_reconst / rs_update /
// rs_replace).  Vectors up to g_coalesce_max join a batch of concurrent
// calls of the same shape:
//   join (or open) a filling batch -> copy own inputs into own stripe slot
//   -> the last ready member launches the batch once the GPU is free (one
//   launch for every stripe that joined) -> each member copies its own
//   outputs back and leaves; the batch is reused when all have left.
// Copies run on the callers' own threads, in parallel; two batches let one
// fill while the other runs.  A lone caller's call is one launch, as before.
int host_call(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* src, uint8_t* const* dst,
              size_t size, bool accumulate) {
    if (size > 0 && g_reg_count.load(std::memory_order_relaxed) > 0) {
        // every vector in memory the caller registered (rs_host_register) and
        // 16-byte aligned: one zero-copy launch over the caller's own bytes
        const uint8_t* in[kMaxVects];
        uint8_t* out[kMaxVects];
        bool direct = true;
        for (int i = 0; i < cols && direct; ++i)
            direct = (in[i] = registered_device_ptr(src[i], size)) && (reinterpret_cast<uintptr_t>(src[i]) & 15) == 0;
        for (int r = 0; r < rows && direct; ++r)
            direct = (out[r] = registered_device_ptr(dst[r], size)) && (reinterpret_cast<uintptr_t>(dst[r]) & 15) == 0;
        if (direct) {
            Region region("registered-memory call");
            // small calls: the resident engine straight over the caller's memory
            const int erc = engine_call_addr(rs, mat, rows, cols, in, out, size, accumulate);
            if (erc != RS_ERR_INVAL) return erc;
            std::lock_guard<std::mutex> lk(rs->stage_mu);
            if (!rs->stream)
                RS_TRY(hip_ok(hipStreamCreateWithFlags(&rs->stream, hipStreamNonBlocking), "stream create"));
            if (rs->zc_pending) RS_TRY(sync(rs));
            const int rc = matmul(rs, mat, rows, cols, in, 0, out, 0, 1, size, accumulate, rs->stream);
            engine_warm_async(rs);  // (a cold engine declined this call: it restarts behind it, on the warmer thread)
            const int src_rc = flag_sync(rs->stream, rs->stream_flag, "host-call stream sync");
            return rc ? rc : src_rc;
        }
    }
    if (size > g_coalesce_max || size == 0) {
        std::lock_guard<std::mutex> lk(rs->stage_mu);
        return host_product(rs, mat, rows, cols, src, dst, size, accumulate);
    }
    if (g_engine_direct) {
        const size_t pitch = rup(size, 64), stride = pitch * static_cast<size_t>(rows + cols);
        if (engine_accepts(rows, cols, stride) && !engine_cold_now(rs)) {
            using clk = std::chrono::steady_clock;
            clk::time_point t0, t1, t2;
            if (g_phase_trace) t0 = clk::now();
            // inputs into device memory the host writes through the BAR when
            // the platform has it (posted writes; the engine reads them from
            // HBM), outputs (and an Update / Replace's old parity) in a pinned
            // block; else the whole stripe in the pinned block
            const size_t in_bytes = pitch * static_cast<size_t>(cols);
            size_t vcap = 0;
            uint8_t* vin = g_engine_vram ? host_writable_vram_get(rs->device, in_bytes, &vcap) : nullptr;
            PinnedBlock blk;
            const int prc = pinned_get(vin ? stride - in_bytes : stride, &blk);
            if (prc) {
                host_writable_vram_put(rs->device, vin, vcap);
                return prc;
            }
            uint8_t* in_host = vin ? vin : blk.host;
            uint8_t* out_host = vin ? blk.host : blk.host + in_bytes;
            for (int i = 0; i < cols; ++i) std::memcpy(in_host + static_cast<size_t>(i) * pitch, src[i], size);
            if (accumulate)
                for (int r = 0; r < rows; ++r) std::memcpy(out_host + static_cast<size_t>(r) * pitch, dst[r], size);
            if (g_phase_trace) t1 = clk::now();
            int rc;
            if (vin) {
                const uint8_t* in[kMaxVects];
                uint8_t* out[kMaxVects];
                uint8_t* out_dev = blk.dev;
                for (int i = 0; i < cols; ++i) in[i] = vin + static_cast<size_t>(i) * pitch;
                for (int r = 0; r < rows; ++r) out[r] = out_dev + static_cast<size_t>(r) * pitch;
                rc = engine_call_addr(rs, mat, rows, cols, in, out, pitch, accumulate);
            } else {
                rc = engine_call(rs, mat, rows, cols, blk.dev, pitch, stride, 1, accumulate, false);
            }
            if (g_phase_trace) t2 = clk::now();
            if (rc == RS_OK)
                for (int r = 0; r < rows; ++r) std::memcpy(dst[r], out_host + static_cast<size_t>(r) * pitch, size);
            pinned_put(blk);
            host_writable_vram_put(rs->device, vin, vcap);
            if (g_phase_trace && rc == RS_OK) {
                phase_add(kPhCopyIn, t0, t1);
                phase_add(kPhCopyOut, t2, clk::now());
            }
            if (rc != RS_ERR_INVAL) return rc;
        }
    }
    const auto t_enter = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(rs->co_mu);
    if (!rs->co_stream && hip_ok(hipStreamCreateWithFlags(&rs->co_stream, hipStreamNonBlocking), "stream create")) {
        rs->co_stream = nullptr;
        return RS_ERR_DEVICE;
    }
    ++rs->co_active;
    CoBatch* b = nullptr;
    int idx = -1;
    while (!b) {
        for (CoBatch& c : rs->co)
            if (c.state == CoBatch::kFilling && c.joined < c.cap && same_shape(c, mat, rows, cols, size, accumulate)) {
                b = &c;
                break;
            }
        if (!b)
            for (CoBatch& c : rs->co)
                if (c.state == CoBatch::kIdle) {
                    const int rc = init_batch(c, mat, rows, cols, size, accumulate);
                    if (rc) {
                        --rs->co_active;
                        return rc;
                    }
                    b = &c;
                    break;
                }
        if (!b) co_wait(rs, lk);
    }
    idx = b->joined++;
    const bool alone = rs->co_active == 1;
    lk.unlock();
    using clk = std::chrono::steady_clock;
    clk::time_point t_joined, t_ready, t_ran, t_done;
    if (g_phase_trace) t_joined = clk::now();

    // copy in: own stripe slot [cols inputs | rows outputs (accumulate)]
    uint8_t* slot = b->host + static_cast<size_t>(idx) * b->stride;
    {
        uint8_t* cd[2 * kMaxVects];
        const uint8_t* cs[2 * kMaxVects];
        int n = 0;
        for (int i = 0; i < cols; ++i, ++n) {
            cd[n] = slot + static_cast<size_t>(i) * b->pitch;
            cs[n] = src[i];
        }
        if (accumulate)
            for (int r = 0; r < rows; ++r, ++n) {
                cd[n] = slot + static_cast<size_t>(cols + r) * b->pitch;
                cs[n] = dst[r];
            }
        if (alone) parallel_copy(cd, cs, n, size);  // the copy pool serves one call at a time
        else
            for (int i = 0; i < n; ++i) std::memcpy(cd[i], cs[i], size);
    }

    if (g_phase_trace) t_ready = clk::now();
    lk.lock();
    ++b->ready;  // (no wake-up: the member that completes the batch launches it itself)
    bool ran = false;
    while (b->state != CoBatch::kDone) {
        if (b->state == CoBatch::kFilling && rs->co_running < g_co_running && b->ready == b->joined) {
            if (g_coalesce_linger_us > 0 && b->joined < b->cap) {
                // group-commit window: give other callers until the deadline to join
                const auto now = std::chrono::steady_clock::now();
                if (!b->launchable) {
                    b->launchable = true;
                    b->deadline = now + std::chrono::microseconds(g_coalesce_linger_us);
                }
                if (now < b->deadline) {
                    rs->co_cv.wait_until(lk, b->deadline);
                    continue;
                }
            }
            b->state = CoBatch::kRunning;
            ++rs->co_running;
            const int n = b->joined;
            lk.unlock();
            rs->co_launches.fetch_add(1, std::memory_order_relaxed);
            rs->co_calls.fetch_add(static_cast<uint64_t>(n), std::memory_order_relaxed);
            if (g_phase_trace) t_ran = clk::now();
            const int rc = run_batch(rs, *b, n);
            if (g_phase_trace) t_done = clk::now();
            ran = true;
            lk.lock();
            b->rc = rc;
            b->state = CoBatch::kDone;
            --rs->co_running;
            co_changed(rs);
            break;
        }
        co_wait(rs, lk);
    }
    const int rc = b->rc;
    lk.unlock();
    clk::time_point t_out;
    if (g_phase_trace) {
        t_out = clk::now();
        phase_add(kPhJoin, t_enter, t_joined);
        phase_add(kPhCopyIn, t_joined, t_ready);
        phase_add(kPhWaitRun, t_ready, ran ? t_ran : t_out);
        if (ran) phase_add(kPhWake, t_done, t_out);
    }

    if (g_host_trace) {
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_enter).count();
        if (us > 200) std::fprintf(stderr, "host_call slow: %.1f us to batch done (joined %d)\n", us, b->joined);
    }
    if (rc == RS_OK) {  // copy out: own output rows
        uint8_t* cd[kMaxVects];
        const uint8_t* cs[kMaxVects];
        for (int r = 0; r < rows; ++r) {
            cd[r] = dst[r];
            cs[r] = slot + static_cast<size_t>(cols + r) * b->pitch;
        }
        if (alone) parallel_copy(cd, cs, rows, size);
        else
            for (int r = 0; r < rows; ++r) std::memcpy(cd[r], cs[r], size);
    }
    if (g_phase_trace) phase_add(kPhCopyOut, t_out, clk::now());

    lk.lock();
    if (++b->released == b->joined) {
        b->state = CoBatch::kIdle;
        co_changed(rs);
    }
    --rs->co_active;
    return rc;
}

}  // namespace detail
}  // namespace rsamd

extern "C" {

int rs_encode(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n) {
    return abi_guard([&]() -> int {
        if (!rs || (n > 0 && (!vects || !lens))) return RS_ERR_INVAL;
        RS_TRY(check_encode(rs, lens, n));
        RS_TRY(ensure_device(rs));
        DeviceGuard g(rs->device);
        return host_call(rs, rs->gen(), rs->p, rs->d, vects, vects + rs->d, lens[0], false);
    });
}

int rs_reconst(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n, const int* survived, int ns,
               const int* need, int nn) {
    return abi_guard([&]() -> int {
        if (!rs || (nn > 0 && !need) || (ns > 0 && !survived)) return RS_ERR_INVAL;
        ReconstPlan pl;
        int rc = plan_reconst(rs, survived, ns, need, nn, pl.vs, &pl.nvs, pl.nr, &pl.nnr, &pl.dn);
        if (rc == RS_ERR_NO_NEED_RECONST) return RS_OK;  // rs.go:225-228
        if (rc) return rc;
        if (!vects || !lens) return RS_ERR_INVAL;
        const int d = rs->d;
        int parity_rc = RS_OK;
        RS_TRY(check_reconst_passes(rs, pl, lens, n, &parity_rc));
        const int rows = parity_rc ? pl.dn : pl.nnr;  // see rs_reconst_dev
        if (rows > 0) {
            RS_TRY(ensure_device(rs));
            DeviceGuard g(rs->device);
            const uint8_t* src[kMaxVects];
            uint8_t* dst[kMaxVects];
            for (int i = 0; i < d; ++i) src[i] = vects[pl.vs[i]];
            for (int i = 0; i < rows; ++i) dst[i] = vects[pl.nr[i]];
            std::vector<uint8_t> m;
            RS_TRY(combined_matrix(rs, pl.vs, pl.nr, rows, pl.dn, m));
            RS_TRY(host_call(rs, m.data(), rows, d, src, dst, lens[pl.vs[0]], false));
        }
        return parity_rc;
    });
}

int rs_update(rs_t* rs, const uint8_t* old_data, size_t old_len, const uint8_t* new_data, size_t new_len, int row,
              uint8_t* const* parity, const size_t* parity_lens, int np) {
    return abi_guard([&]() -> int {
        if (!rs || (np > 0 && (!parity || !parity_lens))) return RS_ERR_INVAL;
        RS_TRY(check_update(rs, old_len, new_len, row, parity_lens, np));
        if (!old_data || !new_data) return RS_ERR_INVAL;
        RS_TRY(ensure_device(rs));
        DeviceGuard g(rs->device);
        std::vector<uint8_t> gm = update_matrix(rs, row);
        return update_ranges(rs, new_len, [&](uint64_t off, uint64_t n) {
            const uint8_t* src[2] = {old_data + off, new_data + off};
            uint8_t* dst[kMaxVects];
            for (int j = 0; j < rs->p; ++j) dst[j] = parity[j] + off;
            return host_call(rs, gm.data(), rs->p, 2, src, dst, n, true);
        });
    });
}

int rs_replace(rs_t* rs, const uint8_t* const* data, const size_t* data_lens, int nd, const int* replace_rows, int nr,
               uint8_t* const* parity, const size_t* parity_lens, int np) {
    return abi_guard([&]() -> int {
        if (!rs || (nd > 0 && (!data || !data_lens)) || (nr > 0 && !replace_rows) ||
            (np > 0 && (!parity || !parity_lens)))
            return RS_ERR_INVAL;
        RS_TRY(check_replace(rs, data_lens, nd, replace_rows, nr, parity_lens, np));
        RS_TRY(ensure_device(rs));
        DeviceGuard g(rs->device);
        std::vector<uint8_t> gm = replace_matrix(rs, replace_rows, nr);
        return update_ranges(rs, data_lens[0], [&](uint64_t off, uint64_t n) {
            const uint8_t* src[kMaxVects];
            uint8_t* dst[kMaxVects];
            for (int i = 0; i < nr; ++i) src[i] = data[i] + off;
            for (int j = 0; j < rs->p; ++j) dst[j] = parity[j] + off;
            return host_call(rs, gm.data(), rs->p, nr, src, dst, n, true);
        });
    });
}

}  // extern "C"
