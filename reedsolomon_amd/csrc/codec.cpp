// codec.cpp — host side of librsamd: the reference's codec driver
// (rs.go, matrix.go) re-expressed around a device GF(2^8) matrix product.
//
// What runs here (small, per call or per erasure pattern):
//   * argument checks in the reference's exact order and error codes
//     (checkEncode rs.go:119-134, checkReconst :264-325, checkUpdate
//     :456-477, checkReplace :536-570);
//   * encoding-matrix construction (matrix.go:37-54), Gauss-Jordan inverse
//     (matrix.go:85-147) and the survivor-bitmap inverse cache (rs.go:33-39,
//     70-74, 382-420);
//   * conversion of a small coefficient matrix into per-coefficient device
//     perm tables, uploaded once per distinct matrix (registry below).
// What runs on the GPU: every byte of every vector (kernels.hip).
#include <cstdio>
#include <algorithm>
#include <cstdlib>

#include <immintrin.h>

#include "codec_internal.hpp"

#if defined(__x86_64__) || defined(__i386__)
#include <cpuid.h>
#endif
#include "jit.hpp"

using namespace rsamd;
using namespace rsamd::detail;

namespace rsamd {
namespace detail {

// ---------------------------------------------------------------- matrix.go

// makeEncodeMatrix matrix.go:37-54: identity over a Cauchy block 1/(i^j).
std::vector<uint8_t> make_encode_matrix(int d, int p) {
    std::vector<uint8_t> m(static_cast<size_t>(d + p) * d, 0);
    for (int i = 0; i < d; ++i) m[i * d + i] = 1;
    size_t off = static_cast<size_t>(d) * d;
    for (int i = d; i < d + p; ++i)
        for (int j = 0; j < d; ++j) m[off++] = gf_inv(static_cast<uint8_t>(i ^ j));
    return m;
}

// Gauss-Jordan of invert() below on the augmented rows [left | inv], the
// row operations as split-nibble products on 32-byte vectors (what the
// reference's gmu_amd64.s does for vectors, here for matrix rows): the same
// pivot order and the same field arithmetic, so the same bytes.
namespace {
struct NibTables {  // per v: v * i (i = 0..15), then v * (i << 4)
    alignas(32) uint8_t t[256][32];
    NibTables() {
        const auto& T = gf();
        for (int v = 0; v < 256; ++v)
            for (int i = 0; i < 16; ++i) {
                t[v][i] = T.mul[v][i];
                t[v][16 + i] = T.mul[v][i << 4];
            }
    }
};
const NibTables& nib() {
    static const NibTables n;
    return n;
}

__attribute__((target("avx2"))) inline __m256i nib_mul(__m256i x, const uint8_t* tv) {
    const __m256i lo_t = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i*>(tv)));
    const __m256i hi_t = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i*>(tv + 16)));
    const __m256i m = _mm256_set1_epi8(0x0f);
    const __m256i lo = _mm256_shuffle_epi8(lo_t, _mm256_and_si256(x, m));
    const __m256i hi = _mm256_shuffle_epi8(hi_t, _mm256_and_si256(_mm256_srli_epi16(x, 4), m));
    return _mm256_xor_si256(lo, hi);
}

__attribute__((target("avx2"))) int invert_avx2(const uint8_t* src, int n, uint8_t* out) {
    const int w = (2 * n + 31) & ~31;  // augmented row bytes, whole vectors
    std::vector<uint8_t> aug(static_cast<size_t>(n) * w + 32, 0);
    uint8_t* a = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(aug.data()) + 31) & ~uintptr_t{31});
    for (int i = 0; i < n; ++i) {
        std::memcpy(a + static_cast<size_t>(i) * w, src + static_cast<size_t>(i) * n, n);
        a[static_cast<size_t>(i) * w + n + i] = 1;
    }
    const auto& T = gf();
    const auto& N = nib();
    const int nv = w / 32;
    for (int i = 0; i < n; ++i) {
        uint8_t* ri = a + static_cast<size_t>(i) * w;
        if (ri[i] == 0) {
            int j = i + 1;
            while (j < n && a[static_cast<size_t>(j) * w + i] == 0) ++j;
            if (j == n) return RS_ERR_SINGULAR_MATRIX;
            std::swap_ranges(ri, ri + w, a + static_cast<size_t>(j) * w);
        }
        if (ri[i] != 1) {
            const uint8_t* tv = N.t[T.inv[ri[i]]];
            for (int k = 0; k < nv; ++k) {
                __m256i* p = reinterpret_cast<__m256i*>(ri) + k;
                _mm256_store_si256(p, nib_mul(_mm256_load_si256(p), tv));
            }
        }
        for (int j = 0; j < n; ++j) {
            uint8_t* rj = a + static_cast<size_t>(j) * w;
            if (j == i || !rj[i]) continue;
            const uint8_t* tv = N.t[rj[i]];
            for (int k = 0; k < nv; ++k) {
                __m256i* p = reinterpret_cast<__m256i*>(rj) + k;
                const __m256i src_v = _mm256_load_si256(reinterpret_cast<const __m256i*>(ri) + k);
                _mm256_store_si256(p, _mm256_xor_si256(_mm256_load_si256(p), nib_mul(src_v, tv)));
            }
        }
    }
    for (int i = 0; i < n; ++i) std::memcpy(out + static_cast<size_t>(i) * n, a + static_cast<size_t>(i) * w + n, n);
    return RS_OK;
}

// (env RSAMD_INVERT_SCALAR=1: the byte-table row operations, for A/B and for
// testing that path on an AVX2 host)
const bool g_has_avx2 = __builtin_cpu_supports("avx2") && !std::getenv("RSAMD_INVERT_SCALAR");
}  // namespace

// invert matrix.go:85-147 (Gauss-Jordan; a zero pivot swaps with the first
// lower row that has a non-zero entry in the pivot column; the result is
// bit-identical to the reference's).  AVX2 row operations where the host
// has them (invert_avx2, same steps), else byte-table ones.
int invert(const uint8_t* src, size_t len, int n, uint8_t* out) {
    if (static_cast<size_t>(n) * n != len) return RS_ERR_NOT_SQUARE;
    if (g_has_avx2 && n > 0) return invert_avx2(src, n, out);
    std::vector<uint8_t> left(src, src + len), inv(len, 0);
    for (int i = 0; i < n; ++i) inv[i * n + i] = 1;
    auto swap_rows = [n](std::vector<uint8_t>& m, int a, int b) {
        std::swap_ranges(m.begin() + a * n, m.begin() + (a + 1) * n, m.begin() + b * n);
    };
    const auto& T = gf();
    for (int i = 0; i < n; ++i) {
        if (left[i * n + i] == 0) {
            int j = i + 1;
            while (j < n && left[j * n + i] == 0) ++j;
            if (j == n) return RS_ERR_SINGULAR_MATRIX;
            swap_rows(left, i, j);
            swap_rows(inv, i, j);
        }
        const uint8_t piv = left[i * n + i];
        if (piv != 1) {
            const uint8_t v = T.inv[piv];
            for (int j = 0; j < n; ++j) {
                left[i * n + j] = T.mul[left[i * n + j]][v];
                inv[i * n + j] = T.mul[inv[i * n + j]][v];
            }
        }
        for (int j = 0; j < n; ++j) {
            if (j == i) continue;
            const uint8_t v = left[j * n + i];
            if (!v) continue;
            const uint8_t* mv = T.mul[v];
            for (int k = 0; k < n; ++k) {
                left[j * n + k] ^= mv[left[i * n + k]];
                inv[j * n + k] ^= mv[inv[i * n + k]];
            }
        }
    }
    std::memcpy(out, inv.data(), len);
    return RS_OK;
}

uint64_t cache_key(const int* survived, int ns) {  // makeInverseCacheKey rs.go:414-420
    uint64_t key = 0;
    for (int k = 0; k < ns; ++k) {
        const unsigned s = static_cast<uint8_t>(survived[k]);  // Go: 1 << uint8(i)
        key += s < 64 ? (uint64_t{1} << s) : 0;
    }
    return key;
}

// ---------------------------------------------------------------- device product

int ensure_device(rs_t* rs) {
    std::lock_guard<std::mutex> lk(rs->dev_mu);
    if (rs->device_ready) return RS_OK;
    int count = 0;
    RS_TRY(hip_ok(hipGetDeviceCount(&count), "hipGetDeviceCount"));
    if (count <= 0) return dev_fail(hipErrorNoDevice, "hipGetDeviceCount");
    if (rs->device < 0) {
        int cur = 0;
        RS_TRY(hip_ok(hipGetDevice(&cur), "hipGetDevice"));
        rs->device = cur;
    }
    if (rs->device >= count) return dev_fail(hipErrorInvalidDevice, "device ordinal");
    if (rs->device < 64) g_devices_used.fetch_or(uint64_t{1} << rs->device, std::memory_order_acq_rel);
    rs->device_ready = true;
    return RS_OK;
}

std::atomic<uint64_t> g_devices_used{0};

size_t g_registry_max = size_t{1} << 14;
// First sight of a matrix in a small launch (at most this many bytes of input
// vectors): the launch reads the tables in place from the mapped staging
// slot, with no device allocation, upload copy or upload event on the
// caller's path; the matrix's second use uploads them (get_tables).
// rs_tune("table_inplace_max", bytes), 0 = always upload at first sight.
size_t g_tab_inplace_max = size_t{2} << 20;
// Table staging slots and the first-sight arena in device memory the host
// writes through the BAR (uncached, hipDeviceMallocUncached; the engine's
// host_writable_vram_get): a first-sight launch then reads its tables from
// local HBM instead of across PCIe (new 10+4 pattern, small synchronous
// Reconst 23.7 -> 21.7 us), and an upload is a
// device-to-device copy.  Off by default: the one full GPU run with it on
// failed with hipErrorIllegalAddress in a runtime pageable copy of another
// test (cause not identified), so until that is understood
// the default keeps host memory.  Platforms that map no device memory for
// the CPU keep coherent pinned host memory either way.  Taken by slots
// allocated after a change; rs_tune("table_stage_vram", 0 default | 1),
// env RSAMD_TAB_VRAM.
int g_tab_stage_vram = [] {
    const char* e = std::getenv("RSAMD_TAB_VRAM");
    return e ? (std::atoi(e) ? 1 : 0) : 0;
}();
// The first-sight arena per handle (get_tables): ~400 new 10+4 matrices.
constexpr size_t kTabArenaBytes = size_t{1} << 20;

thread_local char g_last_dev_err[192] = {0};

int dev_fail(hipError_t e, const char* where) {
    std::snprintf(g_last_dev_err, sizeof g_last_dev_err, "%s: %s (%d)", where, hipGetErrorName(e),
                  static_cast<int>(e));
    return RS_ERR_DEVICE;
}

// Perm tables for a rows x cols coefficient matrix, laid out
// [col][rows_pad][5] dwords (rows padded to a multiple of 8 so that every
// kernel row group reads inside the allocation), followed - for rows <= 4 -
// by the same tables as the 4-row kernels' LDS image [rup(cols, 4)][20]
// (zero rows and columns as padding), which those kernels stage with a plain
// copy.  Uploaded once per distinct matrix and reused by every later launch.
// The upload is asynchronous on the launching stream (pinned staging slots):
// a synchronous copy from pageable memory waited for every kernel already
// queued, which put a full GPU drain in front of every new erasure pattern
// (a rebuild storm of one-off patterns: profiles/r04/).  A later launch on
// another stream waits for the upload's event.  Caller holds tab_mu until its
// launch is enqueued: a full registry is recycled after a device sync, so no
// table may be handed out and launched across a recycle.
//
// First sight in a small launch (launch_in_bytes <= table_inplace_max, and
// the caller passes inplace_slot), no host call on the caller's path beyond
// the launch itself: a small synchronous Reconst of a pattern new to the
// process spent ~12 of its 33 us in the upload's host calls (hipMalloc,
// hipMemcpyAsync, event create and two records;
// profiles/r05/first_sight_api_trace/), and a rebuild storm of one-off
// patterns never reuses its tables.
//  * the first-sight arena (host-writable device memory, table_stage_vram):
//    the host writes the tables there through the BAR and the registry entry
//    points at them; the launch reads them from HBM.  The matrix's next use
//    copies them to ordinary (cached) device memory.  Arena space comes back
//    only with the registry, after its device drain; a full arena falls
//    through to
//  * a staging slot read in place (pinned or VRAM): *inplace_slot names the
//    slot, and the caller records the slot's `done` event behind its launch
//    (the slot is reused only after that).  No registry entry is made: the
//    matrix's next use uploads.
int get_tables(rs_t* rs, const uint8_t* mat, int rows, int cols, hipStream_t stream, const uint32_t** out,
               int* rows_pad_out, uint64_t launch_in_bytes, int* inplace_slot) {
    if (inplace_slot) *inplace_slot = -1;
    const int rows_pad = static_cast<int>(rup(rows, 8));
    std::string key(reinterpret_cast<const char*>(&rows), sizeof rows);
    key.append(reinterpret_cast<const char*>(&cols), sizeof cols);
    key.append(reinterpret_cast<const char*>(mat), static_cast<size_t>(rows) * cols);
    auto it = rs->tables.find(key);
    if (it != rs->tables.end() && it->second.arena) {
        // second use of a matrix whose tables sit in the first-sight arena:
        // to ordinary device memory (a device-to-device copy on this stream;
        // the arena copy stays valid for launches still reading it)
        rs_t::TableEntry& te = it->second;
        uint32_t* dptr = nullptr;
        hipEvent_t ev = nullptr;
        if (hipMalloc(&dptr, te.bytes) != hipSuccess) {
            (void)hipGetLastError();
            *out = te.dev;  // (no memory: keep reading the arena copy)
            *rows_pad_out = rows_pad;
            return RS_OK;
        }
        hipError_t e = hipMemcpyAsync(dptr, te.dev, te.bytes, hipMemcpyDeviceToDevice, stream);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventRecord(ev, stream);
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(stream);
            if (ev) (void)hipEventDestroy(ev);
            (void)hipFree(dptr);
            return dev_fail(e, "table move out of the first-sight arena");
        }
        te.dev = dptr;
        te.arena = false;
        te.ready = ev;
        te.stream = stream;
        ++rs->tab_uploads;
        *out = dptr;
        *rows_pad_out = rows_pad;
        return RS_OK;
    }
    if (it != rs->tables.end()) {
        rs_t::TableEntry& te = it->second;
        if (te.ready) {
            if (hipEventQuery(te.ready) == hipSuccess) {
                (void)hipEventDestroy(te.ready);
                te.ready = nullptr;
            } else if (stream != te.stream) {
                RS_TRY(hip_ok(hipStreamWaitEvent(stream, te.ready, 0), "table upload wait"));
            }
        }
        *out = te.dev;
        *rows_pad_out = rows_pad;
        return RS_OK;
    }
    if (rs->tables.size() >= g_registry_max) {
        // Bounded registry: drain the device before recycling table memory
        // (the resident host-call engine first: a device sync waits for it)
        std::lock_guard<std::mutex> elk(rs->eng_mu);
        RS_TRY(engine_drain(rs));  // calls in flight complete first (a stopped instance would strand them)
        engine_stop(rs);
        engines_quiesce();  // other handles' instances on this device would hold the sync for their idle window
        RS_TRY(hip_ok(hipDeviceSynchronize(), "table registry drain"));
        for (auto& kv : rs->tables) {
            if (!kv.second.arena) (void)hipFree(kv.second.dev);
            if (kv.second.ready) (void)hipEventDestroy(kv.second.ready);
        }
        rs->tables.clear();
        rs->tab_arena_off = 0;  // (drained above: no launch reads the arena)
    }
    const bool small = inplace_slot && g_tab_inplace_max && launch_in_bytes <= g_tab_inplace_max;
    bool inplace = false;
    if (small) {
        if (rs->tab_seen.size() >= 4096) rs->tab_seen.clear();
        uint64_t h = 0xcbf29ce484222325ull;  // FNV-1a over the key (rows, cols, matrix bytes)
        for (unsigned char ch : key) h = (h ^ ch) * 0x100000001b3ull;
        inplace = rs->tab_seen.insert(h).second;  // first sight: in place; a second one uploads
    }
    const size_t main_dw = static_cast<size_t>(cols) * rows_pad * 5;
    const size_t img_dw = rows <= 4 ? rup(cols, 4) * 20 : 0;
    // wide kernels (rows > 8): [column pair][rows_pad][12] dwords, per (pair,
    // row) T0a T2a T0b T2b | T1a T3a T1b T3b | T4a T4b 0 0 (the dwords v_perm
    // takes from VGPRs first, as two 64-bit pairs); an odd last column's
    // partner has zero tables
    const size_t wide_dw = rows > 8 ? static_cast<size_t>((cols + 1) / 2) * rows_pad * 12 : 0;
    const size_t bytes = (main_dw + img_dw + wide_dw) * 4;
    // built in host memory, then one streaming copy into its place (arena or
    // staging slot; VRAM is write-combined: no reads of it, and the stores
    // are fenced before any launch or copy can read them)
    thread_local std::vector<uint32_t> build;
    build.assign(bytes / 4, 0u);
    uint32_t* host = build.data();
    for (int c = 0; c < cols; ++c)
        for (int r = 0; r < rows; ++r) {
            uint32_t t[5];
            perm_table(mat[static_cast<size_t>(r) * cols + c], t);
            std::memcpy(&host[(static_cast<size_t>(c) * rows_pad + r) * 5], t, sizeof t);
            if (img_dw) std::memcpy(&host[main_dw + static_cast<size_t>(c) * 20 + r * 5], t, sizeof t);
            if (wide_dw) {
                uint32_t* w = &host[main_dw + img_dw + (static_cast<size_t>(c / 2) * rows_pad + r) * 12];
                const int h = c & 1;
                w[2 * h] = t[0];
                w[2 * h + 1] = t[2];
                w[4 + 2 * h] = t[1];
                w[5 + 2 * h] = t[3];
                w[8 + h] = t[4];
            }
        }
    if (small && g_tab_stage_vram) {
        if (!rs->tab_arena) {
            size_t cap = 0;
            rs->tab_arena = host_writable_vram_get(rs->device, kTabArenaBytes, &cap);
            rs->tab_arena_cap = rs->tab_arena ? cap : 0;
            rs->tab_arena_off = 0;
        }
        const size_t at = rup(rs->tab_arena_off, size_t{256});
        if (rs->tab_arena && at + bytes <= rs->tab_arena_cap) {
            uint8_t* dst = rs->tab_arena + at;
            std::memcpy(dst, host, bytes);
            _mm_sfence();
            rs->tab_arena_off = at + bytes;
            rs_t::TableEntry te;
            te.dev = reinterpret_cast<uint32_t*>(dst);
            te.arena = true;
            te.bytes = bytes;
            rs->tables.emplace(std::move(key), te);
            ++rs->tab_inplace;
            *out = te.dev;
            *rows_pad_out = rows_pad;
            return RS_OK;
        }
    }
    rs_t::TabStage& st = rs->tab_stage[rs->tab_stage_next];
    rs->tab_stage_next = (rs->tab_stage_next + 1) % rs_t::kTabStages;
    if (st.pending) {  // the copy enqueued from this slot kTabStages uploads ago
        RS_TRY(hip_ok(hipEventSynchronize(st.done), "table staging slot"));
        st.pending = false;
    }
    if (!st.done) RS_TRY(hip_ok(hipEventCreateWithFlags(&st.done, hipEventDisableTiming), "table staging event"));
    if (st.cap < bytes) {
        if (st.host && st.vram) host_writable_vram_put(rs->device, st.host, st.cap);
        else if (st.host) coherent_put(st.host, st.cap);
        st.host = nullptr;
        st.dev_host = nullptr;
        st.cap = 0;
        const size_t cap = rup(bytes, size_t{64} << 10);
        size_t vcap = 0;
        uint8_t* v = g_tab_stage_vram ? host_writable_vram_get(rs->device, cap, &vcap) : nullptr;
        if (v) {  // device memory the host writes: read in place from HBM
            st.host = v;
            st.dev_host = v;
            st.cap = vcap;
            st.vram = true;
        } else {  // coherent and mapped pinned host memory (recycled blocks): read in place over PCIe
            size_t ccap = 0;
            void* hd = nullptr;
            st.host = coherent_get(cap, &ccap, &hd);
            if (!st.host) return RS_ERR_NOMEM;
            st.dev_host = static_cast<const uint8_t*>(hd);
            st.cap = ccap;
            st.vram = false;
        }
    }
    std::memcpy(st.host, host, bytes);
    if (st.vram) _mm_sfence();
    if (inplace && st.dev_host) {
        *inplace_slot = static_cast<int>(&st - rs->tab_stage);
        *out = reinterpret_cast<const uint32_t*>(st.dev_host);
        *rows_pad_out = rows_pad;
        ++rs->tab_inplace;
        return RS_OK;
    }
    uint32_t* dptr = nullptr;
    if (hipMalloc(&dptr, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return RS_ERR_NOMEM;
    }
    rs_t::TableEntry te;
    te.dev = dptr;
    te.stream = stream;
    hipError_t e = hipMemcpyAsync(dptr, st.host, bytes, st.vram ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                                  stream);
    if (e == hipSuccess) e = hipEventRecord(st.done, stream);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&te.ready, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(te.ready, stream);
    if (e != hipSuccess) {
        (void)hipStreamSynchronize(stream);
        if (te.ready) (void)hipEventDestroy(te.ready);
        (void)hipFree(dptr);
        return dev_fail(e, "table upload");
    }
    st.pending = true;
    ++rs->tab_uploads;
    rs->tables.emplace(std::move(key), te);
    *out = dptr;
    *rows_pad_out = rows_pad;
    return RS_OK;
}

// One launch of the product: out[r] (=|^=) sum_c mat[r][c] * in[c] on every
// stripe.  in_ptrs/out_ptrs are stripe-0 addresses; vector v of stripe s adds
// s * ss[sid[v]] (sid == nullptr: all inputs use ss[0], all outputs ss[1]).
int matmul_ex(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* in_ptrs,
              const uint8_t* in_sid, uint8_t* const* out_ptrs, const uint8_t* out_sid, const int64_t ss[4],
              int nstripes, uint64_t len, bool accumulate, hipStream_t stream, const int32_t* stripe_ids) {
    if (rows <= 0 || cols <= 0 || nstripes <= 0 || len == 0) return RS_OK;
    if (rows + cols > kMaxPtrs) return RS_ERR_INVAL;
    MatmulArgs a;
    std::memset(&a, 0, sizeof a);
    std::lock_guard<std::mutex> lk(rs->tab_mu);  // table lookup through launch (get_tables)
    int slot = -1;
    int rc = get_tables(rs, mat, rows, cols, stream, &a.tables, &a.rows_pad,
                        static_cast<uint64_t>(nstripes) * len * static_cast<uint64_t>(cols), &slot);
    if (rc) return rc;
    a.img4 = rows <= 4 ? a.tables + static_cast<size_t>(cols) * a.rows_pad * 5 : nullptr;
    a.wide = rows > 8 ? a.tables + static_cast<size_t>(cols) * a.rows_pad * 5 : nullptr;
    a.host_mat = mat;
    a.rows = rows;
    a.cols = cols;
    a.nstripes = nstripes;
    a.accumulate = accumulate ? 1 : 0;
    a.len = len;
    for (int i = 0; i < 4; ++i) a.ss[i] = ss[i];
    a.stripe_ids = stripe_ids;
    for (int c = 0; c < cols; ++c) {
        a.ptr[c] = reinterpret_cast<uint64_t>(in_ptrs[c]);
        a.sid[c] = in_sid ? in_sid[c] : 0;
    }
    for (int r = 0; r < rows; ++r) {
        a.ptr[cols + r] = reinterpret_cast<uint64_t>(out_ptrs[r]);
        a.sid[cols + r] = out_sid ? out_sid[r] : 1;
    }
    hipError_t e = launch_gf_matmul(a, stream);
    if (slot >= 0) {  // tables read in place: the slot is reused after this launch
        rs_t::TabStage& st = rs->tab_stage[slot];
        const hipError_t er = hipEventRecord(st.done, stream);
        if (er == hipSuccess) st.pending = true;
        else (void)hipStreamSynchronize(stream);
        if (e == hipSuccess) e = er;
    }
    return e == hipSuccess ? RS_OK : dev_fail(e, "kernel launch");
}

int matmul(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* in_ptrs, int64_t in_ss,
           uint8_t* const* out_ptrs, int64_t out_ss, int nstripes, uint64_t len, bool accumulate,
           hipStream_t stream) {
    const int64_t ss[4] = {in_ss, out_ss, 0, 0};
    return matmul_ex(rs, mat, rows, cols, in_ptrs, nullptr, out_ptrs, nullptr, ss, nstripes, len, accumulate,
                     stream);
}

// ---------------------------------------------------------------- reference checks

int check_encode(const rs_t* rs, const size_t* lens, int n) {  // checkEncode rs.go:119-134
    if (rs->d + rs->p != n) return RS_ERR_MISMATCH_VECTS;
    const size_t size = lens[0];
    if (size == 0) return RS_ERR_ZERO_VECT_SIZE;
    for (int i = 1; i < n; ++i)
        if (lens[i] != size) return RS_ERR_MISMATCH_VECT_SIZE;
    return RS_OK;
}

// checkEncode of the temporary RS built by reconst rs.go:375-380 over the
// vectors idx[0..cnt).
int check_encode_idx(const size_t* lens, const int* idx, int cnt) {
    const size_t size = lens[idx[0]];
    if (size == 0) return RS_ERR_ZERO_VECT_SIZE;
    for (int i = 1; i < cnt; ++i)
        if (lens[idx[i]] != size) return RS_ERR_MISMATCH_VECT_SIZE;
    return RS_OK;
}

int check_vect_idx(const int* idx, int cnt, int n) {  // checkVectIdx rs.go:250-258
    for (int k = 0; k < cnt; ++k)
        if (idx[k] < 0 || idx[k] >= n) return RS_ERR_ILLEGAL_VECTS;
    return RS_OK;
}

// checkReconst rs.go:264-325
int plan_reconst(const rs_t* rs, const int* survived, int ns, const int* need, int nn, int* vs, int* nvs,
                 int* nr, int* nnr, int* dn) {
    const int d = rs->d, p = rs->p;
    *nvs = *nnr = *dn = 0;
    if (nn <= 0) return RS_ERR_NO_NEED_RECONST;
    if (ns < 0) return RS_ERR_INVAL;
    int rc = check_vect_idx(survived, ns, d + p);
    if (rc) return rc;
    rc = check_vect_idx(need, nn, d + p);
    if (rc) return rc;
    enum : uint8_t { kUnknown = 0, kSurvived = 1, kNeed = 2 };
    uint8_t status[kMaxVects];
    std::memset(status, ns == 0 ? kSurvived : kUnknown, sizeof status);
    for (int k = 0; k < ns; ++k) status[survived[k]] = kSurvived;
    bool full_data = false;
    for (int k = 0; k < nn; ++k) {
        status[need[k]] = kNeed;  // need overrides survived
        if (need[k] >= d) full_data = true;
    }
    if (full_data)  // rebuilding parity needs every data vector
        for (int i = 0; i < d; ++i)
            if (status[i] == kUnknown) status[i] = kNeed;
    for (int i = 0; i < d + p; ++i) {
        if (status[i] == kSurvived) vs[(*nvs)++] = i;
        else if (status[i] == kNeed) {
            if (i < d) ++*dn;
            nr[(*nnr)++] = i;
        }
    }
    if (*nvs < d || *nnr > p) return RS_ERR_TOO_MANY_LOST;
    return RS_OK;
}

// getReconstMatrixFromCache rs.go:394-412 + makeEncMatrixForReconst
// matrix.go:68-79: inverse of the encoding-matrix rows of the first d
// survivors, through the survivor-bitmap cache when enabled.
int get_inverse(rs_t* rs, const int* survived_d, std::vector<uint8_t>& inv) {
    const int d = rs->d;
    const uint64_t key = cache_key(survived_d, d);
    if (rs->cache_enabled) {
        std::lock_guard<std::mutex> lk(rs->cache_mu);
        auto it = rs->cache.find(key);
        if (it != rs->cache.end()) {
            inv = it->second;
            return RS_OK;
        }
    }
    std::vector<uint8_t> sub(static_cast<size_t>(d) * d);
    for (int i = 0; i < d; ++i)
        std::memcpy(&sub[static_cast<size_t>(i) * d], &rs->enc[static_cast<size_t>(survived_d[i]) * d], d);
    inv.resize(sub.size());
    int rc = invert(sub.data(), sub.size(), d, inv.data());
    if (rc) return rc;
    if (rs->cache_enabled && rs->cache_n.fetch_add(1) + 1 <= rs->cache_max) {
        std::lock_guard<std::mutex> lk(rs->cache_mu);
        rs->cache.emplace(key, inv);
    }
    return RS_OK;
}

// The coefficients over the survivors vs[0, d) of every data vector U_l not
// among them (C: u x d, row l for U_l), from the u x u block only: the parity
// survivors P among vs[:d] give enc[P][U] D_U = P ^ enc[P][K] D_K (K = the
// data survivors), so with Minv = (enc[P][U])^-1
//   coef_l(q) = Minv[l][j]                        (vs[q] = P_j)
//               ^_j Minv[l][j] * enc[P_j][vs[q]]  (vs[q] in K).
// A vector's coefficients over d independent survivors are unique, so these
// are exactly rows U of the inverse of the d x d survivor submatrix
// (matrix.go:56-64, 85-147), at O(u^3 + u^2 d) instead of Gauss-Jordan over
// all d rows: 200+56 losing 56 data vectors, ~0.4 instead of ~3.4 ms.  A
// duplicate or dependent survivor gives RS_ERR_SINGULAR_MATRIX, as the full
// inverse would.
static int unknown_data_rows(const rs_t* rs, const int* vs, std::vector<int>& U, std::vector<uint8_t>& C) {
    const int d = rs->d;
    bool in_vs[kMaxVects] = {};
    for (int q = 0; q < d; ++q) in_vs[vs[q]] = true;
    U.clear();
    for (int i = 0; i < d; ++i)
        if (!in_vs[i]) U.push_back(i);
    std::vector<int> pq;  // positions q of the parity survivors in vs[:d]
    for (int q = 0; q < d; ++q)
        if (vs[q] >= d) pq.push_back(q);
    const int u = static_cast<int>(U.size());
    if (static_cast<int>(pq.size()) != u) return RS_ERR_SINGULAR_MATRIX;  // (repeated survivors)
    C.assign(static_cast<size_t>(u) * d, 0);
    if (u == 0) return RS_OK;
    std::vector<uint8_t> M(static_cast<size_t>(u) * u), Minv(M.size());
    for (int j = 0; j < u; ++j)
        for (int l = 0; l < u; ++l)
            M[static_cast<size_t>(j) * u + l] = rs->enc[static_cast<size_t>(vs[pq[j]]) * d + U[l]];
    RS_TRY(invert(M.data(), M.size(), u, Minv.data()));
    const auto& T = gf();
    // G[j][q] = enc[P_j][vs[q]] over the data survivors (0 at the parity
    // survivors' positions), so each row is sum_j Minv[l][j] * G[j] with a
    // contiguous inner loop
    std::vector<uint8_t> G(static_cast<size_t>(u) * d, 0);
    for (int j = 0; j < u; ++j) {
        const uint8_t* e = &rs->enc[static_cast<size_t>(vs[pq[j]]) * d];
        for (int q = 0; q < d; ++q)
            if (vs[q] < d) G[static_cast<size_t>(j) * d + q] = e[vs[q]];
    }
    for (int l = 0; l < u; ++l) {
        const uint8_t* mi = &Minv[static_cast<size_t>(l) * u];
        uint8_t* row = &C[static_cast<size_t>(l) * d];
        for (int j = 0; j < u; ++j) {
            if (!mi[j]) continue;
            const uint8_t* mt = T.mul[mi[j]];
            const uint8_t* g = &G[static_cast<size_t>(j) * d];
            for (int q = 0; q < d; ++q) row[q] ^= mt[g[q]];
        }
        for (int j = 0; j < u; ++j) row[pq[j]] = mi[j];  // the parity survivors' own coefficients
    }
    return RS_OK;
}

// getReconstMatrix rs.go:382-392 + makeReconstMatrix matrix.go:56-64:
// rows `need` (data indexes) of the inverse; for codes beyond 64 vectors
// (no reference cache) from the reduced system above.
int reconst_matrix(rs_t* rs, const int* survived_d, const int* need, int nn, uint8_t* out) {
    const int d = rs->d;
    if (!rs->cache_enabled) {
        std::vector<int> U;
        std::vector<uint8_t> C;
        RS_TRY(unknown_data_rows(rs, survived_d, U, C));
        for (int i = 0; i < nn; ++i) {
            uint8_t* row = out + static_cast<size_t>(i) * d;
            const auto it = std::find(U.begin(), U.end(), need[i]);
            if (it != U.end()) {
                std::memcpy(row, &C[static_cast<size_t>(it - U.begin()) * d], d);
            } else {  // a survivor itself: its unit row
                std::memset(row, 0, d);
                for (int q = 0; q < d; ++q)
                    if (survived_d[q] == need[i]) {
                        row[q] = 1;
                        break;
                    }
            }
        }
        return RS_OK;
    }
    std::vector<uint8_t> inv;
    RS_TRY(get_inverse(rs, survived_d, inv));
    for (int i = 0; i < nn; ++i)
        std::memcpy(out + static_cast<size_t>(i) * d, &inv[static_cast<size_t>(need[i]) * d], d);
    return RS_OK;
}

// One-pass Reconst matrix (nnr x d) over the first d survivors vs[:d]:
//   lost data row  i : inv[i]                       (reconstData rs.go:327-349)
//   lost parity row l: enc[l] * inv                 (reconstParity rs.go:351-373 re-encodes
//                                                    the rebuilt data: enc[l]*(inv*S) = (enc[l]*inv)*S)
// GF(2^8) arithmetic is exact, so the bytes equal the reference's two passes
// (survivor data rows of inv are unit rows, reproducing those survivors).
// With no data lost, vs[:d] = 0..d-1, inv = I and no inverse is computed
// (as in the reference, which then only runs reconstParity).
int combined_matrix(rs_t* rs, const int* vs, const int* nr, int nnr, int dn, std::vector<uint8_t>& m) {
    const int d = rs->d;
    if (dn > 0 && !rs->cache_enabled) {
        // codes beyond 64 vectors: the reduced system (unknown_data_rows),
        // and the recent patterns' matrices cached by (survivors, need)
        std::string key(64, '\0');
        auto set = [&](int base, int v) { key[static_cast<size_t>(base + v / 8)] |= static_cast<char>(1 << (v % 8)); };
        for (int q = 0; q < d; ++q) set(0, vs[q]);
        for (int r = 0; r < nnr; ++r) set(32, nr[r]);
        {
            std::lock_guard<std::mutex> lk(rs->wide_mu);
            auto it = rs->wide_cache.find(key);
            if (it != rs->wide_cache.end()) {
                m = it->second;
                return RS_OK;
            }
        }
        std::vector<int> U;
        std::vector<uint8_t> C;
        RS_TRY(unknown_data_rows(rs, vs, U, C));
        m.assign(static_cast<size_t>(nnr) * d, 0);
        const auto& T = gf();
        for (int r = 0; r < nnr; ++r) {
            uint8_t* row = &m[static_cast<size_t>(r) * d];
            const int v = nr[r];
            if (v < d) {  // a lost data vector: one of U (needed data is never a survivor)
                const auto it = std::find(U.begin(), U.end(), v);
                if (it == U.end()) return RS_ERR_INVAL;
                std::memcpy(row, &C[static_cast<size_t>(it - U.begin()) * d], d);
                continue;
            }
            // a lost parity row: enc[v] over the data, the unknown data through C
            const uint8_t* e = &rs->enc[static_cast<size_t>(v) * d];
            for (int q = 0; q < d; ++q)
                if (vs[q] < d) row[q] = e[vs[q]];
            for (size_t l = 0; l < U.size(); ++l) {
                const uint8_t f = e[U[l]];
                if (!f) continue;
                const uint8_t* mt = T.mul[f];
                const uint8_t* cr = &C[l * d];
                for (int q = 0; q < d; ++q) row[q] ^= mt[cr[q]];
            }
        }
        std::lock_guard<std::mutex> lk(rs->wide_mu);
        if (rs->wide_cache.size() >= 1024) rs->wide_cache.clear();
        rs->wide_cache.emplace(std::move(key), m);
        return RS_OK;
    }
    m.assign(static_cast<size_t>(nnr) * d, 0);
    std::vector<uint8_t> inv;
    if (dn > 0) RS_TRY(get_inverse(rs, vs, inv));
    const auto& T = gf();
    for (int r = 0; r < nnr; ++r) {
        uint8_t* row = &m[static_cast<size_t>(r) * d];
        const int v = nr[r];
        if (v < d) {
            std::memcpy(row, &inv[static_cast<size_t>(v) * d], d);
        } else if (dn == 0) {
            std::memcpy(row, &rs->enc[static_cast<size_t>(v) * d], d);
        } else {
            const uint8_t* e = &rs->enc[static_cast<size_t>(v) * d];
            for (int t = 0; t < d; ++t) {
                if (!e[t]) continue;
                const uint8_t* mt = T.mul[e[t]];
                const uint8_t* ir = &inv[static_cast<size_t>(t) * d];
                for (int c = 0; c < d; ++c) row[c] ^= mt[ir[c]];
            }
        }
    }
    return RS_OK;
}

int check_update(const rs_t* rs, size_t old_len, size_t new_len, int row, const size_t* plens, int np) {
    if (np != rs->p) return RS_ERR_MISMATCH_PARITY_NUM;  // checkUpdate rs.go:456-477
    const size_t size = new_len;
    if (size == 0) return RS_ERR_ZERO_VECT_SIZE;
    if (size != old_len) return RS_ERR_MISMATCH_VECT_SIZE;
    for (int i = 0; i < np; ++i)
        if (plens[i] != size) return RS_ERR_MISMATCH_VECT_SIZE;
    if (row >= rs->d || row < 0) return RS_ERR_ILLEGAL_VECT_INDEX;
    return RS_OK;
}

int check_replace(const rs_t* rs, const size_t* dlens, int nd, const int* rows, int nr, const size_t* plens,
                  int np) {
    if (nd > rs->d) return RS_ERR_TOO_MANY_REPLACE;  // checkReplace rs.go:536-570
    if (nr != nd) return RS_ERR_MISMATCH_REPLACE;
    if (np != rs->p) return RS_ERR_MISMATCH_PARITY_NUM;
    if (nd <= 0) return RS_ERR_INVAL;  // reference indexes data[0] and panics
    const size_t size = dlens[0];
    if (size == 0) return RS_ERR_ZERO_VECT_SIZE;
    for (int i = 0; i < nd; ++i)
        if (dlens[i] != size) return RS_ERR_MISMATCH_VECT_SIZE;
    for (int i = 0; i < np; ++i)
        if (plens[i] != size) return RS_ERR_MISMATCH_VECT_SIZE;
    for (int i = 0; i < nr; ++i)
        if (rows[i] >= rs->d || rows[i] < 0) return RS_ERR_ILLEGAL_VECT_INDEX;
    return RS_OK;
}

// Update's matrix: p x 2, both columns G[j][row] (g*old ^ g*new == g*(old^new),
// so xorsimd's step rs.go:432-433 folds into the product).
bool ref_update_skip(int l1d, uint64_t size, uint64_t* lo, uint64_t* hi) {
    if (l1d <= 0) return false;
    const uint64_t split = static_cast<uint64_t>(l1d) / 2;  // getSplitSize rs.go:158-173
    if (size < split) return false;  // chunks of (n>>4)<<4 bytes, then a < 16-byte tail on its own
    const uint64_t last = size % split;
    if (last < 16 || (last & 15) == 0) return false;
    *lo = size - last;
    *hi = *lo + (last & ~uint64_t{15});
    return true;
}

std::vector<uint8_t> update_matrix(const rs_t* rs, int row) {
    std::vector<uint8_t> m(static_cast<size_t>(rs->p) * 2);
    for (int j = 0; j < rs->p; ++j) m[2 * j] = m[2 * j + 1] = rs->gen()[static_cast<size_t>(j) * rs->d + row];
    return m;
}

std::vector<uint8_t> replace_matrix(const rs_t* rs, const int* rows, int nr) {  // rs.go:506-514
    std::vector<uint8_t> m(static_cast<size_t>(rs->p) * nr);
    for (int i = 0; i < rs->p; ++i)
        for (int j = 0; j < nr; ++j) m[static_cast<size_t>(i) * nr + j] = rs->gen()[static_cast<size_t>(i) * rs->d + rows[j]];
    return m;
}

// The reference's two passes check their own argument sizes in order
// (reconstData, then reconstParity after the data is rebuilt).  Returns the
// data-pass check result and, through *parity_rc, the parity-pass one.
int check_reconst_passes(const rs_t* rs, const ReconstPlan& pl, const size_t* lens, int n, int* parity_rc) {
    const int d = rs->d, pn = pl.nnr - pl.dn;
    int idx[2 * kMaxVects];
    *parity_rc = RS_OK;
    if (pl.dn > 0) {
        for (int i = 0; i < d; ++i) idx[i] = pl.vs[i];
        for (int i = 0; i < pl.dn; ++i) idx[d + i] = pl.nr[i];
        for (int i = 0; i < d + pl.dn; ++i)
            if (idx[i] >= n) return RS_ERR_INVAL;  // the reference indexes past len(vects) and panics
        RS_TRY(check_encode_idx(lens, idx, d + pl.dn));
    }
    if (pn > 0) {
        for (int i = 0; i < d; ++i) idx[i] = i;
        for (int i = 0; i < pn; ++i) idx[d + i] = pl.nr[pl.dn + i];
        for (int i = 0; i < d + pn && *parity_rc == RS_OK; ++i)
            if (idx[i] >= n) *parity_rc = RS_ERR_INVAL;
        if (*parity_rc == RS_OK) *parity_rc = check_encode_idx(lens, idx, d + pn);
    }
    return RS_OK;
}

}  // namespace detail
}  // namespace rsamd

// ======================================================================
// C ABI: handle, matrices, planning, knobs (the calls themselves are in
// host_calls.cpp, batches.cpp and host_batches.cpp)
// ======================================================================
extern "C" {

const char* rs_strerror(int code) {
    switch (code) {
        case RS_OK: return "";
        case RS_ERR_ILLEGAL_VECTS: return "illegal data/parity number: <= 0 or data+parity > 256";
        case RS_ERR_MISMATCH_VECTS: return "too few/many vectors given";
        case RS_ERR_ZERO_VECT_SIZE: return "vector size is 0";
        case RS_ERR_MISMATCH_VECT_SIZE: return "vectors size mismatched";
        case RS_ERR_NO_NEED_RECONST: return "no need reconst";
        case RS_ERR_TOO_MANY_LOST: return "too many lost";
        case RS_ERR_MISMATCH_PARITY_NUM: return "parity number mismatched";
        case RS_ERR_ILLEGAL_VECT_INDEX: return "illegal vect index";
        case RS_ERR_TOO_MANY_REPLACE: return "too many data for replacing";
        case RS_ERR_MISMATCH_REPLACE: return "number of replaceRows and data mismatch";
        case RS_ERR_NOT_SQUARE: return "not a square matrix";
        case RS_ERR_SINGULAR_MATRIX: return "matrix is singular";
        case RS_ERR_INVAL: return "invalid argument (the reference panics on this input)";
        case RS_ERR_DEVICE: return "HIP device error";
        case RS_ERR_NOMEM: return "out of host memory";
        default: return "unknown error";
    }
}

int rs_version(void) { return 100; }

// cpu.X86.Cache.L1D as the reference's getSplitSize reads it (rs.go:158-159):
// the L1 data cache size of this host from CPUID, -1 when it cannot be
// detected, 0 on a non-x86 host.  templexxx/cpu v0.0.1 (go.mod:4) is not in
// the container; this restates the CPUID sources such a library reads:
// deterministic cache parameters (leaf 4 on Intel, leaf 0x8000001D on AMD
// with topology extensions), else AMD's leaf 0x80000005 ECX[31:24] KiB.
int rs_host_l1d(void) {
#if defined(__x86_64__) || defined(__i386__)
    static const int l1d = [] {
        unsigned a, b, c, d;
        if (!__get_cpuid(0, &a, &b, &c, &d)) return -1;
        const unsigned max_leaf = a;
        const bool amd = b == 0x68747541u;  // "Auth"enticAMD
        auto leaf_params = [](unsigned leaf) -> int {
            for (unsigned sub = 0; sub < 16; ++sub) {
                unsigned a2, b2, c2, d2;
                __cpuid_count(leaf, sub, a2, b2, c2, d2);
                const unsigned type = a2 & 31, level = (a2 >> 5) & 7;
                if (type == 0) break;
                if (type == 1 && level == 1)  // data cache, level 1
                    return static_cast<int>(((b2 >> 22) + 1) * (((b2 >> 12) & 0x3ff) + 1) * ((b2 & 0xfff) + 1) *
                                            (c2 + 1));
            }
            return -1;
        };
        if (!amd && max_leaf >= 4) {
            const int v = leaf_params(4);
            if (v > 0) return v;
        }
        if (amd && __get_cpuid(0x80000000u, &a, &b, &c, &d)) {
            const unsigned max_ext = a;
            if (max_ext >= 0x8000001Du && __get_cpuid(0x80000001u, &a, &b, &c, &d) && (c >> 22 & 1)) {
                const int v = leaf_params(0x8000001Du);
                if (v > 0) return v;
            }
            if (max_ext >= 0x80000005u && __get_cpuid(0x80000005u, &a, &b, &c, &d) && (c >> 24))
                return static_cast<int>((c >> 24) * 1024);
        }
        return -1;
    }();
    return l1d;
#else
    return 0;
#endif
}

int rs_set_ref_l1d(rs_t* rs, int l1d) {
    if (!rs) return RS_ERR_INVAL;
    if (l1d == -1) {
        const int host = rs_host_l1d();
        l1d = host > 0 ? host : 32 * 1024;  // rs.go:159-161: unknown (-1) or not x86 (0) -> 32 KiB
    }
    if (l1d != 0 && l1d < 32) return RS_ERR_INVAL;  // a split of at least 16 bytes (rs.go:169-172)
    rs->ref_l1d.store(l1d, std::memory_order_relaxed);
    return RS_OK;
}

int rs_ref_l1d(const rs_t* rs) { return rs ? rs->ref_l1d.load(std::memory_order_relaxed) : 0; }

// Source digest stamped by reedsolomon_amd/build.py (SHA-256 over the build's
// sources and flags).  The marker stays in .rodata so build.py can read the
// digest of a library file without loading it.
#ifndef RSAMD_BUILD_ID
#define RSAMD_BUILD_ID "unstamped"
#endif
__attribute__((used)) static const char k_build_stamp[] = "RSAMD_BUILD_ID=" RSAMD_BUILD_ID;

const char* rs_build_id(void) { return k_build_stamp + sizeof("RSAMD_BUILD_ID=") - 1; }

int rs_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : -1;
}

int rs_new(int data_num, int parity_num, int device, rs_t** out) {
    return abi_guard([&]() -> int {
        if (!out) return RS_ERR_INVAL;
        *out = nullptr;
        const int d = data_num, p = parity_num;
        if (d <= 0 || p <= 0 || d + p > kMaxVects) return RS_ERR_ILLEGAL_VECTS;  // rs.go:61-63
        rs_t* rs = new (std::nothrow) rs_codec();
        if (!rs) return RS_ERR_NOMEM;
        rs->d = d;
        rs->p = p;
        rs->enc = make_encode_matrix(d, p);
        if (d + p <= 64) {  // rs.go:70-74 (the cache key is a 64-bit bitmap)
            rs->cache_enabled = true;
            rs->cache_max = kMaxInverseCacheBytes / static_cast<uint64_t>(d) / static_cast<uint64_t>(d);
        }
        rs->device = device;
        *out = rs;
        return RS_OK;
    });
}

void rs_free(rs_t* rs) { delete rs; }

int rs_data_num(const rs_t* rs) { return rs ? rs->d : 0; }

int rs_parity_num(const rs_t* rs) { return rs ? rs->p : 0; }

int rs_device(const rs_t* rs) { return rs ? rs->device : -1; }

int rs_gen_matrix(const rs_t* rs, uint8_t* out) {
    return abi_guard([&]() -> int {
        if (!rs || !out) return RS_ERR_INVAL;
        std::memcpy(out, rs->gen(), static_cast<size_t>(rs->p) * rs->d);
        return RS_OK;
    });
}

int rs_enc_matrix(const rs_t* rs, uint8_t* out) {
    return abi_guard([&]() -> int {
        if (!rs || !out) return RS_ERR_INVAL;
        std::memcpy(out, rs->enc.data(), rs->enc.size());
        return RS_OK;
    });
}

uint8_t rs_gf_mul(uint8_t a, uint8_t b) { return gf_mul(a, b); }

int rs_tune(const char* name, int value) {
    return abi_guard([&]() -> int {
        if (!name) return RS_ERR_INVAL;
        LaunchTuning& t = tuning();
        const std::string n(name);
        if (n == "max_grid") t.max_grid = value;
        else if (n == "vpt") t.vpt = value == 2 ? 2 : 1;
        else if (n == "nt_store") t.nt_store = value;
#ifdef RSAMD_EXPERIMENTS  // code-shape experiments: librsamd_exp.so only (the product has no "var")
        else if (n == "var") t.var = value;
        else if (n == "jit_nobar") g_jit_nobar = value < 0 ? 0 : value > 3 ? 3 : value;  // timing diagnostic, wrong results
#endif
        else if (n == "lds_pad") t.lds_pad = value;
        else if (n == "lane_bytes") t.lane_bytes = value == 16 ? 16 : 8;
        else if (n == "block8") t.block8 = value == 128 ? 128 : 256;
        else if (n == "bitslice") t.bitslice = value ? 1 : 0;
        else if (n == "bs_waves") t.bs_waves = value < 0 ? 0 : value > 8 ? 8 : value;
        else if (n == "jit") g_jit_mode = value < 0 ? 0 : value > 2 ? 2 : value;
        else if (n == "jit_min_rows") g_jit_min_rows = value < 1 ? 1 : value;
        else if (n == "jit_min_acc_cols") g_jit_min_acc_cols = value < 1 ? 1 : value;
        else if (n == "jit_min_launches") g_jit_min_launches = value < 1 ? 1 : value;
        else if (n == "jit_pf") g_jit_pf = value < 1 ? 1 : value > 6 ? 6 : value;
        else if (n == "jit_sync") g_jit_sync = value < 0 ? 0 : value > 64 ? 64 : value;
        else if (n == "jit_waves") g_jit_waves = value < 0 ? 0 : value > 8 ? 8 : value;
        else if (n == "jit_layout") g_jit_layout = value == 1 || value == 2 ? value : 0;
        else if (n == "jit_group_waves")  // a power of two (the kernel shifts by log2): 1, 2, 4 or 8
            g_jit_group_waves = value >= 8 ? 8 : value >= 4 ? 4 : value >= 2 ? 2 : 1;
        else if (n == "jit_path_rows") g_jit_path_rows = value < 1 ? 1 : value > 16 ? 16 : value;
        else if (n == "jit_share") g_jit_share = value ? 1 : 0;
        else if (n == "jit_share_deep") g_jit_share_deep = value < 0 ? -1 : value ? 1 : 0;
        else if (n == "jit_share_dma") g_jit_share_dma = value < 2 ? 0 : value > 8 ? 8 : value;
        else if (n == "jit_share_ahead") g_jit_share_ahead = value ? 1 : 0;
        else if (n == "jit_gray") g_jit_gray = value ? 1 : 0;
        else if (n == "jit_split_cols") g_jit_split_cols = value < 0 ? 0 : value;
        else if (n == "jit_share_cols") g_jit_share_cols = value < 0 ? -1 : value > 2 ? 2 : value < 1 ? 1 : value;
        else if (n == "jit_wide_pf") g_jit_wide_pf = value < 1 ? 1 : value > 4 ? 4 : value;
        else if (n == "jit_wide_waves") g_jit_wide_waves = value < 0 ? 0 : value > 8 ? 8 : value;
        else if (n == "jit_disk_cache") g_jit_disk_cache = value ? 1 : 0;
        else if (n == "jit_backend") g_jit_backend = value < 0 ? 0 : value > 2 ? 2 : value;
        else if (n == "jit_min_bytes") g_jit_min_bytes = value < 0 ? 0 : static_cast<uint64_t>(value);
        else if (n == "multi_gpu_plan") t.multi_gpu_plan = value < 0 ? -1 : value;
        else if (n == "bs_block") t.bs_block = (value == 64 || value == 128 || value == 256) ? value : 0;
        else if (n == "wide_block") t.wide_block = value == 128 ? 128 : 256;
        else if (n == "wide_single_pass") t.wide_single_pass = value ? 1 : 0;
        else if (n == "host_engine") g_engine = value ? 1 : 0;
        else if (n == "host_engine_waves") g_engine_waves = value < 1 ? 1 : value > kEngineMaxGroups ? kEngineMaxGroups : value;
        else if (n == "host_engine_group_waves")
            g_engine_group_waves = value < 1 ? 1 : value > kEngineMaxGroupWaves ? kEngineMaxGroupWaves : value;
        else if (n == "host_engine_wg_units") g_engine_wg_units = value < 0 ? 0 : value;
        else if (n == "host_engine_poll_gap") g_engine_poll_gap = value < 0 ? 0 : value > 1000 ? 1000 : value;
        else if (n == "host_engine_yield_us") g_engine_yield_us = value < 0 ? 0 : value;
        else if (n == "host_engine_idle_us") g_engine_idle_us = value < 20 ? 20 : value > 100000 ? 100000 : value;
        else if (n == "host_engine_vram") g_engine_vram = value ? 1 : 0;
        else if (n == "host_engine_split_rows") g_engine_split_rows = value < 0 ? 0 : value > 2 ? 2 : value;
        else if (n == "host_engine_cold_launch") g_engine_cold_launch = value ? 1 : 0;
        else if (n == "host_flag_sync") g_host_flag_sync = value ? 1 : 0;
        else if (n == "host_engine_life_us") g_engine_life_us = value < 100 ? 100 : value > 1000000 ? 1000000 : value;
        else if (n == "host_engine_max_bytes") g_engine_max_bytes = value < 0 ? 0 : static_cast<size_t>(value);
        else if (n == "host_pinned_max") g_pinned_max = value < 0 ? 0 : static_cast<size_t>(value);
        else if (n == "host_zc_max") g_zc_max = value < 0 ? SIZE_MAX : static_cast<size_t>(value);
        else if (n == "host_batch_zc") g_host_batch_zc = value;
        else if (n == "host_unregister_revoke") g_unregister_revoke = value ? 1 : 0;
        else if (n == "host_dma_1d") g_host_dma_1d = value;
        else if (n == "host_pageable_stage") g_host_pageable_stage = value;
        else if (n == "host_pageable_slot") g_pageable_slot = value < 4096 ? 4096 : static_cast<size_t>(value);
        else if (n == "host_copy_nt") g_copy_nt = value ? 1 : 0;
        else if (n == "host_copy_coalesce") g_copy_coalesce = value ? 1 : 0;
        else if (n == "bind_numa") g_bind_numa = value;
        else if (n == "table_registry_max") g_registry_max = value < 1 ? 1 : static_cast<size_t>(value);
        else if (n == "table_inplace_max") g_tab_inplace_max = value < 0 ? 0 : static_cast<size_t>(value);
        else if (n == "table_stage_vram") g_tab_stage_vram = value ? 1 : 0;
        else if (n == "host_coalesce_linger_us") g_coalesce_linger_us = value < 0 ? 0 : value;
        else if (n == "host_engine_direct") g_engine_direct = value ? 1 : 0;
        else if (n == "host_coalesce_running") g_co_running = value < 1 ? 1 : value > 2 ? 2 : value;
        else if (n == "host_coalesce_max") g_coalesce_max = value < 0 ? 0 : static_cast<size_t>(value);
        else if (n == "host_chunk") g_chunk = value < 4096 ? 4096 : static_cast<size_t>(value) & ~size_t{4095};
        else if (n == "host_chunk_split") g_chunk_split = value < 0 ? 0 : static_cast<size_t>(value);
        else return RS_ERR_INVAL;
        return RS_OK;
    });
}

int rs_matrix_invert(const uint8_t* m, size_t m_len, int n, uint8_t* out) {
    return abi_guard([&]() -> int {
        if (n < 0 || (!m && m_len) || !out) return RS_ERR_INVAL;
        return invert(m, m_len, n, out);
    });
}

uint64_t rs_inverse_cache_key(const int* survived, int ns) { return cache_key(survived, ns); }

const char* rs_last_device_error(void) { return g_last_dev_err; }

int rs_host_engine_stats(const rs_t* rs, uint64_t* calls, uint64_t* launches) {
    return abi_guard([&]() -> int {
        if (!rs) return RS_ERR_INVAL;
        if (calls) *calls = rs->eng_calls.load(std::memory_order_relaxed);
        if (launches) *launches = rs->eng_launches.load(std::memory_order_relaxed);
        return RS_OK;
    });
}

int rs_host_call_stats(const rs_t* rs, uint64_t* launches, uint64_t* calls) {
    return abi_guard([&]() -> int {
        if (!rs) return RS_ERR_INVAL;
        if (launches) *launches = rs->co_launches.load(std::memory_order_relaxed);
        if (calls) *calls = rs->co_calls.load(std::memory_order_relaxed);
        return RS_OK;
    });
}

int64_t rs_inverse_cache_size(const rs_t* rs) {
    if (!rs) return -1;
    std::lock_guard<std::mutex> lk(const_cast<rs_t*>(rs)->cache_mu);
    return static_cast<int64_t>(rs->cache.size());
}

int rs_plan_reconst(const rs_t* rs, const int* survived, int ns, const int* need, int nn, int* vs, int* nvs,
                    int* nr, int* nnr, int* dn) {
    return abi_guard([&]() -> int {
        if (!rs || !vs || !nvs || !nr || !nnr || !dn) return RS_ERR_INVAL;
        return plan_reconst(rs, survived, ns, need, nn, vs, nvs, nr, nnr, dn);
    });
}

int rs_reconst_matrix(rs_t* rs, const int* survived_d, const int* need, int nn, uint8_t* out) {
    return abi_guard([&]() -> int {
        if (!rs || !survived_d || (nn && (!need || !out))) return RS_ERR_INVAL;
        RS_TRY(check_vect_idx(survived_d, rs->d, rs->d + rs->p));
        for (int i = 0; i < nn; ++i)
            if (need[i] < 0 || need[i] >= rs->d) return RS_ERR_INVAL;
        return reconst_matrix(rs, survived_d, need, nn, out);
    });
}

}  // extern "C"

int rs_jit_stats(uint64_t* compiled, uint64_t* failed, uint64_t* launches, double* compile_ms) {
    return abi_guard([&]() -> int {
        jit_stats(compiled, failed, launches, compile_ms);
        return RS_OK;
    });
}

int rs_coef_table_stats(const rs_t* rs, uint64_t* uploads, uint64_t* inplace) {
    return abi_guard([&]() -> int {
        if (!rs) return RS_ERR_INVAL;
        std::lock_guard<std::mutex> lk(const_cast<rs_t*>(rs)->tab_mu);
        if (uploads) *uploads = rs->tab_uploads;
        if (inplace) *inplace = rs->tab_inplace;
        return RS_OK;
    });
}

int rs_jit_table_stats(uint64_t* entries, uint64_t* evictions) {
    return abi_guard([&]() -> int {
        jit_table_stats(entries, evictions);
        return RS_OK;
    });
}

int rs_jit_cache_stats(uint64_t* hits, uint64_t* misses, uint64_t* writes, uint64_t* rejects) {
    return abi_guard([&]() -> int {
        jit_cache_stats(hits, misses, writes, rejects);
        return RS_OK;
    });
}

int rs_jit_prepare(rs_t* rs, const uint8_t* mat, int rows, int cols, int accumulate, int wait) {
    return abi_guard([&]() -> int {
        if (!rs || !mat || rows < kJitMinRows || rows > jit_max_rows() || cols < 1 || cols > jit_max_cols())
            return RS_ERR_INVAL;
        RS_TRY(ensure_device(rs));
        DeviceGuard g(rs->device);
        return jit_prepare(mat, rows, cols, accumulate != 0, wait != 0);
    });
}

int64_t rs_jit_asm_source(const uint8_t* mat, int rows, int cols, int accumulate, char* buf, size_t len) {
    try {
        std::string s;
        const int rc = jit_asm_source_text(mat, rows, cols, accumulate != 0, &s);
        if (rc) return -rc;
        if (buf && len) {
            const size_t n = s.size() < len - 1 ? s.size() : len - 1;
            std::memcpy(buf, s.data(), n);
            buf[n] = 0;
        }
        return static_cast<int64_t>(s.size()) + 1;
    } catch (...) {
        return -RS_ERR_NOMEM;
    }
}

int rs_jit_compile_check(const uint8_t* mat, int rows, int cols, int accumulate, double* ms) {
    return abi_guard([&]() -> int { return jit_compile_check(mat, rows, cols, accumulate != 0, ms); });
}

int rs_jit_encoder_check(const uint8_t* mat, int rows, int cols, int accumulate, size_t* code_bytes) {
    return abi_guard([&]() -> int { return jit_encoder_check(mat, rows, cols, accumulate != 0, code_bytes); });
}
