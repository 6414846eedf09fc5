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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/rs_amd.h"
#include "gf256.hpp"
#include "host_pool.hpp"
#include "kernels.hpp"

using namespace rsamd;

#define RS_TRY(x)                 \
    do {                          \
        int rc_ = (x);            \
        if (rc_) return rc_;      \
    } while (0)

namespace {

constexpr int kMaxVects = 256;                              // rs.go:47
constexpr uint64_t kMaxInverseCacheBytes = 16ull << 20;     // rs.go:50
constexpr size_t kMaxRegistryEntries = 1 << 14;

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

// invert matrix.go:85-147 (Gauss-Jordan; a zero pivot swaps with the first
// lower row that has a non-zero entry in the pivot column; the result is
// bit-identical to the reference's).
int invert(const uint8_t* src, size_t len, int n, uint8_t* out) {
    if (static_cast<size_t>(n) * n != len) return RS_ERR_NOT_SQUARE;
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

}  // namespace

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

    // device state (created lazily; the handle works on a GPU-less host)
    std::mutex dev_mu;
    int device = -1;
    bool device_ready = false;

    std::mutex tab_mu;  // coefficient-table registry: matrix bytes -> device perm tables
    std::map<std::string, uint32_t*> tables;

    std::mutex stage_mu;  // staging for the host-memory entry points
    uint8_t* stage = nullptr;
    size_t stage_bytes = 0;
    uint8_t* hstage = nullptr;  // pinned host mirror of `stage` (small-vector fast path)
    size_t hstage_bytes = 0;
    uint8_t* slots = nullptr;   // device staging slots of the staged (non-zero-copy) host path
    bool zc_pending = false;    // a zero-copy kernel may still be using hstage
    hipEvent_t chunk_ev[3] = {nullptr, nullptr, nullptr};  // host-call chunk pipeline slots
    hipStream_t stream = nullptr;

    // Upload ring for per-call device descriptors (multi-pattern Reconst):
    // pinned host slot -> device slot on a private copy stream, so the copy
    // for call n+1 overlaps call n's kernel instead of stalling the stream.
    static constexpr int kUploadSlots = 4;
    struct UploadSlot {
        uint8_t* host = nullptr;
        uint8_t* dev = nullptr;
        size_t cap = 0;
        hipEvent_t copied = nullptr, done = nullptr;
        bool in_flight = false;
    };
    std::mutex up_mu;
    UploadSlot up[kUploadSlots];
    int up_next = 0;
    hipStream_t up_stream = nullptr;

    const uint8_t* gen() const { return enc.data() + static_cast<size_t>(d) * d; }

    ~rs_codec() {
        if (!device_ready) return;
        DeviceGuard g(device);
        if (stream) (void)hipStreamSynchronize(stream);
        (void)hipDeviceSynchronize();
        for (auto& kv : tables) (void)hipFree(kv.second);
        for (UploadSlot& u : up) {
            if (u.host) (void)hipHostFree(u.host);
            if (u.dev) (void)hipFree(u.dev);
            if (u.copied) (void)hipEventDestroy(u.copied);
            if (u.done) (void)hipEventDestroy(u.done);
        }
        if (up_stream) (void)hipStreamDestroy(up_stream);
        if (stage) (void)hipFree(stage);
        if (hstage) (void)hipHostFree(hstage);
        for (hipEvent_t e : chunk_ev)
            if (e) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {

int ensure_device(rs_t* rs) {
    std::lock_guard<std::mutex> lk(rs->dev_mu);
    if (rs->device_ready) return RS_OK;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return RS_ERR_DEVICE;
    if (rs->device < 0) {
        int cur = 0;
        if (hipGetDevice(&cur) != hipSuccess) return RS_ERR_DEVICE;
        rs->device = cur;
    }
    if (rs->device >= count) return RS_ERR_DEVICE;
    rs->device_ready = true;
    return RS_OK;
}

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
    // A pinned host buffer of `bytes` to fill (slot free for reuse on return).
    int acquire(size_t bytes, uint8_t** host) {
        rs_codec::UploadSlot& u = rs_->up[rs_->up_next];
        rs_->up_next = (rs_->up_next + 1) % rs_codec::kUploadSlots;
        if (!rs_->up_stream && hipStreamCreateWithFlags(&rs_->up_stream, hipStreamNonBlocking) != hipSuccess) {
            rs_->up_stream = nullptr;
            return RS_ERR_DEVICE;
        }
        if (u.in_flight) {  // the kernel that read this slot's device copy has finished
            if (hipEventSynchronize(u.done) != hipSuccess) return RS_ERR_DEVICE;
            u.in_flight = false;
        }
        if (!u.copied && (hipEventCreateWithFlags(&u.copied, hipEventDisableTiming) != hipSuccess ||
                          hipEventCreateWithFlags(&u.done, hipEventDisableTiming) != hipSuccess))
            return RS_ERR_DEVICE;
        if (u.cap < bytes) {
            if (u.host) (void)hipHostFree(u.host);
            if (u.dev) (void)hipFree(u.dev);
            u.host = nullptr;
            u.dev = nullptr;
            u.cap = 0;
            size_t cap = (bytes + (size_t{64} << 10) - 1) & ~((size_t{64} << 10) - 1);
            if (hipHostMalloc(reinterpret_cast<void**>(&u.host), cap, hipHostMallocDefault) != hipSuccess) {
                u.host = nullptr;
                return RS_ERR_NOMEM;
            }
            if (hipMalloc(reinterpret_cast<void**>(&u.dev), cap) != hipSuccess) {
                (void)hipHostFree(u.host);
                u.host = nullptr;
                u.dev = nullptr;
                return RS_ERR_NOMEM;
            }
            u.cap = cap;
        }
        slot_ = &u;
        bytes_ = bytes;
        *host = u.host;
        return RS_OK;
    }
    // Copy the filled host buffer to the device and make `st` wait for it.
    int upload(hipStream_t st, uint8_t** dev) {
        st_ = st;
        if (hipMemcpyAsync(slot_->dev, slot_->host, bytes_, hipMemcpyHostToDevice, rs_->up_stream) != hipSuccess ||
            hipEventRecord(slot_->copied, rs_->up_stream) != hipSuccess ||
            hipStreamWaitEvent(st, slot_->copied, 0) != hipSuccess)
            return RS_ERR_DEVICE;
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

// Perm tables for a rows x cols coefficient matrix, laid out
// [col][rows_pad][5] dwords (rows padded to a multiple of 8 so that every
// kernel row group reads inside the allocation).  Uploaded once per distinct
// matrix and reused by every later launch.
int get_tables(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint32_t** out, int* rows_pad_out) {
    const int rows_pad = static_cast<int>(rup(rows, 8));
    std::string key(reinterpret_cast<const char*>(&rows), sizeof rows);
    key.append(reinterpret_cast<const char*>(&cols), sizeof cols);
    key.append(reinterpret_cast<const char*>(mat), static_cast<size_t>(rows) * cols);
    std::lock_guard<std::mutex> lk(rs->tab_mu);
    auto it = rs->tables.find(key);
    if (it != rs->tables.end()) {
        *out = it->second;
        *rows_pad_out = rows_pad;
        return RS_OK;
    }
    if (rs->tables.size() >= kMaxRegistryEntries) {
        // Bounded registry: drain the device before recycling table memory.
        if (hipDeviceSynchronize() != hipSuccess) return RS_ERR_DEVICE;
        for (auto& kv : rs->tables) (void)hipFree(kv.second);
        rs->tables.clear();
    }
    std::vector<uint32_t> host(static_cast<size_t>(cols) * rows_pad * 5, 0);
    for (int c = 0; c < cols; ++c)
        for (int r = 0; r < rows; ++r)
            perm_table(mat[static_cast<size_t>(r) * cols + c], &host[(static_cast<size_t>(c) * rows_pad + r) * 5]);
    uint32_t* dptr = nullptr;
    if (hipMalloc(&dptr, host.size() * 4) != hipSuccess) return RS_ERR_DEVICE;
    if (hipMemcpy(dptr, host.data(), host.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(dptr);
        return RS_ERR_DEVICE;
    }
    rs->tables.emplace(std::move(key), dptr);
    *out = dptr;
    *rows_pad_out = rows_pad;
    return RS_OK;
}

// One launch of the product: out[r] (=|^=) sum_c mat[r][c] * in[c] on every
// stripe.  in_ptrs/out_ptrs are stripe-0 addresses; vector v of stripe s adds
// s * ss[sid[v]] (sid == nullptr: all inputs use ss[0], all outputs ss[1]).
int matmul_ex(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* in_ptrs,
              const uint8_t* in_sid, uint8_t* const* out_ptrs, const uint8_t* out_sid, const int64_t ss[4],
              int nstripes, uint64_t len, bool accumulate, hipStream_t stream, const int32_t* stripe_ids = nullptr) {
    if (rows <= 0 || cols <= 0 || nstripes <= 0 || len == 0) return RS_OK;
    if (rows + cols > kMaxPtrs) return RS_ERR_INVAL;
    MatmulArgs a;
    std::memset(&a, 0, sizeof a);
    int rc = get_tables(rs, mat, rows, cols, &a.tables, &a.rows_pad);
    if (rc) return rc;
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
    return launch_gf_matmul(a, stream) == hipSuccess ? RS_OK : RS_ERR_DEVICE;
}

int matmul(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* const* in_ptrs, int64_t in_ss,
           uint8_t* const* out_ptrs, int64_t out_ss, int nstripes, uint64_t len, bool accumulate,
           hipStream_t stream) {
    const int64_t ss[4] = {in_ss, out_ss, 0, 0};
    return matmul_ex(rs, mat, rows, cols, in_ptrs, nullptr, out_ptrs, nullptr, ss, nstripes, len, accumulate,
                     stream);
}

// Address of vector v (0..d+p) of stripe 0 and its stride selector under a layout.
struct LayoutAddr {
    const rs_layout_t* L;
    int d;
    uint8_t* ptr(int v) const {
        return v < d ? L->data_base + v * L->data_vect_stride : L->parity_base + (v - d) * L->parity_vect_stride;
    }
    uint8_t sid(int v) const { return v < d ? 0 : 1; }
};

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

// getReconstMatrix rs.go:382-392 + makeReconstMatrix matrix.go:56-64:
// rows `need` (data indexes) of the inverse.
int reconst_matrix(rs_t* rs, const int* survived_d, const int* need, int nn, uint8_t* out) {
    const int d = rs->d;
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


// ---------------------------------------------------------------- host staging

// Vectors up to this size go through the pinned host mirror: the caller's
// bytes are memcpy'd into pinned memory and each direction is ONE DMA over
// contiguous slots, instead of one pageable copy (staged by the runtime) per
// vector.  Larger vectors use the runtime's pipelined pageable copies.
size_t g_pinned_max = 256 * 1024;
// Host calls on vectors up to this size take the chunked zero-copy pipeline
// (host_matmul: the kernel reads and writes the pinned mirror over PCIe, no
// DMA set-up either way); larger ones the runtime's pageable copies, which
// measured 7 % faster at 4 MiB (profiles/r01/host_latency.log).
size_t g_zc_max = 2 * 1024 * 1024;

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
    if (!rs->stream && hipStreamCreateWithFlags(&rs->stream, hipStreamNonBlocking) != hipSuccess)
        return RS_ERR_DEVICE;
    if (need > rs->stage_bytes) {
        if (rs->stage) {
            (void)hipStreamSynchronize(rs->stream);
            (void)hipFree(rs->stage);
            rs->stage = nullptr;
            rs->stage_bytes = 0;
        }
        if (hipMalloc(&rs->stage, need) != hipSuccess) return RS_ERR_DEVICE;
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
    return hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, rs->stream) == hipSuccess ? RS_OK : RS_ERR_DEVICE;
}
int d2h(rs_t* rs, uint8_t* dst, const uint8_t* src, size_t n) {
    return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, rs->stream) == hipSuccess ? RS_OK : RS_ERR_DEVICE;
}
int sync(rs_t* rs) { return hipStreamSynchronize(rs->stream) == hipSuccess ? RS_OK : RS_ERR_DEVICE; }

int stage_in(rs_t* rs, const uint8_t* const* src, int n, size_t size, size_t pitch, int first, int total_slots) {
    if (n <= 0) return RS_OK;
    uint8_t* dev = rs->stage + static_cast<size_t>(first) * pitch;
    if (use_pinned(rs, total_slots, pitch)) {
        uint8_t* h = rs->hstage + static_cast<size_t>(first) * pitch;
        for (int i = 0; i < n; ++i) std::memcpy(h + static_cast<size_t>(i) * pitch, src[i], size);
        return h2d(rs, dev, h, static_cast<size_t>(n - 1) * pitch + size);
    }
    for (int i = 0; i < n; ++i) RS_TRY(h2d(rs, dev + static_cast<size_t>(i) * pitch, src[i], size));
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
    for (int i = 0; i < n; ++i) RS_TRY(d2h(rs, dst[i], dev + static_cast<size_t>(i) * pitch, size));
    return sync(rs);
}


// Column-chunk size of the host-call pipeline (bytes per vector per chunk).
size_t g_chunk = 128 * 1024;
// Total copy bytes of one chunk above which the staging copies are split
// over the host copy pool.
constexpr size_t kParallelCopyMin = 512 * 1024;

// dst[i] <- src[i] (n vectors, len bytes each) on the copy pool, in
// 64 KiB pieces so every thread gets work.
void parallel_copy(uint8_t* const* dst, const uint8_t* const* src, int n, size_t len) {
    const size_t piece = 64 * 1024;
    const size_t per = (len + piece - 1) / piece;
    const size_t total = per * static_cast<size_t>(n);
    if (len * static_cast<size_t>(n) < kParallelCopyMin || total <= 1) {
        for (int i = 0; i < n; ++i) std::memcpy(dst[i], src[i], len);
        return;
    }
    CopyPool::get().run(total, [&](size_t k) {
        const size_t v = k / per, off = (k % per) * piece;
        const size_t b = std::min(piece, len - off);
        std::memcpy(dst[v] + off, src[v] + off, b);
    });
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
    if (!rs->stream && hipStreamCreateWithFlags(&rs->stream, hipStreamNonBlocking) != hipSuccess)
        return RS_ERR_DEVICE;
    // chunk: <= g_chunk per vector and <= 8 MiB per slot, 4 KiB multiple
    size_t C = rup(size, 256);
    const size_t cap = std::max<size_t>(4096, std::min(g_chunk, (size_t{8} << 20) / nvec) & ~size_t{4095});
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
    if (hipHostGetDevicePointer(&dbase, rs->hstage, 0) != hipSuccess || !dbase) return RS_ERR_DEVICE;
    for (int i = 0; i < ns; ++i)
        if (!rs->chunk_ev[i] && hipEventCreateWithFlags(&rs->chunk_ev[i], hipEventDisableTiming) != hipSuccess) {
            rs->chunk_ev[i] = nullptr;
            return RS_ERR_DEVICE;
        }
    auto hslot = [&](size_t c, int v) { return rs->hstage + (c % ns) * slot + static_cast<size_t>(v) * C; };
    auto dslot = [&](size_t c, int v) {
        return static_cast<uint8_t*>(dbase) + (c % ns) * slot + static_cast<size_t>(v) * C;
    };
    auto clen = [&](size_t c) { return std::min(C, size - c * C); };
    auto finish = [&](size_t c) -> int {  // wait for chunk c, copy its outputs back
        if (hipEventSynchronize(rs->chunk_ev[c % ns]) != hipSuccess) return RS_ERR_DEVICE;
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
        if (rc == RS_OK && hipEventRecord(rs->chunk_ev[c % ns], rs->stream) != hipSuccess) rc = RS_ERR_DEVICE;
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

// Bytes spanned by a [S][nvec][len] batch with non-negative strides.
size_t batch_extent(int64_t ss, int64_t vs, int nstripes, int nvec, size_t len) {
    return static_cast<size_t>(nstripes - 1) * static_cast<size_t>(ss) +
           static_cast<size_t>(nvec - 1) * static_cast<size_t>(vs) + len;
}

// Zero-copy host batches (on by default): kernels read and write pinned host
// memory over PCIe directly.  Measured on MI355X: 72 GiB/s of (k+m)*vec for
// 10+4 encode at 8 KiB-1 MiB vectors vs 13-57 GiB/s for the DMA pipeline.
int g_host_batch_zc = 1;

hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Reconst on one stripe whose vectors are addressed by `ptr` (host staging
// slots or caller device pointers).  Shared by rs_reconst / rs_reconst_dev /
// rs_reconst_batch.  `before_parity` lets the host path copy the rebuilt data
// back before the parity check runs (the reference returns the parity-pass
// error with the data already rebuilt).
struct ReconstPlan {
    int vs[kMaxVects], nr[kMaxVects];
    int nvs = 0, nnr = 0, dn = 0;
};

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

}  // namespace

// ======================================================================
// C ABI
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

int rs_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : -1;
}

int rs_new(int data_num, int parity_num, int device, rs_t** out) {
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
}

void rs_free(rs_t* rs) { delete rs; }

int rs_data_num(const rs_t* rs) { return rs ? rs->d : 0; }
int rs_parity_num(const rs_t* rs) { return rs ? rs->p : 0; }

int rs_gen_matrix(const rs_t* rs, uint8_t* out) {
    if (!rs || !out) return RS_ERR_INVAL;
    std::memcpy(out, rs->gen(), static_cast<size_t>(rs->p) * rs->d);
    return RS_OK;
}

int rs_enc_matrix(const rs_t* rs, uint8_t* out) {
    if (!rs || !out) return RS_ERR_INVAL;
    std::memcpy(out, rs->enc.data(), rs->enc.size());
    return RS_OK;
}

uint8_t rs_gf_mul(uint8_t a, uint8_t b) { return gf_mul(a, b); }

int rs_tune(const char* name, int value) {
    if (!name) return RS_ERR_INVAL;
    LaunchTuning& t = tuning();
    const std::string n(name);
    if (n == "max_grid") t.max_grid = value;
    else if (n == "vpt") t.vpt = value == 2 ? 2 : 1;
    else if (n == "nt_store") t.nt_store = value;
    else if (n == "var") t.var = value;
    else if (n == "lds_pad") t.lds_pad = value;
    else if (n == "stage_late") t.stage_late = value;
    else if (n == "host_pinned_max") g_pinned_max = value < 0 ? 0 : static_cast<size_t>(value);
    else if (n == "host_zc_max") g_zc_max = value < 0 ? SIZE_MAX : static_cast<size_t>(value);
    else if (n == "host_batch_zc") g_host_batch_zc = value;
    else if (n == "host_chunk") g_chunk = value < 4096 ? 4096 : static_cast<size_t>(value) & ~size_t{4095};
    else return RS_ERR_INVAL;
    return RS_OK;
}

int rs_matrix_invert(const uint8_t* m, size_t m_len, int n, uint8_t* out) {
    if (n < 0 || (!m && m_len) || !out) return RS_ERR_INVAL;
    return invert(m, m_len, n, out);
}

uint64_t rs_inverse_cache_key(const int* survived, int ns) { return cache_key(survived, ns); }

int64_t rs_inverse_cache_size(const rs_t* rs) {
    if (!rs) return -1;
    std::lock_guard<std::mutex> lk(const_cast<rs_t*>(rs)->cache_mu);
    return static_cast<int64_t>(rs->cache.size());
}

int rs_plan_reconst(const rs_t* rs, const int* survived, int ns, const int* need, int nn, int* vs, int* nvs,
                    int* nr, int* nnr, int* dn) {
    if (!rs || !vs || !nvs || !nr || !nnr || !dn) return RS_ERR_INVAL;
    return plan_reconst(rs, survived, ns, need, nn, vs, nvs, nr, nnr, dn);
}

int rs_reconst_matrix(rs_t* rs, const int* survived_d, const int* need, int nn, uint8_t* out) {
    if (!rs || !survived_d || (nn && (!need || !out))) return RS_ERR_INVAL;
    RS_TRY(check_vect_idx(survived_d, rs->d, rs->d + rs->p));
    for (int i = 0; i < nn; ++i)
        if (need[i] < 0 || need[i] >= rs->d) return RS_ERR_INVAL;
    return reconst_matrix(rs, survived_d, need, nn, out);
}

// ---------------------------------------------------------------- Encode

int rs_encode(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n) {
    if (!rs || (n > 0 && (!vects || !lens))) return RS_ERR_INVAL;
    RS_TRY(check_encode(rs, lens, n));
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    std::lock_guard<std::mutex> lk(rs->stage_mu);
    return host_product(rs, rs->gen(), rs->p, rs->d, vects, vects + rs->d, lens[0], false);
}

int rs_encode_dev(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n, void* stream) {
    if (!rs || (n > 0 && (!vects || !lens))) return RS_ERR_INVAL;
    RS_TRY(check_encode(rs, lens, n));
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    return matmul(rs, rs->gen(), rs->p, rs->d, vects, 0, vects + rs->d, 0, 1, lens[0], false, as_stream(stream));
}

int rs_encode_batch_layout(rs_t* rs, const rs_layout_t* L, int nstripes, size_t len, void* stream) {
    if (!rs || !L || nstripes < 0 || (nstripes > 0 && (!L->data_base || !L->parity_base))) return RS_ERR_INVAL;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    if (nstripes == 0) return RS_OK;
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    const LayoutAddr A{L, rs->d};
    const uint8_t* in[kMaxVects];
    uint8_t* out[kMaxVects];
    for (int i = 0; i < rs->d; ++i) in[i] = A.ptr(i);
    for (int j = 0; j < rs->p; ++j) out[j] = A.ptr(rs->d + j);
    return matmul(rs, rs->gen(), rs->p, rs->d, in, L->data_stripe_stride, out, L->parity_stripe_stride, nstripes,
                  len, false, as_stream(stream));
}

int rs_encode_batch(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride, int nstripes, size_t len,
                    void* stream) {
    if (!rs || nstripes < 0 || (nstripes > 0 && !base)) return RS_ERR_INVAL;
    const rs_layout_t L{base, stripe_stride, vect_stride, base + rs->d * vect_stride, stripe_stride, vect_stride};
    return rs_encode_batch_layout(rs, &L, nstripes, len, stream);
}

// ---------------------------------------------------------------- Reconst

int rs_reconst(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n, const int* survived, int ns,
               const int* need, int nn) {
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
        std::lock_guard<std::mutex> lk(rs->stage_mu);
        const uint8_t* src[kMaxVects];
        uint8_t* dst[kMaxVects];
        for (int i = 0; i < d; ++i) src[i] = vects[pl.vs[i]];
        for (int i = 0; i < rows; ++i) dst[i] = vects[pl.nr[i]];
        std::vector<uint8_t> m;
        RS_TRY(combined_matrix(rs, pl.vs, pl.nr, rows, pl.dn, m));
        RS_TRY(host_product(rs, m.data(), rows, d, src, dst, lens[pl.vs[0]], false));
    }
    return parity_rc;
}

int rs_reconst_dev(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n, const int* survived, int ns,
                   const int* need, int nn, void* stream) {
    if (!rs || (nn > 0 && !need) || (ns > 0 && !survived)) return RS_ERR_INVAL;
    ReconstPlan pl;
    int rc = plan_reconst(rs, survived, ns, need, nn, pl.vs, &pl.nvs, pl.nr, &pl.nnr, &pl.dn);
    if (rc == RS_ERR_NO_NEED_RECONST) return RS_OK;
    if (rc) return rc;
    if (!vects || !lens) return RS_ERR_INVAL;
    const int d = rs->d;
    int parity_rc = RS_OK;
    RS_TRY(check_reconst_passes(rs, pl, lens, n, &parity_rc));
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    const uint8_t* in[kMaxVects];
    uint8_t* out[kMaxVects];
    for (int i = 0; i < d; ++i) in[i] = vects[pl.vs[i]];
    // Parity pass would fail its checks: rebuild the data only, then report
    // the parity-pass error (the reference's order).  Otherwise one pass.
    const int rows = parity_rc ? pl.dn : pl.nnr;
    if (rows > 0) {
        std::vector<uint8_t> m;
        RS_TRY(combined_matrix(rs, pl.vs, pl.nr, rows, pl.dn, m));
        for (int i = 0; i < rows; ++i) out[i] = vects[pl.nr[i]];
        RS_TRY(matmul(rs, m.data(), rows, d, in, 0, out, 0, 1, lens[pl.vs[0]], false, as_stream(stream)));
    }
    return parity_rc;
}

int rs_reconst_batch_layout(rs_t* rs, const rs_layout_t* L, int nstripes, size_t len, const int* survived, int ns,
                            const int* need, int nn, void* stream) {
    if (!rs || !L || nstripes < 0 || (nn > 0 && !need) || (ns > 0 && !survived)) return RS_ERR_INVAL;
    ReconstPlan pl;
    int rc = plan_reconst(rs, survived, ns, need, nn, pl.vs, &pl.nvs, pl.nr, &pl.nnr, &pl.dn);
    if (rc == RS_ERR_NO_NEED_RECONST) return RS_OK;
    if (rc) return rc;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    if (nstripes == 0) return RS_OK;
    if (!L->data_base || !L->parity_base) return RS_ERR_INVAL;
    const int d = rs->d;
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    // One pass: every lost vector from the first d survivors (combined_matrix).
    std::vector<uint8_t> m;
    RS_TRY(combined_matrix(rs, pl.vs, pl.nr, pl.nnr, pl.dn, m));
    const LayoutAddr A{L, d};
    const int64_t ss[4] = {L->data_stripe_stride, L->parity_stripe_stride, 0, 0};
    const uint8_t* in[kMaxVects];
    uint8_t* out[kMaxVects];
    uint8_t isid[kMaxVects], osid[kMaxVects];  // stride selectors (copied into the dword kernel array)
    for (int i = 0; i < d; ++i) {
        in[i] = A.ptr(pl.vs[i]);
        isid[i] = A.sid(pl.vs[i]);
    }
    for (int i = 0; i < pl.nnr; ++i) {
        out[i] = A.ptr(pl.nr[i]);
        osid[i] = A.sid(pl.nr[i]);
    }
    return matmul_ex(rs, m.data(), pl.nnr, d, in, isid, out, osid, ss, nstripes, len, false, as_stream(stream));
}

int rs_reconst_batch(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride, int nstripes, size_t len,
                     const int* survived, int ns, const int* need, int nn, void* stream) {
    if (!rs || nstripes < 0 || (nstripes > 0 && !base)) return RS_ERR_INVAL;
    const rs_layout_t L{base, stripe_stride, vect_stride, base + rs->d * vect_stride, stripe_stride, vect_stride};
    return rs_reconst_batch_layout(rs, &L, nstripes, len, survived, ns, need, nn, stream);
}

int rs_reconst_batch_multi(rs_t* rs, const rs_layout_t* L, int nstripes, size_t len, const uint64_t* need_masks,
                           void* stream) {
    if (!rs || !L || nstripes < 0 || (nstripes > 0 && !need_masks)) return RS_ERR_INVAL;
    const int d = rs->d, p = rs->p;
    if (d + p > 64) return RS_ERR_INVAL;  // masks are 64-bit survivor bitmaps, like the cache key
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    const uint64_t valid = (d + p == 64) ? ~uint64_t{0} : ((uint64_t{1} << (d + p)) - 1);
    // Group stripes by erasure pattern (host, O(S)); validate every pattern before any launch.
    std::unordered_map<uint64_t, std::vector<int32_t>> groups;
    for (int s = 0; s < nstripes; ++s) {
        const uint64_t m = need_masks[s];
        if (!m) continue;
        if (m & ~valid) return RS_ERR_ILLEGAL_VECTS;
        groups[m].push_back(s);
    }
    if (groups.empty()) return RS_OK;
    struct Group {
        uint64_t mask;
        ReconstPlan pl;
        size_t off, n;
    };
    std::vector<Group> plan;
    std::vector<int32_t> ids;
    ids.reserve(nstripes);
    for (auto& kv : groups) {
        Group gr;
        gr.mask = kv.first;
        int need[64], nn = 0;
        for (int v = 0; v < d + p; ++v)
            if (kv.first >> v & 1) need[nn++] = v;
        int rc = plan_reconst(rs, nullptr, 0, need, nn, gr.pl.vs, &gr.pl.nvs, gr.pl.nr, &gr.pl.nnr, &gr.pl.dn);
        if (rc) return rc;  // RS_ERR_TOO_MANY_LOST for a pattern beyond p erasures
        gr.off = ids.size();
        gr.n = kv.second.size();
        ids.insert(ids.end(), kv.second.begin(), kv.second.end());
        plan.push_back(gr);
    }
    if (!L->data_base || !L->parity_base) return RS_ERR_INVAL;
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    hipStream_t st = as_stream(stream);

    // Single launch over all stripes when every pattern has <= 4 outputs and
    // the layout takes the 16-byte vector path; otherwise one launch per
    // pattern over a stripe-id list (below).
    bool single = len % 16 == 0 && len < (size_t{1} << 31);
    for (const Group& gr : plan) single = single && gr.pl.nnr <= 4;
    for (int v = 0; v < d + p && single; ++v)
        single = (reinterpret_cast<uintptr_t>(LayoutAddr{L, d}.ptr(v)) & 15) == 0;
    single = single && (L->data_stripe_stride & 15) == 0 && (L->parity_stripe_stride & 15) == 0;
    if (single) {
        const int npat = static_cast<int>(plan.size());
        const int tdw = multi_table_dwords(d);
        const size_t tab_bytes = static_cast<size_t>(npat) * tdw * 4;
        const size_t desc_bytes = static_cast<size_t>(npat) * sizeof(PatternDesc);
        const size_t pat_bytes = static_cast<size_t>(nstripes) * 4;
        int nout_max = 0;
        for (const Group& gr : plan) nout_max = gr.pl.nnr > nout_max ? gr.pl.nnr : nout_max;
        UploadLease lease(rs);
        uint8_t* host = nullptr;
        RS_TRY(lease.acquire(tab_bytes + desc_bytes + pat_bytes, &host));
        std::memset(host, 0, tab_bytes + desc_bytes);
        uint32_t* tabs = reinterpret_cast<uint32_t*>(host);
        PatternDesc* descs = reinterpret_cast<PatternDesc*>(host + tab_bytes);
        int32_t* spat = reinterpret_cast<int32_t*>(host + tab_bytes + desc_bytes);
        for (int s = 0; s < nstripes; ++s) spat[s] = -1;
        for (int gi = 0; gi < npat; ++gi) {
            const Group& gr = plan[gi];
            std::vector<uint8_t> m;
            RS_TRY(combined_matrix(rs, gr.pl.vs, gr.pl.nr, gr.pl.nnr, gr.pl.dn, m));
            uint32_t* img = tabs + static_cast<size_t>(gi) * tdw;
            for (int i = 0; i < d; ++i)
                for (int r = 0; r < gr.pl.nnr; ++r) perm_table(m[static_cast<size_t>(r) * d + i], img + i * 20 + r * 5);
            PatternDesc& pd = descs[gi];
            pd.tab_off = static_cast<uint32_t>(gi * tdw);
            pd.nout = static_cast<uint32_t>(gr.pl.nnr);
            for (int i = 0; i < d; ++i) pd.in_idx[i] = static_cast<uint32_t>(gr.pl.vs[i]);
            for (int r = 0; r < gr.pl.nnr; ++r) pd.out_idx[r] = static_cast<uint32_t>(gr.pl.nr[r]);
            for (size_t t = 0; t < gr.n; ++t) spat[ids[gr.off + t]] = gi;
        }
        uint8_t* dev = nullptr;
        RS_TRY(lease.upload(st, &dev));
        MatmulArgs a;
        std::memset(&a, 0, sizeof a);
        a.tables = reinterpret_cast<const uint32_t*>(dev);
        a.rows = nout_max;
        a.cols = d;
        a.nstripes = nstripes;
        a.len = len;
        a.ss[0] = L->data_stripe_stride;
        a.ss[1] = L->parity_stripe_stride;
        const LayoutAddr A{L, d};
        for (int v = 0; v < d + p; ++v) {
            a.ptr[v] = reinterpret_cast<uint64_t>(A.ptr(v));
            a.sid[v] = A.sid(v);
        }
        return launch_gf_multi(a, reinterpret_cast<const PatternDesc*>(dev + tab_bytes),
                               reinterpret_cast<const int32_t*>(dev + tab_bytes + desc_bytes), st) == hipSuccess
                   ? RS_OK
                   : RS_ERR_DEVICE;
    }

    UploadLease lease(rs);
    uint8_t* hids = nullptr;
    RS_TRY(lease.acquire(ids.size() * sizeof(int32_t), &hids));
    std::memcpy(hids, ids.data(), ids.size() * sizeof(int32_t));
    uint8_t* dev_ids = nullptr;
    RS_TRY(lease.upload(st, &dev_ids));
    const int32_t* dids = reinterpret_cast<const int32_t*>(dev_ids);
    int rc = RS_OK;
    const LayoutAddr A{L, d};
    const int64_t ss[4] = {L->data_stripe_stride, L->parity_stripe_stride, 0, 0};
    const uint8_t* in[kMaxVects];
    uint8_t* out[kMaxVects];
    uint8_t isid[kMaxVects], osid[kMaxVects];
    for (const Group& gr : plan) {  // one launch per distinct pattern (combined_matrix)
        if (rc) break;
        const ReconstPlan& pl = gr.pl;
        std::vector<uint8_t> m;
        rc = combined_matrix(rs, pl.vs, pl.nr, pl.nnr, pl.dn, m);
        if (rc) break;
        for (int i = 0; i < d; ++i) {
            in[i] = A.ptr(pl.vs[i]);
            isid[i] = A.sid(pl.vs[i]);
        }
        for (int i = 0; i < pl.nnr; ++i) {
            out[i] = A.ptr(pl.nr[i]);
            osid[i] = A.sid(pl.nr[i]);
        }
        rc = matmul_ex(rs, m.data(), pl.nnr, d, in, isid, out, osid, ss, static_cast<int>(gr.n), len, false, st,
                       dids + gr.off);
    }
    return rc;
}

// ---------------------------------------------------------------- Update

int rs_update(rs_t* rs, const uint8_t* old_data, size_t old_len, const uint8_t* new_data, size_t new_len, int row,
              uint8_t* const* parity, const size_t* parity_lens, int np) {
    if (!rs || (np > 0 && (!parity || !parity_lens))) return RS_ERR_INVAL;
    RS_TRY(check_update(rs, old_len, new_len, row, parity_lens, np));
    if (!old_data || !new_data) return RS_ERR_INVAL;
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    std::lock_guard<std::mutex> lk(rs->stage_mu);
    const uint8_t* src[2] = {old_data, new_data};
    std::vector<uint8_t> gm = update_matrix(rs, row);
    return host_product(rs, gm.data(), rs->p, 2, src, parity, new_len, true);
}

int rs_update_dev(rs_t* rs, const uint8_t* old_data, size_t old_len, const uint8_t* new_data, size_t new_len, int row,
                  uint8_t* const* parity, const size_t* parity_lens, int np, void* stream) {
    if (!rs || (np > 0 && (!parity || !parity_lens))) return RS_ERR_INVAL;
    RS_TRY(check_update(rs, old_len, new_len, row, parity_lens, np));
    if (!old_data || !new_data) return RS_ERR_INVAL;
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    const uint8_t* in[2] = {old_data, new_data};
    std::vector<uint8_t> gm = update_matrix(rs, row);
    return matmul(rs, gm.data(), rs->p, 2, in, 0, parity, 0, 1, new_len, true, as_stream(stream));
}

int rs_update_batch(rs_t* rs, const uint8_t* old_base, int64_t old_stride, const uint8_t* new_base,
                    int64_t new_stride, int row, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                    int nstripes, size_t len, void* stream) {
    if (!rs || nstripes < 0) return RS_ERR_INVAL;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    if (row >= rs->d || row < 0) return RS_ERR_ILLEGAL_VECT_INDEX;
    if (nstripes == 0) return RS_OK;
    if (!old_base || !new_base || !base) return RS_ERR_INVAL;
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    const uint8_t* in[2] = {old_base, new_base};
    const uint8_t isid[2] = {0, 1};
    uint8_t* out[kMaxVects];
    uint8_t osid[kMaxVects];
    for (int j = 0; j < rs->p; ++j) {
        out[j] = base + (rs->d + j) * vect_stride;
        osid[j] = 2;
    }
    const int64_t ss[4] = {old_stride, new_stride, stripe_stride, 0};
    std::vector<uint8_t> gm = update_matrix(rs, row);
    return matmul_ex(rs, gm.data(), rs->p, 2, in, isid, out, osid, ss, nstripes, len, true, as_stream(stream));
}

// ---------------------------------------------------------------- Replace

int rs_replace(rs_t* rs, const uint8_t* const* data, const size_t* data_lens, int nd, const int* replace_rows, int nr,
               uint8_t* const* parity, const size_t* parity_lens, int np) {
    if (!rs || (nd > 0 && (!data || !data_lens)) || (nr > 0 && !replace_rows) ||
        (np > 0 && (!parity || !parity_lens)))
        return RS_ERR_INVAL;
    RS_TRY(check_replace(rs, data_lens, nd, replace_rows, nr, parity_lens, np));
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    std::lock_guard<std::mutex> lk(rs->stage_mu);
    std::vector<uint8_t> gm = replace_matrix(rs, replace_rows, nr);
    return host_product(rs, gm.data(), rs->p, nr, data, parity, data_lens[0], true);
}

int rs_replace_dev(rs_t* rs, const uint8_t* const* data, const size_t* data_lens, int nd, const int* replace_rows,
                   int nr, uint8_t* const* parity, const size_t* parity_lens, int np, void* stream) {
    if (!rs || (nd > 0 && (!data || !data_lens)) || (nr > 0 && !replace_rows) ||
        (np > 0 && (!parity || !parity_lens)))
        return RS_ERR_INVAL;
    RS_TRY(check_replace(rs, data_lens, nd, replace_rows, nr, parity_lens, np));
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    std::vector<uint8_t> gm = replace_matrix(rs, replace_rows, nr);
    return matmul(rs, gm.data(), rs->p, nr, data, 0, parity, 0, 1, data_lens[0], true, as_stream(stream));
}

int rs_replace_batch(rs_t* rs, const uint8_t* data_base, int64_t data_stripe_stride, int64_t data_vect_stride,
                     const int* replace_rows, int nr, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                     int nstripes, size_t len, void* stream) {
    if (!rs || nstripes < 0 || (nr > 0 && !replace_rows)) return RS_ERR_INVAL;
    if (nr > rs->d) return RS_ERR_TOO_MANY_REPLACE;
    if (nr <= 0) return RS_ERR_INVAL;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    for (int i = 0; i < nr; ++i)
        if (replace_rows[i] >= rs->d || replace_rows[i] < 0) return RS_ERR_ILLEGAL_VECT_INDEX;
    if (nstripes == 0) return RS_OK;
    if (!data_base || !base) return RS_ERR_INVAL;
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    const uint8_t* in[kMaxVects];
    uint8_t* out[kMaxVects];
    for (int i = 0; i < nr; ++i) in[i] = data_base + i * data_vect_stride;
    for (int j = 0; j < rs->p; ++j) out[j] = base + (rs->d + j) * vect_stride;
    std::vector<uint8_t> gm = replace_matrix(rs, replace_rows, nr);
    return matmul(rs, gm.data(), rs->p, nr, in, data_stripe_stride, out, stripe_stride, nstripes, len, true,
                  as_stream(stream));
}

// ---------------------------------------------------------------- host-resident pipeline

int rs_host_register(void* ptr, size_t bytes) {
    if (!ptr || !bytes) return RS_ERR_INVAL;
    // mapped: kernels may address it directly (zero-copy host batches)
    return hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable) == hipSuccess
               ? RS_OK
               : RS_ERR_DEVICE;
}

int rs_host_device_pointer(const void* host_ptr, size_t bytes, void** dev_ptr) {
    if (!host_ptr || !bytes || !dev_ptr) return RS_ERR_INVAL;
    *dev_ptr = nullptr;
    uint8_t* d = nullptr;
    RS_TRY(host_device_range(host_ptr, bytes, &d));
    *dev_ptr = d;
    return RS_OK;
}

int rs_host_unregister(void* ptr) {
    if (!ptr) return RS_ERR_INVAL;
    return hipHostUnregister(ptr) == hipSuccess ? RS_OK : RS_ERR_DEVICE;
}

// Host-resident encode: a three-stage pipeline over a ring of `streams`
// device slots.  H2D copies run on one stream, kernels on a second, D2H on a
// third, linked by events, so the copy engines of both PCIe directions and
// the CUs work on different chunks at the same time:
//     h2d:  [wait slot free] copy data(c)  -> ev_in[slot]
//     comp: [wait ev_in]     encode(c)     -> ev_enc[slot]
//     d2h:  [wait ev_enc]    copy parity(c)-> ev_free[slot]
int rs_encode_host_batch(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride, int nstripes,
                         size_t len, int stripes_per_chunk, int streams) {
    if (!rs || nstripes < 0 || (nstripes > 0 && !base)) return RS_ERR_INVAL;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    if (nstripes == 0) return RS_OK;
    if (stripes_per_chunk <= 0) stripes_per_chunk = 8;
    int slots = streams <= 0 ? 3 : std::min(streams, 8);
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    const int d = rs->d, p = rs->p;
    uint8_t* zc = nullptr;
    if (g_host_batch_zc && stripe_stride >= 0 && vect_stride >= 0 &&
        host_device_range(base, batch_extent(stripe_stride, vect_stride, nstripes, d + p, len), &zc) == RS_OK) {
        // pinned / registered caller memory: one launch straight over it
        std::lock_guard<std::mutex> lk(rs->stage_mu);
        if (!rs->stream && hipStreamCreateWithFlags(&rs->stream, hipStreamNonBlocking) != hipSuccess)
            return RS_ERR_DEVICE;
        const uint8_t* in[kMaxVects];
        uint8_t* out[kMaxVects];
        for (int i = 0; i < d; ++i) in[i] = zc + i * vect_stride;
        for (int j = 0; j < p; ++j) out[j] = zc + (d + j) * vect_stride;
        int rc = matmul(rs, rs->gen(), p, d, in, stripe_stride, out, stripe_stride, nstripes, len, false,
                        rs->stream);
        if (hipStreamSynchronize(rs->stream) != hipSuccess && rc == RS_OK) rc = RS_ERR_DEVICE;
        return rc;
    }
    // [S][d+p][len] with 256-B-multiple len: data and parity of a stripe are contiguous rows
    const bool dense = vect_stride == static_cast<int64_t>(len) && len % 256 == 0;
    const size_t pitch = dense ? len : rup(len, 256);
    const int64_t dstripe = static_cast<int64_t>(pitch) * (d + p);
    const size_t slot_bytes = static_cast<size_t>(dstripe) * stripes_per_chunk;
    std::lock_guard<std::mutex> lk(rs->stage_mu);
    uint8_t* ring = nullptr;
    if (hipMalloc(&ring, slot_bytes * slots) != hipSuccess) return RS_ERR_DEVICE;
    hipStream_t sh = nullptr, sc = nullptr, sd = nullptr;
    std::vector<hipEvent_t> ev_in(slots), ev_enc(slots), ev_free(slots);
    int rc = RS_OK;
    if (hipStreamCreateWithFlags(&sh, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&sc, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&sd, hipStreamNonBlocking) != hipSuccess)
        rc = RS_ERR_DEVICE;
    for (int i = 0; i < slots && rc == RS_OK; ++i)
        if (hipEventCreateWithFlags(&ev_in[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ev_enc[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ev_free[i], hipEventDisableTiming) != hipSuccess)
            rc = RS_ERR_DEVICE;
    auto ok = [&](hipError_t e) {
        if (e != hipSuccess && rc == RS_OK) rc = RS_ERR_DEVICE;
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
        if (dense) {  // one 2-D copy: cn rows of d*len bytes
            if (!ok(hipMemcpy2DAsync(dev, dstripe, hb, stripe_stride, static_cast<size_t>(d) * len, cn,
                                     hipMemcpyHostToDevice, sh)))
                break;
        } else {
            for (int i = 0; i < d; ++i)
                if (!ok(hipMemcpy2DAsync(dev + i * pitch, dstripe, hb + i * vect_stride, stripe_stride, len, cn,
                                         hipMemcpyHostToDevice, sh)))
                    break;
        }
        if (!ok(hipEventRecord(ev_in[slot], sh)) || !ok(hipStreamWaitEvent(sc, ev_in[slot], 0))) break;
        for (int i = 0; i < d; ++i) in[i] = dev + i * pitch;
        for (int j = 0; j < p; ++j) out[j] = dev + (d + j) * pitch;
        rc = matmul(rs, rs->gen(), p, d, in, dstripe, out, dstripe, cn, len, false, sc);
        if (rc) break;
        if (!ok(hipEventRecord(ev_enc[slot], sc)) || !ok(hipStreamWaitEvent(sd, ev_enc[slot], 0))) break;
        if (dense) {
            if (!ok(hipMemcpy2DAsync(hb + d * vect_stride, stripe_stride, dev + d * pitch, dstripe,
                                     static_cast<size_t>(p) * len, cn, hipMemcpyDeviceToHost, sd)))
                break;
        } else {
            for (int j = 0; j < p; ++j)
                if (!ok(hipMemcpy2DAsync(hb + (d + j) * vect_stride, stripe_stride, dev + (d + j) * pitch, dstripe,
                                         len, cn, hipMemcpyDeviceToHost, sd)))
                    break;
        }
        if (!ok(hipEventRecord(ev_free[slot], sd))) break;
    }
    for (hipStream_t s : {sh, sc, sd})
        if (s) {
            if (hipStreamSynchronize(s) != hipSuccess) rc = RS_ERR_DEVICE;
            (void)hipStreamDestroy(s);
        }
    for (int i = 0; i < slots; ++i)
        for (hipEvent_t e : {ev_in[i], ev_enc[i], ev_free[i]})
            if (e) (void)hipEventDestroy(e);
    (void)hipFree(ring);
    return rc;
}

// ---------------------------------------------------------------- device groups

struct rs_group {
    std::vector<rs_t*> members;
};

int rs_group_new(int data_num, int parity_num, const int* devices, int ndev, rs_group_t** out) {
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
}

void rs_group_free(rs_group_t* g) {
    if (!g) return;
    for (rs_t* r : g->members) rs_free(r);
    delete g;
}

int rs_group_size(const rs_group_t* g) { return g ? static_cast<int>(g->members.size()) : 0; }

rs_t* rs_group_codec(rs_group_t* g, int i) {
    return g && i >= 0 && i < static_cast<int>(g->members.size()) ? g->members[i] : nullptr;
}

int rs_group_encode_host_batch(rs_group_t* g, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                               int nstripes, size_t len, int stripes_per_chunk, int streams) {
    if (!g || g->members.empty() || nstripes < 0 || (nstripes > 0 && !base)) return RS_ERR_INVAL;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    const int n = static_cast<int>(g->members.size());
    std::vector<int> rc(n, RS_OK);
    std::vector<std::thread> th;
    for (int i = 0; i < n; ++i) {
        const int lo = static_cast<int>(static_cast<int64_t>(nstripes) * i / n);
        const int hi = static_cast<int>(static_cast<int64_t>(nstripes) * (i + 1) / n);
        if (hi <= lo) continue;
        auto job = [&, i, lo, hi] {
            rc[i] = rs_encode_host_batch(g->members[i], base + static_cast<int64_t>(lo) * stripe_stride,
                                         stripe_stride, vect_stride, hi - lo, len, stripes_per_chunk, streams);
        };
        try {
            th.emplace_back(job);
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
    if (!rs || nstripes < 0 || (nstripes > 0 && (!base || !need_masks))) return RS_ERR_INVAL;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    if (nstripes == 0) return RS_OK;
    if (stripe_stride < 0 || vect_stride < 0) return RS_ERR_INVAL;
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    const int d = rs->d, p = rs->p;
    uint8_t* zc = nullptr;
    RS_TRY(host_device_range(base, batch_extent(stripe_stride, vect_stride, nstripes, d + p, len), &zc));
    rs_layout_t L{zc, stripe_stride, vect_stride, zc + static_cast<int64_t>(d) * vect_stride, stripe_stride,
                  vect_stride};
    std::lock_guard<std::mutex> lk(rs->stage_mu);
    if (!rs->stream && hipStreamCreateWithFlags(&rs->stream, hipStreamNonBlocking) != hipSuccess)
        return RS_ERR_DEVICE;
    int rc = rs_reconst_batch_multi(rs, &L, nstripes, len, need_masks, rs->stream);
    if (hipStreamSynchronize(rs->stream) != hipSuccess && rc == RS_OK) rc = RS_ERR_DEVICE;
    return rc;
}

int rs_group_reconst_host_batch_multi(rs_group_t* g, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                                      int nstripes, size_t len, const uint64_t* need_masks) {
    if (!g || g->members.empty() || nstripes < 0 || (nstripes > 0 && (!base || !need_masks))) return RS_ERR_INVAL;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    const int n = static_cast<int>(g->members.size());
    std::vector<int> rc(n, RS_OK);
    std::vector<std::thread> th;
    for (int i = 0; i < n; ++i) {
        const int lo = static_cast<int>(static_cast<int64_t>(nstripes) * i / n);
        const int hi = static_cast<int>(static_cast<int64_t>(nstripes) * (i + 1) / n);
        if (hi <= lo) continue;
        auto job = [&, i, lo, hi] {
            rc[i] = rs_reconst_host_batch_multi(g->members[i], base + static_cast<int64_t>(lo) * stripe_stride,
                                                stripe_stride, vect_stride, hi - lo, len, need_masks + lo);
        };
        try {
            th.emplace_back(job);
        } catch (...) {
            job();
        }
    }
    for (std::thread& t : th) t.join();
    for (int r : rc)
        if (r) return r;
    return RS_OK;
}

// ---------------------------------------------------------------- XOR primitive

int rs_xor_batch(rs_t* rs, const uint8_t* src_base, int64_t src_stripe_stride, int64_t src_vect_stride, int nsrc,
                 uint8_t* dst_base, int64_t dst_stripe_stride, int nstripes, size_t len, void* stream) {
    if (!rs || nsrc <= 0 || nsrc + 1 > kMaxPtrs || nstripes < 0) return RS_ERR_INVAL;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    if (nstripes == 0) return RS_OK;
    if (!src_base || !dst_base) return RS_ERR_INVAL;
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    std::vector<uint8_t> ones(static_cast<size_t>(nsrc), 1);
    const uint8_t* in[kMaxPtrs];
    for (int c = 0; c < nsrc; ++c) in[c] = src_base + c * src_vect_stride;
    uint8_t* out[1] = {dst_base};
    return matmul(rs, ones.data(), 1, nsrc, in, src_stripe_stride, out, dst_stripe_stride, nstripes, len, false,
                  as_stream(stream));
}

// ---------------------------------------------------------------- generic product

int rs_gf_matmul_batch(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* in_base,
                       int64_t in_stripe_stride, int64_t in_vect_stride, const int* in_map, uint8_t* out_base,
                       int64_t out_stripe_stride, int64_t out_vect_stride, const int* out_map, int nstripes,
                       size_t len, int accumulate, void* stream) {
    if (!rs || !mat || rows <= 0 || cols <= 0 || rows + cols > kMaxPtrs || nstripes < 0) return RS_ERR_INVAL;
    if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
    if (nstripes == 0) return RS_OK;
    if (!in_base || !out_base) return RS_ERR_INVAL;
    RS_TRY(ensure_device(rs));
    DeviceGuard g(rs->device);
    const uint8_t* in[kMaxPtrs];
    uint8_t* out[kMaxPtrs];
    for (int c = 0; c < cols; ++c) in[c] = in_base + (in_map ? in_map[c] : c) * in_vect_stride;
    for (int r = 0; r < rows; ++r) out[r] = out_base + (out_map ? out_map[r] : r) * out_vect_stride;
    return matmul(rs, mat, rows, cols, in, in_stripe_stride, out, out_stripe_stride, nstripes, len, accumulate != 0,
                  as_stream(stream));
}

}  // extern "C"
