// batches.cpp — device-resident calls: one stripe on caller device pointers
// (rs_*_dev), batches of stripes under a layout (rs_*_batch*), a different
// erasure pattern per stripe (rs_reconst_batch_multi), the XOR primitive and
// the generic product.  All asynchronous on the caller's stream.
#include <algorithm>
#include <array>

#include "codec_internal.hpp"

using namespace rsamd;
using namespace rsamd::detail;

extern "C" {

int rs_encode_dev(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n, void* stream) {
    return abi_guard([&]() -> int {
        if (!rs || (n > 0 && (!vects || !lens))) return RS_ERR_INVAL;
        RS_TRY(check_encode(rs, lens, n));
        RS_TRY(ensure_device(rs));
        DeviceGuard g(rs->device);
        return matmul(rs, rs->gen(), rs->p, rs->d, vects, 0, vects + rs->d, 0, 1, lens[0], false, as_stream(stream));
    });
}

int rs_encode_batch_layout(rs_t* rs, const rs_layout_t* L, int nstripes, size_t len, void* stream) {
    return abi_guard([&]() -> int {
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
    });
}

int rs_encode_batch(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride, int nstripes, size_t len,
                    void* stream) {
    return abi_guard([&]() -> int {
        if (!rs || nstripes < 0 || (nstripes > 0 && !base)) return RS_ERR_INVAL;
        const rs_layout_t L{base, stripe_stride, vect_stride, base + rs->d * vect_stride, stripe_stride, vect_stride};
        return rs_encode_batch_layout(rs, &L, nstripes, len, stream);
    });
}

int rs_reconst_dev(rs_t* rs, uint8_t* const* vects, const size_t* lens, int n, const int* survived, int ns,
                   const int* need, int nn, void* stream) {
    return abi_guard([&]() -> int {
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
    });
}

int rs_reconst_batch_layout(rs_t* rs, const rs_layout_t* L, int nstripes, size_t len, const int* survived, int ns,
                            const int* need, int nn, void* stream) {
    return abi_guard([&]() -> int {
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
    });
}

int rs_reconst_batch(rs_t* rs, uint8_t* base, int64_t stripe_stride, int64_t vect_stride, int nstripes, size_t len,
                     const int* survived, int ns, const int* need, int nn, void* stream) {
    return abi_guard([&]() -> int {
        if (!rs || nstripes < 0 || (nstripes > 0 && !base)) return RS_ERR_INVAL;
        const rs_layout_t L{base, stripe_stride, vect_stride, base + rs->d * vect_stride, stripe_stride, vect_stride};
        return rs_reconst_batch_layout(rs, &L, nstripes, len, survived, ns, need, nn, stream);
    });
}

}  // extern "C"

namespace {

// Group stripes by erasure pattern (host, O(S)): pat_of[s] = the pattern
// index of stripe s (-1 for a zero mask); keyw holds each pattern's W mask
// words in first-seen order (npat x W, the layout the GPU planner reads),
// counts its stripes.  Batches hold few distinct patterns, often in runs: the
// previous stripe's pattern, then a linear scan while there are at most kScan
// patterns, then an open-addressing hash of pattern indexes holding every
// pattern.  W is the mask width in words (1 or 4), so the common one-word
// masks compare and hash as one integer (a node-based map cost ~150 ns per new
// pattern, 4-word keys with a 16-key scan ahead of the hash ~80, and copying
// 4,096 patterns out as 32-byte keys took a fresh mmap'ed block and its page
// faults on every call: most of a many-pattern call once the GPU plans the
// patterns).  Returns RS_ERR_ILLEGAL_VECTS for a bit at or above nvec.
template <int W>
int group_patterns(const uint64_t* m, int nstripes, int nvec, std::vector<int32_t>& pat_of, std::vector<uint64_t>& keyw,
                   std::vector<size_t>& counts) {
    typedef std::array<uint64_t, W> Key;
    auto hash = [](const Key& k) {
        uint64_t h = 0x9E3779B97F4A7C15ull;
        for (uint64_t w : k) h = (h ^ w) * 0xBF58476D1CE4E5B9ull;
        // a product's low bits see only the low bits of its input: fold the
        // high half down twice so a code's top vectors (bits 32-63 for 32+32)
        // reach the slot index too
        h = (h ^ (h >> 32)) * 0x94D049BB133111EBull;
        return static_cast<size_t>(h ^ (h >> 32));
    };
    uint64_t top[W];  // bits a stripe may set, per word
    for (int w = 0; w < W; ++w) {
        const int lo = w * 64;
        top[w] = nvec >= lo + 64 ? ~uint64_t{0} : nvec <= lo ? 0 : (uint64_t{1} << (nvec - lo)) - 1;
    }
    auto key_at = [&](size_t k) {
        Key r;
        for (int w = 0; w < W; ++w) r[w] = keyw[k * W + w];
        return r;
    };
    std::vector<int32_t> slots;  // pattern index per hash slot, -1 = empty (power-of-two size)
    auto slot_of = [&](const Key& key) -> size_t {  // the key's slot, or the empty one it would take
        size_t h = hash(key) & (slots.size() - 1);
        while (slots[h] >= 0 && key_at(static_cast<size_t>(slots[h])) != key) h = (h + 1) & (slots.size() - 1);
        return h;
    };
    auto rehash = [&](size_t size) {  // every pattern into a table of `size` slots
        slots.assign(size, -1);
        for (size_t k = 0; k < counts.size(); ++k) slots[slot_of(key_at(k))] = static_cast<int32_t>(k);
    };
    constexpr int kScan = 16;
    int last = -1;
    for (int s = 0; s < nstripes; ++s) {
        Key key;
        uint64_t any = 0, bad = 0;
        for (int w = 0; w < W; ++w) {
            key[w] = m[static_cast<size_t>(s) * W + w];
            any |= key[w];
            bad |= key[w] & ~top[w];
        }
        if (!any) continue;
        if (bad) return RS_ERR_ILLEGAL_VECTS;
        int gi = -1;
        if (last >= 0 && key_at(static_cast<size_t>(last)) == key) {
            gi = last;
        } else {
            const int n = static_cast<int>(counts.size());
            size_t h = 0;
            if (slots.empty()) {
                for (int k = 0; k < n && gi < 0; ++k)
                    if (key_at(static_cast<size_t>(k)) == key) gi = k;
            } else {
                h = slot_of(key);
                gi = slots[h];
            }
            if (gi < 0) {
                gi = n;
                for (int w = 0; w < W; ++w) keyw.push_back(key[w]);
                counts.push_back(0);
                if (!slots.empty() && 2 * (n + 1) <= static_cast<int>(slots.size()))
                    slots[h] = gi;
                else if (n + 1 >= kScan)  // build at kScan patterns, then double at load 1/2
                    rehash(slots.empty() ? 256 : slots.size() * 2);
            }
        }
        pat_of[static_cast<size_t>(s)] = gi;
        ++counts[static_cast<size_t>(gi)];
        last = gi;
    }
    return RS_OK;
}
}  // namespace

namespace rsamd {
namespace detail {

// rs_reconst_batch_multi / rs_reconst_batch_multi256 (masks of 1 or 4 words).
int reconst_multi(rs_t* rs, const rs_layout_t* L, int nstripes, size_t len, MaskView masks, void* stream) {
    {
        if (!rs || !L || nstripes < 0 || (nstripes > 0 && !masks.m)) return RS_ERR_INVAL;
        const int d = rs->d, p = rs->p;
        if (d + p > 64 * masks.words) return RS_ERR_INVAL;  // the mask cannot name every vector
        if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
        // Group stripes by erasure pattern and validate every pattern before
        // any launch (group_patterns above).
        std::vector<int32_t> pat_of(static_cast<size_t>(nstripes), -1);
        std::vector<uint64_t> keyw;  // npat x masks.words
        std::vector<size_t> counts;
        const int rc_g = masks.words == 1 ? group_patterns<1>(masks.m, nstripes, d + p, pat_of, keyw, counts)
                                          : group_patterns<4>(masks.m, nstripes, d + p, pat_of, keyw, counts);
        if (rc_g) return rc_g;
        const size_t npat_all = counts.size();
        auto key_word = [&](size_t gi, int w) { return keyw[gi * static_cast<size_t>(masks.words) + w]; };
        if (npat_all == 0) return RS_OK;
        // Every pattern's plan_reconst error before any device work: with no
        // survivor list the needed vectors are the mask's, and more than p of
        // them is RS_ERR_TOO_MANY_LOST (nothing else can fail there).
        int nn_max = 0;
        for (size_t gi = 0; gi < npat_all; ++gi) {
            int nn = 0;
            for (int w = 0; w < masks.words; ++w) nn += __builtin_popcountll(key_word(gi, w));
            if (nn > p) return RS_ERR_TOO_MANY_LOST;
            nn_max = nn > nn_max ? nn : nn_max;
        }
        if (!L->data_base || !L->parity_base) return RS_ERR_INVAL;
        RS_TRY(ensure_device(rs));
        DeviceGuard g(rs->device);
        hipStream_t st = as_stream(stream);

        // Single launch over all stripes when every pattern has <= 8 outputs and
        // the layout takes the 16-byte vector path; otherwise one launch per
        // pattern over a stripe-id list (below).
        bool single = nn_max <= kMultiMaxOut && len % 16 == 0 && len < (size_t{1} << 31) &&
                      (len / 1024 + 1) * static_cast<uint64_t>(nstripes) < (uint64_t{1} << 31);  // grid < 2^31 chunks
        for (int v = 0; v < d + p && single; ++v)
            single = (reinterpret_cast<uintptr_t>(LayoutAddr{L, d}.ptr(v)) & 15) == 0;
        single = single && (L->data_stripe_stride & 15) == 0 && (L->parity_stripe_stride & 15) == 0;
        // (the GPU planner costs ~6 us more than the host's for a handful of
        // patterns and less from ~16 patterns at d = 10, ~8 at 20, ~5 at 32:
        // profiles/r05/multi_planner_small_counts.log)
        // the one launch over every stripe, from the tables / descriptors /
        // stripe -> pattern map in device memory (a.rows: the most outputs)
        auto launch_single = [&](const uint32_t* tabs, const PatternDesc* descs, const int32_t* spat) {
            MatmulArgs a;
            std::memset(&a, 0, sizeof a);
            a.tables = tabs;
            a.rows = nn_max;
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
            return hip_ok(launch_gf_multi(a, descs, spat, st), "multi-pattern kernel launch");
        };
        const int gpu_plan = tuning().multi_gpu_plan;
        const bool use_gpu_plan = gpu_plan < 0 ? npat_all * static_cast<size_t>(d) >= 160
                                               : gpu_plan > 0 && npat_all >= static_cast<size_t>(gpu_plan);
        if (single && use_gpu_plan) {
            // Plan on the GPU (gf_plan_multi, kernels.hip): the distinct masks
            // and the stripe -> pattern map go into a mapped pinned buffer the
            // planner reads in place (no copy, no cross-stream wait: those
            // cost ~24 us of a 75 us call); the field tables are device
            // constants, and the parity rows are Cauchy, so the planner derives
            // every entry it needs.  It copies the map into the device slot and
            // writes the table images and descriptors behind it, then the
            // multi kernel runs.
            const int npat = static_cast<int>(npat_all);
            const int tdw = multi_table_dwords(d, nn_max);
            auto al16 = [](size_t x) { return (x + 15) & ~size_t{15}; };
            const size_t mask_b = al16(static_cast<size_t>(npat) * masks.words * 8);
            const size_t pat_b = al16(static_cast<size_t>(nstripes) * 4);
            const size_t tab_b = static_cast<size_t>(npat) * tdw * 4;
            const size_t desc_b = static_cast<size_t>(npat) * sizeof(PatternDesc);
            UploadLease lease(rs);
            uint8_t* host = nullptr;
            RS_TRY(lease.acquire(mask_b + pat_b, &host, pat_b + tab_b + desc_b));
            // (a pinned slot without a device address cannot be read in
            // place: the host planner below serves the call instead, advisor r05)
            if (lease.mappable()) {
                std::memcpy(host, keyw.data(), keyw.size() * sizeof(uint64_t));  // (npat x words, as grouped)
                std::memcpy(host + mask_b, pat_of.data(), static_cast<size_t>(nstripes) * 4);
                const uint8_t* hdev = nullptr;
                uint8_t* dev = nullptr;
                RS_TRY(lease.map(st, &hdev, &dev));
                PlanArgs pa;
                pa.masks = reinterpret_cast<const uint64_t*>(hdev);
                pa.pat_src = reinterpret_cast<const int32_t*>(hdev + mask_b);
                pa.pat_dst = reinterpret_cast<int32_t*>(dev);
                pa.tabs = reinterpret_cast<uint32_t*>(dev + pat_b);
                pa.descs = reinterpret_cast<PatternDesc*>(dev + pat_b + tab_b);
                pa.npat = npat;
                pa.words = masks.words;
                pa.d = d;
                pa.p = p;
                pa.tdw = tdw;
                pa.nstripes = nstripes;
                pa.img_rows = multi_image_rows(nn_max);
                RS_TRY(hip_ok(launch_gf_plan_multi(pa, st), "multi-pattern planner launch"));
                return launch_single(pa.tabs, pa.descs, pa.pat_dst);
            }
        }
        struct Group {
            ReconstPlan pl;
            size_t off, n;
        };
        std::vector<Group> plan;
        plan.reserve(npat_all);
        size_t off = 0;
        for (size_t gi = 0; gi < npat_all; ++gi) {
            Group gr;
            int need[kMaxVects], nn = 0;
            for (int v = 0; v < d + p; ++v)
                if (key_word(gi, v >> 6) >> (v & 63) & 1) need[nn++] = v;
            int rc = plan_reconst(rs, nullptr, 0, need, nn, gr.pl.vs, &gr.pl.nvs, gr.pl.nr, &gr.pl.nnr, &gr.pl.dn);
            if (rc) return rc;  // (validated above)
            gr.off = off;
            gr.n = counts[gi];
            off += gr.n;
            plan.push_back(gr);
        }
        if (single) {
            const int npat = static_cast<int>(plan.size());
            const int tdw = multi_table_dwords(d, nn_max);
            const int cw = multi_image_rows(nn_max) * 5;
            const size_t tab_bytes = static_cast<size_t>(npat) * tdw * 4;
            const size_t desc_bytes = static_cast<size_t>(npat) * sizeof(PatternDesc);
            const size_t pat_bytes = static_cast<size_t>(nstripes) * 4;
            UploadLease lease(rs);
            uint8_t* host = nullptr;
            RS_TRY(lease.acquire(tab_bytes + desc_bytes + pat_bytes, &host));
            std::memset(host, 0, tab_bytes + desc_bytes);
            uint32_t* tabs = reinterpret_cast<uint32_t*>(host);
            PatternDesc* descs = reinterpret_cast<PatternDesc*>(host + tab_bytes);
            int32_t* spat = reinterpret_cast<int32_t*>(host + tab_bytes + desc_bytes);
            std::memcpy(spat, pat_of.data(), pat_bytes);
            for (int gi = 0; gi < npat; ++gi) {
                const Group& gr = plan[gi];
                std::vector<uint8_t> m;
                RS_TRY(combined_matrix(rs, gr.pl.vs, gr.pl.nr, gr.pl.nnr, gr.pl.dn, m));
                uint32_t* img = tabs + static_cast<size_t>(gi) * tdw;
                for (int i = 0; i < d; ++i)
                    for (int r = 0; r < gr.pl.nnr; ++r) perm_table(m[static_cast<size_t>(r) * d + i], img + i * cw + r * 5);
                PatternDesc& pd = descs[gi];
                pd.tab_off = static_cast<uint32_t>(gi * tdw);
                pd.nout = static_cast<uint32_t>(gr.pl.nnr);
                for (int i = 0; i < d; ++i) pd.in_idx[i] = static_cast<uint16_t>(gr.pl.vs[i]);
                for (int r = 0; r < gr.pl.nnr; ++r) pd.out_idx[r] = static_cast<uint32_t>(gr.pl.nr[r]);
            }
            uint8_t* dev = nullptr;
            RS_TRY(lease.upload(st, &dev));
            return launch_single(reinterpret_cast<const uint32_t*>(dev), reinterpret_cast<const PatternDesc*>(dev + tab_bytes),
                                 reinterpret_cast<const int32_t*>(dev + tab_bytes + desc_bytes));
        }

        // stripe ids grouped by pattern, in stripe order within a pattern
        UploadLease lease(rs);
        uint8_t* hids = nullptr;
        RS_TRY(lease.acquire(off * sizeof(int32_t), &hids));
        {
            int32_t* ids = reinterpret_cast<int32_t*>(hids);
            std::vector<size_t> next(plan.size());
            for (size_t gi = 0; gi < plan.size(); ++gi) next[gi] = plan[gi].off;
            for (int s = 0; s < nstripes; ++s)
                if (pat_of[s] >= 0) ids[next[pat_of[s]]++] = s;
        }
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
}

}  // namespace detail
}  // namespace rsamd

extern "C" {

int rs_reconst_batch_multi(rs_t* rs, const rs_layout_t* L, int nstripes, size_t len, const uint64_t* need_masks,
                           void* stream) {
    return abi_guard([&]() -> int { return reconst_multi(rs, L, nstripes, len, MaskView{need_masks, 1}, stream); });
}

int rs_reconst_batch_multi256(rs_t* rs, const rs_layout_t* L, int nstripes, size_t len, const uint64_t* need_masks,
                              void* stream) {
    return abi_guard([&]() -> int { return reconst_multi(rs, L, nstripes, len, MaskView{need_masks, 4}, stream); });
}

int rs_update_dev(rs_t* rs, const uint8_t* old_data, size_t old_len, const uint8_t* new_data, size_t new_len, int row,
                  uint8_t* const* parity, const size_t* parity_lens, int np, void* stream) {
    return abi_guard([&]() -> int {
        if (!rs || (np > 0 && (!parity || !parity_lens))) return RS_ERR_INVAL;
        RS_TRY(check_update(rs, old_len, new_len, row, parity_lens, np));
        if (!old_data || !new_data) return RS_ERR_INVAL;
        RS_TRY(ensure_device(rs));
        DeviceGuard g(rs->device);
        std::vector<uint8_t> gm = update_matrix(rs, row);
        return update_ranges(rs, new_len, [&](uint64_t off, uint64_t n) {
            const uint8_t* in[2] = {old_data + off, new_data + off};
            uint8_t* out[kMaxVects];
            for (int j = 0; j < rs->p; ++j) out[j] = parity[j] + off;
            return matmul(rs, gm.data(), rs->p, 2, in, 0, out, 0, 1, n, true, as_stream(stream));
        });
    });
}

int rs_update_batch(rs_t* rs, const uint8_t* old_base, int64_t old_stride, const uint8_t* new_base,
                    int64_t new_stride, int row, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                    int nstripes, size_t len, void* stream) {
    return abi_guard([&]() -> int {
        if (!rs || nstripes < 0) return RS_ERR_INVAL;
        if (len == 0) return RS_ERR_ZERO_VECT_SIZE;
        if (row >= rs->d || row < 0) return RS_ERR_ILLEGAL_VECT_INDEX;
        if (nstripes == 0) return RS_OK;
        if (!old_base || !new_base || !base) return RS_ERR_INVAL;
        RS_TRY(ensure_device(rs));
        DeviceGuard g(rs->device);
        const uint8_t isid[2] = {0, 1};
        uint8_t osid[kMaxVects];
        for (int j = 0; j < rs->p; ++j) osid[j] = 2;
        const int64_t ss[4] = {old_stride, new_stride, stripe_stride, 0};
        std::vector<uint8_t> gm = update_matrix(rs, row);
        return update_ranges(rs, len, [&](uint64_t off, uint64_t n) {
            const uint8_t* in[2] = {old_base + off, new_base + off};
            uint8_t* out[kMaxVects];
            for (int j = 0; j < rs->p; ++j) out[j] = base + (rs->d + j) * vect_stride + off;
            return matmul_ex(rs, gm.data(), rs->p, 2, in, isid, out, osid, ss, nstripes, n, true, as_stream(stream));
        });
    });
}

int rs_replace_dev(rs_t* rs, const uint8_t* const* data, const size_t* data_lens, int nd, const int* replace_rows,
                   int nr, uint8_t* const* parity, const size_t* parity_lens, int np, void* stream) {
    return abi_guard([&]() -> int {
        if (!rs || (nd > 0 && (!data || !data_lens)) || (nr > 0 && !replace_rows) ||
            (np > 0 && (!parity || !parity_lens)))
            return RS_ERR_INVAL;
        RS_TRY(check_replace(rs, data_lens, nd, replace_rows, nr, parity_lens, np));
        RS_TRY(ensure_device(rs));
        DeviceGuard g(rs->device);
        std::vector<uint8_t> gm = replace_matrix(rs, replace_rows, nr);
        return update_ranges(rs, data_lens[0], [&](uint64_t off, uint64_t n) {
            const uint8_t* in[kMaxVects];
            uint8_t* out[kMaxVects];
            for (int i = 0; i < nr; ++i) in[i] = data[i] + off;
            for (int j = 0; j < rs->p; ++j) out[j] = parity[j] + off;
            return matmul(rs, gm.data(), rs->p, nr, in, 0, out, 0, 1, n, true, as_stream(stream));
        });
    });
}

int rs_replace_batch(rs_t* rs, const uint8_t* data_base, int64_t data_stripe_stride, int64_t data_vect_stride,
                     const int* replace_rows, int nr, uint8_t* base, int64_t stripe_stride, int64_t vect_stride,
                     int nstripes, size_t len, void* stream) {
    return abi_guard([&]() -> int {
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
        std::vector<uint8_t> gm = replace_matrix(rs, replace_rows, nr);
        return update_ranges(rs, len, [&](uint64_t off, uint64_t n) {
            const uint8_t* in[kMaxVects];
            uint8_t* out[kMaxVects];
            for (int i = 0; i < nr; ++i) in[i] = data_base + i * data_vect_stride + off;
            for (int j = 0; j < rs->p; ++j) out[j] = base + (rs->d + j) * vect_stride + off;
            return matmul(rs, gm.data(), rs->p, nr, in, data_stripe_stride, out, stripe_stride, nstripes, n, true,
                          as_stream(stream));
        });
    });
}

int rs_xor_batch(rs_t* rs, const uint8_t* src_base, int64_t src_stripe_stride, int64_t src_vect_stride, int nsrc,
                 uint8_t* dst_base, int64_t dst_stripe_stride, int nstripes, size_t len, void* stream) {
    return abi_guard([&]() -> int {
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
    });
}

int rs_gf_matmul_batch(rs_t* rs, const uint8_t* mat, int rows, int cols, const uint8_t* in_base,
                       int64_t in_stripe_stride, int64_t in_vect_stride, const int* in_map, uint8_t* out_base,
                       int64_t out_stripe_stride, int64_t out_vect_stride, const int* out_map, int nstripes,
                       size_t len, int accumulate, void* stream) {
    return abi_guard([&]() -> int {
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
    });
}

}  // extern "C"
