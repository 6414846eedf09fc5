// jit_asm.cpp — run-time bit-sliced kernels emitted directly as gfx950
// assembly and assembled by the code-object manager (comgr), instead of
// C++ compiled by hiprtc.
//
// Why: hiprtc runs the whole LLVM pipeline over a straight-line network of
// thousands of XORs: 1.2-1.5 s for a 10 x 8 matrix (0.85 s of it fixed cost:
// headers, device libraries) and 6-16 s for 16 x 32 .. 16 x 64,
// too slow for erasure patterns seen a few times, and out of reach for
// networks wider than 16 rows.  The network needs no optimiser: register
// allocation is fixed by the layout below, and assembling is linear in its
// size (tens of ms).
//
// Kernel contract (AsmArgs, jit.hpp).  Grid x = 2 KiB chunks of each vector,
// grid y = stripes of the launch; a workgroup is NW waves over the same
// chunk.  Lane t of a wave owns 32 bytes of every vector: four 8-byte pieces
// at 8t + 512k (k = 0..3) of the chunk, so each wave instruction moves 512
// contiguous bytes (the perm-table kernels' dwordx2 pattern).  Wave w
// computes rows [w*RW, w*RW + RW) of the matrix (rows past the matrix are
// not emitted); with NW > 1 the waves load the same input lines, the first
// fetch going to HBM and the others hitting the CU's L1 / the XCD's L2.
//
// Per column: the 8 dwords of the lane's 32 bytes (four buffer_load_dwordx2
// ... nt, issued `pf` columns ahead) go through an 8x8 bit transpose (12 swaps
// of 4 VALU: two shifts and two v_bfi_b32, in place) into bit-planes; the
// XORs of each 4-plane half's subsets that the column uses are formed once;
// output plane i of row r takes one subset of each half (v_bitop3 xor3).  At
// the end each row's planes are transposed back and stored (buffer
// store_dwordx2 ... nt), XORed with the old output bytes first in accumulate
// mode.  Vector v of stripe s is at ptr[v] + s * 16 * stride16[v], addressed
// through a buffer descriptor whose range is `body` bytes: lanes past the
// vector body read zeros and their stores are dropped, so no lane masks.
#include "jit_asm.hpp"

#include <amd_comgr/amd_comgr.h>

#include <algorithm>

#include <chrono>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <vector>

namespace rsamd {

namespace {

uint8_t gmul8(uint8_t a, uint8_t b) {  // GF(2^8), polynomial 0x11d
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        const bool hi = a & 0x80;
        a = static_cast<uint8_t>(a << 1);
        if (hi) a ^= 0x1d;
        b >>= 1;
    }
    return r;
}

class Asm {
public:
    std::string out;
    void line(const char* fmt, ...) __attribute__((format(printf, 2, 3))) {
        char buf[256];
        va_list ap;
        va_start(ap, fmt);
        std::vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        out += '\t';
        out += buf;
        out += '\n';
    }
    void label(const std::string& l) { out += l + ":\n"; }
};

// SGPRs
constexpr int kSKarg = 0;      // s[0:1] kernarg segment pointer
constexpr int kSWgX = 2;       // workgroup id x: chunk
constexpr int kSWgY = 3;       // workgroup id y: launch stripe
constexpr int kSStripe = 4;    // stripe index (through stripe_ids)
constexpr int kSWave = 5;      // wave index in the workgroup
constexpr int kSTmp = 8;       // s[8:11] scratch
constexpr int kSDescIn = 12;   // s[12:15] input buffer descriptor
constexpr int kSDescOut = 16;  // s[16:19] output buffer descriptor
constexpr int kSStage = 20;    // s[20:27] two (ptr lo, ptr hi, stride16, -) staging slots
constexpr int kSMask = 28;     // s[28:33] transpose masks
constexpr int kSgprs = 34;
// VGPRs
constexpr int kVTid = 0;       // work-item id
constexpr int kVOff = 1;       // lane's byte offset in the vectors (chunk * 2048 + 8 * lane)
constexpr int kVT0 = 2, kVT1 = 3;  // transpose temporaries
constexpr int kVSlots = 4;     // pf slots of 8 (64-bit aligned pairs)

const uint32_t kMasks[6] = {0x0F0F0F0Fu, 0xF0F0F0F0u, 0x33333333u, 0xCCCCCCCCu, 0x55555555u, 0xAAAAAAAAu};

struct Layout {
    int pf, slots_end, sub, acc, vgprs;
};

// In-place 8x8 bit transpose of v[r[0]..r[7]] (bs_transpose8, kernels.hip):
// swap(a, b, s, m): b = (m & (a >> s)) | (~m & b); a = ((m << s) & (b << s)) | (~(m << s) & a)
void transpose8(Asm& A, const int (&r)[8]) {
    auto swap = [&](int a, int b, int s, int mi) {
        A.line("v_lshrrev_b32 v%d, %d, v%d", kVT0, s, a);
        A.line("v_lshlrev_b32 v%d, %d, v%d", kVT1, s, b);
        A.line("v_bfi_b32 v%d, s%d, v%d, v%d", b, kSMask + mi, kVT0, b);
        A.line("v_bfi_b32 v%d, s%d, v%d, v%d", a, kSMask + mi + 1, kVT1, a);
    };
    for (int i = 0; i < 4; ++i) swap(r[i], r[i + 4], 4, 0);
    swap(r[0], r[2], 2, 2);
    swap(r[1], r[3], 2, 2);
    swap(r[4], r[6], 2, 2);
    swap(r[5], r[7], 2, 2);
    for (int i = 0; i < 8; i += 2) swap(r[i], r[i + 1], 1, 4);
}

}  // namespace

std::string asm_source(const uint8_t* mat, int rows, int cols, bool acc, int nw, int pf, int sync, int max_waves,
                       int* vgprs_out) {
    const int rw = (rows + nw - 1) / nw;  // rows per wave
    Layout L;
    L.pf = pf < 1 ? 1 : pf > 4 ? 4 : pf;
    L.slots_end = kVSlots + 8 * L.pf;
    L.sub = L.slots_end;        // 2 x 15 subset registers (index by half * 15 + m - 1; singles unused)
    L.acc = L.sub + 30;
    L.vgprs = L.acc + 8 * rw;
    if (vgprs_out) *vgprs_out = L.vgprs;

    // mask[c][r][i]: input planes j of column c feeding plane i of row r
    std::vector<uint8_t> mask(static_cast<size_t>(cols) * rows * 8);
    for (int c = 0; c < cols; ++c)
        for (int r = 0; r < rows; ++r) {
            const uint8_t g = mat[static_cast<size_t>(r) * cols + c];
            for (int i = 0; i < 8; ++i) {
                uint8_t m = 0;
                for (int j = 0; j < 8; ++j)
                    if ((gmul8(g, static_cast<uint8_t>(1u << j)) >> i) & 1) m |= static_cast<uint8_t>(1u << j);
                mask[(static_cast<size_t>(c) * rows + r) * 8 + i] = m;
            }
        }

    Asm A;
    A.out += "\t.amdgcn_target \"amdgcn-amd-amdhsa--gfx950\"\n\t.amdhsa_code_object_version 6\n\t.text\n";
    A.out += "\t.globl\trs_bs_asm\n\t.p2align\t8\n\t.type\trs_bs_asm,@function\nrs_bs_asm:\n";
    // ---- prologue: stripe, lane offset, wave, masks, descriptor constants
    A.line("s_load_dword s%d, s[%d:%d], 0x%x", kSDescIn + 2, kSKarg, kSKarg + 1,
           static_cast<unsigned>(offsetof(AsmArgs, body)));
    A.line("s_load_dwordx2 s[%d:%d], s[%d:%d], 0x%x", kSTmp, kSTmp + 1, kSKarg, kSKarg + 1,
           static_cast<unsigned>(offsetof(AsmArgs, stripe_ids)));
    A.line("s_load_dword s%d, s[%d:%d], 0x%x", kSTmp + 3, kSKarg, kSKarg + 1,
           static_cast<unsigned>(offsetof(AsmArgs, stripe0)));
    for (int i = 0; i < 6; ++i) A.line("s_mov_b32 s%d, 0x%08x", kSMask + i, kMasks[i]);
    A.line("s_mov_b32 s%d, 0x20000", kSDescIn + 3);
    A.line("s_mov_b32 s%d, 0x20000", kSDescOut + 3);
    A.line("v_and_b32 v%d, 63, v%d", kVOff, kVTid);
    A.line("v_lshlrev_b32 v%d, 3, v%d", kVOff, kVOff);
    A.line("s_lshl_b32 s%d, s%d, 11", kSTmp + 2, kSWgX);
    A.line("v_add_u32 v%d, s%d, v%d", kVOff, kSTmp + 2, kVOff);
    // wave id = bits 6-9 of the work-item id (packed work-item ids: y / z sit
    // in bits 10-29; zero for these 1-D launches, masked anyway)
    A.line("v_and_b32 v%d, 0x3c0, v%d", kVT0, kVTid);
    A.line("v_lshrrev_b32 v%d, 6, v%d", kVT0, kVT0);
    // a VALU write of a VGPR followed at once by v_readfirstlane of it reads
    // the OLD value (one wait state required; measured: the wave id came out
    // as 64, not 1, tools/asm_probe/wave_id.s)
    A.line("s_nop 1");
    A.line("v_readfirstlane_b32 s%d, v%d", kSWave, kVT0);
    A.line("s_waitcnt lgkmcnt(0)");
    A.line("s_mov_b32 s%d, s%d", kSDescOut + 2, kSDescIn + 2);
    A.line("s_add_u32 s%d, s%d, s%d", kSStripe, kSWgY, kSTmp + 3);  // stripe0 + y
    A.line("s_cmp_eq_u64 s[%d:%d], 0", kSTmp, kSTmp + 1);
    A.line("s_cbranch_scc1 .Lstripe_done");
    A.line("s_lshl_b32 s%d, s%d, 2", kSTmp + 2, kSStripe);
    A.line("s_add_u32 s%d, s%d, s%d", kSTmp, kSTmp, kSTmp + 2);
    A.line("s_addc_u32 s%d, s%d, 0", kSTmp + 1, kSTmp + 1);
    A.line("s_load_dword s%d, s[%d:%d], 0x0", kSStripe, kSTmp, kSTmp + 1);
    A.line("s_waitcnt lgkmcnt(0)");
    A.label(".Lstripe_done");
    A.line("s_nop 4");  // (v_readfirstlane -> SGPR read hazard margin)
    // wave w -> its rows' code (long jumps: a wave's straight-line code can
    // exceed the 16-bit branch range); waves without rows leave
    for (int w = 1; w < nw; ++w) {
        const std::string tgt = w * rw < rows ? ".Lwave" + std::to_string(w) : std::string(".Lidle");
        A.line("s_cmp_eq_u32 s%d, %d", kSWave, w);
        A.line("s_cbranch_scc0 .Lnot%d", w);
        A.line("s_getpc_b64 s[%d:%d]", kSTmp, kSTmp + 1);
        A.label(".Lpc" + std::to_string(w));
        A.line("s_add_u32 s%d, s%d, (%s-.Lpc%d)&4294967295", kSTmp, kSTmp, tgt.c_str(), w);
        A.line("s_addc_u32 s%d, s%d, (%s-.Lpc%d)>>32", kSTmp + 1, kSTmp + 1, tgt.c_str(), w);
        A.line("s_setpc_b64 s[%d:%d]", kSTmp, kSTmp + 1);
        A.label(".Lnot" + std::to_string(w));
    }

    for (int w = 0; w < nw; ++w) {
        const int r0 = w * rw, nr = std::min(rw, rows - r0);
        if (nr <= 0) break;
        if (w) A.label(".Lwave" + std::to_string(w));
        // per-wave VMEM queue: ids of issued ops, in order (vmcnt bookkeeping)
        std::vector<int> vq;
        int next_id = 0;
        auto vmem_wait_for = [&](int id) {  // wait until op `id` has completed
            int after = 0;
            bool found = false;
            for (int x : vq) {
                if (found) ++after;
                if (x == id) found = true;
            }
            if (!found) return;
            A.line("s_waitcnt vmcnt(%d)", after > 63 ? 63 : after);
            // everything issued up to and including `id` is done
            std::vector<int> rest;
            bool keep = false;
            for (int x : vq) {
                if (keep) rest.push_back(x);
                if (x == id) keep = true;
            }
            vq.swap(rest);
        };
        // scalar staging of vector v's (ptr, stride16) into stage slot `st`
        auto stage = [&](int v, int st) {
            const int s = kSStage + 4 * st;
            A.line("s_load_dwordx2 s[%d:%d], s[%d:%d], 0x%x", s, s + 1, kSKarg, kSKarg + 1,
                   static_cast<unsigned>(offsetof(AsmArgs, ptr) + 8 * v));
            A.line("s_load_dword s%d, s[%d:%d], 0x%x", s + 2, kSKarg, kSKarg + 1,
                   static_cast<unsigned>(offsetof(AsmArgs, stride16) + 4 * v));
        };
        // descriptor base = ptr + stripe * stride16 * 16, from stage slot `st`
        auto desc = [&](int st, int d) {
            const int s = kSStage + 4 * st;
            A.line("s_waitcnt lgkmcnt(0)");
            A.line("s_mul_i32 s%d, s%d, s%d", kSTmp, kSStripe, s + 2);
            A.line("s_mul_hi_u32 s%d, s%d, s%d", kSTmp + 1, kSStripe, s + 2);
            A.line("s_lshl_b64 s[%d:%d], s[%d:%d], 4", kSTmp, kSTmp + 1, kSTmp, kSTmp + 1);
            A.line("s_add_u32 s%d, s%d, s%d", d, s, kSTmp);
            A.line("s_addc_u32 s%d, s%d, s%d", d + 1, s + 1, kSTmp + 1);
            A.line("s_and_b32 s%d, s%d, 0xffff", d + 1, d + 1);
        };
        auto slot_reg = [&](int c, int j) { return kVSlots + 8 * (c % L.pf) + j; };
        std::vector<int> col_id(static_cast<size_t>(cols), -1);  // last VMEM op of each column's loads
        // a lone wave streams its inputs (nt); the waves of a multi-wave
        // workgroup read the same lines, so those loads keep them cached for
        // the other waves (measured with nt: 64+64 Encode fetched 1.45x its
        // input bytes from HBM, 128+128 2.8x; profiles/r03/pmc_traffic_*.json)
        const char* in_aux = nw > 1 ? "" : " nt";
        auto issue_col = [&](int c) {  // stage(c) was issued into slot c & 1
            desc(c & 1, kSDescIn);
            if (c + 1 < cols) stage(c + 1, (c + 1) & 1);
            for (int k = 0; k < 4; ++k) {
                const int v = slot_reg(c, 2 * k);
                if (k) A.line("buffer_load_dwordx2 v[%d:%d], v%d, s[%d:%d], 0 offen offset:%d%s", v, v + 1, kVOff,
                              kSDescIn, kSDescIn + 3, 512 * k, in_aux);
                else A.line("buffer_load_dwordx2 v[%d:%d], v%d, s[%d:%d], 0 offen%s", v, v + 1, kVOff, kSDescIn,
                            kSDescIn + 3, in_aux);
                vq.push_back(next_id);
                col_id[static_cast<size_t>(c)] = next_id++;
            }
        };
        stage(0, 0);
        for (int c = 0; c < L.pf && c < cols; ++c) issue_col(c);
        auto sub_reg = [&](int half, int m) { return L.sub + half * 15 + m - 1; };
        auto acc_reg = [&](int r, int i) { return L.acc + 8 * r + i; };
        for (int c = 0; c < cols; ++c) {
            vmem_wait_for(col_id[static_cast<size_t>(c)]);
            int pr[8];
            for (int j = 0; j < 8; ++j) pr[j] = slot_reg(c, j);
            transpose8(A, pr);
            // subsets of each half used by this column's rows
            std::string name[2][16];
            for (int half = 0; half < 2; ++half) {
                bool have[16] = {}, used[16] = {}, need[16] = {};
                for (int b = 0; b < 4; ++b) {
                    have[1 << b] = true;
                    name[half][1 << b] = "v" + std::to_string(pr[4 * half + b]);
                }
                for (int r = r0; r < r0 + nr; ++r)
                    for (int i = 0; i < 8; ++i)
                        used[(mask[(static_cast<size_t>(c) * rows + r) * 8 + i] >> (4 * half)) & 15] = true;
                used[0] = false;
                for (int m = 1; m < 16; ++m)
                    if (used[m])
                        for (int x = m; x && !have[x] && !need[x]; x ^= x & -x) need[x] = true;
                for (int pc = 2; pc <= 4; ++pc)
                    for (int m = 1; m < 16; ++m) {
                        if (!need[m] || __builtin_popcount(m) != pc) continue;
                        const int low = m & -m, rest = m ^ low;
                        const int dst = sub_reg(half, m);
                        A.line("v_xor_b32 v%d, %s, %s", dst, name[half][rest].c_str(), name[half][low].c_str());
                        name[half][m] = "v" + std::to_string(dst);
                        have[m] = true;
                    }
            }
            for (int r = r0; r < r0 + nr; ++r)
                for (int i = 0; i < 8; ++i) {
                    const int m = mask[(static_cast<size_t>(c) * rows + r) * 8 + i];
                    const std::string* t[2];
                    int nt = 0;
                    if (m & 15) t[nt++] = &name[0][m & 15];
                    if (m >> 4) t[nt++] = &name[1][m >> 4];
                    const int a = acc_reg(r - r0, i);
                    if (c == 0) {
                        if (nt == 0) A.line("v_mov_b32 v%d, 0", a);
                        else if (nt == 1) A.line("v_mov_b32 v%d, %s", a, t[0]->c_str());
                        else A.line("v_xor_b32 v%d, %s, %s", a, t[0]->c_str(), t[1]->c_str());
                    } else if (nt == 2) {
                        A.line("v_bitop3_b32 v%d, v%d, %s, %s bitop3:0x96", a, a, t[0]->c_str(), t[1]->c_str());
                    } else if (nt == 1) {
                        A.line("v_xor_b32 v%d, v%d, %s", a, a, t[0]->c_str());
                    }
                }
            if (c + L.pf < cols) issue_col(c + L.pf);  // the slot is free again
            // keep the waves within `sync` columns of each other, so the lines
            // the first wave fetched are still cached when the others load them
            if (nw > 1 && sync > 0 && (c + 1) % sync == 0 && c + 1 < cols) A.line("s_barrier");
        }
        // ---- outputs: transpose back, (accumulate: XOR the old bytes), store
        int ostage = 0;
        stage(cols + r0, ostage);
        std::vector<int> old_id(static_cast<size_t>(nr), -1);
        auto old_reg = [&](int r, int j) { return kVSlots + 8 * (r % 2) + j; };  // pf >= 1: 8 regs; 2 rows need 16
        auto issue_old = [&](int r) {  // descriptor of row r is in kSDescOut
            for (int k = 0; k < 4; ++k) {
                const int v = old_reg(r, 2 * k);
                if (k) A.line("buffer_load_dwordx2 v[%d:%d], v%d, s[%d:%d], 0 offen offset:%d", v, v + 1, kVOff,
                              kSDescOut, kSDescOut + 3, 512 * k);
                else A.line("buffer_load_dwordx2 v[%d:%d], v%d, s[%d:%d], 0 offen", v, v + 1, kVOff, kSDescOut,
                            kSDescOut + 3);
                vq.push_back(next_id);
                old_id[static_cast<size_t>(r)] = next_id++;
            }
        };
        for (int r = 0; r < nr; ++r) {
            desc(ostage, kSDescOut);
            if (r + 1 < nr) {
                ostage ^= 1;
                stage(cols + r0 + r + 1, ostage);
            }
            int pr[8];
            for (int j = 0; j < 8; ++j) pr[j] = acc_reg(r, j);
            if (acc) {
                issue_old(r);
                transpose8(A, pr);
                vmem_wait_for(old_id[static_cast<size_t>(r)]);
                for (int j = 0; j < 8; ++j) A.line("v_xor_b32 v%d, v%d, v%d", pr[j], pr[j], old_reg(r, j));
            } else {
                transpose8(A, pr);
            }
            for (int k = 0; k < 4; ++k) {
                if (k) A.line("buffer_store_dwordx2 v[%d:%d], v%d, s[%d:%d], 0 offen offset:%d nt", pr[2 * k],
                              pr[2 * k + 1], kVOff, kSDescOut, kSDescOut + 3, 512 * k);
                else A.line("buffer_store_dwordx2 v[%d:%d], v%d, s[%d:%d], 0 offen nt", pr[0], pr[1], kVOff,
                            kSDescOut, kSDescOut + 3);
                vq.push_back(next_id++);
            }
        }
        A.line("s_endpgm");
    }
    A.label(".Lidle");
    A.line("s_endpgm");
    A.out += ".Lfunc_end0:\n\t.size\trs_bs_asm, .Lfunc_end0-rs_bs_asm\n";
    // ---- kernel descriptor and metadata (code object v6)
    int accum = (L.vgprs + 3) / 4 * 4;
    // occupancy cap: 512 VGPRs per SIMD lane, allocated in granules of 8
    if (max_waves > 1 && max_waves <= 8) accum = std::max(accum, std::min(256, 512 / max_waves / 8 * 8));
    char kd[2048];
    std::snprintf(kd, sizeof kd,
                  "\t.rodata\n\t.p2align\t6\n\t.amdhsa_kernel rs_bs_asm\n"
                  "\t\t.amdhsa_group_segment_fixed_size 0\n\t\t.amdhsa_private_segment_fixed_size 0\n"
                  "\t\t.amdhsa_kernarg_size %zu\n\t\t.amdhsa_user_sgpr_count 2\n"
                  "\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1\n"
                  "\t\t.amdhsa_system_sgpr_workgroup_id_x 1\n\t\t.amdhsa_system_sgpr_workgroup_id_y 1\n"
                  "\t\t.amdhsa_system_vgpr_workitem_id 0\n"
                  "\t\t.amdhsa_next_free_vgpr %d\n\t\t.amdhsa_next_free_sgpr %d\n\t\t.amdhsa_accum_offset %d\n"
                  "\t\t.amdhsa_reserve_vcc 0\n\t\t.amdhsa_ieee_mode 1\n\t\t.amdhsa_dx10_clamp 1\n"
                  "\t.end_amdhsa_kernel\n",
                  sizeof(AsmArgs), accum, kSgprs, accum);
    A.out += kd;
    std::snprintf(kd, sizeof kd,
                  "\t.amdgpu_metadata\n---\namdhsa.kernels:\n  - .agpr_count: 0\n    .args:\n"
                  "      - .offset: 0\n        .size: %zu\n        .value_kind: by_value\n"
                  "    .group_segment_fixed_size: 0\n    .kernarg_segment_align: 8\n"
                  "    .kernarg_segment_size: %zu\n    .max_flat_workgroup_size: %d\n    .name: rs_bs_asm\n"
                  "    .private_segment_fixed_size: 0\n    .sgpr_count: %d\n    .sgpr_spill_count: 0\n"
                  "    .symbol: rs_bs_asm.kd\n    .uniform_work_group_size: 1\n    .vgpr_count: %d\n"
                  "    .vgpr_spill_count: 0\n    .wavefront_size: 64\n"
                  "amdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n"
                  "\t.end_amdgpu_metadata\n",
                  sizeof(AsmArgs), sizeof(AsmArgs), 64 * nw, kSgprs + 6, accum);
    A.out += kd;
    return A.out;
}

// Assemble and link through comgr: relocatable, then executable code object.
bool asm_assemble(const std::string& src, std::vector<char>* code, std::string* log, double* ms) {
    const auto t0 = std::chrono::steady_clock::now();
    amd_comgr_data_t data{};
    amd_comgr_data_set_t in{}, reloc{}, exe{};
    amd_comgr_action_info_t info{};
    bool ok = amd_comgr_create_data(AMD_COMGR_DATA_KIND_SOURCE, &data) == AMD_COMGR_STATUS_SUCCESS;
    ok = ok && amd_comgr_set_data(data, src.size(), src.data()) == AMD_COMGR_STATUS_SUCCESS;
    ok = ok && amd_comgr_set_data_name(data, "rs_bs_asm.s") == AMD_COMGR_STATUS_SUCCESS;
    ok = ok && amd_comgr_create_data_set(&in) == AMD_COMGR_STATUS_SUCCESS;
    ok = ok && amd_comgr_create_data_set(&reloc) == AMD_COMGR_STATUS_SUCCESS;
    ok = ok && amd_comgr_create_data_set(&exe) == AMD_COMGR_STATUS_SUCCESS;
    ok = ok && amd_comgr_data_set_add(in, data) == AMD_COMGR_STATUS_SUCCESS;
    ok = ok && amd_comgr_create_action_info(&info) == AMD_COMGR_STATUS_SUCCESS;
    ok = ok && amd_comgr_action_info_set_isa_name(info, "amdgcn-amd-amdhsa--gfx950") == AMD_COMGR_STATUS_SUCCESS;
    ok = ok && amd_comgr_action_info_set_logging(info, true) == AMD_COMGR_STATUS_SUCCESS;
    auto collect_log = [&](amd_comgr_data_set_t set) {
        size_t n = 0;
        if (amd_comgr_action_data_count(set, AMD_COMGR_DATA_KIND_LOG, &n) != AMD_COMGR_STATUS_SUCCESS) return;
        for (size_t i = 0; i < n; ++i) {
            amd_comgr_data_t lg;
            if (amd_comgr_action_data_get_data(set, AMD_COMGR_DATA_KIND_LOG, i, &lg) != AMD_COMGR_STATUS_SUCCESS)
                continue;
            size_t sz = 0;
            if (amd_comgr_get_data(lg, &sz, nullptr) == AMD_COMGR_STATUS_SUCCESS && sz) {
                std::string s(sz, '\0');
                if (amd_comgr_get_data(lg, &sz, &s[0]) == AMD_COMGR_STATUS_SUCCESS) *log += s;
            }
            amd_comgr_release_data(lg);
        }
    };
    if (ok) {
        ok = amd_comgr_do_action(AMD_COMGR_ACTION_ASSEMBLE_SOURCE_TO_RELOCATABLE, info, in, reloc) ==
             AMD_COMGR_STATUS_SUCCESS;
        if (!ok) collect_log(reloc);
    }
    if (ok) {
        ok = amd_comgr_do_action(AMD_COMGR_ACTION_LINK_RELOCATABLE_TO_EXECUTABLE, info, reloc, exe) ==
             AMD_COMGR_STATUS_SUCCESS;
        if (!ok) collect_log(exe);
    }
    if (ok) {
        amd_comgr_data_t obj;
        ok = amd_comgr_action_data_get_data(exe, AMD_COMGR_DATA_KIND_EXECUTABLE, 0, &obj) == AMD_COMGR_STATUS_SUCCESS;
        if (ok) {
            size_t sz = 0;
            ok = amd_comgr_get_data(obj, &sz, nullptr) == AMD_COMGR_STATUS_SUCCESS && sz > 0;
            if (ok) {
                code->resize(sz);
                ok = amd_comgr_get_data(obj, &sz, code->data()) == AMD_COMGR_STATUS_SUCCESS;
            }
            amd_comgr_release_data(obj);
        }
    }
    amd_comgr_destroy_action_info(info);
    amd_comgr_destroy_data_set(in);
    amd_comgr_destroy_data_set(reloc);
    amd_comgr_destroy_data_set(exe);
    amd_comgr_release_data(data);
    if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return ok;
}

}  // namespace rsamd
