// jit_asm.cpp — run-time bit-sliced kernels generated for one matrix as
// gfx950 machine code.
//
// Why: hiprtc runs the whole LLVM pipeline over a straight-line network of
// thousands of XORs: 1.2-1.5 s for a 10 x 8 matrix and 6-16 s for 16 x 32 ..
// 16 x 64.  The network needs no optimiser: register
// allocation is fixed by the layout below.  Round 3 printed it as assembly
// and had comgr assemble and link it: 12 ms for 5 x 10, ~30 ms for 16 x 16,
// 0.3-0.4 s for 28 x 100 / 64 x 64 and 1.5-1.7 s for 128 x 128 (llvm-mc over
// hundreds of thousands of lines).  The generator now builds the kernel as a
// list of instructions (Prog) that is either printed as assembly (asm_source:
// the CPU emulator's input, and the comgr path kept for comparison) or
// encoded straight into machine code (asm_binary) and dropped into a
// code-object template (asm_link_binary): the template - kernel descriptor,
// metadata, and a .text of the right size class filled with s_endpgm - is
// assembled by comgr once per (waves per workgroup, VGPR budget, size class)
// and reused for every matrix.  tests/test_jit_asm.py checks that the
// encoder's bytes equal comgr's for generated kernels, instruction for
// instruction.
//
// Kernel contract (AsmArgs, jit_asm.hpp).  Grid x = 2 KiB chunks of each
// vector, grid y = stripes of the launch; a workgroup is NW waves over the
// same chunk.  Lane t of a wave owns 32 bytes of every vector: four 8-byte
// pieces at 8t + 512k (k = 0..3) of the chunk, so each wave instruction moves
// 512 contiguous bytes (the perm-table kernels' dwordx2 pattern).  Wave w
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
#include <map>
#include <mutex>
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

// ---------------------------------------------------------------- instructions
//
// Source operands use the hardware's 9-bit operand space: SGPR n = n, inline
// integer k (0..64) = 128 + k, -1 = 193, a 32-bit literal = 255 (value in
// `imm`), VGPR n = 256 + n.
constexpr int kLit = 255;
constexpr int V(int n) { return 256 + n; }
constexpr int C(int k) { return 128 + k; }

enum class K : uint8_t {
    Label,
    SLoad,      // a = sdst, b = dwords (1 | 2), c = sbase, imm = byte offset
    SMovLit,    // a = sdst, imm (d = 1: printed zero-padded)
    SOp1,       // sub: mov | getpc | setpc; a = sdst, b = ssrc
    SOp2,       // sub: add | addc | lshl | lshl64 | mul | mulhi | and; a = sdst, b = src0, c = src1, imm
    SCmp,       // sub: eq32 | eq64; a = src0, b = src1
    SNop,       // a = wait states - 1
    SWaitLgkm0, // a = count (lgkmcnt(a))
    SWaitVm,    // a = count
    SBarrier,
    SEndpgm,
    SBranch,    // sub: scc0 | scc1; a = label
    SAddPcrel,  // sub: lo (s_add_u32 with the literal label(a) - label(b)) | hi (s_addc_u32 with its upper half); c = sdst = src0
    VOp2,       // sub: and | lshl | lshr | add | xor; a = vdst, b = src0, c = vsrc1 (VGPR number), imm
    VMov,       // a = vdst, b = src0
    VReadLane,  // a = sdst, b = VGPR number
    VBfi,       // a = vdst, b = src0, c = src1, d = src2 (9-bit operands)
    VXor3,      // v_bitop3_b32 ... bitop3:0x96; a = vdst, b, c, d = VGPR numbers
    BufLoad2,   // a = vdata, b = vaddr, c = srsrc (first SGPR), d = offset, sub = nt
    BufStore2,  // same
    DsWrite4,   // ds_write_b128: a = vaddr, b = first data VGPR, imm = offset
    DsRead4,    // ds_read_b128: a = first vdst, b = vaddr, imm = offset
    DsRead2,    // ds_read_b64: a = first vdst, b = vaddr, imm = offset
    BufLoadLds4,  // buffer_load_dwordx4 ... lds (LDS-DMA: 16 bytes per lane to LDS at M0 + 16 * lane):
                  // b = vaddr, c = srsrc, sub = nt
};

enum Sub : uint8_t {
    kNone = 0,
    kMov, kGetpc, kSetpc,
    kAdd, kAddc, kLshl, kLshl64, kMul, kMulhi, kAnd, kLshr, kSub, kOr,
    kEq32, kEq64, kGe32,
    kScc0, kScc1,
    kLo, kHi,
    kVAnd, kVLshl, kVLshr, kVAdd, kVXor,
};

struct Ins {
    K k;
    uint8_t sub;
    int16_t a, b, c, d;
    uint32_t imm;
};

struct Prog {
    std::vector<Ins> ins;
    std::vector<std::string> label_names;
    int new_label(const std::string& name) {
        label_names.push_back(name);
        return static_cast<int>(label_names.size()) - 1;
    }
    void put(K k, int sub, int a = 0, int b = 0, int c = 0, int d = 0, uint32_t imm = 0) {
        ins.push_back(Ins{k, static_cast<uint8_t>(sub), static_cast<int16_t>(a), static_cast<int16_t>(b),
                          static_cast<int16_t>(c), static_cast<int16_t>(d), imm});
    }
    void label(int l) { put(K::Label, kNone, l); }
    void s_load(int sdst, int dwords, int sbase, uint32_t off) { put(K::SLoad, kNone, sdst, dwords, sbase, 0, off); }
    void s_mov_lit(int sdst, uint32_t v, bool pad) { put(K::SMovLit, kNone, sdst, 0, 0, pad ? 1 : 0, v); }
    void s_mov(int sdst, int ssrc) { put(K::SOp1, kMov, sdst, ssrc); }
    void s_getpc(int sdst) { put(K::SOp1, kGetpc, sdst, 0); }
    void s_setpc(int ssrc) { put(K::SOp1, kSetpc, 0, ssrc); }
    void s_op2(Sub s, int sdst, int src0, int src1, uint32_t imm = 0) { put(K::SOp2, s, sdst, src0, src1, 0, imm); }
    void s_cmp(Sub s, int src0, int src1) { put(K::SCmp, s, src0, src1); }
    void s_nop(int n) { put(K::SNop, kNone, n); }
    void wait_lgkm0() { put(K::SWaitLgkm0, kNone, 0); }
    void wait_lgkm(int n) { put(K::SWaitLgkm0, kNone, n); }
    void wait_vm(int n) { put(K::SWaitVm, kNone, n); }
    void s_barrier() { put(K::SBarrier, kNone); }
    void s_endpgm() { put(K::SEndpgm, kNone); }
    void branch(Sub s, int label) { put(K::SBranch, s, label); }
    void add_pcrel(Sub s, int sreg, int target, int pc) { put(K::SAddPcrel, s, target, pc, sreg); }
    void v_op2(Sub s, int vdst, int src0, int vsrc1, uint32_t imm = 0) { put(K::VOp2, s, vdst, src0, vsrc1, 0, imm); }
    void v_mov(int vdst, int src0) { put(K::VMov, kNone, vdst, src0); }
    void v_readlane(int sdst, int vsrc) { put(K::VReadLane, kNone, sdst, vsrc); }
    void v_bfi(int vdst, int src0, int src1, int src2) { put(K::VBfi, kNone, vdst, src0, src1, src2); }
    void v_xor3(int vdst, int a, int b, int c) { put(K::VXor3, kNone, vdst, a, b, c); }
    void buf_load2(int vdata, int vaddr, int srsrc, int off, bool nt) {
        put(K::BufLoad2, nt ? 1 : 0, vdata, vaddr, srsrc, off);
    }
    void buf_store2(int vdata, int vaddr, int srsrc, int off) { put(K::BufStore2, 1, vdata, vaddr, srsrc, off); }
    void ds_write4(int vaddr, int vdata, uint32_t off) { put(K::DsWrite4, kNone, vaddr, vdata, 0, 0, off); }
    void ds_read4(int vdst, int vaddr, uint32_t off) { put(K::DsRead4, kNone, vdst, vaddr, 0, 0, off); }
    void ds_read2(int vdst, int vaddr, uint32_t off) { put(K::DsRead2, kNone, vdst, vaddr, 0, 0, off); }
    void buf_load_lds4(int vaddr, int srsrc, bool nt) { put(K::BufLoadLds4, nt ? 1 : 0, 0, vaddr, srsrc); }
};

constexpr int kM0 = 124;  // SGPR operand number of M0

// ---------------------------------------------------------------- text

std::string opnd(int x, uint32_t imm) {  // a 9-bit source operand as assembly text
    char b[32];
    if (x >= 256) std::snprintf(b, sizeof b, "v%d", x - 256);
    else if (x == kLit) std::snprintf(b, sizeof b, "0x%x", imm);
    else if (x >= 128 && x <= 192) std::snprintf(b, sizeof b, "%d", x - 128);
    else if (x >= 193 && x <= 208) std::snprintf(b, sizeof b, "%d", 192 - x);
    else if (x == kM0) std::snprintf(b, sizeof b, "m0");
    else std::snprintf(b, sizeof b, "s%d", x);
    return b;
}

std::string sreg(int n) { return n == kM0 ? std::string("m0") : "s" + std::to_string(n); }

std::string print(const Prog& p) {
    std::string out;
    char b[256];
    auto line = [&](const char* fmt, ...) __attribute__((format(printf, 2, 3))) {
        va_list ap;
        va_start(ap, fmt);
        std::vsnprintf(b, sizeof b, fmt, ap);
        va_end(ap);
        out += '\t';
        out += b;
        out += '\n';
    };
    for (const Ins& i : p.ins) {
        switch (i.k) {
            case K::Label: out += p.label_names[static_cast<size_t>(i.a)] + ":\n"; break;
            case K::SLoad:
                if (i.b == 1) line("s_load_dword s%d, s[%d:%d], 0x%x", i.a, i.c, i.c + 1, i.imm);
                else line("s_load_dwordx2 s[%d:%d], s[%d:%d], 0x%x", i.a, i.a + 1, i.c, i.c + 1, i.imm);
                break;
            case K::SMovLit:
                line(i.d ? "s_mov_b32 %s, 0x%08x" : "s_mov_b32 %s, 0x%x", sreg(i.a).c_str(), i.imm);
                break;
            case K::SOp1:
                if (i.sub == kMov) line("s_mov_b32 %s, %s", sreg(i.a).c_str(), sreg(i.b).c_str());
                else if (i.sub == kGetpc) line("s_getpc_b64 s[%d:%d]", i.a, i.a + 1);
                else line("s_setpc_b64 s[%d:%d]", i.b, i.b + 1);
                break;
            case K::SOp2: {
                static const char* const nm[] = {"s_add_u32", "s_addc_u32", "s_lshl_b32", "s_lshl_b64", "s_mul_i32",
                                                 "s_mul_hi_u32", "s_and_b32", "s_lshr_b32", "s_sub_u32", "s_or_b32"};
                const char* n = nm[i.sub - kAdd];
                if (i.sub == kLshl64)
                    line("%s s[%d:%d], s[%d:%d], %s", n, i.a, i.a + 1, i.b, i.b + 1, opnd(i.c, i.imm).c_str());
                else
                    line("%s s%d, %s, %s", n, i.a, opnd(i.b, i.imm).c_str(), opnd(i.c, i.imm).c_str());
                break;
            }
            case K::SCmp:
                if (i.sub == kEq64) line("s_cmp_eq_u64 s[%d:%d], %s", i.a, i.a + 1, opnd(i.b, 0).c_str());
                else line("%s %s, %s", i.sub == kGe32 ? "s_cmp_ge_u32" : "s_cmp_eq_u32", opnd(i.a, 0).c_str(),
                          opnd(i.b, 0).c_str());
                break;
            case K::SNop: line("s_nop %d", i.a); break;
            case K::SWaitLgkm0: line("s_waitcnt lgkmcnt(%d)", i.a); break;
            case K::SWaitVm: line("s_waitcnt vmcnt(%d)", i.a); break;
            case K::SBarrier: line("s_barrier"); break;
            case K::SEndpgm: line("s_endpgm"); break;
            case K::SBranch:
                line("%s %s", i.sub == kScc0 ? "s_cbranch_scc0" : "s_cbranch_scc1",
                     p.label_names[static_cast<size_t>(i.a)].c_str());
                break;
            case K::SAddPcrel: {
                const std::string& t = p.label_names[static_cast<size_t>(i.a)];
                const std::string& pc = p.label_names[static_cast<size_t>(i.b)];
                if (i.sub == kLo) line("s_add_u32 s%d, s%d, (%s-%s)&4294967295", i.c, i.c, t.c_str(), pc.c_str());
                else line("s_addc_u32 s%d, s%d, (%s-%s)>>32", i.c, i.c, t.c_str(), pc.c_str());
                break;
            }
            case K::VOp2: {
                static const char* const nm[] = {"v_and_b32", "v_lshlrev_b32", "v_lshrrev_b32", "v_add_u32",
                                                 "v_xor_b32"};
                line("%s v%d, %s, v%d", nm[i.sub - kVAnd], i.a, opnd(i.b, i.imm).c_str(), i.c);
                break;
            }
            case K::VMov: line("v_mov_b32 v%d, %s", i.a, opnd(i.b, 0).c_str()); break;
            case K::VReadLane: line("v_readfirstlane_b32 s%d, v%d", i.a, i.b); break;
            case K::VBfi:
                line("v_bfi_b32 v%d, %s, %s, %s", i.a, opnd(i.b, 0).c_str(), opnd(i.c, 0).c_str(),
                     opnd(i.d, 0).c_str());
                break;
            case K::VXor3: line("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96", i.a, i.b, i.c, i.d); break;
            case K::BufLoad2:
            case K::BufStore2: {
                const bool ld = i.k == K::BufLoad2;
                char off[32] = "";
                if (i.d) std::snprintf(off, sizeof off, " offset:%d", i.d);
                line("%s v[%d:%d], v%d, s[%d:%d], 0 offen%s%s", ld ? "buffer_load_dwordx2" : "buffer_store_dwordx2",
                     i.a, i.a + 1, i.b, i.c, i.c + 3, off, i.sub ? " nt" : "");
                break;
            }
            case K::DsWrite4:
                line("ds_write_b128 v%d, v[%d:%d] offset:%u", i.a, i.b, i.b + 3, i.imm);
                break;
            case K::DsRead4:
                line("ds_read_b128 v[%d:%d], v%d offset:%u", i.a, i.a + 3, i.b, i.imm);
                break;
            case K::DsRead2:
                line("ds_read_b64 v[%d:%d], v%d offset:%u", i.a, i.a + 1, i.b, i.imm);
                break;
            case K::BufLoadLds4:
                line("buffer_load_dwordx4 v%d, s[%d:%d], 0 offen%s lds", i.b, i.c, i.c + 3, i.sub ? " nt" : "");
                break;
        }
    }
    return out;
}

// ---------------------------------------------------------------- machine code (gfx950)
//
// Encodings as llvm-mc --mcpu=gfx950 --show-encoding emits them (GFX9
// formats): SOP1/SOP2/SOPC/SOPP/SMEM/VOP1/VOP2/VOP3/MUBUF.  Size in bytes.
int ins_size(const Ins& i) {
    switch (i.k) {
        case K::Label: return 0;
        case K::SLoad: case K::VBfi: case K::VXor3: case K::BufLoad2: case K::BufStore2: return 8;
        case K::DsWrite4: case K::DsRead4: case K::DsRead2: case K::BufLoadLds4: return 8;
        case K::SMovLit: return 8;
        case K::SAddPcrel: return 8;
        case K::SOp2: return (i.b == kLit || i.c == kLit) ? 8 : 4;
        case K::VOp2: return i.b == kLit ? 8 : 4;
        default: return 4;
    }
}

bool encode(const Prog& p, std::vector<uint32_t>* out, std::string* err) {
    std::vector<int64_t> at(p.label_names.size(), -1);
    int64_t pc = 0;
    for (const Ins& i : p.ins) {
        if (i.k == K::Label) at[static_cast<size_t>(i.a)] = pc;
        pc += ins_size(i);
    }
    out->clear();
    out->reserve(static_cast<size_t>(pc / 4));
    auto w = [&](uint32_t x) { out->push_back(x); };
    auto bad = [&](const char* what) {
        if (err) *err = what;
        return false;
    };
    // add addc lshl lshl64 mul mulhi and lshr sub or
    static const uint8_t sop2_op[] = {0x00, 0x04, 0x1c, 0x1d, 0x24, 0x2c, 0x0c, 0x1e, 0x01, 0x0e};
    static const uint8_t vop2_op[] = {0x13, 0x12, 0x10, 0x34, 0x15};              // and lshlrev lshrrev add_u32 xor
    pc = 0;
    for (const Ins& i : p.ins) {
        const int64_t here = pc;
        pc += ins_size(i);
        switch (i.k) {
            case K::Label: break;
            case K::SLoad:  // SMEM: op 0 (dword) / 1 (dwordx2), imm offset
                w(0xc0020000u | (i.b == 2 ? 1u << 18 : 0u) | (static_cast<uint32_t>(i.a) << 6) |
                  (static_cast<uint32_t>(i.c) >> 1));
                if (i.imm >= (1u << 20)) return bad("s_load offset");
                w(i.imm);
                break;
            case K::SMovLit:  // SOP1 s_mov_b32 sdst, literal
                w(0xbe800000u | (static_cast<uint32_t>(i.a) << 16) | 0xffu);
                w(i.imm);
                break;
            case K::SOp1: {
                const uint32_t op = i.sub == kMov ? 0x00 : i.sub == kGetpc ? 0x1c : 0x1d;
                w(0xbe800000u | (static_cast<uint32_t>(i.a) << 16) | (op << 8) | static_cast<uint32_t>(i.b));
                break;
            }
            case K::SOp2:
                if (i.b > 255 || i.c > 255) return bad("SOP2 operand");
                w(0x80000000u | (static_cast<uint32_t>(sop2_op[i.sub - kAdd]) << 23) |
                  (static_cast<uint32_t>(i.a) << 16) | (static_cast<uint32_t>(i.c) << 8) | static_cast<uint32_t>(i.b));
                if (i.b == kLit || i.c == kLit) w(i.imm);
                break;
            case K::SCmp:
                w(0xbf000000u | ((i.sub == kEq64 ? 0x12u : i.sub == kGe32 ? 0x09u : 0x06u) << 16) |
                  (static_cast<uint32_t>(i.b) << 8) | static_cast<uint32_t>(i.a));
                break;
            case K::SNop: w(0xbf800000u | static_cast<uint32_t>(i.a)); break;
            case K::SWaitLgkm0:  // vmcnt 63, expcnt 7, lgkmcnt bits 11:8
                w(0xbf8cc07fu | ((static_cast<uint32_t>(i.a) & 15u) << 8));
                break;
            case K::SWaitVm: {  // vmcnt[3:0] bits 3:0, [5:4] bits 15:14; expcnt 7, lgkmcnt 15
                const uint32_t n = static_cast<uint32_t>(i.a) & 63;
                w(0xbf8c0000u | (n & 15) | ((n >> 4) << 14) | 0x70u | 0xf00u);
                break;
            }
            case K::SBarrier: w(0xbf8a0000u); break;
            case K::SEndpgm: w(0xbf810000u); break;
            case K::SBranch: {
                const int64_t t = at[static_cast<size_t>(i.a)];
                if (t < 0) return bad("branch label");
                const int64_t rel = (t - (here + 4)) / 4;
                if (rel < -32768 || rel > 32767) return bad("branch range");
                w(0xbf800000u | ((i.sub == kScc0 ? 0x04u : 0x05u) << 16) | (static_cast<uint32_t>(rel) & 0xffffu));
                break;
            }
            case K::SAddPcrel: {
                const int64_t t = at[static_cast<size_t>(i.a)], b = at[static_cast<size_t>(i.b)];
                if (t < 0 || b < 0) return bad("pc-relative label");
                const int64_t d = t - b;
                const uint32_t s = static_cast<uint32_t>(i.c);
                // s_add_u32 s, s, literal (low half) | s_addc_u32 s, s, literal (high half),
                // as the assembler encodes the label expressions
                w(0x80000000u | (i.sub == kLo ? 0u : 0x04u << 23) | (s << 16) | (0xffu << 8) | s);
                w(static_cast<uint32_t>(i.sub == kLo ? static_cast<uint64_t>(d) : static_cast<uint64_t>(d) >> 32));
                break;
            }
            case K::VOp2:
                if (i.c > 255) return bad("VOP2 vsrc1");
                w((static_cast<uint32_t>(vop2_op[i.sub - kVAnd]) << 25) | (static_cast<uint32_t>(i.a) << 17) |
                  (static_cast<uint32_t>(i.c) << 9) | static_cast<uint32_t>(i.b));
                if (i.b == kLit) w(i.imm);
                break;
            case K::VMov: w(0x7e000000u | (static_cast<uint32_t>(i.a) << 17) | (0x01u << 9) | static_cast<uint32_t>(i.b)); break;
            case K::VReadLane:
                w(0x7e000000u | (static_cast<uint32_t>(i.a) << 17) | (0x02u << 9) | (256u + static_cast<uint32_t>(i.b)));
                break;
            case K::VBfi:  // VOP3a op 0x1ca
                w(0xd1ca0000u | static_cast<uint32_t>(i.a));
                w(static_cast<uint32_t>(i.b) | (static_cast<uint32_t>(i.c) << 9) | (static_cast<uint32_t>(i.d) << 18));
                break;
            case K::VXor3:  // VOP3 op 0x234, truth table 0x96 spread over ABS / OMOD / NEG
                w(0xd2340200u | static_cast<uint32_t>(i.a));
                w(0xd0000000u | (256u + static_cast<uint32_t>(i.b)) | ((256u + static_cast<uint32_t>(i.c)) << 9) |
                  ((256u + static_cast<uint32_t>(i.d)) << 18));
                break;
            case K::BufLoad2:
            case K::BufStore2: {  // MUBUF op 0x15 / 0x1d, offen, nt = bit 17
                if (i.d < 0 || i.d > 4095) return bad("buffer offset");
                const uint32_t op = i.k == K::BufLoad2 ? 0x15u : 0x1du;
                w(0xe0000000u | (op << 18) | (i.sub ? 1u << 17 : 0u) | (1u << 12) | static_cast<uint32_t>(i.d));
                w(0x80000000u | ((static_cast<uint32_t>(i.c) >> 2) << 16) | (static_cast<uint32_t>(i.a) << 8) |
                  static_cast<uint32_t>(i.b));
                break;
            }
            case K::DsWrite4:  // DS op 0xdf: offset 15:0, op 24:17; addr, data0 << 8
                if (i.imm > 0xffffu) return bad("ds offset");
                w(0xd8000000u | (0xdfu << 17) | i.imm);
                w(static_cast<uint32_t>(i.a) | (static_cast<uint32_t>(i.b) << 8));
                break;
            case K::DsRead4:  // DS op 0xff; addr, vdst << 24
            case K::DsRead2:  // DS op 0x76 (ds_read_b64)
                if (i.imm > 0xffffu) return bad("ds offset");
                w(0xd8000000u | ((i.k == K::DsRead4 ? 0xffu : 0x76u) << 17) | i.imm);
                w(static_cast<uint32_t>(i.b) | (static_cast<uint32_t>(i.a) << 24));
                break;
            case K::BufLoadLds4:  // MUBUF op 0x17 (dwordx4), lds = bit 16, nt = bit 17, offen, offset 0; soffset 0
                w(0xe0000000u | (0x17u << 18) | (i.sub ? 1u << 17 : 0u) | (1u << 16) | (1u << 12));
                w(0x80000000u | ((static_cast<uint32_t>(i.c) >> 2) << 16) | static_cast<uint32_t>(i.b));
                break;
        }
    }
    return true;
}

// SGPRs
constexpr int kSKarg = 0;      // s[0:1] kernarg segment pointer
constexpr int kSWgX = 2;       // workgroup id x: chunk
constexpr int kSWgY = 3;       // workgroup id y: launch stripe
constexpr int kSStripe = 4;    // stripe index (through stripe_ids)
constexpr int kSWave = 5;      // wave index in the workgroup
constexpr int kSGrp = 6;       // layout 1: s6 row group, s7 chunk group
constexpr int kSTmp = 8;       // s[8:11] scratch
constexpr int kSDescIn = 12;   // s[12:15] input buffer descriptor
constexpr int kSDescOut = 16;  // s[16:19] output buffer descriptor
constexpr int kSStage = 20;    // s[20:27] two (ptr lo, ptr hi, stride16, -) staging slots
constexpr int kSMask = 28;     // s[28:33] transpose masks
constexpr int kSgprs = 34;
// VGPRs
constexpr int kVTid = 0;       // work-item id
constexpr int kVOff = 1;       // lane's byte offset in the vectors (chunk * 2048 + 8 * lane)
// Transpose temporaries: the work-item id's register once the prologue has
// used it, and the last subset register (subsets are dead while columns and
// outputs are transposed, and no load ever targets it: the old outputs of
// accumulate mode go to slot registers 0-15 of the subset region at most).
// Two VGPRs fewer than dedicated temporaries: 16-row paths with two columns
// of loads in flight fit 168 VGPRs, i.e. 3 waves per SIMD without the cap.
constexpr int kVT0 = 0;
constexpr int kVSlots = 2;     // pf slots of 8 (64-bit aligned pairs)

const uint32_t kMasks[6] = {0x0F0F0F0Fu, 0xF0F0F0F0u, 0x33333333u, 0xCCCCCCCCu, 0x55555555u, 0xAAAAAAAAu};

struct Layout {
    int pf, slots_end, sub, acc, vgprs;
};

// In-place 8x8 bit transpose of v[r[0]..r[7]] (bs_transpose8, kernels.hip):
// swap(a, b, s, m): b = (m & (a >> s)) | (~m & b); a = ((m << s) & (b << s)) | (~(m << s) & a)
void transpose8(Prog& P, const int (&r)[8], int t1) {
    auto swap = [&](int a, int b, int s, int mi) {
        P.v_op2(kVLshr, kVT0, C(s), a);
        P.v_op2(kVLshl, t1, C(s), b);
        P.v_bfi(b, kSMask + mi, V(kVT0), V(b));
        P.v_bfi(a, kSMask + mi + 1, V(t1), V(a));
    };
    for (int i = 0; i < 4; ++i) swap(r[i], r[i + 4], 4, 0);
    swap(r[0], r[2], 2, 2);
    swap(r[1], r[3], 2, 2);
    swap(r[4], r[6], 2, 2);
    swap(r[5], r[7], 2, 2);
    for (int i = 0; i < 8; i += 2) swap(r[i], r[i + 1], 1, 4);
}

// The kernel's instructions for one matrix (see the file header and
// AsmShape, jit_asm.hpp).
Prog generate(const uint8_t* mat, int rows, int cols, bool acc, const AsmShape& sh, int pf, int sync,
              int* vgprs_out) {
    // layout 1 and 2: row groups over XCD-mapped workgroups; layout 2's
    // workgroup is nw waves with a path each over ONE chunk, sharing columns
    const bool by_group = sh.layout == 1 || sh.layout == 2;
    const bool grouped_share = sh.layout == 2;
    const int nw = sh.nw;
    const int rw = sh.rw;  // rows per code path (per wave in layouts 0 / 2, per workgroup in layout 1)
    const int npaths = (rows + rw - 1) / rw;
    const int G = grouped_share ? sh.groups : npaths;  // row groups (workgroups per chunk group)
    const int nsh = grouped_share ? nw : npaths;       // waves sharing a step's columns
    const bool share = sh.share && (!by_group || grouped_share) && nsh > 1;
    const int K = share && sh.kcols > 1 ? sh.kcols : 1;  // own columns per wave and step
    // (dma: each wave's columns stream into a private LDS ring D steps deep
    // through LDS-DMA loads - no VGPRs held by loads in flight)
    const int D = share && K == 1 && sh.dma >= 2 ? sh.dma : 0;
    const bool deep = share && sh.deep && K == 1 && !D;
    // (ahead: the next column's planes are read from LDS while this one
    // combines - deep does that too, with a second step of loads)
    const bool ahead = share && K == 1 && (deep || sh.ahead);
    const bool gray = sh.gray != 0;
    Layout L;
    // (share: one column of loads in flight per wave, i.e. nw columns of the
    // workgroup - two with deep; the planes read back from LDS get registers
    // of their own, two sets with deep; dma: no load registers, the raw bytes
    // are read from LDS into the plane registers and transposed there)
    L.pf = share ? (D ? 0 : deep ? 2 : K) : pf < 1 ? 1 : pf > 4 ? 4 : pf;
    L.slots_end = kVSlots + 8 * L.pf;
    const int kVPlanes = L.slots_end;
    // subset registers: the XORs of 2-4 planes of each half, 2 x 11; gray:
    // the high half's 11 and one for the low half's subset of the moment
    const int nsub = gray ? 12 : 22;
    L.sub = L.slots_end + (share ? (ahead ? 16 : 8) : 0);
    L.acc = L.sub + nsub;
    const int kVT1 = L.sub + nsub - 1;  // (see kVT0)
    L.vgprs = L.acc + 8 * rw;
    const int kVDma = L.vgprs;  // dma: the lane's LDS-DMA offsets, chunk * 2048 + 16 * lane (+ 1024)
    if (D) L.vgprs += 2;
    const uint32_t raw_base = static_cast<uint32_t>(2 * nsh * K * 2048);  // dma ring, after the plane buffers
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

    Prog P;
    P.ins.reserve(static_cast<size_t>(cols) * (80 + 8 * rw) * static_cast<size_t>(npaths) + 96);
    const int l_stripe_done = P.new_label(".Lstripe_done");
    const int l_idle = P.new_label(".Lidle");
    std::vector<int> l_path(static_cast<size_t>(npaths), -1);
    for (int w = 1; w < npaths; ++w)
        l_path[static_cast<size_t>(w)] = P.new_label((by_group ? ".Lgroup" : ".Lwave") + std::to_string(w));
    // ---- prologue: stripe, lane offset, wave, masks, descriptor constants
    P.s_load(kSDescIn + 2, 1, kSKarg, static_cast<uint32_t>(offsetof(AsmArgs, body)));
    P.s_load(kSTmp, 2, kSKarg, static_cast<uint32_t>(offsetof(AsmArgs, stripe_ids)));
    P.s_load(kSTmp + 3, 1, kSKarg, static_cast<uint32_t>(offsetof(AsmArgs, stripe0)));
    for (int i = 0; i < 6; ++i) P.s_mov_lit(kSMask + i, kMasks[i], true);
    P.s_mov_lit(kSDescIn + 3, 0x20000, false);
    P.s_mov_lit(kSDescOut + 3, 0x20000, false);
    P.v_op2(kVAnd, kVOff, C(63), kVTid);
    P.v_op2(kVLshl, kVOff, C(3), kVOff);
    if (!by_group) {
        P.s_op2(kLshl, kSTmp + 2, kSWgX, C(11));
        P.v_op2(kVAdd, kVOff, kSTmp + 2, kVOff);
    }
    // wave id = bits 6-9 of the work-item id (packed work-item ids: y / z sit
    // in bits 10-29; zero for these 1-D launches, masked anyway)
    P.v_op2(kVAnd, kVT0, kLit, kVTid, 0x3c0);
    P.v_op2(kVLshr, kVT0, C(6), kVT0);
    // a VALU write of a VGPR followed at once by v_readfirstlane of it reads
    // the OLD value (one wait state required; measured: the wave id came out
    // as 64, not 1, tools/asm_probe/wave_id.s)
    P.s_nop(1);
    P.v_readlane(kSWave, kVT0);
    P.wait_lgkm0();
    P.s_mov(kSDescOut + 2, kSDescIn + 2);
    P.s_op2(kAdd, kSStripe, kSWgY, kSTmp + 3);  // stripe0 + y
    P.s_cmp(kEq64, kSTmp, C(0));
    P.branch(kScc1, l_stripe_done);
    P.s_op2(kLshl, kSTmp + 2, kSStripe, C(2));
    P.s_op2(kAdd, kSTmp, kSTmp, kSTmp + 2);
    P.s_op2(kAddc, kSTmp + 1, kSTmp + 1, C(0));
    P.s_load(kSStripe, 1, kSTmp, 0);
    P.wait_lgkm0();
    P.label(l_stripe_done);
    P.s_nop(4);  // (v_readfirstlane -> SGPR read hazard margin)
    if (by_group) {
        // Layout 1: workgroup x -> (chunk group cg, row group g) with the row
        // groups of one chunk group on one XCD, back to back in its dispatch
        // order (the hardware hands workgroup x to XCD x % 8):
        //   x = ((cg / 8) * G + g) * 8 + cg % 8
        // so the G workgroups reading the same input lines share that XCD's
        // L2.  Wave w of the workgroup takes chunk cg * NW + w (layout 2: all
        // waves take chunk cg, one path each: path g * NW + w).
        P.s_op2(kAnd, kSGrp + 1, kSWgX, C(7));       // cg % 8
        P.s_op2(kLshr, kSTmp, kSWgX, C(3));          // q = x / 8
        if (G > 1 && (G & (G - 1)) == 0) {
            int lg = 0;
            while ((1 << lg) < G) ++lg;
            P.s_op2(kAnd, kSGrp, kSTmp, C(G - 1));      // g = q % G
            P.s_op2(kLshr, kSTmp, kSTmp, C(lg));         // q / G
        } else if (G > 1) {
            // cg / 8 = q / G: multiply by ceil(2^32 / G) (exact for q < 2^29 / G)
            const uint32_t magic = static_cast<uint32_t>(((uint64_t{1} << 32) + G - 1) / G);
            P.s_op2(kMulhi, kSTmp + 1, kSTmp, kLit, magic);
            P.s_op2(kMul, kSTmp + 2, kSTmp + 1, C(G));
            P.s_op2(kSub, kSGrp, kSTmp, kSTmp + 2);    // g = q - (q / G) * G
            P.s_mov(kSTmp, kSTmp + 1);
        }  // (G == 1: a single path, no dispatch on g)
        P.s_op2(kLshl, kSTmp, kSTmp, C(3));
        P.s_op2(kOr, kSGrp + 1, kSGrp + 1, kSTmp);   // cg
        // chunk groups past the vector body: nothing to do
        int lg_nw = 0;
        while (!grouped_share && (1 << lg_nw) < nw) ++lg_nw;
        P.s_op2(kAdd, kSTmp, kSDescIn + 2, kLit, static_cast<uint32_t>((2048u << lg_nw) - 1));
        P.s_op2(kLshr, kSTmp, kSTmp, C(11 + lg_nw));
        const int l_go = P.new_label(".Lgo");
        P.s_cmp(kGe32, kSGrp + 1, kSTmp);
        P.branch(kScc0, l_go);  // (.Lidle lies past all the code: out of branch range)
        P.s_endpgm();
        P.label(l_go);
        if (grouped_share) {
            // lane offset = (cg << 11) + 8 * lane; path = g * NW + wave
            if (G == 1) P.s_mov_lit(kSGrp, 0, false);
            P.s_op2(kLshl, kSTmp, kSGrp + 1, C(11));
            P.v_op2(kVAdd, kVOff, kSTmp, kVOff);
            P.s_op2(kMul, kSTmp, kSGrp, C(nw));
            P.s_op2(kAdd, kSGrp, kSTmp, kSWave);
        } else {
            // lane offset = ((cg * NW + wave) << 11) + 8 * lane
            P.s_op2(kLshl, kSTmp, kSGrp + 1, C(lg_nw));
            P.s_op2(kAdd, kSTmp, kSTmp, kSWave);
            P.s_op2(kLshl, kSTmp, kSTmp, C(11));
            P.v_op2(kVAdd, kVOff, kSTmp, kVOff);
        }
    }
    if (D) {
        P.v_op2(kVAnd, kVDma, kLit, kVOff, 0x1f8);        // 8 * lane
        P.v_op2(kVAdd, kVDma, V(kVOff), kVDma);            // chunk * 2048 + 16 * lane
        P.v_op2(kVAdd, kVDma + 1, kLit, kVDma, 1024);
    }
    // path p (layout 0: wave p; layout 1: row group p) -> its rows' code
    // (long jumps: a path's straight-line code can exceed the 16-bit branch
    // range); waves without rows leave
    const int sel = by_group ? kSGrp : kSWave;
    const int nsel = by_group ? npaths : nw;
    for (int w = 1; w < nsel; ++w) {
        const int tgt = w < npaths ? l_path[static_cast<size_t>(w)] : l_idle;
        const int l_not = P.new_label(".Lnot" + std::to_string(w));
        const int l_pc = P.new_label(".Lpc" + std::to_string(w));
        P.s_cmp(kEq32, sel, C(w));
        P.branch(kScc0, l_not);
        P.s_getpc(kSTmp);
        P.label(l_pc);
        P.add_pcrel(kLo, kSTmp, tgt, l_pc);
        P.add_pcrel(kHi, kSTmp + 1, tgt, l_pc);
        P.s_setpc(kSTmp);
        P.label(l_not);
    }

    for (int w = 0; w < npaths; ++w) {
        const int r0 = w * rw, nr = std::min(rw, rows - r0);
        if (nr <= 0) break;
        if (w) P.label(l_path[static_cast<size_t>(w)]);
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
            P.wait_vm(after > 63 ? 63 : after);
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
            P.s_load(s, 2, kSKarg, static_cast<uint32_t>(offsetof(AsmArgs, ptr) + 8 * v));
            P.s_load(s + 2, 1, kSKarg, static_cast<uint32_t>(offsetof(AsmArgs, stride16) + 4 * v));
        };
        // descriptor base = ptr + stripe * stride16 * 16, from stage slot `st`
        auto desc = [&](int st, int d) {
            const int s = kSStage + 4 * st;
            P.wait_lgkm0();
            P.s_op2(kMul, kSTmp, kSStripe, s + 2);
            P.s_op2(kMulhi, kSTmp + 1, kSStripe, s + 2);
            P.s_op2(kLshl64, kSTmp, kSTmp, C(4));
            P.s_op2(kAdd, d, s, kSTmp);
            P.s_op2(kAddc, d + 1, s + 1, kSTmp + 1);
            P.s_op2(kAnd, d + 1, d + 1, kLit, 0xffff);
        };
        auto slot_reg = [&](int c, int j) { return kVSlots + 8 * (c % L.pf) + j; };
        std::vector<int> col_id(static_cast<size_t>(cols), -1);  // last VMEM op of each column's loads
        // an input line read by one wave only is streamed (nt); lines other
        // waves read too (layout 0 with several waves: the same chunk;
        // layout 1 with several row groups: the other groups' workgroups on
        // the same XCD) stay cached for them (measured with nt: 64+64 Encode
        // fetched 1.45x its input bytes from HBM, 128+128 2.8x;
        // profiles/r03/pmc_traffic_*.json)
        const bool in_nt = npaths == 1 || (share && G == 1) || (share && !grouped_share);
        // the columns this wave loads, in order: all of them, or (share) its
        // own column of each step, w, w + nw, ...
        const int wi = grouped_share ? w % nw : w;  // this path's wave in its workgroup
        const int c_first = share ? wi : 0, c_step = share ? nsh : 1;
        auto issue_col = [&](int c) {  // stage(c) was issued into slot (c / c_step) & 1
            const int k_ = c / c_step;
            desc(k_ & 1, kSDescIn);
            if (c + c_step < cols) stage(c + c_step, (k_ + 1) & 1);
            for (int k = 0; k < 4; ++k) {
                P.buf_load2(slot_reg(k_, 2 * k), kVOff, kSDescIn, 512 * k, in_nt);
                vq.push_back(next_id);
                col_id[static_cast<size_t>(c)] = next_id++;
            }
        };
        // dma: column c = c_first + k_ * c_step streams into this wave's ring
        // slot k_ % D (2 KiB as two LDS-DMA loads of 1 KiB, lane-linear)
        auto dma_slot = [&](int k_) { return raw_base + static_cast<uint32_t>(((k_ % std::max(D, 1)) * nsh + wi) * 2048); };
        auto issue_dma = [&](int c) {  // stage(c) was issued into slot (c / c_step) & 1
            const int k_ = c / c_step;
            desc(k_ & 1, kSDescIn);
            if (c + c_step < cols) stage(c + c_step, (k_ + 1) & 1);
            for (int h = 0; h < 2; ++h) {
                P.s_mov_lit(kM0, dma_slot(k_) + 1024u * static_cast<uint32_t>(h), false);
                P.s_nop(0);  // (M0 write -> LDS-DMA: one wait state)
                P.buf_load_lds4(kVDma + h, kSDescIn, in_nt);
                vq.push_back(next_id);
                col_id[static_cast<size_t>(c)] = next_id++;
            }
        };
        if (c_first < cols) {
            stage(c_first, 0);
            if (D) {
                for (int k_ = 0; k_ < D - 1 && c_first + k_ * c_step < cols; ++k_) issue_dma(c_first + k_ * c_step);
            } else {
                for (int k_ = 0; k_ < L.pf && c_first + k_ * c_step < cols; ++k_) issue_col(c_first + k_ * c_step);
            }
        }
        // subset m of a half (2-4 of its planes) -> one of 11 registers (the
        // single planes stay where the transpose left them)
        auto sub_reg = [&](int half, int m) {
            static const int8_t kIdx[16] = {-1, -1, -1, 0, -1, 1, 2, 3, -1, 4, 5, 6, 7, 8, 9, 10};
            return L.sub + (gray ? 0 : half * 11) + kIdx[m];
        };
        auto acc_reg = [&](int r, int i) { return L.acc + 8 * r + i; };
        // output plane (r, i) ^= the column's terms t[0..nt) (the first column sets it)
        auto update = [&](int c, int r, int i, const int* t, int nt) {
            const int a = acc_reg(r - r0, i);
            if (c == 0) {
                if (nt == 0) P.v_mov(a, C(0));
                else if (nt == 1) P.v_mov(a, V(t[0]));
                else P.v_op2(kVXor, a, V(t[0]), t[1]);
            } else if (nt == 2) {
                P.v_xor3(a, a, t[0], t[1]);
            } else if (nt == 1) {
                P.v_op2(kVXor, a, V(a), t[0]);
            }
        };
        // column c's planes in pr[]: its subsets of each half that this
        // path's rows use, then one xor3 per output plane and row
        auto combine = [&](int c, const int (&pr)[8]) {
            int reg[2][16];
            for (int half = gray ? 1 : 0; half < 2; ++half) {
                bool have[16] = {}, used[16] = {}, need[16] = {};
                for (int b = 0; b < 4; ++b) {
                    have[1 << b] = true;
                    reg[half][1 << b] = pr[4 * half + b];
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
                        P.v_op2(kVXor, dst, V(reg[half][rest]), reg[half][low]);
                        reg[half][m] = dst;
                        have[m] = true;
                    }
            }
            if (!gray) {
                for (int r = r0; r < r0 + nr; ++r)
                    for (int i = 0; i < 8; ++i) {
                        const int m = mask[(static_cast<size_t>(c) * rows + r) * 8 + i];
                        int t[2];
                        int nt = 0;
                        if (m & 15) t[nt++] = reg[0][m & 15];
                        if (m >> 4) t[nt++] = reg[1][m >> 4];
                        update(c, r, i, t, nt);
                    }
                return;
            }
            // gray: the outputs grouped by their low-half subset; the subsets
            // visited in Gray-code order, each built in register tl with one
            // XOR / xor3 from the one before or from the planes (single planes
            // are used where they are), its outputs updated right after
            std::vector<std::pair<int, int>> by_lo[16];
            for (int r = r0; r < r0 + nr; ++r)
                for (int i = 0; i < 8; ++i)
                    by_lo[mask[(static_cast<size_t>(c) * rows + r) * 8 + i] & 15].emplace_back(r, i);
            const int tl = L.sub + 11;
            static const int kGray[15] = {1, 3, 2, 6, 7, 5, 4, 12, 13, 15, 14, 10, 11, 9, 8};
            int cur = 0;  // the subset tl holds (0: none)
            for (int gi = -1; gi < 15; ++gi) {
                const int a = gi < 0 ? 0 : kGray[gi];
                if (by_lo[a].empty()) continue;
                int src = -1;
                if (a && (a & (a - 1)) == 0) {
                    src = pr[__builtin_ctz(static_cast<unsigned>(a))];
                } else if (a) {
                    int b[4], nb = 0;
                    const int d = a ^ cur;
                    if (cur && __builtin_popcount(static_cast<unsigned>(d)) <= 2) {
                        for (int x = 0; x < 4; ++x)
                            if (d >> x & 1) b[nb++] = pr[x];
                        if (nb == 1) P.v_op2(kVXor, tl, V(tl), b[0]);
                        else P.v_xor3(tl, tl, b[0], b[1]);
                    } else {
                        for (int x = 0; x < 4; ++x)
                            if (a >> x & 1) b[nb++] = pr[x];
                        if (nb == 2) {
                            P.v_op2(kVXor, tl, V(b[0]), b[1]);
                        } else {
                            P.v_xor3(tl, b[0], b[1], b[2]);
                            if (nb == 4) P.v_op2(kVXor, tl, V(tl), b[3]);
                        }
                    }
                    cur = a;
                    src = tl;
                }
                for (const auto& ri : by_lo[a]) {
                    const int m = mask[(static_cast<size_t>(c) * rows + ri.first) * 8 + ri.second];
                    int t[2];
                    int nt = 0;
                    if (src >= 0) t[nt++] = src;
                    if (m >> 4) t[nt++] = reg[1][m >> 4];
                    update(c, ri.first, ri.second, t, nt);
                }
            }
        };
        if (!share) {
            for (int c = 0; c < cols; ++c) {
                vmem_wait_for(col_id[static_cast<size_t>(c)]);
                int pr[8];
                for (int j = 0; j < 8; ++j) pr[j] = slot_reg(c, j);
                transpose8(P, pr, kVT1);
                combine(c, pr);
                if (c + L.pf < cols) issue_col(c + L.pf);  // the slot is free again
                // keep the waves within `sync` columns of each other, so the lines
                // the first wave fetched are still cached when the others load
                // them (layout 0; in layout 1 every wave of a workgroup runs the
                // same path, so the barriers match there too)
                if (nw > 1 && sync > 0 && (c + 1) % sync == 0 && c + 1 < cols) P.s_barrier();
            }
        } else {
            // Step s: this wave transposes its column s * nw + w into LDS
            // buffer s & 1 (lane t's 8 planes as two 16-byte pieces, 1 KiB
            // apart), loads its next column, and after the barrier combines the
            // step's nw columns from LDS into its rows.  One barrier per step
            // also frees buffer s & 1 for step s + 2: every wave has combined
            // step s before it passes the barrier of step s + 1.  With K > 1
            // (AsmShape::kcols) a step is K columns per wave (half the barriers),
            // column s * nw * K + q * nw + w being the wave's q-th of the step.
            const int per = nsh * K;
            const int steps = (cols + per - 1) / per;
            for (int st = 0; st < steps; ++st) {
                const uint32_t buf = static_cast<uint32_t>(st & 1) * static_cast<uint32_t>(per) * 2048u;
                for (int q = 0; q < K; ++q) {
                    const int c = st * per + q * nsh + wi, k_ = st * K + q;
                    if (c >= cols) break;
                    if (D) {
                        // the column D - 1 steps ahead into the ring slot this
                        // wave read (and waited for) in the previous step
                        if (c + (D - 1) * c_step < cols) issue_dma(c + (D - 1) * c_step);
                        vmem_wait_for(col_id[static_cast<size_t>(c)]);
                        // lane t's four 8-byte pieces (8 t + 512 k) from the ring slot
                        P.v_op2(kVAnd, kVT0, kLit, kVOff, 0x1f8);
                        P.v_op2(kVAdd, kVT0, kLit, kVT0, dma_slot(k_));
                        for (int k = 0; k < 4; ++k) P.ds_read2(kVPlanes + 2 * k, kVT0, 512u * static_cast<uint32_t>(k));
                        P.wait_lgkm0();
                    } else if (sh.nobar < 2) {
                        vmem_wait_for(col_id[static_cast<size_t>(c)]);
                    }
                    int pr[8];
                    for (int j = 0; j < 8; ++j) pr[j] = D ? kVPlanes + j : slot_reg(k_, j);
                    transpose8(P, pr, kVT1);
                    // LDS address of lane t: 16 t (kVT0 is free between transposes)
                    P.v_op2(kVAnd, kVT0, kLit, kVOff, 0x1f8);
                    P.v_op2(kVLshl, kVT0, C(1), kVT0);
                    const uint32_t off = buf + static_cast<uint32_t>(q * nsh + wi) * 2048u;
                    P.ds_write4(kVT0, pr[0], off);
                    P.ds_write4(kVT0, pr[4], off + 1024u);
                    if (sh.nobar < 3) P.wait_lgkm0();  // (the slot registers are read before the next load lands in them)
                    if (!D && c + L.pf * nsh < cols) {
                        issue_col(c + L.pf * nsh);
                        // (its scalar loads back before the LDS reads below, so
                        // lgkmcnt counts LDS reads only, in order)
                        if (deep) P.wait_lgkm0();
                    }
                }
                if (st * per + wi >= cols) {  // no column of this wave in the step: the address still
                    P.v_op2(kVAnd, kVT0, kLit, kVOff, 0x1f8);
                    P.v_op2(kVLshl, kVT0, C(1), kVT0);
                }
                if (!sh.nobar) P.s_barrier();
                const int ncol = std::min(per, cols - st * per);
                auto read = [&](int j) {
                    const uint32_t off = buf + static_cast<uint32_t>(j) * 2048u;
                    const int d = kVPlanes + (ahead ? 8 * (j & 1) : 0);
                    P.ds_read4(d, kVT0, off);
                    P.ds_read4(d + 4, kVT0, off + 1024u);
                };
                read(0);
                for (int j = 0; j < ncol; ++j) {
                    if (ahead && j + 1 < ncol) {
                        // the next column's planes arrive while this one combines
                        // (a count of LDS reads only: the scalar loads still out
                        // are staging, not waited for here, and LDS reads return
                        // in order, so 2 outstanding means read(j) is in)
                        read(j + 1);
                        if (sh.nobar < 3) P.wait_lgkm(2);
                    } else if (sh.nobar < 3) {
                        P.wait_lgkm0();
                    }
                    int pr[8];
                    for (int q = 0; q < 8; ++q) pr[q] = kVPlanes + (ahead ? 8 * (j & 1) : 0) + q;
                    combine(st * per + j, pr);
                    if (!ahead && j + 1 < ncol) read(j + 1);
                }
            }
        }
        // ---- outputs: transpose back, (accumulate: XOR the old bytes), store
        int ostage = 0;
        stage(cols + r0, ostage);
        std::vector<int> old_id(static_cast<size_t>(nr), -1);
        auto old_reg = [&](int r, int j) { return kVSlots + 8 * (r % 2) + j; };  // pf >= 1: 8 regs; 2 rows need 16
        auto issue_old = [&](int r) {  // descriptor of row r is in kSDescOut
            for (int k = 0; k < 4; ++k) {
                P.buf_load2(old_reg(r, 2 * k), kVOff, kSDescOut, 512 * k, false);
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
                transpose8(P, pr, kVT1);
                vmem_wait_for(old_id[static_cast<size_t>(r)]);
                for (int j = 0; j < 8; ++j) P.v_op2(kVXor, pr[j], V(pr[j]), old_reg(r, j));
            } else {
                transpose8(P, pr, kVT1);
            }
            for (int k = 0; k < 4; ++k) {
                P.buf_store2(pr[2 * k], kVOff, kSDescOut, 512 * k);
                vq.push_back(next_id++);
            }
        }
        P.s_endpgm();
    }
    P.label(l_idle);
    P.s_endpgm();
    return P;
}

// VGPRs the kernel declares: what it uses, or more for the occupancy cap
// (512 VGPRs per SIMD lane, allocated in granules of 8).
int declared_vgprs(int used, int max_waves) {
    int accum = (used + 3) / 4 * 4;
    if (max_waves > 1 && max_waves <= 8) accum = std::max(accum, std::min(256, 512 / max_waves / 8 * 8));
    return accum;
}

// Kernel descriptor and metadata (code object v6) of a kernel named rs_bs_asm.
std::string descriptor(int nw, int accum, int lds) {
    char kd[2048];
    std::string s;
    std::snprintf(kd, sizeof kd,
                  "\t.rodata\n\t.p2align\t6\n\t.amdhsa_kernel rs_bs_asm\n"
                  "\t\t.amdhsa_group_segment_fixed_size %d\n\t\t.amdhsa_private_segment_fixed_size 0\n"
                  "\t\t.amdhsa_kernarg_size %zu\n\t\t.amdhsa_user_sgpr_count 2\n"
                  "\t\t.amdhsa_user_sgpr_kernarg_segment_ptr 1\n"
                  "\t\t.amdhsa_system_sgpr_workgroup_id_x 1\n\t\t.amdhsa_system_sgpr_workgroup_id_y 1\n"
                  "\t\t.amdhsa_system_vgpr_workitem_id 0\n"
                  "\t\t.amdhsa_next_free_vgpr %d\n\t\t.amdhsa_next_free_sgpr %d\n\t\t.amdhsa_accum_offset %d\n"
                  "\t\t.amdhsa_reserve_vcc 0\n\t\t.amdhsa_ieee_mode 1\n\t\t.amdhsa_dx10_clamp 1\n"
                  "\t.end_amdhsa_kernel\n",
                  lds, sizeof(AsmArgs), accum, kSgprs, accum);
    s += kd;
    std::snprintf(kd, sizeof kd,
                  "\t.amdgpu_metadata\n---\namdhsa.kernels:\n  - .agpr_count: 0\n    .args:\n"
                  "      - .offset: 0\n        .size: %zu\n        .value_kind: by_value\n"
                  "    .group_segment_fixed_size: %d\n    .kernarg_segment_align: 8\n"
                  "    .kernarg_segment_size: %zu\n    .max_flat_workgroup_size: %d\n    .name: rs_bs_asm\n"
                  "    .private_segment_fixed_size: 0\n    .sgpr_count: %d\n    .sgpr_spill_count: 0\n"
                  "    .symbol: rs_bs_asm.kd\n    .uniform_work_group_size: 1\n    .vgpr_count: %d\n"
                  "    .vgpr_spill_count: 0\n    .wavefront_size: 64\n"
                  "amdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n"
                  "\t.end_amdgpu_metadata\n",
                  sizeof(AsmArgs), lds, sizeof(AsmArgs), 64 * nw, kSgprs + 6, accum);
    s += kd;
    return s;
}

const char* const kHeader =
    "\t.amdgcn_target \"amdgcn-amd-amdhsa--gfx950\"\n\t.amdhsa_code_object_version 6\n\t.text\n"
    "\t.globl\trs_bs_asm\n\t.p2align\t8\n\t.type\trs_bs_asm,@function\nrs_bs_asm:\n";
const char* const kTrailer = ".Lfunc_end0:\n\t.size\trs_bs_asm, .Lfunc_end0-rs_bs_asm\n";

// ---------------------------------------------------------------- ELF

struct Elf64Ehdr {
    unsigned char ident[16];
    uint16_t type, machine;
    uint32_t version;
    uint64_t entry, phoff, shoff;
    uint32_t flags;
    uint16_t ehsize, phentsize, phnum, shentsize, shnum, shstrndx;
};
struct Elf64Shdr {
    uint32_t name, type;
    uint64_t flags, addr, offset, size;
    uint32_t link, info;
    uint64_t addralign, entsize;
};

// File offset and size of the section named `want` in an ELF64 image.
bool elf_section(const std::vector<char>& elf, const char* want, size_t* off, size_t* size) {
    if (elf.size() < sizeof(Elf64Ehdr) || std::memcmp(elf.data(), "\x7f" "ELF", 4) != 0 || elf[4] != 2) return false;
    Elf64Ehdr eh;
    std::memcpy(&eh, elf.data(), sizeof eh);
    if (eh.shentsize != sizeof(Elf64Shdr) || eh.shstrndx >= eh.shnum ||
        eh.shoff + static_cast<uint64_t>(eh.shnum) * sizeof(Elf64Shdr) > elf.size())
        return false;
    auto sh = [&](int i) {
        Elf64Shdr s;
        std::memcpy(&s, elf.data() + eh.shoff + static_cast<size_t>(i) * sizeof(Elf64Shdr), sizeof s);
        return s;
    };
    const Elf64Shdr strs = sh(eh.shstrndx);
    for (int i = 0; i < eh.shnum; ++i) {
        const Elf64Shdr s = sh(i);
        if (strs.offset + s.name + std::strlen(want) + 1 > elf.size()) continue;
        if (std::strcmp(elf.data() + strs.offset + s.name, want) == 0) {
            if (s.offset + s.size > elf.size()) return false;
            *off = s.offset;
            *size = s.size;
            return true;
        }
    }
    return false;
}

// Code-object templates: the kernel descriptor and metadata for (waves per
// workgroup, declared VGPRs, LDS bytes) and a .text of `bytes` filled with s_endpgm,
// assembled by comgr once per process and shape.
struct Template {
    std::vector<char> elf;
    size_t text_off = 0, text_size = 0;
};
std::mutex g_tmpl_mu;
std::map<std::tuple<int, int, size_t, int>, Template>& templates() {
    static auto* m = new std::map<std::tuple<int, int, size_t, int>, Template>;
    return *m;
}

}  // namespace

std::string asm_source(const uint8_t* mat, int rows, int cols, bool acc, const AsmShape& sh, int pf, int sync,
                       int max_waves, int* vgprs_out) {
    int used = 0;
    const Prog P = generate(mat, rows, cols, acc, sh, pf, sync, &used);
    if (vgprs_out) *vgprs_out = used;
    return kHeader + print(P) + kTrailer + descriptor(sh.nw, declared_vgprs(used, max_waves), asm_lds_bytes(sh));
}

bool asm_binary(const uint8_t* mat, int rows, int cols, bool acc, const AsmShape& sh, int pf, int sync,
                std::vector<uint32_t>* code, int* vgprs_out, std::string* err) {
    int used = 0;
    const Prog P = generate(mat, rows, cols, acc, sh, pf, sync, &used);
    if (vgprs_out) *vgprs_out = used;
    return encode(P, code, err);
}

bool asm_text_section(const std::vector<char>& elf, std::vector<char>* text) {
    size_t off = 0, size = 0;
    if (!elf_section(elf, ".text", &off, &size)) return false;
    text->assign(elf.begin() + static_cast<long>(off), elf.begin() + static_cast<long>(off + size));
    return true;
}

bool asm_link_binary(const std::vector<uint32_t>& code, const AsmShape& sh, int vgprs_used, int max_waves,
                     std::vector<char>* elf, std::string* log, double* ms) {
    const auto t0 = std::chrono::steady_clock::now();
    const size_t need = code.size() * 4;
    size_t cls = size_t{16} << 10;
    while (cls < need) cls <<= 1;
    const int accum = declared_vgprs(vgprs_used, max_waves);
    const Template* t = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_tmpl_mu);
        const int lds = asm_lds_bytes(sh);
        auto key = std::make_tuple(sh.nw, accum, cls, lds);
        auto it = templates().find(key);
        if (it == templates().end()) {
            std::string src = kHeader;
            src += "\t.fill " + std::to_string(cls / 4) + ", 4, 0xbf810000\n";  // s_endpgm
            src += kTrailer + descriptor(sh.nw, accum, lds);
            Template nt;
            double ams = 0;
            if (!asm_assemble(src, &nt.elf, log, &ams) || !elf_section(nt.elf, ".text", &nt.text_off, &nt.text_size) ||
                nt.text_size < cls) {
                if (log && log->empty()) *log = "code-object template: no .text of the expected size";
                return false;
            }
            it = templates().emplace(key, std::move(nt)).first;
        }
        t = &it->second;  // (entries are never erased)
    }
    *elf = t->elf;
    std::memcpy(elf->data() + t->text_off, code.data(), need);
    if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return true;
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
        if (!log || amd_comgr_action_data_count(set, AMD_COMGR_DATA_KIND_LOG, &n) != AMD_COMGR_STATUS_SUCCESS) return;
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
