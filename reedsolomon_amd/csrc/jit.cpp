// jit.cpp — run-time generated bit-sliced kernels (hiprtc) for products with
// 5-16 output rows whose matrix is only known at run time.
//
// Why: above 4 output rows the perm-table kernels are VALU-bound (10+8 @ 1 MiB
// Reconst of 8: 5.05-5.18 TB/s, profiles/r02/pmc_sq_10_8.json), while the
// bit-sliced networks generated at build time for fixed generator matrices
// (tools/gen_bitslice.py, gf_bitslice in kernels.hip) need ~22 VALU per
// (column, dword) against ~40 and run at 6.1-6.3 TB/s.  A network needs its
// matrix at code-generation time: selecting subset XORs by a run-time index
// costs a register gather per term (counted at ~40 VALU), so
// the matrix is baked into the code instead — here, at run time.
//
// The generator is the C++ form of tools/gen_bitslice.py: a lane owns 32 bytes
// of every vector as 8 bit-planes (8x8 SWAR transpose); multiplying by a
// constant is GF(2)-linear, so output plane i of row r is a fixed XOR of input
// planes; per column the XORs of each 4-plane half's subsets are formed once
// and every output plane takes one subset of each half (xor3).  Accumulate
// mode (Update / Replace) XORs the old output bytes in after the back
// transpose.
//
// Flow: first sight of a (device, matrix, mode) in a launch moving at least
// jit_min_bytes queues a compile on a worker thread (hiprtc only: the worker
// makes no HIP runtime calls); launches keep taking the perm-table kernels
// until the code object is ready; the launching thread then loads it
// (hipModuleLoadData) and from there on launches the bit-sliced kernel.
// rs_tune("jit", 2) compiles on the launching thread instead.
//
// Code objects persist across processes in an on-disk cache
// (RSAMD_JIT_CACHE_DIR, default $XDG_CACHE_HOME/rsamd/jit or
// ~/.cache/rsamd/jit; rs_tune("jit_disk_cache", 0) turns it off): a file per
// (device arch, hiprtc version, generator version, prelude, argument layout,
// mode, prefetch distance, matrix).  The first sight of a matrix whose code
// object is on disk loads it on the launching thread and launches the
// compiled kernel right away, whatever the launch history: a restarted
// server pays no compile for the matrices it has seen before.  Files are
// written atomically (temporary file + rename) and checked on load (magic,
// two independent key hashes, length, a checksum of the code, ELF magic);
// anything else is ignored and recompiled.  The directory must be the
// user's own and not group / world-writable, and so must each file (created
// 0700 / 0600): otherwise the cache is neither read nor written.
#include "jit.hpp"

#include <hip/hiprtc.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <pthread.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdlib>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <cmath>
#include <mutex>
#include <set>
#include <shared_mutex>
#include <thread>
#include <vector>

#include "jit_asm.hpp"
#include "rs_amd.h"

namespace rsamd {

int g_jit_mode = [] {
    const char* e = std::getenv("RSAMD_JIT");
    return e ? std::atoi(e) : 1;
}();
uint64_t g_jit_min_bytes = uint64_t{8} << 20;
int g_jit_min_launches = 2;
int g_jit_min_rows = kJitMinRows;
int g_jit_min_acc_cols = kJitMinAccCols;
int g_jit_sync = 0;  // rs_tune("jit_sync", n): multi-wave assembly kernels meet at a barrier every n columns (0: never)
// rs_tune("jit_waves", n): assembly kernels declare enough VGPRs to hold at
// most n waves per SIMD (0: as many as their registers allow).  Default 2:
// fewer 2 KiB chunks in flight per CU; 4-15 % faster on every shape measured,
// in-place Reconst most (10+8 of 5: 5.34 -> 6.13 TB/s, profiles/r03/ab_jit_waves.log)
// (env RSAMD_JIT_WAVES)
int g_jit_waves = [] {
    const char* e = std::getenv("RSAMD_JIT_WAVES");
    return e ? std::atoi(e) : 2;
}();
// rs_tune("jit_layout", 0 | 1) / ("jit_group_waves", 1..8): how generated
// kernels of more than 16 rows split their work (AsmShape, jit_asm.hpp):
// rows over the waves of a workgroup (0), row groups over workgroups whose
// waves take consecutive chunks with the same code (1, group_waves waves), or
// (2, the default) as 0 up to group_waves paths and beyond that row groups of
// shared-column workgroups of at most group_waves waves, several per CU:
// 128+128 Encode 1.94 -> 2.00 TB/s; 2-wave groups were slower on 64+64 /
// 200+56 (profiles/r05/ab_layout2_*.log)
int g_jit_layout = [] {
    const char* e = std::getenv("RSAMD_JIT_LAYOUT");
    const int v = e ? std::atoi(e) : 2;
    return v == 1 || v == 2 ? v : 0;
}();
int g_jit_group_waves = 4;
// rs_tune("jit_path_rows", 1..16): rows per code path of generated kernels of
// more than 16 rows (each row holds 8 VGPR accumulators)
int g_jit_path_rows = 16;
// rs_tune("jit_share", 0 | 1): generated kernels of several waves (layout 0)
// share each column's load and transpose through LDS (AsmShape::share):
// 32+32 / 64+64 / 128+128 / 200+56 Encode 4.79 / 2.94 / 1.56 / 2.11 ->
// 5.33 / 3.68 / 2.02 / 2.85 TB/s (profiles/r04/ab_share.log)
int g_jit_share = 1;
// rs_tune("jit_share_deep", -1 | 0 | 1): shared-column kernels with two steps
// of loads in flight and the next column's planes read from LDS ahead
// (-1: for 8-wave workgroups only).  Default off: within 1 % on 128+128 and
// 1-9 % slower elsewhere (fewer waves per SIMD; profiles/r04/ab_share_deep.log)
int g_jit_share_deep = 0;
// rs_tune("jit_split_cols", n): products of 9-16 rows over at least n columns
// run as two 8-row paths of one workgroup, sharing the columns (0: never)
int g_jit_split_cols = 0;
static bool jit_split_small(int rows, int cols) {
    return g_jit_split_cols > 0 && rows > 8 && rows <= 16 && cols >= g_jit_split_cols;
}
// rs_tune("jit_share_cols", 1 | 2 | -1): columns each wave of a shared-column
// kernel loads per step, i.e. one barrier per nw x n columns (-1: 2 for 8-wave
// workgroups, whose occupancy the 8 extra VGPRs do not change)
int g_jit_share_cols = 1;
// rs_tune("jit_share_dma", 0 | 2..8): shared-column kernels stream each wave's
// columns into an LDS ring of n steps by LDS-DMA loads (n - 1 steps ahead, no
// load registers) instead of one step ahead through VGPRs; 0 = off
int g_jit_share_dma = 0;
// rs_tune("jit_share_ahead", 0 | 1): shared-column kernels read the next
// column's planes from LDS while the current one combines (8 more VGPRs)
int g_jit_share_ahead = 0;
// rs_tune("jit_gray", 0 | 1): generated kernels build the low half's subsets
// one at a time in Gray-code order (12 subset registers instead of 22)
int g_jit_gray = 0;
// rs_tune("jit_nobar", 1), experiments build only: a timing diagnostic that
// drops the shared-column barriers (the results are wrong)
int g_jit_nobar = 0;
AsmShape jit_shape(int rows, int cols) {
    AsmShape s = asm_shape(rows, g_jit_layout, g_jit_group_waves, g_jit_path_rows, g_jit_share, g_jit_share_deep,
                           jit_split_small(rows, cols) ? 1 : 0, g_jit_share_cols, g_jit_share_dma, g_jit_share_ahead,
                           g_jit_gray);
    s.nobar = g_jit_nobar;
    return s;
}
int g_jit_pf = 3;  // rs_tune("jit_pf", 1..6): columns whose loads are in flight ahead of the one combined
// Generated kernels of more than 16 rows (several code paths): two columns of
// loads in flight and at most 3 waves per SIMD (their 16-row paths fit 168
// VGPRs then): 32+32 Encode +4 %, 64+64 +7 %, 128+128 +5 % over the
// single-path settings, which lose 2.5 % on 16+16 (profiles/r04/ab_wide_waves3.log);
// rs_tune("jit_wide_pf") / ("jit_wide_waves")
int g_jit_wide_pf = 2;
int g_jit_wide_waves = 3;
int jit_pf_for(int rows, int cols) { return rows > 16 || jit_split_small(rows, cols) ? g_jit_wide_pf : g_jit_pf; }
int jit_waves_for(int rows, int cols) {
    return rows > 16 || jit_split_small(rows, cols) ? g_jit_wide_waves : g_jit_waves;
}
// rs_tune("jit_backend", 2 | 1 | 0): machine code encoded directly into a
// code-object template (jit_asm.cpp) | the same kernel as assembly text
// assembled by comgr | hiprtc C++; env RSAMD_JIT_BACKEND
int g_jit_backend = [] {
    const char* e = std::getenv("RSAMD_JIT_BACKEND");
    const int v = e ? std::atoi(e) : 2;
    return v < 0 ? 0 : v > 2 ? 2 : v;
}();
int jit_max_rows() { return g_jit_backend ? kAsmMaxRows : kJitMaxRows; }
int jit_max_cols() { return g_jit_backend ? kAsmMaxCols : kJitMaxCols; }
int g_jit_disk_cache = [] {  // rs_tune("jit_disk_cache", 0 | 1); env RSAMD_JIT_DISK_CACHE
    const char* e = std::getenv("RSAMD_JIT_DISK_CACHE");
    return e ? (std::atoi(e) ? 1 : 0) : 1;
}();

void jit_evict_now();  // (below: the worker runs it)
namespace detail {
void engines_quiesce();  // engine.cpp
}

namespace {

uint8_t gmul(uint8_t a, uint8_t b) {  // GF(2^8), polynomial 0x11d
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


// Device prelude: the launch arguments (the layout of MatmulArgs, checked by
// the static_asserts the generator appends) and the bit-slice helpers of
// kernels.hip (bs_swap / bs_transpose8 / bs_x3, buffer nt dwordx2 accesses).
const char* const kPrelude = R"RSJIT(
typedef unsigned char u8;
typedef unsigned int u32;
typedef unsigned long long u64;
typedef long long i64;
typedef u32 u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) u8 g_u8;
struct MatmulArgs {
    const u32* tables; const u32* img4; const u32* wide; const u8* host_mat;
    int rows, cols, rows_pad; int nstripes; int accumulate; int units_per_chunk; int nt_store;
    u64 len; u64 body; u64 tail_start; i64 ss[4]; const int* stripe_ids;
    i64 chunks_per_stripe; i64 total_chunks; int cps_shift;
    u64 ptr[260]; u32 sid[260];
};
__device__ __forceinline__ u32x2 ld8(const g_u8* base, u32 off, u32 nbytes) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(base), 0, (int)nbytes, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 2);
}
__device__ __forceinline__ void st8(g_u8* base, u32 off, u32 nbytes, u32x2 v) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(base), 0, (int)nbytes, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)off, 0, 2);
}
__device__ __forceinline__ void bs_swap(u32& a, u32& b, int s, u32 m) {
    const u32 t = ((a >> s) ^ b) & m;
    b ^= t;
    a ^= t << s;
}
__device__ __forceinline__ void bs_transpose8(u32 (&w)[8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) bs_swap(w[i], w[i + 4], 4, 0x0F0F0F0Fu);
    bs_swap(w[0], w[2], 2, 0x33333333u);
    bs_swap(w[1], w[3], 2, 0x33333333u);
    bs_swap(w[4], w[6], 2, 0x33333333u);
    bs_swap(w[5], w[7], 2, 0x33333333u);
#pragma unroll
    for (int i = 0; i < 8; i += 2) bs_swap(w[i], w[i + 1], 1, 0x55555555u);
}
__device__ __forceinline__ u32 bs_x3(u32 a, u32 b, u32 c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

// A workgroup covers 32*BS bytes of every vector; lane t's 32-byte unit is
// four 8-byte pieces at 8t + 2048k (BS = 64) / 8t + 8*BS*k of the chunk.
template <int BS>
__device__ __forceinline__ void rs_bs_body(const MatmulArgs& a) {
    const u32 chunk = blockIdx.x;
    const u32 cps = (u32)a.chunks_per_stripe;
    const u32 su = a.cps_shift >= 0 ? (chunk >> a.cps_shift) : chunk / cps;
    const int s = a.stripe_ids ? a.stripe_ids[su] : (int)su;
    const u32 cb = chunk - su * cps;
    const u32 off = cb * (32u * BS) + 8u * threadIdx.x;
    const u32 nbytes = (u32)a.body;
    auto fetch = [&](int c, u32 (&w)[8]) {
        const g_u8* p = (const g_u8*)a.ptr[c] + (i64)s * a.ss[a.sid[c] & 3];
        u32 o32 = off;
        asm volatile("" : "+v"(o32));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x2 v = ld8(p, o32 + (u32)(k * 8 * BS), nbytes);
            w[2 * k] = v.x;
            w[2 * k + 1] = v.y;
        }
    };
    // accumulate mode: the old output bytes are loaded up front (fetch_out,
    // with the first columns) and XORed in after the back transpose
    auto fetch_out = [&](int r, u32 (&w)[8]) { fetch(RSJ_COLS + r, w); };
    auto store = [&](int r, u32 (&o)[8], const u32 (&old)[8]) {
        bs_transpose8(o);
        const int v = RSJ_COLS + r;
        g_u8* q = (g_u8*)a.ptr[v] + (i64)s * a.ss[a.sid[v] & 3];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            u32x2 x = {o[2 * k], o[2 * k + 1]};
            if (RSJ_ACC) x ^= u32x2{old[2 * k], old[2 * k + 1]};
            st8(q, off + (u32)(k * 8 * BS), nbytes, x);
        }
    };
    RSJ_NETWORK
}
extern "C" __global__ __launch_bounds__(64) void rs_bs_jit_64(const MatmulArgs a) { rs_bs_body<64>(a); }
extern "C" __global__ __launch_bounds__(256) void rs_bs_jit_256(const MatmulArgs a) { rs_bs_body<256>(a); }
)RSJIT";

// The network for one matrix: the statements of BsNet<d, p>::run in
// bitslice_gen.inc, for this matrix (same construction as
// tools/gen_bitslice.py emit()).
std::string network(const uint8_t* mat, int rows, int cols, bool acc) {
    const int kPF = g_jit_pf;
    std::string o;
    char buf[160];
#define line(...)                                      \
    do {                                               \
        std::snprintf(buf, sizeof buf, __VA_ARGS__);   \
        o += buf;                                      \
        o += '\n';                                     \
    } while (0)
    // mask[c][r][i]: input planes j of column c feeding plane i of row r
    std::vector<uint8_t> mask(static_cast<size_t>(cols) * rows * 8);
    for (int c = 0; c < cols; ++c)
        for (int r = 0; r < rows; ++r) {
            const uint8_t g = mat[static_cast<size_t>(r) * cols + c];
            for (int i = 0; i < 8; ++i) {
                uint8_t m = 0;
                for (int j = 0; j < 8; ++j)
                    if ((gmul(g, static_cast<uint8_t>(1u << j)) >> i) & 1) m |= static_cast<uint8_t>(1u << j);
                mask[(static_cast<size_t>(c) * rows + r) * 8 + i] = m;
            }
        }
    line("    u32 A[%d][8];", rows);
    for (int k = 0; k < kPF && k < cols; ++k) {
        line("    u32 N%d[8];", k);
        line("    fetch(%d, N%d);", k, k);
    }
    line("    u32 O[%d][8];", acc ? rows : 1);
    if (acc) line("    for (int r = 0; r < %d; ++r) fetch_out(r, O[r]);", rows);
    for (int c = 0; c < cols; ++c) {
        line("    {");
        line("        u32 P[8];");
        line("        for (int k = 0; k < 8; ++k) P[k] = N%d[k];", c % kPF);
        if (c + kPF < cols) line("        fetch(%d, N%d);", c + kPF, c % kPF);
        line("        bs_transpose8(P);");
        std::string name[2][16];  // per half: expression naming subset m
        for (int half = 0; half < 2; ++half) {
            const int base = 4 * half;
            const char h = half ? 'H' : 'L';
            bool have[16] = {}, used[16] = {};
            for (int b = 0; b < 4; ++b) {
                have[1 << b] = true;
                name[half][1 << b] = "P[" + std::to_string(base + b) + "]";
            }
            for (int r = 0; r < rows; ++r)
                for (int i = 0; i < 8; ++i) used[(mask[(static_cast<size_t>(c) * rows + r) * 8 + i] >> base) & 15] = true;
            used[0] = false;
            bool need[16] = {};
            // want(m): m and the chain m ^ lowbit(m), ... down to a single plane
            for (int m = 1; m < 16; ++m)
                if (used[m])
                    for (int x = m; x && !have[x] && !need[x]; x ^= x & -x) need[x] = true;
            for (int pc = 2; pc <= 4; ++pc)
                for (int m = 1; m < 16; ++m) {
                    if (!need[m] || __builtin_popcount(m) != pc) continue;
                    const int low = m & -m, rest = m ^ low;
                    line("        const u32 %c%d = %s ^ %s;", h, m, name[half][rest].c_str(), name[half][low].c_str());
                    name[half][m] = std::string(1, h) + std::to_string(m);
                    have[m] = true;
                }
        }
        for (int r = 0; r < rows; ++r)
            for (int i = 0; i < 8; ++i) {
                const int m = mask[(static_cast<size_t>(c) * rows + r) * 8 + i];
                const std::string* t[2];
                int nt = 0;
                if (m & 15) t[nt++] = &name[0][m & 15];
                if (m >> 4) t[nt++] = &name[1][m >> 4];
                if (c == 0) {
                    if (nt == 0) line("        A[%d][%d] = 0u;", r, i);
                    else if (nt == 1) line("        A[%d][%d] = %s;", r, i, t[0]->c_str());
                    else line("        A[%d][%d] = %s ^ %s;", r, i, t[0]->c_str(), t[1]->c_str());
                } else if (nt == 2) {
                    line("        A[%d][%d] = bs_x3(A[%d][%d], %s, %s);", r, i, r, i, t[0]->c_str(), t[1]->c_str());
                } else if (nt == 1) {
                    line("        A[%d][%d] ^= %s;", r, i, t[0]->c_str());
                }
            }
        line("    }");
        // pin the running sums per column (no re-association across columns)
        line("#pragma unroll");
        line("    for (int r = 0; r < %d; ++r)", rows);
        line("#pragma unroll");
        line("        for (int i = 0; i < 8; ++i) asm volatile(\"\" : \"+v\"(A[r][i]));");
        line("    __builtin_amdgcn_sched_barrier(0);");
    }
    line("    for (int r = 0; r < %d; ++r) store(r, A[r], O[%s]);", rows, acc ? "r" : "0");
#undef line
    return o;
}

// ---------------------------------------------------------------- on-disk cache

// Bumped whenever network() or the launch contract changes in a way the
// key below does not capture (the prelude text and the MatmulArgs layout are
// hashed into the key).
constexpr uint32_t kJitGenVersion = 5;
constexpr char kDiskMagic[8] = {'R', 'S', 'A', 'M', 'D', 'J', 'I', 'T'};
constexpr uint32_t kDiskFormat = 1;

uint64_t fnv1a(const void* p, size_t n, uint64_t h) {
    const uint8_t* b = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 0x100000001b3ull;
    }
    return h;
}
uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}
// Second, independent hash: splitmix64 over 8-byte words
uint64_t hash2(const std::string& s) {
    uint64_t h = 0x6a09e667f3bcc909ull ^ s.size();
    size_t i = 0;
    for (; i + 8 <= s.size(); i += 8) {
        uint64_t w;
        std::memcpy(&w, s.data() + i, 8);
        h = mix64(h ^ w) + 0x9e3779b97f4a7c15ull;
    }
    uint64_t w = 0;
    std::memcpy(&w, s.data() + i, s.size() - i);
    return mix64(h ^ w ^ 0xff);
}

struct DiskStats {
    std::atomic<uint64_t> hits{0}, misses{0}, writes{0}, rejects{0};
};
DiskStats& disk_stats() {
    static DiskStats* d = new DiskStats;
    return *d;
}

std::string cache_dir() {
    static const std::string dir = [] {
        if (const char* e = std::getenv("RSAMD_JIT_CACHE_DIR")) return std::string(e);
        if (const char* x = std::getenv("XDG_CACHE_HOME"); x && *x) return std::string(x) + "/rsamd/jit";
        if (const char* h = std::getenv("HOME"); h && *h) return std::string(h) + "/.cache/rsamd/jit";
        return std::string();
    }();
    return dir;
}

// The cache holds GPU code this process loads and runs, so it must be the
// caller's alone: a directory or file owned by another user, or writable by
// group / others, could carry code injected by another process (the FNV
// checksum and key hashes catch corruption, not tampering).  Directories are
// created 0700 and files 0600; anything else is not read and not written.
bool private_to_us(const struct stat& st) {
    return st.st_uid == geteuid() && (st.st_mode & (S_IWGRP | S_IWOTH)) == 0;
}

bool cache_dir_private(const std::string& d) {
    struct stat st {};
    return lstat(d.c_str(), &st) == 0 && S_ISDIR(st.st_mode) && private_to_us(st);
}

bool make_dirs(const std::string& d) {
    if (d.empty()) return false;
    std::string cur;
    for (size_t i = 0; i <= d.size(); ++i) {
        if (i == d.size() || d[i] == '/') {
            if (!cur.empty() && mkdir(cur.c_str(), 0700) != 0 && errno != EEXIST) return false;
        }
        if (i < d.size()) cur += d[i];
    }
    return cache_dir_private(d);
}

struct DiskKey {
    std::string text;  // everything the code object depends on
    uint64_t h1 = 0, h2 = 0;
    std::string path() const {
        char name[48];
        std::snprintf(name, sizeof name, "%016llx%016llx.co", static_cast<unsigned long long>(h1),
                      static_cast<unsigned long long>(h2));
        return cache_dir() + "/" + name;
    }
};

struct FileHeader {
    char magic[8];
    uint32_t format, gen;
    uint64_t h1, h2, key_len, code_len, code_sum;
};

std::vector<char> disk_load(const DiskKey& k) {
    std::vector<char> code;
    const std::string path = k.path();
    if (!cache_dir_private(cache_dir())) return code;
    const int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC | O_NOFOLLOW);
    if (fd < 0) return code;
    struct stat st {};
    FileHeader h{};
    bool ok = fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && private_to_us(st) &&
              read(fd, &h, sizeof h) == static_cast<ssize_t>(sizeof h) &&
              std::memcmp(h.magic, kDiskMagic, 8) == 0 && h.format == kDiskFormat && h.gen == kJitGenVersion &&
              h.h1 == k.h1 && h.h2 == k.h2 && h.key_len == k.text.size() && h.code_len > 4 &&
              h.code_len < (uint64_t{256} << 20);
    if (ok) {
        code.resize(h.code_len);
        ok = read(fd, code.data(), code.size()) == static_cast<ssize_t>(code.size()) &&
             fnv1a(code.data(), code.size(), 0xcbf29ce484222325ull) == h.code_sum && code[0] == 0x7f &&
             code[1] == 'E' && code[2] == 'L' && code[3] == 'F';
    }
    close(fd);
    if (!ok) {
        code.clear();
        disk_stats().rejects.fetch_add(1, std::memory_order_relaxed);
    }
    return code;
}

void disk_store(const DiskKey& k, const std::vector<char>& code) {
    const std::string dir = cache_dir();
    if (!make_dirs(dir)) return;
    const std::string path = k.path();
    char tmp_suffix[64];
    std::snprintf(tmp_suffix, sizeof tmp_suffix, ".tmp.%d.%llx", static_cast<int>(getpid()),
                  static_cast<unsigned long long>(mix64(reinterpret_cast<uintptr_t>(&code) ^ k.h1)));
    const std::string tmp = path + tmp_suffix;
    const int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC | O_NOFOLLOW, 0600);
    if (fd < 0) return;
    FileHeader h{};
    std::memcpy(h.magic, kDiskMagic, 8);
    h.format = kDiskFormat;
    h.gen = kJitGenVersion;
    h.h1 = k.h1;
    h.h2 = k.h2;
    h.key_len = k.text.size();
    h.code_len = code.size();
    h.code_sum = fnv1a(code.data(), code.size(), 0xcbf29ce484222325ull);
    bool ok = write(fd, &h, sizeof h) == static_cast<ssize_t>(sizeof h) &&
              write(fd, code.data(), code.size()) == static_cast<ssize_t>(code.size());
    ok = close(fd) == 0 && ok;
    // rename is atomic: a reader sees the old file, no file, or this whole file
    if (ok && rename(tmp.c_str(), path.c_str()) == 0) {
        disk_stats().writes.fetch_add(1, std::memory_order_relaxed);
    } else {
        unlink(tmp.c_str());
    }
}

struct Compiled {
    std::vector<char> code;
    double ms = 0;
    bool ok = false;
    std::string log;
};

Compiled compile_asm(const std::string& src) {
    Compiled out;
    out.ok = asm_assemble(src, &out.code, &out.log, &out.ms);
    return out;
}

Compiled compile_binary_shape(const uint8_t* mat, int rows, int cols, bool acc, const AsmShape& sh, int pf,
                              int sync, int waves) {
    Compiled out;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<uint32_t> code;
    int used = 0;
    if (!asm_binary(mat, rows, cols, acc, sh, pf, sync, &code, &used, &out.log)) return out;
    double lms = 0;
    out.ok = asm_link_binary(code, sh, used, waves, &out.code, &out.log, &lms);
    out.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return out;
}

Compiled compile(const std::string& src) {
    Compiled out;
    const auto t0 = std::chrono::steady_clock::now();
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "rs_bs_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        out.log = "hiprtcCreateProgram failed";
        return out;
    }
    std::vector<const char*> opts = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
#ifdef RSAMD_EXPERIMENTS  // compile-option experiments (librsamd_exp.so only): RSAMD_JIT_OPTS="opt opt ..."
    static std::vector<std::string> extra = [] {
        std::vector<std::string> v;
        if (const char* e = std::getenv("RSAMD_JIT_OPTS")) {
            std::string cur;
            for (const char* c = e;; ++c) {
                if (*c == ' ' || *c == 0) {
                    if (!cur.empty()) v.push_back(cur);
                    cur.clear();
                    if (!*c) break;
                } else {
                    cur += *c;
                }
            }
        }
        return v;
    }();
    for (const std::string& x : extra) opts.push_back(x.c_str());
    if (const char* d = std::getenv("RSAMD_JIT_DUMP")) {  // the generated source, for offline profiling
        if (FILE* f = std::fopen(d, "w")) {
            std::fputs(src.c_str(), f);
            std::fclose(f);
        }
    }
#endif
    const hiprtcResult rc = hiprtcCompileProgram(prog, static_cast<int>(opts.size()), opts.data());
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        if (hiprtcGetProgramLogSize(prog, &n) == HIPRTC_SUCCESS && n > 1) {
            out.log.resize(n);
            hiprtcGetProgramLog(prog, &out.log[0]);
        }
        hiprtcDestroyProgram(&prog);
        return out;
    }
    size_t n = 0;
    if (hiprtcGetCodeSize(prog, &n) == HIPRTC_SUCCESS && n > 0) {
        out.code.resize(n);
        out.ok = hiprtcGetCode(prog, out.code.data()) == HIPRTC_SUCCESS;
    }
    hiprtcDestroyProgram(&prog);
    out.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return out;
}

// ---------------------------------------------------------------- cache

struct Entry {
    enum State { kQueued, kCompiling, kReady, kLoaded, kFailed } state = kQueued;
    bool is_asm = false;  // generated kernel (rs_bs_asm) or hiprtc C++ (rs_bs_jit_64 / _256)
    int nw = 1;           // generated kernels: waves per workgroup
    AsmShape shape;       // ... and how they split the work
    int backend = 1;
    std::string src;      // backends 1 (assembly) and 0 (C++)
    // backend 2 (machine code): the matrix and the generator's settings
    std::vector<uint8_t> mat;
    int rows = 0, cols = 0, pf = 3, sync = 0, waves = 2;
    bool acc = false;
    int dev = 0;
    uint64_t last_use = 0;  // (eviction: least recently looked up first)
    DiskKey disk;  // on-disk cache key (text empty: the disk cache is off)
    std::vector<char> code;
    hipModule_t module = nullptr;
    hipFunction_t fn64 = nullptr, fn256 = nullptr;
};

Compiled compile_binary(const Entry& e) {
    return compile_binary_shape(e.mat.data(), e.rows, e.cols, e.acc, e.shape, e.pf, e.sync, e.waves);
}

constexpr size_t kMaxEntries = 256;  // compiled matrices per process; the older half is evicted beyond

// Backend 2 in the default mode compiles a matrix on the launching thread
// once the time its launches are estimated to have lost on the table kernels
// exceeds the estimated time to generate and load its kernel, so a one-off
// pattern large enough to pay for its kernel gets it on its FIRST launch, and
// a small one only once it recurs.  First sight to loaded, measured on MI355X
// (tools/jit_compile_probe.py, profiles/r04/jit_compile_probe.log): 0.17-0.26
// ms up to 16 x 20, 0.64 ms at 28 x 100, 0.76-0.94 ms at 64 x 64, 2.2 ms at
// 56 x 200, 2.6-3.0 ms at 128 x 128.
double est_compile_us(int rows, int cols) { return 150.0 + 0.15 * rows * cols; }
// Microseconds per byte moved that a product with `rows` outputs loses on the
// table kernels: those run 5-8 rows at ~5 TB/s (VALU-bound) and more rows on
// the single-pass wide kernel at ~3.4 TB/s for 16 rows, falling about as
// 1 / rows beyond; compiled kernels run ~6 TB/s up to 32 rows, 3.7 at 64 and
// 2.0 at 128 (shared columns): about 6 x (32 / rows)^0.8.
double lost_us_per_byte(int rows) {
    const double fb = rows <= 8 ? 5.0 : std::min(5.0, 3.4 * 16.0 / rows);  // TB/s = 1e6 bytes per us
    const double jt = rows <= 32 ? 6.0 : 6.0 * std::pow(32.0 / rows, 0.8);
    return std::max(0.0, 1.0 / fb - 1.0 / jt) * 1e-6;
}
constexpr size_t kMaxSeen = 4096;  // matrices counted but not compiled yet (cleared when full)

struct Seen {
    uint64_t launches = 0, bytes = 0;
    double lost_us = 0;  // backend 2: time its launches are estimated to have lost on the table kernels
    bool disk_checked = false;  // no code object on disk for it at first sight
};

void jit_atexit_hook();
void jit_atexit();

struct Jit {
    std::mutex mu;
    std::condition_variable cv;
    std::map<std::string, std::shared_ptr<Entry>> entries;  // key: device, mode, rows, cols, matrix
    std::map<std::string, Seen> seen;  // background mode: launches / bytes of matrices not compiled yet
    std::deque<std::shared_ptr<Entry>> queue;
    std::thread worker;
    bool stop = false;
    uint64_t compiled = 0, failed = 0, evictions = 0, loads = 0;
    double load_ms = 0;  // in hipModuleLoadData (diagnostics: env RSAMD_JIT_TRACE prints these at exit)
    double compile_ms = 0;
    std::atomic<uint64_t> launches{0};

    void run_one(const std::shared_ptr<Entry>& e) {  // caller does not hold mu
        Compiled c = e->backend == 2 ? compile_binary(*e) : e->is_asm ? compile_asm(e->src) : compile(e->src);
        // The compiler libraries hiprtc loads on its first compile register
        // their static destructors then, i.e. after jit_atexit: those ran
        // first at exit and a compile still in flight on the worker crashed
        // (SIGSEGV at exit of tools/gpu_stress.py).  Registering once more
        // after the first compile puts the join ahead of them (atexit runs in
        // reverse order); jit_atexit is idempotent.
        static std::once_flag late;
        std::call_once(late, [] { std::atexit(jit_atexit_hook); });
        if (c.ok && !e->disk.text.empty()) disk_store(e->disk, c.code);
        std::lock_guard<std::mutex> lk(mu);
        if (c.ok) {
            e->code = std::move(c.code);
            e->state = Entry::kReady;
            ++compiled;
            compile_ms += c.ms;
        } else {
            e->state = Entry::kFailed;
            ++failed;
            std::fprintf(stderr, "librsamd: run-time kernel compile failed (perm-table kernels stay in use): %s\n",
                         c.log.substr(0, 2000).c_str());
        }
        e->src.clear();
        e->src.shrink_to_fit();
        e->mat.clear();
        e->mat.shrink_to_fit();
    }

    void work() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return stop || !queue.empty() || evict_task; });
            if (stop) return;
            if (evict_task) {  // posted by a launch (jit_launch_guard): done here, off the launch path
                evict_task = false;
                lk.unlock();
                jit_evict_now();
                lk.lock();
                continue;
            }
            std::shared_ptr<Entry> e = queue.front();
            queue.pop_front();
            e->state = Entry::kCompiling;
            lk.unlock();
            run_one(e);
            lk.lock();
        }
    }

    pid_t owner = 0;  // the process that started the worker
    uint64_t use_clock = 0;
    std::atomic<bool> evict_wanted{false};
    bool evict_task = false;  // an eviction is queued for the worker (under mu)

    // Caller holds mu.  Starts the worker thread if this object has none (a
    // forked child works on a fresh object: jit() below).
    void ensure_worker() {
        if (worker.joinable()) return;
        // load the compiler library hiprtc would load on its first compile
        // now, so its static destructors are registered before jit_atexit and
        // run after it (atexit order)
        static void* const comgr = dlopen("libamd_comgr.so.3", RTLD_NOW | RTLD_GLOBAL);
        (void)comgr;
        static const bool registered = std::atexit(jit_atexit) == 0;
        (void)registered;
        owner = getpid();
        worker = std::thread([this] { work(); });
    }
};

// Never destroyed (a std::thread destructor on a joinable thread aborts); the
// process that started the worker joins it at exit: the compile in flight
// finishes (hiprtc only), queued ones are dropped.  A forked child inherits
// the object but not its worker thread, possibly with `mu` or the eviction
// lock held by that thread at the fork and with modules loaded into the
// parent's HIP context: the child's pthread_atfork handler gives it a fresh
// Jit and eviction lock instead (the inherited ones are left alone, never
// destroyed; advisor r05).
Jit* g_jit = nullptr;
// Launches hold this shared from the lookup of a compiled kernel until it is
// enqueued; eviction holds it exclusively, drains the devices and unloads.
std::shared_mutex* g_evict_mu = nullptr;

void jit_fork_child() {
    g_jit = new Jit;
    g_evict_mu = new std::shared_mutex;
}

Jit& jit() {
    static const bool init = [] {
        g_jit = new Jit;
        g_evict_mu = new std::shared_mutex;
        return pthread_atfork(nullptr, nullptr, jit_fork_child) == 0;
    }();
    (void)init;
    return *g_jit;
}

std::shared_mutex& evict_mu() {
    (void)jit();
    return *g_evict_mu;
}

void jit_trace_report() {
    Jit& j = jit();
    std::fprintf(stderr, "{\"jit_trace\": {\"compiled\": %llu, \"compile_ms\": %.3f, \"loads\": %llu, "
                 "\"load_ms\": %.3f, \"evictions\": %llu}}\n",
                 static_cast<unsigned long long>(j.compiled), j.compile_ms, static_cast<unsigned long long>(j.loads),
                 j.load_ms, static_cast<unsigned long long>(j.evictions));
}

void jit_trace_register() {
    static const bool on = std::getenv("RSAMD_JIT_TRACE") != nullptr && std::atexit(jit_trace_report) == 0;
    (void)on;
}

void jit_atexit() {
    Jit& j = jit();
    if (!j.worker.joinable()) return;
    if (j.owner != getpid()) return;
    {
        std::lock_guard<std::mutex> lk(j.mu);
        j.stop = true;
    }
    j.cv.notify_all();
    if (j.worker.joinable()) j.worker.join();
}

void jit_atexit_hook() { jit_atexit(); }

}  // namespace

std::string jit_source(const uint8_t* mat, int rows, int cols, bool accumulate) {
    std::string s = "#define RSJ_COLS " + std::to_string(cols) + "\n#define RSJ_ACC " +
                    std::string(accumulate ? "1" : "0") + "\n";
    std::string pre(kPrelude);
    const size_t at = pre.find("RSJ_NETWORK");
    s += pre.substr(0, at) + "\n" + network(mat, rows, cols, accumulate) + pre.substr(at + std::strlen("RSJ_NETWORK"));
    // the kernel's argument layout must equal the host's
    s += "static_assert(sizeof(MatmulArgs) == " + std::to_string(sizeof(MatmulArgs)) + ", \"MatmulArgs size\");\n";
    s += "static_assert(__builtin_offsetof(MatmulArgs, ptr) == " + std::to_string(offsetof(MatmulArgs, ptr)) +
         ", \"MatmulArgs ptr\");\n";
    s += "static_assert(__builtin_offsetof(MatmulArgs, stripe_ids) == " +
         std::to_string(offsetof(MatmulArgs, stripe_ids)) + ", \"MatmulArgs stripe_ids\");\n";
    s += "static_assert(__builtin_offsetof(MatmulArgs, cps_shift) == " +
         std::to_string(offsetof(MatmulArgs, cps_shift)) + ", \"MatmulArgs cps_shift\");\n";
    return s;
}

int jit_compile_check(const uint8_t* mat, int rows, int cols, bool accumulate, double* ms) {
    if (!mat || rows < 1 || rows > jit_max_rows() || cols < 1 || cols > jit_max_cols()) return RS_ERR_INVAL;
    Compiled c =
        g_jit_backend == 2 ? compile_binary_shape(mat, rows, cols, accumulate, jit_shape(rows, cols), jit_pf_for(rows, cols),
                                                  g_jit_sync, jit_waves_for(rows, cols))
        : g_jit_backend    ? compile_asm(asm_source(mat, rows, cols, accumulate, jit_shape(rows, cols), jit_pf_for(rows, cols),
                                                    g_jit_sync, jit_waves_for(rows, cols), nullptr))
                           : compile(jit_source(mat, rows, cols, accumulate));
    if (ms) *ms = c.ms;
    if (!c.ok) std::fprintf(stderr, "librsamd: jit compile check failed: %s\n", c.log.substr(0, 4000).c_str());
    return c.ok ? RS_OK : RS_ERR_DEVICE;
}

int jit_encoder_check(const uint8_t* mat, int rows, int cols, bool accumulate, size_t* code_bytes) {
    if (!mat || rows < 1 || rows > kAsmMaxRows || cols < 1 || cols > kAsmMaxCols) return RS_ERR_INVAL;
    const AsmShape sh = jit_shape(rows, cols);
    std::vector<uint32_t> bin;
    int used = 0;
    std::string err;
    if (!asm_binary(mat, rows, cols, accumulate, sh, jit_pf_for(rows, cols), g_jit_sync, &bin, &used, &err)) {
        std::fprintf(stderr, "librsamd: encoder failed: %s\n", err.c_str());
        return RS_ERR_DEVICE;
    }
    Compiled c = compile_asm(
        asm_source(mat, rows, cols, accumulate, sh, jit_pf_for(rows, cols), g_jit_sync, jit_waves_for(rows, cols), nullptr));
    std::vector<char> text;
    if (!c.ok || !asm_text_section(c.code, &text)) {
        std::fprintf(stderr, "librsamd: encoder check: assembly failed: %s\n", c.log.substr(0, 2000).c_str());
        return RS_ERR_DEVICE;
    }
    if (code_bytes) *code_bytes = bin.size() * 4;
    const size_t n = bin.size() * 4;
    if (text.size() < n) {
        std::fprintf(stderr, "librsamd: encoder check: %zu bytes encoded, the assembler's .text has %zu\n", n,
                     text.size());
        return RS_ERR_DEVICE;
    }
    const char* b = reinterpret_cast<const char*>(bin.data());
    for (size_t i = 0; i < n; i += 4)
        if (std::memcmp(b + i, text.data() + i, 4) != 0) {
            uint32_t x, y;
            std::memcpy(&x, b + i, 4);
            std::memcpy(&y, text.data() + i, 4);
            std::fprintf(stderr, "librsamd: encoder check: byte %zu differs: encoder %08x, assembler %08x\n", i, x, y);
            return RS_ERR_DEVICE;
        }
    for (size_t i = n; i < text.size(); ++i)  // (the assembler's .text may end with alignment padding)
        if (text[i] != 0) {
            std::fprintf(stderr, "librsamd: encoder check: the assembler's .text goes on past byte %zu\n", n);
            return RS_ERR_DEVICE;
        }
    return RS_OK;
}

void jit_stats(uint64_t* compiled, uint64_t* failed, uint64_t* launches, double* compile_ms) {
    Jit& j = jit();
    std::lock_guard<std::mutex> lk(j.mu);
    if (compiled) *compiled = j.compiled;
    if (failed) *failed = j.failed;
    if (launches) *launches = j.launches.load();
    if (compile_ms) *compile_ms = j.compile_ms;
}

void jit_count_launch() { jit().launches.fetch_add(1, std::memory_order_relaxed); }

void jit_table_stats(uint64_t* entries, uint64_t* evictions) {
    Jit& j = jit();
    std::lock_guard<std::mutex> lk(j.mu);
    if (entries) *entries = j.entries.size();
    if (evictions) *evictions = j.evictions;
}

void jit_cache_stats(uint64_t* hits, uint64_t* misses, uint64_t* writes, uint64_t* rejects) {
    DiskStats& d = disk_stats();
    if (hits) *hits = d.hits.load();
    if (misses) *misses = d.misses.load();
    if (writes) *writes = d.writes.load();
    if (rejects) *rejects = d.rejects.load();
}

// gcnArchName of a device ("gfx950:sramecc+:xnack-"), cached; caller holds jit().mu
static const std::string& device_arch(int dev) {
    static std::map<int, std::string> archs;
    auto it = archs.find(dev);
    if (it != archs.end()) return it->second;
    hipDeviceProp_t prop;
    std::string name = hipGetDeviceProperties(&prop, dev) == hipSuccess ? std::string(prop.gcnArchName) : "";
    return archs.emplace(dev, name).first->second;
}

// Everything the code object for this launch shape depends on.
static DiskKey disk_key(const std::string& arch, const MatmulArgs& a) {
    static const std::string fixed = [] {
        int maj = 0, mnr = 0;
        (void)hiprtcVersion(&maj, &mnr);
        char b[160];
        std::snprintf(b, sizeof b, "gen %u hiprtc %d.%d args %zu/%zu/%zu/%zu prelude %016llx", kJitGenVersion, maj, mnr,
                      sizeof(MatmulArgs), offsetof(MatmulArgs, ptr), offsetof(MatmulArgs, stripe_ids),
                      offsetof(MatmulArgs, cps_shift),
                      static_cast<unsigned long long>(fnv1a(kPrelude, std::strlen(kPrelude), 0xcbf29ce484222325ull)));
        return std::string(b);
    }();
    DiskKey k;
    k.text = arch + '\n' + fixed + (g_jit_backend == 2 ? " bin " : g_jit_backend ? " asm " : " hiprtc ") + '\n';
    k.text += static_cast<char>(a.accumulate ? 1 : 0);
    k.text += static_cast<char>(a.rows);
    k.text += static_cast<char>(a.cols);
    k.text += static_cast<char>(g_jit_backend ? jit_pf_for(a.rows, a.cols) : g_jit_pf);
    k.text += static_cast<char>(g_jit_backend ? g_jit_sync : 0);
    k.text += static_cast<char>(g_jit_backend ? jit_waves_for(a.rows, a.cols) : 0);
    k.text += static_cast<char>(g_jit_backend ? g_jit_layout : 0);
    k.text += static_cast<char>(g_jit_backend ? g_jit_group_waves : 0);
    k.text += static_cast<char>(g_jit_backend ? g_jit_path_rows : 0);
    k.text += static_cast<char>(g_jit_backend ? g_jit_share : 0);
    k.text += static_cast<char>(g_jit_backend ? g_jit_share_deep : 0);
    k.text += static_cast<char>(g_jit_backend ? g_jit_share_dma : 0);
    k.text += static_cast<char>(g_jit_backend && jit_split_small(a.rows, a.cols) ? 1 : 0);
    k.text += static_cast<char>(g_jit_backend ? g_jit_share_cols : 0);
    k.text += static_cast<char>(g_jit_backend ? g_jit_share_ahead : 0);
    k.text += static_cast<char>(g_jit_backend ? g_jit_gray : 0);
    k.text += static_cast<char>(g_jit_backend ? g_jit_nobar : 0);
    k.text.append(reinterpret_cast<const char*>(a.host_mat), static_cast<size_t>(a.rows) * a.cols);
    k.h1 = fnv1a(k.text.data(), k.text.size(), 0xcbf29ce484222325ull);
    k.h2 = hash2(k.text);
    return k;
}

// mode: 1 background after recurrence, 2 compile on this thread, 3 queue now
static JitKernel lookup(const MatmulArgs& a, int bs, uint64_t launch_bytes, int mode) {
    const int backend = g_jit_backend;
    if (!mode || !a.host_mat || a.rows < 1 || a.rows > jit_max_rows() || a.cols < 1 || a.cols > jit_max_cols())
        return {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return {};
    Jit& j = jit();
    std::shared_ptr<Entry> e;
    std::unique_lock<std::mutex> lk(j.mu);
    // the generated code is gfx950 code (v_bitop3, buffer nt): other devices
    // keep the perm-table kernels (no compile is ever attempted for them)
    const std::string& arch = device_arch(dev);
    if (arch.compare(0, 6, "gfx950") != 0) return {};
    std::string key(reinterpret_cast<const char*>(&dev), sizeof dev);
    key += static_cast<char>(backend);
    key += static_cast<char>(a.accumulate ? 1 : 0);
    key += static_cast<char>(a.rows);
    key += static_cast<char>(a.rows >> 8);
    key += static_cast<char>(a.cols);
    key += static_cast<char>(a.cols >> 8);
    key += static_cast<char>(backend ? jit_pf_for(a.rows, a.cols) : g_jit_pf);
    key += static_cast<char>(backend ? g_jit_sync : 0);
    key += static_cast<char>(backend ? jit_waves_for(a.rows, a.cols) : 0);
    key += static_cast<char>(backend ? g_jit_layout : 0);
    key += static_cast<char>(backend ? g_jit_group_waves : 0);
    key += static_cast<char>(backend ? g_jit_path_rows : 0);
    key += static_cast<char>(backend ? g_jit_share : 0);
    key += static_cast<char>(backend ? g_jit_share_deep : 0);
    key += static_cast<char>(backend ? g_jit_share_dma : 0);
    key += static_cast<char>(backend && jit_split_small(a.rows, a.cols) ? 1 : 0);
    key += static_cast<char>(backend ? g_jit_share_cols : 0);
    key += static_cast<char>(backend ? g_jit_share_ahead : 0);
    key += static_cast<char>(backend ? g_jit_gray : 0);
    key += static_cast<char>(backend ? g_jit_nobar : 0);
    key.append(reinterpret_cast<const char*>(a.host_mat), static_cast<size_t>(a.rows) * a.cols);
    {
        auto it = j.entries.find(key);
        if (it == j.entries.end()) {
            if (j.entries.size() >= kMaxEntries) {  // full: evict the older half before a later launch
                j.evict_wanted.store(true, std::memory_order_release);
                return {};
            }
            // a code object on disk (another process, an earlier run): load it
            // now whatever the launch history; checked once per matrix
            DiskKey dk;
            Seen* h = nullptr;
            if (mode == 1) {
                if (j.seen.size() >= kMaxSeen) j.seen.clear();
                h = &j.seen[key];
            }
            // (backend 2 builds a kernel about as fast as it would read the
            // file: no disk cache, so a storm of one-off patterns writes nothing)
            if (backend != 2 && g_jit_disk_cache && !cache_dir().empty() && !(h && h->disk_checked)) {
                dk = disk_key(arch, a);
                std::vector<char> code = disk_load(dk);
                if (h) h->disk_checked = true;
                if (!code.empty()) {
                    disk_stats().hits.fetch_add(1, std::memory_order_relaxed);
                    if (h) j.seen.erase(key);
                    e = std::make_shared<Entry>();
                    e->is_asm = backend != 0;
                    e->backend = backend;
                    e->shape = jit_shape(a.rows, a.cols);
                    e->nw = e->shape.nw;
                    e->code = std::move(code);
                    e->state = Entry::kReady;
                    e->disk = std::move(dk);
                    it = j.entries.emplace(key, e).first;
                } else {
                    disk_stats().misses.fetch_add(1, std::memory_order_relaxed);
                }
            }
        }
        if (it == j.entries.end()) {
            if (mode == 1) {
                Seen& h = j.seen[key];
                ++h.launches;
                h.bytes += launch_bytes;
                if (backend == 2) {
                    // compile once it pays for itself (est_compile_us above)
                    h.lost_us += static_cast<double>(launch_bytes) * lost_us_per_byte(a.rows);
                    if (h.lost_us < est_compile_us(a.rows, a.cols)) return {};
                } else if (h.launches < static_cast<uint64_t>(g_jit_min_launches) || h.bytes < g_jit_min_bytes) {
                    // compile only a matrix that recurs: a one-off erasure pattern
                    // would cost a compile (seconds of host time) and never pay it back
                    return {};
                }
                j.seen.erase(key);
            }
            e = std::make_shared<Entry>();
            e->is_asm = backend != 0;
            e->backend = backend;
            e->shape = jit_shape(a.rows, a.cols);
            e->nw = e->shape.nw;
            if (backend == 2) {
                e->mat.assign(a.host_mat, a.host_mat + static_cast<size_t>(a.rows) * a.cols);
                e->rows = a.rows;
                e->cols = a.cols;
                e->acc = a.accumulate != 0;
                e->pf = jit_pf_for(a.rows, a.cols);
                e->sync = g_jit_sync;
                e->waves = jit_waves_for(a.rows, a.cols);
            } else {
                e->src = e->is_asm ? asm_source(a.host_mat, a.rows, a.cols, a.accumulate != 0, e->shape,
                                                jit_pf_for(a.rows, a.cols), g_jit_sync, jit_waves_for(a.rows, a.cols), nullptr)
                                   : jit_source(a.host_mat, a.rows, a.cols, a.accumulate != 0);
            }
            if (backend != 2 && g_jit_disk_cache && !cache_dir().empty()) e->disk = disk_key(arch, a);
            e->dev = dev;
            j.entries.emplace(key, e);
            if (mode == 2 || (mode == 1 && backend == 2)) {
                e->state = Entry::kCompiling;
                lk.unlock();
                j.run_one(e);  // on this thread
                lk.lock();
            } else {
                j.queue.push_back(e);
                j.ensure_worker();
                j.cv.notify_one();
                return {};
            }
        } else {
            e = it->second;
        }
        e->dev = dev;
        e->last_use = ++j.use_clock;
        auto result = [&]() -> JitKernel {
            JitKernel k;
            k.is_asm = e->is_asm;
            k.nw = e->nw;
            k.layout = e->shape.layout;
            k.groups = e->shape.groups;
            k.fn = e->is_asm ? e->fn64 : (bs == 256 ? e->fn256 : e->fn64);
            return k;
        };
        if (e->state == Entry::kLoaded) return result();
        if (e->state != Entry::kReady) return {};
        // load the code object on this device (launching thread, under mu)
        hipModule_t m = nullptr;
        hipFunction_t f64 = nullptr, f256 = nullptr;
        const auto tl = std::chrono::steady_clock::now();
        const bool loaded = hipModuleLoadData(&m, e->code.data()) == hipSuccess;
        ++j.loads;
        j.load_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tl).count();
        jit_trace_register();
        const bool ok = loaded &&
                        (e->is_asm ? hipModuleGetFunction(&f64, m, "rs_bs_asm") == hipSuccess
                                   : hipModuleGetFunction(&f64, m, "rs_bs_jit_64") == hipSuccess &&
                                         hipModuleGetFunction(&f256, m, "rs_bs_jit_256") == hipSuccess);
        if (!ok) {
            (void)hipGetLastError();
            e->state = Entry::kFailed;
            ++j.failed;
            std::fprintf(stderr, "librsamd: run-time kernel load failed (perm-table kernels stay in use)\n");
            return {};
        }
        e->module = m;
        e->fn64 = f64;
        e->fn256 = f256;
        e->state = Entry::kLoaded;
        e->code.clear();
        e->code.shrink_to_fit();
        return result();
    }
}

// The older half of the compiled kernels leaves.  Under exclusive
// g_evict_mu (every launch that looked one up is enqueued) they are taken out
// of the lookup, so no later launch can find them; the locks are then
// released (launches go on, on the kernels that stay) while the devices that
// ran them drain, and only then are their modules unloaded.
void jit_evict_now() {
    Jit& j = jit();
    std::vector<std::shared_ptr<Entry>> victims;
    std::set<int> devs;
    {
        std::unique_lock<std::shared_mutex> ex(evict_mu());
        std::lock_guard<std::mutex> lk(j.mu);
        if (!j.evict_wanted.load(std::memory_order_acquire)) return;
        std::vector<std::pair<uint64_t, std::string>> loaded;
        for (auto& kv : j.entries)
            if (kv.second->state == Entry::kLoaded || kv.second->state == Entry::kFailed ||
                kv.second->state == Entry::kReady)
                loaded.emplace_back(kv.second->last_use, kv.first);
        std::sort(loaded.begin(), loaded.end());
        loaded.resize(std::max<size_t>(loaded.size() / 2, std::min<size_t>(loaded.size(), 1)));
        for (auto& x : loaded) {
            auto it = j.entries.find(x.second);
            if (it->second->module) devs.insert(it->second->dev);
            victims.push_back(std::move(it->second));
            j.entries.erase(it);
        }
        ++j.evictions;
        j.evict_wanted.store(false, std::memory_order_release);
    }
    if (!devs.empty()) {
        detail::engines_quiesce();  // (resident host-call engines would hold the sync for their idle window)
        int cur = 0;
        (void)hipGetDevice(&cur);
        for (int dv : devs) {
            (void)hipSetDevice(dv);
            (void)hipDeviceSynchronize();
        }
        (void)hipSetDevice(cur);
    }
    for (auto& e : victims)
        if (e->module) (void)hipModuleUnload(e->module);
}

static void jit_evict() { jit_evict_now(); }

// A launch never drains the device itself: a full kernel table queues the
// eviction on the worker (this launch takes the table kernels meanwhile).
std::shared_lock<std::shared_mutex> jit_launch_guard() {
    Jit& j = jit();
    if (j.evict_wanted.load(std::memory_order_acquire)) {
        std::lock_guard<std::mutex> lk(j.mu);
        if (j.evict_wanted.load(std::memory_order_acquire) && !j.evict_task) {
            j.evict_task = true;
            j.ensure_worker();
            j.cv.notify_one();
        }
    }
    return std::shared_lock<std::shared_mutex>(evict_mu());
}

JitKernel jit_kernel_for(const MatmulArgs& a, int bs, uint64_t launch_bytes) {
    return lookup(a, bs, launch_bytes, g_jit_mode);
}

int jit_asm_source_text(const uint8_t* mat, int rows, int cols, bool accumulate, std::string* out) {
    if (!mat || rows < 1 || rows > kAsmMaxRows || cols < 1 || cols > kAsmMaxCols) return RS_ERR_INVAL;
    *out = asm_source(mat, rows, cols, accumulate, jit_shape(rows, cols), jit_pf_for(rows, cols), g_jit_sync, jit_waves_for(rows, cols),
                      nullptr);
    return RS_OK;
}

int jit_prepare(const uint8_t* mat, int rows, int cols, bool accumulate, bool wait) {
    if (!mat || rows < kJitMinRows || rows > jit_max_rows() || cols < 1 || cols > jit_max_cols()) return RS_ERR_INVAL;
    MatmulArgs a;
    std::memset(&a, 0, sizeof a);
    a.host_mat = mat;
    a.rows = rows;
    a.cols = cols;
    a.accumulate = accumulate ? 1 : 0;
    JitKernel k = lookup(a, 64, ~uint64_t{0}, wait ? 2 : 3);
    if (!k.fn && jit().evict_wanted.load(std::memory_order_acquire)) {  // full: make room, then once more
        jit_evict();
        k = lookup(a, 64, ~uint64_t{0}, wait ? 2 : 3);
    }
    return (k.fn || !wait) ? RS_OK : RS_ERR_DEVICE;
}

}  // namespace rsamd
