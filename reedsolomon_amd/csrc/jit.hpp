// jit.hpp — run-time generated bit-sliced kernels for matrices with 5-16
// output rows that are only known at run time (Reconst of 5-16 lost vectors,
// Encode of codes without a generated network, Update / Replace with 5-16
// parity rows).  See jit.cpp and DESIGN.md §3 "Run-time bit-sliced kernels".
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <shared_mutex>
#include <string>

#include "kernels.hpp"

namespace rsamd {

// 9-16 rows: 138-221 VGPRs, no scratch (16 x 16: 2 waves/SIMD); the perm-table
// kernels run those in row groups of 8 that re-read every input
constexpr int kJitMinRows = 5, kJitMaxRows = 16, kJitMaxCols = 64;
// XOR-accumulate launches (Update / Replace) with fewer columns are not
// compiled: 1 = every one (with the old outputs loaded up front the compiled
// kernels measured 10+8 Update 6.08 vs 5.73 TB/s, Replace of 3 rows 6.13 vs
// 5.60, 16+8 Replace 6.16 vs 6.09, 16+8 Update 6.07 vs 6.23;
// profiles/r02/ab_jit_acc.log)
constexpr int kJitMinAccCols = 1;
extern int g_jit_min_acc_cols;
extern int g_jit_min_rows;         // rs_tune("jit_min_rows"): launches with fewer output rows stay on the table kernels     // rs_tune("jit_min_acc_cols"), default kJitMinAccCols

// rs_tune("jit", 0 | 1 | 2): off / compile in the background on first sight
// and launch the perm-table kernels until the code is ready (default) /
// compile on the launching thread (tests, benchmarks).
extern int g_jit_mode;
// rs_tune("jit_min_bytes"): backends 0 / 1 (hiprtc, comgr: seconds / tens of
// ms per matrix): a matrix whose launches moved fewer bytes in total starts no
// compile.  Backend 2 (machine code, 0.2-3 ms) compiles a matrix on the
// launching thread once its launches' estimated loss on the table kernels
// exceeds its estimated compile time (jit.cpp, est_compile_us).
extern uint64_t g_jit_min_bytes;
extern int g_jit_pf;
extern int g_jit_layout;        // rs_tune("jit_layout")
extern int g_jit_group_waves;   // rs_tune("jit_group_waves")
extern int g_jit_path_rows;     // rs_tune("jit_path_rows")
extern int g_jit_share;         // rs_tune("jit_share")
extern int g_jit_share_deep;    // rs_tune("jit_share_deep")
extern int g_jit_split_cols;    // rs_tune("jit_split_cols")
extern int g_jit_share_cols;    // rs_tune("jit_share_cols")
extern int g_jit_share_dma;     // rs_tune("jit_share_dma")
extern int g_jit_share_ahead;   // rs_tune("jit_share_ahead")
extern int g_jit_gray;          // rs_tune("jit_gray")
extern int g_jit_nobar;         // rs_tune("jit_nobar"), experiments build only
extern int g_jit_wide_pf, g_jit_wide_waves;  // rs_tune("jit_wide_pf" / "jit_wide_waves"): kernels of > 16 rows
extern int g_jit_sync;
extern int g_jit_waves;
// rs_tune("jit_min_launches"): background mode compiles a matrix once it has
// been launched this many times, moving jit_min_bytes in total (default 2)
extern int g_jit_min_launches;

// rs_tune("jit_backend", 2 | 1 | 0): kernels generated as gfx950 machine code
// dropped into a code-object template (jit_asm.cpp; default) | the same
// kernels as assembly assembled by comgr (12 ms - 1.7 s per matrix) | C++
// compiled by hiprtc (1-16 s, up to 16 x 64); both generated forms go up to
// 128 rows x 256 columns
extern int g_jit_backend;
int jit_max_rows();
int jit_max_cols();

// A compiled kernel for a launch: the hiprtc kernels take MatmulArgs and a
// 1-D grid of chunks (rs_bs_jit_64 / _256); the assembly kernel takes AsmArgs
// (jit_asm.hpp), grid (2 KiB chunks, stripes) and nw waves per workgroup.
struct JitKernel {
    hipFunction_t fn = nullptr;
    bool is_asm = false;
    int nw = 1;
    int layout = 0, groups = 1;  // generated kernels: AsmShape (jit_asm.hpp)
};
// The compiled kernel for this launch's matrix (a.host_mat, a.rows, a.cols,
// a.accumulate) on the current device (hiprtc kernels: `bs`-lane
// workgroups, 64 or 256), or fn == nullptr (JIT off, shape not covered, not
// compiled yet, or failed).
JitKernel jit_kernel_for(const MatmulArgs& a, int bs, uint64_t launch_bytes);
// Held from jit_kernel_for until its kernel is enqueued: compiled kernels are
// only evicted (the older half, once 256 are loaded; devices drained first)
// while no launch holds it.
std::shared_lock<std::shared_mutex> jit_launch_guard();
// The assembly source the generator emits for a matrix (tests: the CPU
// emulator in tests/asm_emu.py runs it against the oracle).
int jit_asm_source_text(const uint8_t* mat, int rows, int cols, bool accumulate, std::string* out);
void jit_count_launch();

// The kernel source for one matrix (rows x cols, row-major); exposed for the
// CPU tests (rs_jit_compile_check).
std::string jit_source(const uint8_t* mat, int rows, int cols, bool accumulate);
// Compile only (no device needed): RS_OK or RS_ERR_DEVICE.
int jit_compile_check(const uint8_t* mat, int rows, int cols, bool accumulate, double* ms);
// The generator's machine code (backend 2) equals comgr's assembly of its
// text (backend 1) byte for byte: RS_OK, or RS_ERR_DEVICE (first difference
// on stderr).  No device needed.
int jit_encoder_check(const uint8_t* mat, int rows, int cols, bool accumulate, size_t* code_bytes);
// Compile (wait: on this thread, and load on the current device) or queue
// the kernel for a matrix now, whatever its launch history (rs_jit_prepare).
int jit_prepare(const uint8_t* mat, int rows, int cols, bool accumulate, bool wait);
void jit_stats(uint64_t* compiled, uint64_t* failed, uint64_t* launches, double* compile_ms);
void jit_table_stats(uint64_t* entries, uint64_t* evictions);
// On-disk code-object cache: first-sight lookups that found a valid file,
// that found none, files written, files rejected on load (corrupt / stale).
void jit_cache_stats(uint64_t* hits, uint64_t* misses, uint64_t* writes, uint64_t* rejects);
extern int g_jit_disk_cache;  // rs_tune("jit_disk_cache", 0 | 1)

}  // namespace rsamd
