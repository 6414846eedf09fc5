// kernels.hpp — launch interface of the GF(2^8) matrix-product kernels.
//
// Everything in the reference's hot path reduces to one primitive
// (rs.go:175-203 encodePart over gmu.go:4-9 / gmu_amd64.s):
//     out[r] (=|^=) XOR_c  G[r][c] (x) in[c]          byte-wise
// applied to every stripe of a batch.  One launch computes it for all rows,
// all columns and all stripes; a lane keeps its slice of every output row in
// VGPRs, so each input byte is read from HBM once and each output byte is
// written once (no d*p call fan-out, no chunking for cache).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace rsamd {

constexpr int kMaxPtrs = 260;  // inputs + outputs of one launch (d+p <= 256, Update adds 1)

// Kernel arguments (passed by value, ~3.2 KB of kernarg).  Vector v of
// stripe s is at  ptr[v] + s * ss[sid[v]]: each vector picks one of four
// stripe strides, so inputs and outputs may live in differently strided
// regions (e.g. data and parity in separate buffers).
struct MatmulArgs {
    const uint32_t* tables;   // device perm tables, [cols][rows_pad][5] dwords
    const uint32_t* img4;     // the same as a 4-row LDS image [rup(cols, 4)][20] (rows <= 4), or null
    const uint8_t* host_mat;  // HOST copy of the rows x cols matrix (launch dispatch only; never read on device)
    int rows, cols, rows_pad;
    int nstripes;
    int accumulate;           // 0: overwrite (Encode), 1: XOR into out (updateOnly)
    int units_per_chunk;      // lane units (16 or 8 bytes) per workgroup-chunk (block * vpt)
    int nt_store;             // non-temporal output stores (overwrite mode)
    uint64_t len;             // bytes per vector
    uint64_t body;            // bytes handled by the vector kernel (multiple of 16)
    uint64_t tail_start;      // first byte handled by the byte kernel
    int64_t ss[4];            // stripe strides in bytes, selected per vector by sid
    const int32_t* stripe_ids;  // optional device list: launch stripe i is stripe stripe_ids[i]
    int64_t chunks_per_stripe;
    int64_t total_chunks;
    int cps_shift;            // log2(chunks_per_stripe) when a power of two, else -1
    uint64_t ptr[kMaxPtrs];   // inputs [0, cols), outputs [cols, cols+rows)
    uint32_t sid[kMaxPtrs];   // stride selector of each vector (0..3); dwords so the
                              // kernel reads them with scalar loads
};

// Multi-pattern mode: one pattern of rs_reconst_batch_multi.  tab_off is the
// dword offset (in MatmulArgs::tables) of the pattern's LDS image:
// multi_table_dwords(cols) dwords laid out [column][4 rows x 5 dwords], zero
// padded (rows >= nout, columns >= cols).
struct PatternDesc {
    uint32_t tab_off;
    uint32_t nout;        // <= 4 outputs
    uint16_t in_idx[256];  // the d input vectors (indexes into MatmulArgs::ptr; d+p <= 256)
    uint32_t out_idx[4];  // the output vectors
};
int multi_table_dwords(int cols);
hipError_t launch_gf_multi(MatmulArgs& a, const PatternDesc* pats, const int32_t* stripe_pat, hipStream_t stream);

// Host-call engine (engine.cpp): a resident kernel that serves small
// synchronous host calls through a doorbell in host memory instead of one
// launch + stream sync per call (DESIGN.md §5 "Host-call engine").
// Everything below lives in fine-grained (coherent) pinned host memory that
// the kernel reads and writes over PCIe.
constexpr int kEngineMaxRows = 8, kEngineMaxCols = 32, kEngineMaxWaves = 64;
struct EngineHeader {      // one 64-byte line; the host writes seq0 and seq1 LAST
    uint64_t seq0;         // doorbell value (first word of the line)
    uint64_t base;         // device address of stripe 0, vector 0
    uint64_t stride;       // bytes between stripes
    uint32_t pitch;        // bytes between the vectors of a stripe (16-byte multiple)
    uint32_t units;        // 16-byte units per vector (pitch / 16: whole slots, padding included)
    uint32_t nstripes;
    uint16_t rows, cols;   // <= kEngineMaxRows / kEngineMaxCols
    uint32_t flags;        // bit 0: XOR into the output rows (Update / Replace); bit 1: the buffer is
                           // coherent (fine-grained) memory, no cache invalidate / write-back needed
    uint32_t tab_id;       // identity of EngineRing::tables (reloaded into LDS when it changes)
    uint64_t reserved;
    uint64_t seq1;         // doorbell value again (last word of the line)
};
static_assert(sizeof(EngineHeader) == 64, "one cache line, seq1 in its last word");
struct EngineRing {
    EngineHeader hdr;
    uint64_t stop;                      // host -> kernel: leave now
    uint64_t pad[7];
    uint64_t done[kEngineMaxWaves];     // workgroup w -> host: last doorbell value it completed
    uint32_t tables[kEngineMaxCols * kEngineMaxRows * 5];  // perm tables, [col][row][5] dwords
};
// Launch the resident engine: `waves` workgroups of 64 lanes on `stream`,
// serving doorbells after `start`; each workgroup leaves on `stop` or after
// `idle_ticks` of the 100 MHz realtime counter without a doorbell.
hipError_t launch_engine(EngineRing* ring_dev, int waves, uint64_t start, uint64_t idle_ticks, hipStream_t stream);

// Launch tuning knobs (read from the environment once).
struct LaunchTuning {
    int max_grid;     // cap on workgroups of the vector kernel (0 = one per chunk)
    int vpt;          // 16-byte units per lane per chunk (1 or 2)
    int nt_store;     // non-temporal parity stores
    int var;          // experimental 10+4 code shape (RSAMD_VAR), -1 = default
    int lds_pad;      // minimum dynamic LDS per workgroup (caps occupancy; experiments)
    int lane_bytes;   // one-chunk and multi-pattern kernels: bytes per lane unit (8 default | 16)
    int block8;       // one-chunk kernels with 8-byte units: lanes per workgroup (256 or 128)
    int bitslice;     // bit-sliced Encode for the generated fixed generator matrices (1 default | 0)
    int bs_block;     // bit-sliced Encode: lanes per workgroup (64 | 128 | 256; 0 = per-layout rule)
    int wide_block;   // 16-byte-unit one-chunk kernels (3-8 rows over runtime columns): lanes (256 | 128)
};
LaunchTuning& tuning();

// Enqueue the product on `stream`.  Splits the work into the 16-byte vector
// body (aligned pointers/strides) and a byte-granular remainder.  Returns a
// hipError_t.
hipError_t launch_gf_matmul(MatmulArgs& a, hipStream_t stream);

// Human-readable name of the vector kernel instantiation that
// launch_gf_matmul picks for (rows, cols, accumulate) — used by the profiler
// scripts to find the dominant kernel in rocprof output.
const char* vector_kernel_name(int rows, int cols, int accumulate);

}  // namespace rsamd
