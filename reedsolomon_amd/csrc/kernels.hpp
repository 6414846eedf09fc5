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
    const uint32_t* wide;     // the same for the wide kernels (rows > 8): [column pair][rows_pad][12], or null
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
// multi_table_dwords(cols, max_out) dwords laid out [column][R rows x 5
// dwords], R = multi_image_rows(max_out) (4, or 8 when a pattern of the batch
// has more than 4 outputs), zero padded (rows >= nout, columns >= cols).
constexpr int kMultiMaxOut = 8;
struct PatternDesc {
    uint32_t tab_off;
    uint32_t nout;        // <= kMultiMaxOut outputs
    uint16_t in_idx[256];  // the d input vectors (indexes into MatmulArgs::ptr; d+p <= 256)
    uint32_t out_idx[kMultiMaxOut];  // the output vectors
};
__host__ __device__ inline int multi_image_rows(int max_out) { return max_out > 4 ? 8 : 4; }
int multi_table_dwords(int cols, int max_out);
hipError_t launch_gf_multi(MatmulArgs& a, const PatternDesc* pats, const int32_t* stripe_pat, hipStream_t stream);
// GPU planner of the multi-pattern kernel's inputs (gf_plan_multi): for each
// distinct need mask, the pattern's table image (tdw dwords at tabs + i * tdw)
// and its descriptor, as reconst_multi builds them on the host.  Every pattern
// must need 1-kMultiMaxOut vectors, none past d + p (validated on the host).
struct PlanArgs {
    const uint64_t* masks;    // npat x words need masks (mapped pinned host memory, read in place)
    const int32_t* pat_src;   // stripe -> pattern map, nstripes (mapped pinned host memory)
    int32_t* pat_dst;         // its device copy, for the multi kernel (the planner copies it)
    uint32_t* tabs;
    PatternDesc* descs;
    int npat, words, d, p, tdw, nstripes;
    int img_rows;             // multi_image_rows(the batch's most outputs): 4 or 8
};
hipError_t launch_gf_plan_multi(const PlanArgs& a, hipStream_t stream);
// Copy `bytes` (a multiple of 16) from mapped pinned host memory (its device
// address) to device memory with a kernel on `stream`: the upload ring's copy
// (UploadLease::upload) without a DMA engine or a cross-stream wait.
hipError_t launch_copy_in(uint8_t* dst, const uint8_t* src_host_dev, size_t bytes, hipStream_t stream);

// Host-call engine (engine.cpp): a resident kernel that serves small
// synchronous host calls through doorbells in host memory instead of one
// launch + stream sync per call (DESIGN.md §5 "Host-call engine").
// Everything below lives in fine-grained (coherent) pinned host memory that
// the kernel reads and writes over PCIe.  Calls are numbered 1, 2, ...; call
// q is described in slot q % kEngineSlots, so up to kEngineSlots calls can be
// in flight (the host reuses a slot only once every workgroup is past it).
constexpr int kEngineMaxRows = 8, kEngineMaxCols = 32;
constexpr int kEngineMaxGroups = 64, kEngineMaxGroupWaves = 8;  // workgroups; waves (of 64 lanes) per workgroup
constexpr int kEnginePtrLines = 6;  // vector-address lines: 7 addresses + a tag each, >= 40 addresses
constexpr int kEngineSlots = 8;
struct EngineHeader {      // one 64-byte line; the host writes seq0 and seq1 LAST
    uint64_t seq0;         // call number (first word of the line)
    uint64_t base;         // device address of stripe 0, vector 0 (batch mode)
    uint64_t stride;       // bytes between stripes
    uint32_t pitch;        // bytes between the vectors of a stripe (16-byte multiple; batch mode)
    uint32_t units;        // 16-byte units per vector (whole slots, padding included)
    uint32_t nstripes;
    uint16_t rows, cols;   // <= kEngineMaxRows / kEngineMaxCols
    uint32_t flags;        // bit 0: XOR into the output rows (Update / Replace); bit 1: the buffer is
                           // coherent (fine-grained) memory, no cache invalidate / write-back needed;
                           // bit 2: workgroup 0 writes EngineRing::stamp (diagnostics);
                           // bit 3: address mode: vector i of the (single) stripe is at
                           // EngineSlot::ptr[i / 7][i % 7] instead of base + i * pitch;
                           // bit 4: rows across waves (wave r of each workgroup computes row r;
                           // a lone call, rows <= waves per workgroup);
                           // bits 8-15: first workgroup of the call, 16-23: its workgroups
                           // (wrapping; the others pass the call without work)
    uint32_t tab_id;       // identity of the slot's tables (reloaded into LDS when it changes)
    uint64_t stop;         // host -> kernel: instances with an epoch up to this leave (polled with the doorbell)
    uint64_t seq1;         // call number again (last word of the line)
};
static_assert(sizeof(EngineHeader) == 64, "one cache line, seq1 in its last word");
// Everything the kernel polls is in a slot's first 7 lines: the header and
// the address lines, each address line tagged with its call's number in its
// last word (a line read before the host rewrote it shows an old tag).
struct EngineSlot {
    EngineHeader hdr;
    uint64_t ptr[kEnginePtrLines][8];   // address mode: [line][0..6] device addresses, [line][7] tag
    uint32_t tables[kEngineMaxCols * kEngineMaxRows * 5];  // perm tables, [col][row][5] dwords
};
struct EngineRing {
    EngineSlot slot[kEngineSlots];
    uint64_t done[kEngineMaxGroups];    // workgroup w -> host: last call it completed
    uint64_t gone[kEngineMaxGroups];    // workgroup w -> host: epoch of the instance it left
    uint64_t stamp[8];                  // diagnostics (flags bit 2), workgroup 0, 100 MHz realtime:
                                        // call seen, tables ready, stores done, released, call number
};
// Launch the resident engine instance `epoch`: `groups` workgroups of
// `waves_per_group` waves on `stream`; workgroup w serves the calls after
// max(start, done[w]), in order.  Wave 0 of each workgroup polls the slot of
// its next call.  Each workgroup leaves when that slot's stop word reaches
// its epoch, after `idle_ticks` of the 100 MHz realtime counter without a
// call, or once it has run `life_ticks` (checked between calls; bounds how
// long a device-wide synchronisation can wait for the instance), and records
// `epoch` in its `gone` word.
// poll_gap_ticks > 0: two doorbell reads in flight, the second issued that
// many ticks after the first (pipelined polls); 0: one read per round trip.
// vslots != nullptr: the call slots live there (device memory the host
// writes through the BAR, engine.cpp) instead of in ring->slot.
hipError_t launch_engine(EngineRing* ring_dev, const EngineSlot* vslots, int groups, int waves_per_group,
                         uint64_t start, uint64_t epoch, uint64_t idle_ticks, uint64_t life_ticks,
                         uint32_t poll_gap_ticks, hipStream_t stream);

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
    int wide_single_pass;  // > 8 rows without a compiled network: single-pass wide kernels (1) | row groups of 8 (0)
    int bs_waves;     // bit-sliced Encode: at most this many waves per SIMD (LDS padding; 0 = as many as fit; default 2)
    int multi_gpu_plan;  // rs_reconst_batch_multi: plan on the GPU from this many distinct patterns (0 = host,
                         // -1 = when patterns x d >= 160, where it starts to pay)
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
