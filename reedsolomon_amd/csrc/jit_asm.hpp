// jit_asm.hpp — run-time bit-sliced kernels emitted as gfx950 assembly
// (jit_asm.cpp): the kernel-argument block and the generator / assembler.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <tuple>
#include <vector>

#include "kernels.hpp"

namespace rsamd {

// Kernel arguments of the generated kernels (by value, 3,136 bytes).  Vector v
// (inputs [0, cols), outputs [cols, cols + rows)) of stripe s is at
// ptr[v] + s * 16 * stride16[v]; launch stripe y (grid y, offset by stripe0
// for launches of more than 65,535 stripes) is stripe stripe_ids[stripe0 + y]
// (stripe_ids == 0: stripe0 + y).  `body` bytes of each vector are processed
// (a multiple of 16; the rest is the byte kernel's).
struct AsmArgs {
    uint32_t body;
    uint32_t stripe0;
    uint64_t stripe_ids;
    uint64_t ptr[kMaxPtrs];
    uint32_t stride16[kMaxPtrs];
};
static_assert(offsetof(AsmArgs, ptr) == 16 && offsetof(AsmArgs, stride16) == 16 + 8 * kMaxPtrs, "AsmArgs layout");

constexpr int kAsmMaxRows = 128, kAsmMaxCols = 256;  // (up to 8 waves of 16 rows)
constexpr int kAsmChunk = 2048;                      // bytes of each vector per workgroup

// How a generated kernel splits the work (every row of a code path keeps 8
// bit-plane accumulators in VGPRs, so a path holds 16 rows at most):
//   layout 0: a workgroup is nw waves over the same 2 KiB chunk of every
//     vector, wave w computing rows [w * rw, w * rw + rw) - the waves of a CU
//     run different code;
//   layout 1: a workgroup is nw waves over nw consecutive 2 KiB chunks, all
//     computing one row group [g * rw, g * rw + rw) with the same code; the G
//     row groups of a chunk group are G workgroups placed on one XCD back to
//     back (grid x = ceil(chunk groups / 8) * 8 * G), sharing its L2.
//   layout 2 (with share, more than group_waves paths): a workgroup is nw
//     waves over the same 2 KiB chunk, each computing its own path
//     (g * nw + w) and sharing the columns through LDS as below; the G row
//     groups of a chunk are G workgroups on one XCD back to back, as in
//     layout 1, so their reads of the chunk's inputs hit that XCD's L2.
//     Smaller workgroups than layout 0's for > 4 x 16 rows: several per CU.
//   share (layout 0 with several waves): the waves share the column work
//     through LDS instead of each loading and transposing every column:
//     in step s wave w loads and transposes column s * nw + w and writes its
//     bit-planes to LDS; after a barrier every wave combines the nw columns
//     of the step into its own rows (two LDS buffers, 2 x nw x 2 KiB).
struct AsmShape {
    int layout = 0;
    int nw = 1;   // waves per workgroup
    int rw = 1;   // rows per code path
    int groups = 1;  // layouts 1 / 2: row groups G (layout 1: = code paths; layout 2: paths / nw)
    int share = 0;   // layout 0, nw > 1: columns shared through LDS
    int deep = 0;    // share: two steps of loads in flight and the next column's planes read ahead
    int kcols = 1;   // share: columns each wave loads per step (one barrier per nw * kcols columns)
    int dma = 0;     // share: each wave's columns stream into a private LDS ring of `dma` steps through
                     // LDS-DMA loads (buffer_load_dwordx4 ... lds), dma - 1 steps ahead; 0 = register loads
    int ahead = 0;   // share: the next column's planes are read from LDS while this one combines
                     // (a second set of 8 plane registers; the loads stay one step ahead)
    int nobar = 0;   // DIAGNOSTIC (experiments build only, wrong results): shared columns without barriers
                     // (1), also without the column loads' vmcnt waits (2), also without the LDS waits (3)
    int gray = 0;    // the low half's subsets are built one at a time into one register, in Gray-code
                     // order, the outputs they feed updated right after (12 subset registers, not 22)
};
// deep: -1 = when the workgroup has 8 waves (one workgroup per CU whatever
// the registers: the extra 24 VGPRs cost no occupancy), 0 / 1 = off / on.
// split_small: a product of 9-16 rows runs as two paths of at most 8 rows
// (half the accumulator registers per wave) instead of one.
inline AsmShape asm_shape_base(int rows, int layout, int group_waves, int path_rows, int share, int deep,
                               int split_small, int kcols, int dma) {
    AsmShape s;
    const int pr = path_rows < 1 ? 1 : path_rows > 16 ? 16 : path_rows;
    const int paths = rows <= 16 ? (split_small && rows > 8 ? 2 : 1) : (rows + pr - 1) / pr;
    if (layout == 2 && share && rows > 16) {
        // row groups of shared-column workgroups: at most group_waves paths
        // (waves) per workgroup, G workgroups per chunk, rows spread evenly
        const int gw = group_waves < 2 ? 2 : group_waves > 8 ? 8 : group_waves;
        const int G = (paths + gw - 1) / gw;
        if (G > 1) {
            s.layout = 2;
            s.groups = G;
            s.nw = (paths + G - 1) / G;
            const int np = G * s.nw;
            s.rw = (rows + np - 1) / np;
            if ((np - 1) * s.rw < rows) {  // every path has rows
                s.share = 1;
                s.deep = 0;
                s.kcols = 1;
                s.dma = dma >= 2 ? (dma > 8 ? 8 : dma) : 0;
                return s;
            }
            s = AsmShape{};
        }
        layout = 0;  // one group: layout 0 is the same kernel
    }
    s.layout = layout == 1 ? 1 : 0;
    s.rw = (rows + paths - 1) / paths;
    // (layout 1: a power of two, the kernel maps chunks with shifts)
    s.nw = s.layout ? (group_waves >= 8 ? 8 : group_waves >= 4 ? 4 : group_waves >= 2 ? 2 : 1) : paths;
    s.groups = s.layout ? paths : 1;
    s.share = (share && !s.layout && paths > 1) ? 1 : 0;
    s.deep = s.share && (deep < 0 ? s.nw >= 8 : deep > 0) ? 1 : 0;
    s.kcols = s.share ? (kcols < 0 ? (s.nw >= 8 ? 2 : 1) : kcols < 1 ? 1 : kcols > 2 ? 2 : kcols) : 1;
    if (s.kcols > 1) s.deep = 0;
    s.dma = (s.share && s.kcols == 1 && dma >= 2) ? (dma > 8 ? 8 : dma) : 0;
    if (s.dma) s.deep = 0;
    return s;
}
inline AsmShape asm_shape(int rows, int layout, int group_waves, int path_rows = 16, int share = 0,
                          int deep = -1, int split_small = 0, int kcols = 1, int dma = 0, int ahead = 0,
                          int gray = 0) {
    AsmShape s = asm_shape_base(rows, layout, group_waves, path_rows, share, deep, split_small, kcols, dma);
    s.gray = gray ? 1 : 0;
    s.ahead = (ahead && s.share && s.kcols == 1 && !s.deep) ? 1 : 0;
    return s;
}
// LDS bytes per workgroup of a generated kernel.
//   dma (share): wave w's columns of steps s .. s + dma - 1 land in its ring
//     slots (s % dma) behind the plane buffers, (2 + dma) x nw x 2 KiB in all.
inline int asm_lds_bytes(const AsmShape& s) { return s.share ? (2 * s.kcols + s.dma) * s.nw * 2048 : 0; }
// Waves per workgroup of layout 0 (16 rows per wave at most).
inline int asm_waves(int rows) { return asm_shape(rows, 0, 1).nw; }
// (path_rows: products of more than 16 rows run in code paths of at most
// this many rows - fewer rows, fewer VGPRs, more waves per SIMD)

// The assembly source of the kernel for a rows x cols matrix (row-major),
// accumulate (XOR into the outputs) or overwrite, split as `shape` says,
// pf columns of loads in flight.  *vgprs receives the VGPRs per lane.
// sync > 0: the waves of a multi-wave workgroup meet at s_barrier every
// `sync` columns; max_waves > 1: the kernel declares enough VGPRs that at
// most that many waves share a SIMD (0: as many as its registers allow).
std::string asm_source(const uint8_t* mat, int rows, int cols, bool accumulate, const AsmShape& shape, int pf,
                       int sync, int max_waves, int* vgprs);
// Assemble + link (comgr) into a code object; false with the log on failure.
bool asm_assemble(const std::string& src, std::vector<char>* code, std::string* log, double* ms);
// The same kernel as asm_source, encoded directly as gfx950 machine code (no
// assembler): the bytes of its .text.  false (with *err) if an operand does
// not fit its encoding.
bool asm_binary(const uint8_t* mat, int rows, int cols, bool accumulate, const AsmShape& shape, int pf, int sync,
                std::vector<uint32_t>* code, int* vgprs_used, std::string* err);
// A code object for machine code from asm_binary: a template (kernel
// descriptor and metadata for the shape's waves per workgroup and LDS, the declared VGPRs,
// .text of the next size class) assembled once per process and shape, with
// the code copied into its .text.
bool asm_link_binary(const std::vector<uint32_t>& code, const AsmShape& shape, int vgprs_used, int max_waves,
                     std::vector<char>* elf, std::string* log, double* ms);
// The .text section of a code object (tests: encoder vs assembler).
bool asm_text_section(const std::vector<char>& elf, std::vector<char>* text);

}  // namespace rsamd
