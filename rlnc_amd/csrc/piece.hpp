// piece.hpp — launch interface of the call-latency kernel in piece.hip (internal to librlnc_hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rlnc {

constexpr int kPieceCols = 1024;     // columns per workgroup (64 lanes x 16 bytes)
constexpr int kPieceMaxWaves = 16;   // source-splitting waves per workgroup

// out[r][0:width) = XOR_j coef[r][j] · in[j][0:width)  (r < n_out, j < n_in)
// in, out, in_row, out_row 16-byte aligned; in_row (and out_row when n_out > 1) >= round16(width): the last 16-byte
// slot of a row is read and written whole.  coef and out may be pinned host memory.
// Completion (flag != nullptr): the grid's x blocks are cut into chunks of chunk_blocks workgroups per output row;
// chunk c = row · chunks_per_row + x / chunk_blocks sets flag[c] = epoch (system scope) once all its workgroups'
// stores are visible.  count: piece_chunks() device words, zero before the first launch (each chunk's last workgroup
// zeroes its word again).
constexpr int kPieceInline = 256;  // coefficient bytes carried in the kernel arguments (one output row, n_in <= this)

struct PieceParams {
    const uint8_t *in;
    int64_t in_row;
    const uint8_t *coef;
    int64_t coef_row;
    uint8_t *out;
    int64_t out_row;
    int64_t width;
    int n_in, n_out;
    uint32_t *count;
    uint32_t *flag;
    uint32_t epoch;
    int chunk_blocks;
    // split > 1: the sources are also split over `split` workgroups per (row, column block) (grid z): each stores its
    // partial 1 KiB (part: split · n_out · gx slabs of 64 uint4, device memory, write-through) and adds to the block's
    // counter (pcount: n_out · gx device words, zero before the first launch); the last to add XORs the others' partials
    // in, re-arms the counter and goes on as a split = 1 workgroup (output row slot, chunk counting)
    int split;
    uint4 *part;
    uint32_t *pcount;
    // coef == nullptr: the coefficients are these bytes (n_out == 1): read from the kernel-argument segment in device
    // memory instead of across PCIe from pinned host memory (a round trip at the head of every workgroup)
    uint8_t coef_inline[kPieceInline];
    // col_waves != 0 (split == 1 only): the waves of a workgroup split the columns instead of the sources -- wave w
    // owns column block blockIdx.x · W + w and walks every source, no LDS reduction -- so a workgroup covers
    // W · kPieceCols columns and a narrow call launches W times fewer workgroups (chunk_blocks still counts workgroups)
    int col_waves;
};

// columns one workgroup covers for `waves` waves per workgroup
inline int64_t piece_cols_per_wg(const PieceParams &p, int waves) { return int64_t(kPieceCols) * (p.col_waves ? waves : 1); }

int piece_waves(int n_in);  // waves per workgroup for n_in sources
int piece_split(int n_in, int64_t blocks);  // workgroups per (row, column block) for n_in sources over `blocks` of them
int piece_chunks(const PieceParams &p, int waves);
hipError_t launch_piece(const PieceParams &p, int waves, hipStream_t s);
// dst row j = src row j (j < n) over width bytes on the call kernel's column-block grid (src may be pinned host memory)
hipError_t launch_piece_upload(const uint8_t *src, int64_t src_row, uint8_t *dst, int64_t dst_row, int64_t width, int n,
                               hipStream_t s);

}  // namespace rlnc
