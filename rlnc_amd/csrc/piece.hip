// piece.hip — the object API's call-latency kernel: a few output rows, each out[r][0:width) =
// XOR_j coef[r][j] · in[j][0:width) over GF(2^8), written straight into pinned host memory, with per-chunk
// completion flags the host spins on while it copies finished chunks into the caller's buffer.
//
// Encoder::code_with_buf (encoder.rs:241-250), Recoder::recode_with_buf (recoder.rs:122-153) and the data side of
// Decoder::get_decoded_data (decoder.rs:136-160) at the reference's small bench shapes (1 MB objects: one coded piece
// is 4-64 KiB over 16-256 sources) cost the reference 11-22 us on one EPYC core.  A GPU call there is latency, not
// bandwidth: the launch and completion round trip alone is 8-9 us on this box (scripts/ubench_call_latency.hip,
// profiles/r04_call_latency.jsonl).  So this kernel
//   * splits the sources (k) across the waves of a workgroup instead of walking them in one lane -- the GPU form of
//     the reference's `parallel` split-then-XOR-reduce (encoder.rs:175-222): a workgroup owns 1 KiB of columns (16
//     bytes a lane), each of its W waves multiplies ceil(k / W) source rows and the W partial sums meet in LDS;
//   * reads the coefficients where the host left them (pinned memory: no H2D copy before the launch), one per lane,
//     and turns each lane's coefficient into its 3-bit-split v_perm tables (kernels.hip) in registers; the wave then
//     broadcasts row j's tables with v_readlane (no LDS table stage, no barrier before the arithmetic);
//   * writes the output rows into pinned host memory (no D2H copy after it) with write-through stores and, per chunk
//     of workgroups, counts finished workgroups in device memory; the chunk's last one raises its host flag, so the
//     host copies chunk c into the caller's buffer while the device still writes chunk c + 1, and never calls
//     hipStreamSynchronize (≈ 3 us of the round trip).  No release fence anywhere: a fence writes back the XCD's L2
//     (1.7-6.5 us), per workgroup -- 1 MiB rows took 4x longer with one (profiles/r04_object_api_bench.txt).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gf256.hpp"
#include "kernels_common.hpp"
#include "piece.hpp"

namespace rlnc {

namespace {

constexpr int kPF = 16;  // source rows in flight per lane
constexpr int kSysWriteThrough = 17;  // buffer cache-policy bits sc0 | sc1: write-through to system scope
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rl(uint32_t v, int lane) {
    return uint32_t(__builtin_amdgcn_readlane(int(v), lane));
}

// acc ^= c·x for the 16 bytes of x, c's tables t (wave-uniform)
__device__ __forceinline__ void mac16(uint32_t (&acc)[4], const uint4 x, uint32_t t0lo, uint32_t t0hi, uint32_t t1lo,
                                      uint32_t t1hi, uint32_t t2) {
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t s0 = w[q] & 0x07070707u, s1 = (w[q] >> 3) & 0x07070707u, s2 = (w[q] >> 6) & 0x03030303u;
        acc[q] = xor3(xor3(acc[q], vperm(t0hi, t0lo, s0), vperm(t1hi, t1lo, s1)), vperm(t2, t2, s2), 0u);
    }
}

// grid (ceil(width / columns per workgroup), n_out, split); block 64·W threads (W = 1, 2, 4, 8 or 16 waves)
__global__ __launch_bounds__(64 * kPieceMaxWaves) void gf_piece_kernel(PieceParams p) {
    __shared__ uint4 red[kPieceMaxWaves - 1][64];
    const int W = int(blockDim.x) >> 6;
    const int w = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
    const int row = int(blockIdx.y);
    // this workgroup's sources: part z of `split` (z = blockIdx.z), then wave w's share of them
    const int RS = (p.n_in + p.split - 1) / p.split;
    const int s0 = min(p.n_in, int(blockIdx.z) * RS), s1 = min(p.n_in, s0 + RS);
    const int R = p.col_waves ? s1 - s0 : (s1 - s0 + W - 1) / W;
    const int r0 = p.col_waves ? s0 : min(s1, s0 + w * R), r1 = min(s1, r0 + R);
    const int64_t cblk = p.col_waves ? int64_t(blockIdx.x) * W + w : int64_t(blockIdx.x);
    const int64_t col = cblk * kPieceCols + lane * 16;
    const bool live = col < p.width;
    // source rows are padded to 16 bytes (in_row >= round16(width)): the last slot loads whole.  Every load is
    // unconditional from a valid address (lanes past the width read column 0, rows past the batch its last row), so
    // the loads stay plain global loads with no per-lane select
    const uint8_t *src = p.in + (live ? col : 0);
    const uint8_t *coef = p.coef ? p.coef + int64_t(row) * p.coef_row : p.coef_inline;
    uint32_t acc[4] = {0u, 0u, 0u, 0u};
    for (int b0 = r0; b0 < r1; b0 += 64) {
        const int nb = min(64, r1 - b0);
        uint4 x[kPF];
        // the first rows' loads go out before the coefficient read (a PCIe round trip when it sits in host memory)
#pragma unroll
        for (int u = 0; u < kPF; ++u) x[u] = *reinterpret_cast<const uint4 *>(src + int64_t(b0 + min(u, nb - 1)) * p.in_row);
        uint32_t t0lo, t0hi, t1lo, t1hi, t2;
        perm_table_regs(lane < nb ? coef[b0 + lane] : 0u, t0lo, t0hi, t1lo, t1hi, t2);
        for (int j0 = 0; j0 < nb; j0 += kPF) {
#pragma unroll
            for (int u = 0; u < kPF; ++u) {
                const int j = j0 + u;
                if (j < nb) {  // wave-uniform
                    const uint4 xv = x[u];
                    if (j + kPF < nb) x[u] = *reinterpret_cast<const uint4 *>(src + int64_t(b0 + j + kPF) * p.in_row);
                    mac16(acc, xv, rl(t0lo, j), rl(t0hi, j), rl(t1lo, j), rl(t1hi, j), rl(t2, j));
                }
            }
        }
    }
    if (W > 1 && !p.col_waves) {
        if (w > 0) red[w - 1][lane] = make_uint4(acc[0], acc[1], acc[2], acc[3]);
        __syncthreads();
        if (w == 0)
            for (int v = 0; v < W - 1; ++v) {
                const uint4 o = red[v][lane];
                acc[0] ^= o.x;
                acc[1] ^= o.y;
                acc[2] ^= o.z;
                acc[3] ^= o.w;
            }
    }
    if (p.split > 1) {
        // every wave but wave 0 is done; wave 0 publishes this workgroup's partial and counts it (the hand-off form of
        // MI355X_MICROARCH.md §inter-workgroup visibility: write-through stores drained by s_waitcnt vmcnt(0), one
        // lane's agent-scope add, the last adder -- told by the value its add returned -- loads the others' bytes with
        // write-through loads), and only the last of the block's `split` workgroups goes on to the output
        if (w > 0) return;
        const int64_t blk = int64_t(row) * gridDim.x + blockIdx.x;
        const __amdgpu_buffer_rsrc_t prs =
            __builtin_amdgcn_make_buffer_rsrc(p.part + blk * p.split * 64, 0, 0x7FFFFFFF, 0x00020000);
        const u32x4 mine = {acc[0], acc[1], acc[2], acc[3]};
        __builtin_amdgcn_raw_buffer_store_b128(mine, prs, int((blockIdx.z * 64 + lane) * 16), 0, kSysWriteThrough);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint32_t prev = 0;
        if (lane == 0) prev = __hip_atomic_fetch_add(p.pcount + blk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        prev = uint32_t(__shfl(int(prev), 0));
        if (prev != uint32_t(p.split - 1)) return;
        if (lane == 0) __hip_atomic_store(p.pcount + blk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int z = 0; z < p.split; ++z) {
            if (z == int(blockIdx.z)) continue;
            const u32x4 o = __builtin_amdgcn_raw_buffer_load_b128(prs, (z * 64 + lane) * 16, 0, kSysWriteThrough);
            acc[0] ^= o.x;
            acc[1] ^= o.y;
            acc[2] ^= o.z;
            acc[3] ^= o.w;
        }
    }
    // the output row is padded to 16 bytes too (out_row >= round16(width)): the last slot stores whole.  Stores are
    // write-through to system scope (sc0 sc1), so no release fence (an L2 write-back per workgroup) is needed before
    // the workgroup is counted: every storing wave drains its stores, the workgroup meets at a barrier, one lane adds
    // to the chunk's counter (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms), and the chunk's last
    // workgroup raises the host flag with a write-through store
    if ((w == 0 || p.col_waves) && live) {
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(p.out + int64_t(row) * p.out_row, 0, 0x7FFFFFFF, 0x00020000);
        const u32x4 v = {acc[0], acc[1], acc[2], acc[3]};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, int(col), 0, kSysWriteThrough);
    }
    if (p.flag == nullptr) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (p.split == 1) __syncthreads();  // (split > 1: wave 0 is the only one left)
    if (p.chunk_blocks == 1) {  // a flag per workgroup: no counter
        if (threadIdx.x == 0)
            __hip_atomic_store(p.flag + int64_t(row) * gridDim.x + blockIdx.x, p.epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    if (threadIdx.x == 0) {
        const int cpr = (int(gridDim.x) + p.chunk_blocks - 1) / p.chunk_blocks;  // chunks per row
        const int cx = int(blockIdx.x) / p.chunk_blocks;
        const int chunk = row * cpr + cx;
        const unsigned in_chunk = unsigned(min(p.chunk_blocks, int(gridDim.x) - cx * p.chunk_blocks));
        const unsigned prev = __hip_atomic_fetch_add(p.count + chunk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == in_chunk - 1) {
            __hip_atomic_store(p.count + chunk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(p.flag + chunk, p.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Recoder::new's upload of small objects: dst row j = src row j (src: pinned host memory), on the call kernel's grid
// (x = 1 KiB column block, one workgroup per block) so that each block's lines are written through the L2 of the XCD
// the recode call's workgroup for that block runs on, and its loads hit there instead of HBM (the DMA upload leaves
// them cold: 1.2-1.8 us per call, profiles/r06_objwarm_ab.txt).  width, src_row, dst_row multiples of 16.
__global__ __launch_bounds__(256) void piece_upload_kernel(const uint8_t *src, int64_t src_row, uint8_t *dst,
                                                          int64_t dst_row, int64_t width, int n) {
    const int W = int(blockDim.x) >> 6;
    const int w = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
    const int64_t col = int64_t(blockIdx.x) * kPieceCols + lane * 16;
    if (col >= width) return;
    for (int j = w; j < n; j += W)
        *reinterpret_cast<uint4 *>(dst + int64_t(j) * dst_row + col) =
            *reinterpret_cast<const uint4 *>(src + int64_t(j) * src_row + col);
}

}  // namespace

hipError_t launch_piece_upload(const uint8_t *src, int64_t src_row, uint8_t *dst, int64_t dst_row, int64_t width, int n,
                               hipStream_t s) {
    if (n <= 0 || width <= 0 || ((width | src_row | dst_row) & 15) || src_row < width || dst_row < width ||
        ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15))
        return hipErrorInvalidValue;
    const int64_t gx = (width + kPieceCols - 1) / kPieceCols;
    if (gx > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(piece_upload_kernel, dim3(unsigned(gx)), dim3(256), 0, s, src, src_row, dst, dst_row, width, n);
    return hipGetLastError();
}

// rows per wave: 2-8 for up to 32 sources (4 waves), 8-16 for up to 128 (8 waves), 16 waves beyond -- the fastest of
// 2/4/8/16 waves at each of the reference's 1 MB bench shapes (profiles/r04_piece_waves_ab.txt; one wave per source
// measured 1-1.5 us slower at 16-64 sources: more waves to launch and to reduce)
int piece_waves(int n_in) { return n_in <= 32 ? 4 : n_in <= 128 ? 8 : kPieceMaxWaves; }

// More than 128 sources over few column blocks (the 1 MB encode at k = 256: 5 blocks): about 64 sources per workgroup,
// at most 32 workgroups per block.  The hand-off (partial stores drained, the counter, the last workgroup's loads)
// costs ~2-3 us, which only pays where a workgroup would otherwise walk 16 sources a wave: 1 MB encode at k = 256
// kernel 12.1 -> 8.9 us (call 17.0-17.3 -> 14.2-15.1), while at 128 sources (k = 128 encode, k = 256 recode) the
// split measured no faster or slower (profiles/r04_split_ab.txt).  Wide rows keep one workgroup per block (enough
// workgroups already; the partials would be extra traffic).
int piece_split(int n_in, int64_t blocks) {
    if (n_in <= 128 || blocks >= 64) return 1;
    return std::min(32, (n_in + 63) / 64);
}

int piece_chunks(const PieceParams &p, int waves) {
    const int64_t cw = piece_cols_per_wg(p, waves);
    const int64_t gx = (p.width + cw - 1) / cw;
    return int((gx + p.chunk_blocks - 1) / p.chunk_blocks) * p.n_out;
}

hipError_t launch_piece(const PieceParams &p, int waves, hipStream_t s) {
    const int64_t cw = piece_cols_per_wg(p, waves);
    const int64_t gx = (p.width + cw - 1) / cw;
    if (p.n_in <= 0 || p.n_out <= 0 || p.n_out > 65535 || gx <= 0 || gx > 0x7FFFFFFFLL || p.chunk_blocks <= 0)
        return hipErrorInvalidValue;
    if (p.coef == nullptr && (p.n_out != 1 || p.n_in > kPieceInline)) return hipErrorInvalidValue;
    if (waves != 1 && waves != 2 && waves != 4 && waves != 8 && waves != 16) return hipErrorInvalidValue;
    if (p.split < 1 || p.split > 64 || (p.split > 1 && (p.part == nullptr || p.pcount == nullptr))) return hipErrorInvalidValue;
    if (p.col_waves && p.split != 1) return hipErrorInvalidValue;
    if ((reinterpret_cast<uintptr_t>(p.in) | reinterpret_cast<uintptr_t>(p.out) | uintptr_t(p.in_row) |
         uintptr_t(p.out_row)) & 15)
        return hipErrorInvalidValue;
    const int64_t padded = (p.width + 15) & ~int64_t(15);
    if (padded > 0x7FFFFFF0LL) return hipErrorInvalidValue;  // 32-bit buffer offsets within a row
    if (p.in_row < padded || (p.n_out > 1 && p.out_row < padded)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gf_piece_kernel, dim3(unsigned(gx), unsigned(p.n_out), unsigned(p.split)), dim3(64 * waves), 0, s,
                       p);
    return hipGetLastError();
}

}  // namespace rlnc
