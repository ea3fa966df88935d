// kernels.hip — hand-written gfx950 (CDNA4) kernels for the RLNC GF(2^8) hot path.
//
// The reference's one hot primitive is dst ^= c·src over GF(2^8) (src/common/simd/mod.rs:89-119), called
// k times per coded piece by the encoder (encoder.rs:138-141), n times per recoded piece
// (recoder.rs:146-150) and ≈k² times per object by the decoder's RREF (decoder_matrix.rs:143-211).
// On MI355X that call is far too small to launch (1 MiB ≈ 0.13 µs of HBM time), so the device operator
// is the matrix form Out = Coef ⊗ In (kernels.hpp) with one workgroup per 4 KiB column block × row tile.
//
// GF multiply on CDNA4 without MFMA (byte-field arithmetic, not a dense FP contraction):
//   c·x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6]      (3-bit split; T0/T1 8 entries, T2 4 entries)
// Each table fits in two VGPR dwords, and v_perm_b32 looks up FOUR bytes per instruction (one per byte
// lane of the selector), so one multiply-accumulate of a 32-bit word costs 3 v_perm_b32 + 1.5 v_bitop3_b32
// (3-way XOR).  The per-coefficient tables are built once per workgroup into LDS and read back as
// broadcast ds_read_b128/b32 (every lane reads the same address).  The selectors depend only on the
// source word, so they are computed once per source row and reused by all NT output rows of the tile.
//
// A second variant (NibbleLds) keeps the reference's 4-bit split tables (simd_mul_table.rs:36-80,
// LOW[c][x&15] ^ HIGH[c][x>>4]) in LDS and looks them up one byte per lane per ds_read_u8, i.e. the
// north-star's literal design; it is kept as the ablation baseline.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "../../include/rlnc_hip.h"
#include "gf256.hpp"
#include "bsj_tile.hpp"
#include "kernels.hpp"
#include "kernels_common.hpp"

namespace rlnc {

namespace {

// main loop of the 2-source perm kernel over one coefficient chunk (tables already in LDS)
template <int NT, bool VEC>
__device__ __forceinline__ void perm_chunk(const MatmulParams &p, const uint8_t *rowp, int kc, int nbytes,
                                           const uint4 (*s_t01)[NT], const uint32_t (*s_t2)[NT], uint32_t (&acc)[NT][4]) {
    const uint4 zero = make_uint4(0, 0, 0, 0);
    uint4 na = ld16<VEC>(rowp, nbytes);
    uint4 nb = kc > 1 ? ld16<VEC>(rowp + p.in_row, nbytes) : zero;
    for (int j = 0; j < kc; j += 2) {
        const uint4 xa = na, xb = nb;
        // software prefetch of the next row pair while this pair is multiplied
        if (j + 2 < kc) na = ld16<VEC>(rowp + int64_t(j + 2) * p.in_row, nbytes);
        nb = (j + 3 < kc) ? ld16<VEC>(rowp + int64_t(j + 3) * p.in_row, nbytes) : zero;
        const Sel a = selectors(xa);
        const Sel b = selectors(xb);
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const uint4 ta = s_t01[j][i];
            const uint32_t ta2 = s_t2[j][i];
            const uint4 tb = s_t01[j + 1][i];  // zero table when j+1 == kc
            const uint32_t tb2 = s_t2[j + 1][i];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t r = xor3(acc[i][q], vperm(ta.y, ta.x, a.s0[q]), vperm(ta.w, ta.z, a.s1[q]));
                r = xor3(r, vperm(ta2, ta2, a.s2[q]), vperm(tb.y, tb.x, b.s0[q]));
                acc[i][q] = xor3(r, vperm(tb.w, tb.z, b.s1[q]), vperm(tb2, tb2, b.s2[q]));
            }
        }
    }
}

// VEC: every lane owns a full, aligned 16-byte slot (all blocks but a ragged/unaligned tail)
template <int NT, bool VEC>
__global__ __launch_bounds__(kThreads) void gf_matmul_perm_kernel(MatmulParams p, int row_tiles, int col_blocks) {
    __shared__ uint4 s_t01[kKC][NT];
    __shared__ uint32_t s_t2[kKC][NT];

    const Tile t = make_tile<NT>(p, row_tiles, col_blocks);
    const uint8_t *in_base = p.in + int64_t(t.obj) * p.in_obj + t.col;
    const uint8_t *coef_base = p.coef + int64_t(t.obj) * p.coef_obj + int64_t(t.row0) * p.coef_row;

    uint32_t acc[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0u;

    for (int j0 = 0; j0 < p.n_in; j0 += kKC) {
        const int kc = min(kKC, p.n_in - j0);
        if (j0) __syncthreads();  // the previous chunk's tables are consumed
        for (int e = threadIdx.x; e < kKC * NT; e += kThreads) {
            const int i = e % NT, j = e / NT;
            const uint8_t c = (i < t.rows_here && j < kc) ? coef_base[int64_t(i) * p.coef_row + j0 + j] : uint8_t(0);
            const PermTable pt = make_perm_table(c);
            s_t01[j][i] = make_uint4(pt.t0lo, pt.t0hi, pt.t1lo, pt.t1hi);
            s_t2[j][i] = pt.t2;
        }
        __syncthreads();
        if (VEC || t.nbytes > 0)
            perm_chunk<NT, VEC>(p, in_base + int64_t(j0) * p.in_row, kc, t.nbytes, s_t01, s_t2, acc);
    }
    store_tile<NT, VEC>(p, t, acc);
    copy_header(p, t);
}

// Narrow operands (< one 4 KiB column block: the ragged k + L tail of a recode, small pieces).  The work is a
// chain over the sources, so it is latency-bound: one workgroup per (object, NT-row tile) builds the tables of ALL
// its (source, row) coefficients at once (one barrier, no per-chunk rebuild), then each lane walks the sources
// with PF source rows in flight; full 16-byte slots load and store as vectors (AL), the last partial one bytewise.
// (The perm kernel it replaces here -- two rows in flight, tables per 32-source chunk -- took 91 us for configs[3]'s
// 64-byte tail: profiles/r02_narrow_ab.txt.)
template <int NT, bool AL>
__global__ __launch_bounds__(kThreads) void gf_matmul_narrow_kernel(MatmulParams p, int row_tiles) {
    extern __shared__ uint4 narrow_lds[];  // [n_in][NT] of (t0lo, t0hi, t1lo, t1hi), then [n_in][NT] of t2
    constexpr int PF = 8;
    const int rt = int(blockIdx.x) % row_tiles, obj = int(blockIdx.x) / row_tiles;
    const int row0 = rt * NT, rows_here = min(NT, p.n_out - row0);
    uint4 *t01 = narrow_lds;
    uint32_t *t2 = reinterpret_cast<uint32_t *>(narrow_lds + p.n_in * NT);
    const uint8_t *coef_base = p.coef + int64_t(obj) * p.coef_obj + int64_t(row0) * p.coef_row;
    for (int e = threadIdx.x; e < p.n_in * NT; e += kThreads) {
        const int i = e % NT, j = e / NT;
        const PermTable pt = make_perm_table(i < rows_here ? coef_base[int64_t(i) * p.coef_row + j] : uint8_t(0));
        t01[e] = make_uint4(pt.t0lo, pt.t0hi, pt.t1lo, pt.t1hi);
        t2[e] = pt.t2;
    }
    if (p.hdr != nullptr) {  // coded-piece header (encoder.rs:246-248) when the whole product is narrow
        uint8_t *h = p.hdr + int64_t(obj) * p.hdr_obj + int64_t(row0) * p.hdr_row;
        for (int e = threadIdx.x; e < rows_here * p.n_in; e += kThreads) {
            const int i = e / p.n_in, j = e % p.n_in;
            h[int64_t(i) * p.hdr_row + j] = coef_base[int64_t(i) * p.coef_row + j];
        }
    }
    __syncthreads();
    for (int64_t col = int64_t(threadIdx.x) * kBytesPerThread; col < p.width; col += int64_t(kColBlock)) {
        const int nbytes = int(min<int64_t>(kBytesPerThread, p.width - col));
        const uint8_t *in = p.in + int64_t(obj) * p.in_obj + col;
        uint32_t acc[NT][4];
#pragma unroll
        for (int i = 0; i < NT; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0u;
        for (int j0 = 0; j0 < p.n_in; j0 += PF) {
            uint4 x[PF];
#pragma unroll
            for (int u = 0; u < PF; ++u) x[u] = load16<AL>(in + int64_t(min(j0 + u, p.n_in - 1)) * p.in_row, nbytes);
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                const int j = j0 + u;
                if (j >= p.n_in) break;
                const Sel a = selectors(x[u]);
#pragma unroll
                for (int i = 0; i < NT; ++i) {
                    const uint4 ta = t01[j * NT + i];
                    const uint32_t ta2 = t2[j * NT + i];
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        acc[i][q] = xor3(xor3(acc[i][q], vperm(ta.y, ta.x, a.s0[q]), vperm(ta.w, ta.z, a.s1[q])),
                                         vperm(ta2, ta2, a.s2[q]), 0u);
                }
            }
        }
        uint8_t *out = p.out + int64_t(obj) * p.out_obj + int64_t(row0) * p.out_row + col;
#pragma unroll
        for (int i = 0; i < NT; ++i)
            if (i < rows_here)
                store16<AL>(out + int64_t(i) * p.out_row, make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]),
                            nbytes);
    }
}

constexpr int kNarrowRows = 4;
inline size_t narrow_lds_bytes(int n_in) { return size_t(n_in) * kNarrowRows * 20; }
constexpr size_t kNarrowMaxLds = 64 * 1024;

hipError_t launch_narrow(const MatmulParams &p, bool aligned, hipStream_t s) {
    const int row_tiles = (p.n_out + kNarrowRows - 1) / kNarrowRows;
    const int64_t total = int64_t(p.n_obj) * row_tiles;
    if (total > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    const size_t lds = narrow_lds_bytes(p.n_in);
    if (aligned)
        hipLaunchKernelGGL((gf_matmul_narrow_kernel<kNarrowRows, true>), dim3(unsigned(total)), dim3(kThreads), lds, s,
                           p, row_tiles);
    else
        hipLaunchKernelGGL((gf_matmul_narrow_kernel<kNarrowRows, false>), dim3(unsigned(total)), dim3(kThreads), lds, s,
                           p, row_tiles);
    return hipGetLastError();
}

// Streaming variant for few output rows (n_out <= 3: one coded piece per pass is HBM-bound, ~1 multiply-add
// per source byte read): the perm kernel's arithmetic with PF source rows in flight per lane (it keeps one
// row pair), loaded non-temporally (each source byte is read once).  Whole aligned 4 KiB blocks only.

constexpr int kStreamFormDefault = 11;  // stream3<PF 1, VW 2, 64-bit shifts>: profiles/r02_stream_ab.txt
constexpr int kStreamPF = 2;            // rows in flight of gf_matmul_stream_kernel (2..16 A/B: r01_stream_pf_ab.txt)

template <int NT, int PF>
__global__ __launch_bounds__(kThreads) void gf_matmul_stream_kernel(MatmulParams p, int row_tiles, int col_blocks) {
    __shared__ uint4 s_t01[kKC][NT];
    __shared__ uint32_t s_t2[kKC][NT];
    const Tile t = make_tile<NT>(p, row_tiles, col_blocks);
    const uint8_t *in_base = p.in + int64_t(t.obj) * p.in_obj + t.col;
    const uint8_t *coef_base = p.coef + int64_t(t.obj) * p.coef_obj + int64_t(t.row0) * p.coef_row;
    uint32_t acc[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0u;
    for (int j0 = 0; j0 < p.n_in; j0 += kKC) {
        const int kc = min(kKC, p.n_in - j0);
        if (j0) __syncthreads();
        for (int e = threadIdx.x; e < kKC * NT; e += kThreads) {
            const int i = e % NT, j = e / NT;
            const uint8_t c = (i < t.rows_here && j < kc) ? coef_base[int64_t(i) * p.coef_row + j0 + j] : uint8_t(0);
            const PermTable pt = make_perm_table(c);
            s_t01[j][i] = make_uint4(pt.t0lo, pt.t0hi, pt.t1lo, pt.t1hi);
            s_t2[j][i] = pt.t2;
        }
        __syncthreads();
        const uint8_t *rowp = in_base + int64_t(j0) * p.in_row;
        // rows past the chunk re-read its last row (in bounds, unconditional: the loads stay countable, so
        // the compiler waits for the oldest one only instead of draining all PF)
        uint4 buf[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) buf[u] = ld16_nt(rowp + int64_t(min(u, kc - 1)) * p.in_row);
        for (int jb = 0; jb < kc; jb += PF) {
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                const int j = jb + u;
                if (j >= kc) break;
                const uint4 x = buf[u];
                buf[u] = ld16_nt(rowp + int64_t(min(j + PF, kc - 1)) * p.in_row);
                const Sel a = selectors(x);
#pragma unroll
                for (int i = 0; i < NT; ++i) {
                    const uint4 ta = s_t01[j][i];
                    const uint32_t ta2 = s_t2[j][i];
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        acc[i][q] = xor3(xor3(acc[i][q], vperm(ta.y, ta.x, a.s0[q]), vperm(ta.w, ta.z, a.s1[q])),
                                         vperm(ta2, ta2, a.s2[q]), 0u);
                }
            }
        }
    }
    store_tile<NT, true>(p, t, acc);
    copy_header(p, t);
}


// One-block streaming form with VW 16-byte slots per lane (slot v at column v * 4 KiB of a VW * 4 KiB block:
// every table read feeds VW x the bytes, VW x PF loads in flight per lane) and optionally 64-bit-shift selectors.
// tail > 0: the grid carries one more workgroup per (object, row tile) after the blocks, for the ragged tail of
// `tail` (< 4 KiB) bytes at column p.width -- saves the tail's own launch (≈ 13 us of a one-piece encode call)
template <int NT>
__device__ __forceinline__ void stream_tail(const MatmulParams &p, int row_tiles, int64_t tail, int64_t u,
                                            const uint4 (*s_t01)[NT], const uint32_t (*s_t2)[NT]) {
    const int obj = int(u / row_tiles), rt = int(u % row_tiles);
    const int row0 = rt * NT, rows_here = min(NT, p.n_out - row0), kc = p.n_in;
    const int64_t col = p.width + int64_t(threadIdx.x) * kBytesPerThread;
    const int nbytes = int(max<int64_t>(0, min<int64_t>(kBytesPerThread, p.width + tail - col)));
    if (nbytes == 0) return;
    const uint8_t *rowp = p.in + int64_t(obj) * p.in_obj + col;
    uint32_t acc[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0u;
    for (int j0 = 0; j0 < kc; j0 += 4) {  // four source rows in flight
        uint4 x[4];
#pragma unroll
        for (int u2 = 0; u2 < 4; ++u2) x[u2] = load16<true>(rowp + int64_t(min(j0 + u2, kc - 1)) * p.in_row, nbytes);
#pragma unroll
        for (int u2 = 0; u2 < 4; ++u2) {
            const int j = j0 + u2;
            if (j >= kc) break;
            const Sel a = selectors(x[u2]);
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                const uint4 ta = s_t01[j][i];
                const uint32_t ta2 = s_t2[j][i];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    acc[i][q] = xor3(xor3(acc[i][q], vperm(ta.y, ta.x, a.s0[q]), vperm(ta.w, ta.z, a.s1[q])),
                                     vperm(ta2, ta2, a.s2[q]), 0u);
            }
        }
    }
    uint8_t *outp = p.out + int64_t(obj) * p.out_obj + int64_t(row0) * p.out_row + col;
#pragma unroll
    for (int i = 0; i < NT; ++i)
        if (i < rows_here)
            store16<true>(outp + int64_t(i) * p.out_row, make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]), nbytes);
}

template <int NT, int PF, int VW, bool SH64>
__global__ __launch_bounds__(kThreads) void gf_matmul_stream3_kernel(MatmulParams p, int row_tiles, int col_blocks,
                                                                     int64_t tail) {
    __shared__ uint4 s_t01[kKC][NT];
    __shared__ uint32_t s_t2[kKC][NT];
    const int64_t blocks = int64_t(p.n_obj) * row_tiles * col_blocks;
    if (int64_t(blockIdx.x) >= blocks) {  // a ragged-tail workgroup: its tables, then the tail
        const int64_t u = int64_t(blockIdx.x) - blocks;
        const int rt = int(u % row_tiles), obj = int(u / row_tiles), row0 = rt * NT;
        const int rows_here = min(NT, p.n_out - row0);
        const uint8_t *coef_base = p.coef + int64_t(obj) * p.coef_obj + int64_t(row0) * p.coef_row;
        for (int e = threadIdx.x; e < kKC * NT; e += kThreads) {
            const int i = e % NT, j = e / NT;
            const uint8_t c = (i < rows_here && j < p.n_in) ? coef_base[int64_t(i) * p.coef_row + j] : uint8_t(0);
            const PermTable pt = make_perm_table(c);
            s_t01[j][i] = make_uint4(pt.t0lo, pt.t0hi, pt.t1lo, pt.t1hi);
            s_t2[j][i] = pt.t2;
        }
        __syncthreads();
        stream_tail<NT>(p, row_tiles, tail, u, s_t01, s_t2);
        return;
    }
    int rt, cb, obj;
    decode_block(int(blocks), row_tiles, col_blocks, rt, cb, obj);
    const int row0 = rt * NT;
    const int rows_here = min(NT, p.n_out - row0);
    const int kc = p.n_in;
    const uint8_t *rowp = p.in + int64_t(obj) * p.in_obj + int64_t(cb) * kColBlock * VW + threadIdx.x * kBytesPerThread;
    uint4 buf[PF][VW];
#pragma unroll
    for (int u = 0; u < PF; ++u)
#pragma unroll
        for (int v = 0; v < VW; ++v) buf[u][v] = ld16_nt(rowp + int64_t(min(u, kc - 1)) * p.in_row + v * kColBlock);
    const uint8_t *coef_base = p.coef + int64_t(obj) * p.coef_obj + int64_t(row0) * p.coef_row;
    for (int e = threadIdx.x; e < kKC * NT; e += kThreads) {
        const int i = e % NT, j = e / NT;
        const uint8_t c = (i < rows_here && j < kc) ? coef_base[int64_t(i) * p.coef_row + j] : uint8_t(0);
        const PermTable pt = make_perm_table(c);
        s_t01[j][i] = make_uint4(pt.t0lo, pt.t0hi, pt.t1lo, pt.t1hi);
        s_t2[j][i] = pt.t2;
    }
    __syncthreads();
    uint32_t acc[NT][VW][4];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int v = 0; v < VW; ++v) acc[i][v][0] = acc[i][v][1] = acc[i][v][2] = acc[i][v][3] = 0u;
    for (int jb = 0; jb < kc; jb += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const int j = jb + u;
            if (j >= kc) break;
            Sel a[VW];
#pragma unroll
            for (int v = 0; v < VW; ++v) {
                a[v] = SH64 ? selectors64(buf[u][v]) : selectors(buf[u][v]);
                buf[u][v] = ld16_nt(rowp + int64_t(min(j + PF, kc - 1)) * p.in_row + v * kColBlock);
            }
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                const uint4 ta = s_t01[j][i];
                const uint32_t ta2 = s_t2[j][i];
#pragma unroll
                for (int v = 0; v < VW; ++v)
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        acc[i][v][q] = xor3(xor3(acc[i][v][q], vperm(ta.y, ta.x, a[v].s0[q]), vperm(ta.w, ta.z, a[v].s1[q])),
                                            vperm(ta2, ta2, a[v].s2[q]), 0u);
            }
        }
    }
    uint8_t *outp = p.out + int64_t(obj) * p.out_obj + int64_t(row0) * p.out_row + int64_t(cb) * kColBlock * VW +
                    threadIdx.x * kBytesPerThread;
#pragma unroll
    for (int i = 0; i < NT; ++i)
        if (i < rows_here)
#pragma unroll
            for (int v = 0; v < VW; ++v)
                *reinterpret_cast<uint4 *>(outp + int64_t(i) * p.out_row + v * kColBlock) =
                    make_uint4(acc[i][v][0], acc[i][v][1], acc[i][v][2], acc[i][v][3]);
    if (p.hdr != nullptr && cb == 0) {
        uint8_t *h = p.hdr + int64_t(obj) * p.hdr_obj + int64_t(row0) * p.hdr_row;
        for (int e = threadIdx.x; e < rows_here * p.n_in; e += kThreads) {
            const int i = e / p.n_in, jj = e % p.n_in;
            h[int64_t(i) * p.hdr_row + jj] = coef_base[int64_t(i) * p.coef_row + jj];
        }
    }
}

template <int NT, int PF, int VW, bool SH64>
hipError_t launch_stream3(const MatmulParams &q, int row_tiles, int col_blocks, hipStream_t s, int64_t tail) {
    if (col_blocks % VW) return launch_stream3<NT, PF, 1, SH64>(q, row_tiles, col_blocks, s, tail);
    const int64_t total = int64_t(q.n_obj) * row_tiles * (col_blocks / VW) + (tail > 0 ? int64_t(q.n_obj) * row_tiles : 0);
    if (total > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((gf_matmul_stream3_kernel<NT, PF, VW, SH64>), dim3(unsigned(total)), dim3(kThreads), 0, s, q,
                       row_tiles, col_blocks / VW, tail);
    return hipGetLastError();
}

// Narrow-operand kernel (A/B knob, read once): RLNC_NARROW = 0 takes the round-1 perm path (two rows per workgroup)
int narrow_form() {
    static const int f = [] {
        const char *e = getenv("RLNC_NARROW");
        return e ? atoi(e) : 1;
    }();
    return f;
}

// Single-pass stream kernel form; RLNC_STREAM_FORM (A/B knob, read once): 11 = gf_matmul_stream3_kernel, 0 =
// gf_matmul_stream_kernel<NT, 2> (the other measured forms: profiles/r02_stream_ab.txt, git history before round 4)
int stream_form() {
    static const int f = [] {
        const char *e = getenv("RLNC_STREAM_FORM");
        return e ? atoi(e) : kStreamFormDefault;
    }();
    return f;
}

// tail_done: the stream3 forms also take the ragged tail (p.width - full bytes) in the same launch
template <int NT>
hipError_t launch_stream(const MatmulParams &p, int64_t full, hipStream_t s, bool &tail_done) {
    MatmulParams q = p;
    q.width = full;
    const int row_tiles = (p.n_out + NT - 1) / NT;
    const int col_blocks = int(full / kColBlock);
    const int64_t tail = p.width - full;
    tail_done = false;
    if (p.n_in <= kKC) {
        tail_done = true;
        // a launch too small to fill the device (one coded piece of a small object: latency-bound) keeps four rows
        // in flight per lane over one 4 KiB slot instead of one row pair over two
        if (stream_form() == 11 && int64_t(p.n_obj) * row_tiles * col_blocks < 1024)
            return launch_stream3<NT, 4, 1, true>(q, row_tiles, col_blocks, s, tail);
        switch (stream_form()) {
            case 11: return launch_stream3<NT, 1, 2, true>(q, row_tiles, col_blocks, s, tail);
            default: tail_done = false; break;
        }
    }
    const int64_t total = int64_t(p.n_obj) * row_tiles * col_blocks;
    if (total > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((gf_matmul_stream_kernel<NT, kStreamPF>), dim3(unsigned(total)), dim3(kThreads), 0, s, q,
                       row_tiles, col_blocks);
    return hipGetLastError();
}

// Ablation baseline: the reference's 4-bit split (LOW/HIGH nibble tables, simd_mul_table.rs:36-80) in
// LDS, one ds_read_u8 per nibble per byte per lane.
template <int NT, bool ALIGNED>
__global__ __launch_bounds__(kThreads) void gf_matmul_nibble_kernel(MatmulParams p, int row_tiles, int col_blocks) {
    __shared__ uint8_t s_tab[kKC][NT][32];  // [0:16) LOW[c][i]=c·i, [16:32) HIGH[c][i]=c·(i<<4)

    int rt, cb, obj;
    decode_block(p.n_obj * row_tiles * col_blocks, row_tiles, col_blocks, rt, cb, obj);
    const int row0 = rt * NT;
    const int rows_here = min(NT, p.n_out - row0);
    const int64_t col = int64_t(cb) * kColBlock + int64_t(threadIdx.x) * kBytesPerThread;
    const int nbytes = col < p.width ? int(min<int64_t>(kBytesPerThread, p.width - col)) : 0;
    const uint8_t *in_base = p.in + int64_t(obj) * p.in_obj + col;
    const uint8_t *coef_base = p.coef + int64_t(obj) * p.coef_obj + int64_t(row0) * p.coef_row;

    uint32_t acc[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0u;

    for (int j0 = 0; j0 < p.n_in; j0 += kKC) {
        const int kc = min(kKC, p.n_in - j0);
        if (j0) __syncthreads();
        for (int e = threadIdx.x; e < kKC * NT * 16; e += kThreads) {
            const int v = e & 15, i = (e >> 4) % NT, j = (e >> 4) / NT;
            const uint8_t c = (i < rows_here && j < kc) ? coef_base[int64_t(i) * p.coef_row + j0 + j] : uint8_t(0);
            s_tab[j][i][v] = gf_mul_slow(c, uint8_t(v));
            s_tab[j][i][16 + v] = gf_mul_slow(c, uint8_t(v << 4));
        }
        __syncthreads();
        if (nbytes > 0) {
            for (int j = 0; j < kc; ++j) {
                const uint4 x = load16<ALIGNED>(in_base + int64_t(j0 + j) * p.in_row, nbytes);
                const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int i = 0; i < NT; ++i) {
                    const uint8_t *t = s_tab[j][i];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        uint32_t r = 0;
#pragma unroll
                        for (int bb = 0; bb < 4; ++bb) {
                            const uint32_t byte = (w[q] >> (8 * bb)) & 0xFFu;
                            r |= uint32_t(t[byte & 15] ^ t[16 + (byte >> 4)]) << (8 * bb);
                        }
                        acc[i][q] ^= r;
                    }
                }
            }
        }
    }
    if (nbytes > 0) {
        uint8_t *out_base = p.out + int64_t(obj) * p.out_obj + int64_t(row0) * p.out_row + col;
#pragma unroll
        for (int i = 0; i < NT; ++i)
            if (i < rows_here)
                store16<ALIGNED>(out_base + int64_t(i) * p.out_row,
                                 make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]), nbytes);
    }
    if (p.hdr != nullptr && cb == 0) {
        uint8_t *h = p.hdr + int64_t(obj) * p.hdr_obj + int64_t(row0) * p.hdr_row;
        for (int e = threadIdx.x; e < rows_here * p.n_in; e += kThreads) {
            const int i = e / p.n_in, j = e % p.n_in;
            h[int64_t(i) * p.hdr_row + j] = coef_base[int64_t(i) * p.coef_row + j];
        }
    }
}

template <int NT, bool VEC>
hipError_t launch_one(const MatmulParams &p, int64_t width, hipStream_t s, MatmulVariant v) {
    const int row_tiles = (p.n_out + NT - 1) / NT;
    const int col_blocks = int((width + kColBlock - 1) / kColBlock);
    const int64_t total = int64_t(p.n_obj) * row_tiles * col_blocks;
    if (total <= 0) return hipSuccess;
    if (total > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    MatmulParams q = p;
    q.width = width;
    const dim3 grid{unsigned(total)}, block{unsigned(kThreads)};
    if (v == MatmulVariant::NibbleLds)
        hipLaunchKernelGGL((gf_matmul_nibble_kernel<NT, VEC>), grid, block, 0, s, q, row_tiles, col_blocks);
    else
        hipLaunchKernelGGL((gf_matmul_perm_kernel<NT, VEC>), grid, block, 0, s, q, row_tiles, col_blocks);
    return hipGetLastError();
}

// Aligned operands: whole 4 KiB column blocks go to the branch-free vector kernel, a ragged tail block
// (width % 4096) to a second launch of the byte-granular kernel.  Unaligned operands: byte kernel only.
template <int NT>
hipError_t launch_nt(const MatmulParams &p, hipStream_t s, MatmulVariant v, bool aligned) {
    if (!aligned) return launch_one<NT, false>(p, p.width, s, v);
    const int64_t full = (p.width / kColBlock) * kColBlock;
    if (full > 0) {
        hipError_t e = launch_one<NT, true>(p, full, s, v);
        if (e != hipSuccess) return e;
    }
    if (full == p.width) return hipSuccess;
    MatmulParams t = p;
    t.in = p.in + full;
    t.out = p.out + full;
    if (full > 0) t.hdr = nullptr;  // the header rows were written by the first launch
    return launch_one<NT, false>(t, p.width - full, s, v);
}


// ---------------------------------------------------------------------------------------------------
// Bit-sliced variant with one code block per coefficient (gen_bsjump.py has the derivation): the (row,
// source) work is a call into block c -- 16 v_bitop3_b32 XOR3s with the combination registers baked in and
// only the accumulator relative to the row slot -- instead of 32 GPR-index-relative XORs + 16 M0 writes.
// ---------------------------------------------------------------------------------------------------
// The program, its constants and the tile body: bsj_tile.hpp.  The shared programs' blocks are packed at their own
// sizes (gen_bsjump.py), at these offsets from the table base:
__constant__ uint32_t kBsjSharedOff[256] = RLNC_BSJ_SOFFSETS;

// stream[obj][row tile][j][row in tile] = c · RLNC_BSJ_BLOCK_BYTES (c = 0 for rows past n_out); ABS: the
// block's absolute address (64-bit, the shared-set programs call it directly): base + kBsjSharedOff[c]
template <bool ABS>
__global__ __launch_bounds__(256) void bsj_offset_kernel(const uint8_t *coef, int64_t coef_obj, int64_t coef_row,
                                                         int n_out, int n_in, int row_tiles, int tile_rows,
                                                         void *stream, uint64_t base) {
    const int64_t per_obj = int64_t(row_tiles) * n_in * tile_rows;
    const int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const int obj = blockIdx.y;
    if (e >= per_obj) return;
    const int i = int(e % tile_rows);
    const int j = int((e / tile_rows) % n_in);
    const int rt = int(e / (int64_t(tile_rows) * n_in));
    const int row = rt * tile_rows + i;
    const uint32_t c = row < n_out ? coef[int64_t(obj) * coef_obj + int64_t(row) * coef_row + j] : 0u;
    if constexpr (ABS)
        static_cast<uint64_t *>(stream)[int64_t(obj) * per_obj + e] = base + kBsjSharedOff[c];
    else
        static_cast<uint32_t *>(stream)[int64_t(obj) * per_obj + e] = c * uint32_t(RLNC_BSJ_BLOCK_BYTES);
}



template <int W, bool SHARE = false>
__global__ __launch_bounds__(64 * W) void gf_matmul_bsj_kernel(MatmulParams p, const void *stream, int row_tiles,
                                                               int col_blocks, uint64_t *probe) {
    static_assert(!SHARE || W == 4 || W == 8, "the shared-set programs are generated for 4 and 8 waves");
    int rt, cb, obj;
    decode_block(p.n_obj * row_tiles * col_blocks, row_tiles, col_blocks, rt, cb, obj);
    bsj_tile<W, SHARE, false>(p, stream, row_tiles, rt, cb, obj, 1u, nullptr);
}

// the shared program's probe launch: stores its block table's address and returns (bsj_shared_base)
__global__ __launch_bounds__(256) void gf_matmul_bsj_probe_kernel(MatmulParams p, const void *stream, uint64_t *probe) {
    bsj_tile<4, true, false>(p, stream, 1, 0, 0, 0, 1u, probe);
}

// waves per workgroup: 8 output rows each, at most 4 (a 32-row tile), no more than the rows need
inline int bsj_waves(int n_out) { return n_out <= 8 ? 1 : n_out <= 16 ? 2 : 4; }
// wide = variant 8: 64-row tiles of 8 waves (shared program) above 32 output rows
inline int bsj_waves(int n_out, bool wide) { return wide && n_out > 32 ? 8 : bsj_waves(n_out); }

// Whole 4 KiB column blocks of 16-byte-aligned operands; the ragged tail goes to the perm kernel.
bool bsj_eligible(const MatmulParams &p, bool aligned) {
    return aligned && p.width >= kBsjColBlock && p.n_out >= 4 && p.in_row < (int64_t(1) << 32) &&
           p.out_row < (int64_t(1) << 32);
}

size_t bsj_scratch_bytes(const MatmulParams &p, bool wide) {
    const int tile_rows = kBsjWaveRows * bsj_waves(p.n_out, wide);
    const int64_t tiles = (p.n_out + tile_rows - 1) / tile_rows;
    // 8 bytes per entry (absolute addresses of the shared program, 4 otherwise) + one source: the main loop
    // loads the entries of the source after the last one
    return size_t(int64_t(p.n_obj) * tiles * p.n_in * tile_rows * 8 + 512);
}

// Address of the shared-set program's block table on the current device: one probe launch per device (the
// code object does not move while the process runs).  Synchronous on `s` the first time only; base = 0 when
// that first time is inside a stream capture (the caller then takes the relative-offset program).
static hipError_t bsj_shared_base(hipStream_t s, void *scratch, uint64_t &base) {
    static std::mutex mu;
    static uint64_t bases[64] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lock(mu);
    base = 0;
    if (bases[dev] == 0) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if ((e = hipStreamIsCapturing(s, &cs)) != hipSuccess) return e;
        if (cs != hipStreamCaptureStatusNone) return hipSuccess;
        MatmulParams q{};
        q.n_obj = 1;
        q.n_out = 1;
        q.n_in = 1;
        uint64_t *slot = static_cast<uint64_t *>(scratch);
        hipLaunchKernelGGL(gf_matmul_bsj_probe_kernel, dim3(1), dim3(256), 0, s, q, scratch, slot);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        uint64_t h = 0;
        if ((e = hipMemcpyAsync(&h, slot, 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (h == 0) return hipErrorLaunchFailure;
        bases[dev] = h;
    }
    base = bases[dev];
    return hipSuccess;
}

}  // namespace

// The block-address stream of a bit-sliced jump product (one bsj_offset_kernel launch) and the launch geometry of its
// whole 4 KiB column blocks (kernels.hpp BsjPlan)
hipError_t bsj_prepare(const MatmulParams &p, hipStream_t s, void *scratch, size_t scratch_bytes, bool share,
                       bool wide, BsjPlan &b) {
    b.full = (p.width / kBsjColBlock) * kBsjColBlock;
    if (scratch == nullptr || scratch_bytes < bsj_scratch_bytes(p, share && wide)) return hipErrorInvalidValue;
    int W = bsj_waves(p.n_out, share && wide);
    bool abs = share && W >= 4;  // the shared-set programs call absolute block addresses
    uint64_t base = 0;
    if (abs) {
        hipError_t e = bsj_shared_base(s, scratch, base);
        if (e != hipSuccess) return e;
        abs = base != 0;  // first use inside a stream capture: the (bit-identical) variant-6 program this time
        share = abs;
        if (!abs) W = bsj_waves(p.n_out);
    }
    const int tile_rows = kBsjWaveRows * W;
    b.waves = W;
    b.share = share;
    b.row_tiles = (p.n_out + tile_rows - 1) / tile_rows;
    b.col_blocks = int(b.full / kBsjColBlock);
    b.total = int64_t(p.n_obj) * b.row_tiles * b.col_blocks;
    if (b.total > 0x7FFFFFFFLL || p.n_obj > 65535) return hipErrorInvalidValue;
    if (p.bsj_stream != nullptr && p.bsj_stream_rows == tile_rows && (p.bsj_stream_abs != 0) == abs) {
        // written already: by the small-object elimination (4-byte offsets) or by launch_bsj_stream ahead
        b.stream = const_cast<void *>(p.bsj_stream);
        return hipSuccess;
    }
    b.stream = scratch;
    const int64_t per_obj = int64_t(b.row_tiles) * p.n_in * tile_rows;
    if ((per_obj + 255) / 256 > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    const dim3 og(unsigned((per_obj + 255) / 256), unsigned(p.n_obj));
    if (abs)
        hipLaunchKernelGGL(bsj_offset_kernel<true>, og, dim3(256), 0, s, p.coef, p.coef_obj, p.coef_row, p.n_out,
                           p.n_in, b.row_tiles, tile_rows, b.stream, base);
    else
        hipLaunchKernelGGL(bsj_offset_kernel<false>, og, dim3(256), 0, s, p.coef, p.coef_obj, p.coef_row, p.n_out,
                           p.n_in, b.row_tiles, tile_rows, b.stream, uint64_t(0));
    return hipGetLastError();
}

namespace {

hipError_t launch_bsj(const MatmulParams &p, hipStream_t s, void *scratch, size_t scratch_bytes, int64_t &full,
                      bool share, bool wide) {
    BsjPlan b;
    hipError_t e = bsj_prepare(p, s, scratch, scratch_bytes, share, wide, b);
    full = b.full;
    if (e != hipSuccess) return e;
    MatmulParams q = p;
    q.width = b.full;
    // the marker scan of undecided objects in the tiles (MatmulParams::scan_need) when each object is one workgroup's
    // whole tile (the 1- and 2-wave programs are never the shared ones, whatever b.share says)
    const bool scan = p.scan_status != nullptr && p.scan_need != nullptr && b.waves <= 2 && b.row_tiles == 1 &&
                      b.col_blocks == 1 && b.full == p.width && p.width == kBsjColBlock && p.n_out == p.scan_k &&
                      p.out_row == p.width && p.out_obj == int64_t(p.scan_k) * p.width;
    if (!scan) q.scan_status = nullptr;
    const dim3 grid(unsigned(b.total));
    if (b.waves == 1)
        hipLaunchKernelGGL(gf_matmul_bsj_kernel<1>, grid, dim3(64), 0, s, q, b.stream, b.row_tiles, b.col_blocks,
                           nullptr);
    else if (b.waves == 2)
        hipLaunchKernelGGL(gf_matmul_bsj_kernel<2>, grid, dim3(128), 0, s, q, b.stream, b.row_tiles, b.col_blocks,
                           nullptr);
    else if (b.waves == 8)
        hipLaunchKernelGGL((gf_matmul_bsj_kernel<8, true>), grid, dim3(512), 0, s, q, b.stream, b.row_tiles,
                           b.col_blocks, nullptr);
    else if (b.share)
        hipLaunchKernelGGL((gf_matmul_bsj_kernel<4, true>), grid, dim3(256), 0, s, q, b.stream, b.row_tiles,
                           b.col_blocks, nullptr);
    else
        hipLaunchKernelGGL(gf_matmul_bsj_kernel<4>, grid, dim3(256), 0, s, q, b.stream, b.row_tiles, b.col_blocks,
                           nullptr);
    const hipError_t e2 = hipGetLastError();
    if (e2 == hipSuccess && scan && p.scan_done != nullptr) *p.scan_done = true;
    return e2;
}

// ---------------------------------------------------------------------------------------------------
// Ragged batches (wire.hip: rlnc_encode_ragged / rlnc_recode_ragged / rlnc_decode_ragged): objects of different
// shapes and buffers in ONE launch per kernel stage, driven by a device-side descriptor table (RaggedObj).  A
// workgroup finds its object by binary search over the objects' first workgroups (wg0), then runs exactly the tile
// the uniform kernels run for that object.
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ int ragged_find(const RaggedObj *objs, int n, int64_t w, bool by_idx) {
    int lo = 0, hi = n - 1;  // the last object whose start is <= w (starts ascend)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        const int64_t start = by_idx ? objs[mid].idx0 : objs[mid].wg0;
        if (start <= w)
            lo = mid;
        else
            hi = mid - 1;
    }
    return __builtin_amdgcn_readfirstlane(lo);
}

// XCD-aware global work index (as decode_block): XCD b & 7 gets a contiguous range of the launch's work items
__device__ __forceinline__ int64_t xcd_work_index(int64_t total) {
    const int64_t b = blockIdx.x;
    if ((total & 7) == 0) return (b & 7) * (total >> 3) + (b >> 3);
    return b;
}

__device__ __forceinline__ MatmulParams ragged_params(const RaggedObj &d) {
    MatmulParams q{};
    q.in = d.in + d.col0;
    q.coef = d.coef;
    q.out = d.out + d.col0;
    q.hdr = d.hdr;
    q.in_row = d.in_row;
    q.coef_row = d.coef_row;
    q.out_row = d.out_row;
    q.hdr_row = d.hdr_row;
    q.n_out = d.n_out;
    q.n_in = d.n_in;
    q.width = d.width;
    q.n_obj = 1;
    return q;
}

// the block-address stream of every object of the table (all wave classes at once): entry e of object o is the
// code block of coefficient c = coef[row][j] (0 past n_out), laid out [rt][j][row in tile] from objs[o].idx0 (in
// 8-byte units), as bsj_offset_kernel lays out one object -- its absolute address for the 4- and 8-wave classes, its
// 4-byte offset for the 1- and 2-wave ones (whose half-used space the table still reserves at 8 bytes an entry)
__global__ __launch_bounds__(256) void ragged_offset_kernel(const RaggedObj *objs, int n, int64_t entries,
                                                            uint64_t *stream, uint64_t base) {
    const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (e >= entries) return;
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (objs[mid].idx0 <= e)
            lo = mid;
        else
            hi = mid - 1;
    }
    const RaggedObj &d = objs[lo];
    const int64_t l = e - d.idx0;
    const int tr = d.tile_rows;
    const int i = int(l % tr);
    const int j = int((l / tr) % d.n_in);
    const int rt = int(l / (int64_t(tr) * d.n_in));
    const int row = rt * tr + i;
    const uint32_t c = row < d.n_out ? d.coef[int64_t(row) * d.coef_row + j] : 0u;
    if (tr > 16)  // the shared-set programs (4 and 8 waves): absolute block addresses
        stream[e] = base + kBsjSharedOff[c];
    else  // 1 and 2 waves: block offsets, 4 bytes each, packed from the object's first entry
        reinterpret_cast<uint32_t *>(stream + d.idx0)[l] = c * uint32_t(RLNC_BSJ_BLOCK_BYTES);
}

template <int W>
__global__ __launch_bounds__(64 * W) void gf_matmul_bsj_ragged_kernel(const RaggedObj *objs, int n, int64_t total,
                                                                      const uint64_t *stream) {
    // 1 and 2 waves: objects of <= 16 rows have one row tile, so no two workgroups share source rows (nothing for an
    // XCD's L2 to keep); the table lists them by source count, most first, and the launch order spreads them over the
    // XCDs and CUs as they come -- the long tiles start first and side by side, not wherever an XCD's contiguous range
    // of the launch happens to hold them (8-row recodes of 16-130 sources: profiles/r04_ragged_ab.txt)
    const int64_t w = W <= 2 ? int64_t(blockIdx.x) : xcd_work_index(total);
    const int o = ragged_find(objs, n, w, false);
    const RaggedObj &d = objs[o];
    const int64_t l = w - d.wg0;
    const int rt = int(l % d.row_tiles), cb = int(l / d.row_tiles);
    const MatmulParams q = ragged_params(d);
    bsj_tile<W, (W >= 4), false>(q, stream + d.idx0, d.row_tiles, rt, cb, 0, 1u, nullptr);
}

// tails and shapes the bit-sliced program does not take: the perm kernel's tile on one object (byte-granular
// loads, vector ones for full slots of an aligned object)
template <bool AL>
__device__ __forceinline__ void perm_ragged_tile(const MatmulParams &q, int rt, int cb) {
    constexpr int NT = kRaggedPermRows;
    __shared__ uint4 s_t01[kKC][NT];
    __shared__ uint32_t s_t2[kKC][NT];
    Tile t;
    t.obj = 0;
    t.cb = cb;
    t.row0 = rt * NT;
    t.rows_here = min(NT, q.n_out - t.row0);
    t.col = int64_t(cb) * kColBlock + int64_t(threadIdx.x) * kBytesPerThread;
    t.nbytes = t.col < q.width ? int(min<int64_t>(kBytesPerThread, q.width - t.col)) : 0;
    const uint8_t *in_base = q.in + t.col;
    const uint8_t *coef_base = q.coef + int64_t(t.row0) * q.coef_row;
    uint32_t acc[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0u;
    for (int j0 = 0; j0 < q.n_in; j0 += kKC) {
        const int kc = min(kKC, q.n_in - j0);
        if (j0) __syncthreads();
        for (int e = threadIdx.x; e < kKC * NT; e += kThreads) {
            const int i = e % NT, j = e / NT;
            const uint8_t c = (i < t.rows_here && j < kc) ? coef_base[int64_t(i) * q.coef_row + j0 + j] : uint8_t(0);
            const PermTable pt = make_perm_table(c);
            s_t01[j][i] = make_uint4(pt.t0lo, pt.t0hi, pt.t1lo, pt.t1hi);
            s_t2[j][i] = pt.t2;
        }
        __syncthreads();
        if (t.nbytes > 0) {
            const uint8_t *rowp = in_base + int64_t(j0) * q.in_row;
            for (int j = 0; j < kc; ++j) {
                const uint4 x = load16<AL>(rowp + int64_t(j) * q.in_row, t.nbytes);
                const Sel a = selectors(x);
#pragma unroll
                for (int i = 0; i < NT; ++i) {
                    const uint4 ta = s_t01[j][i];
                    const uint32_t ta2 = s_t2[j][i];
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq)
                        acc[i][qq] = xor3(xor3(acc[i][qq], vperm(ta.y, ta.x, a.s0[qq]), vperm(ta.w, ta.z, a.s1[qq])),
                                          vperm(ta2, ta2, a.s2[qq]), 0u);
                }
            }
        }
    }
    if (t.nbytes > 0) {
        uint8_t *out_base = q.out + int64_t(t.row0) * q.out_row + t.col;
#pragma unroll
        for (int i = 0; i < NT; ++i)
            if (i < t.rows_here)
                store16<AL>(out_base + int64_t(i) * q.out_row, make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]),
                            t.nbytes);
    }
    copy_header(q, t);
}

// A partial column block (the < 4 KiB tail of an object -- a recode's k coefficient bytes after its bit-sliced
// blocks, a narrow piece): S = ceil(bytes / 16) slots, so a one-lane-per-slot tile leaves most of the workgroup idle
// and walks all n_in sources one dependent load after another (~1 us each: 124 us for the 130-source recode tails of
// scripts/ragged_rate.py).  Here the sources are split over G = min(256 / S2, 32) lane groups (S2 = S rounded up to a
// power of two): group g takes sources g, g + G, ... with PF rows in flight, each lane builds the perm tables of its
// (row, source) coefficients in registers (no LDS table chunks, no barriers in the loop), and the G partial products
// are XOR-reduced through LDS.
template <bool AL>
__device__ __forceinline__ void perm_ragged_split_tile(const MatmulParams &q, int rt, int cb, uint4 *red) {
    constexpr int NT = kRaggedPermRows, PF = 4;
    const int tid = threadIdx.x;
    const int64_t c0 = int64_t(cb) * kColBlock;
    const int S = int((min<int64_t>(kColBlock, q.width - c0) + 15) / 16);
    int lg = 0;
    while ((1 << lg) < S) ++lg;
    const int S2 = 1 << lg, G = min(kThreads >> lg, 32);
    const int slot = tid & (S2 - 1), g = tid >> lg;
    const int row0 = rt * NT, rows_here = min(NT, q.n_out - row0);
    const int64_t col = c0 + int64_t(slot) * kBytesPerThread;
    const int nbytes = (g < G && slot < S) ? int(min<int64_t>(kBytesPerThread, q.width - col)) : 0;
    const uint8_t *coef_base = q.coef + int64_t(row0) * q.coef_row;
    uint32_t acc[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0u;
    if (nbytes > 0) {
        const uint8_t *in = q.in + col;
        for (int j0 = g; j0 < q.n_in; j0 += G * PF) {
            uint4 x[PF];
#pragma unroll
            for (int u = 0; u < PF; ++u)  // clamped: past n_in re-read the last source (its product is skipped)
                x[u] = load16<AL>(in + int64_t(min(j0 + u * G, q.n_in - 1)) * q.in_row, nbytes);
#pragma unroll
            for (int u = 0; u < PF; ++u) {
                const int j = j0 + u * G;
                if (j >= q.n_in) break;
                const Sel a = selectors(x[u]);
#pragma unroll
                for (int i = 0; i < NT; ++i) {
                    if (i >= rows_here) break;
                    uint32_t t0lo, t0hi, t1lo, t1hi, t2;
                    perm_table_regs(coef_base[int64_t(i) * q.coef_row + j], t0lo, t0hi, t1lo, t1hi, t2);
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq)
                        acc[i][qq] = xor3(xor3(acc[i][qq], vperm(t0hi, t0lo, a.s0[qq]), vperm(t1hi, t1lo, a.s1[qq])),
                                          vperm(t2, t2, a.s2[qq]), 0u);
                }
            }
        }
    }
    if (G > 1) {  // red[i][g][slot]: the G partials of row i, slot
#pragma unroll
        for (int i = 0; i < NT; ++i)
            if (g < G) red[(i * G + g) * S2 + slot] = make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
        __syncthreads();
    }
    // output (row i, slot): one lane each, XOR of its G partials
    for (int e = tid; e < NT * S2; e += kThreads) {
        const int i = e >> lg, sl = e & (S2 - 1);
        if (i >= rows_here || sl >= S) continue;
        const int64_t oc = c0 + int64_t(sl) * kBytesPerThread;
        const int nb = int(min<int64_t>(kBytesPerThread, q.width - oc));
        uint4 v;
        if (G > 1) {
            v = red[(i * G) * S2 + sl];
            for (int gg = 1; gg < G; ++gg) {
                const uint4 r = red[(i * G + gg) * S2 + sl];
                v.x ^= r.x;
                v.y ^= r.y;
                v.z ^= r.z;
                v.w ^= r.w;
            }
        } else {  // G = 1 (S2 = 256): lane e = slot e holds row i's product itself
            v = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int ii = 0; ii < NT; ++ii)
                if (ii == i) v = make_uint4(acc[ii][0], acc[ii][1], acc[ii][2], acc[ii][3]);
        }
        store16<AL>(q.out + int64_t(row0 + i) * q.out_row + oc, v, nb);
    }
    Tile t;
    t.obj = 0;
    t.cb = cb;
    t.row0 = row0;
    t.rows_here = rows_here;
    copy_header(q, t);
}

__global__ __launch_bounds__(kThreads) void gf_matmul_perm_ragged_kernel(const RaggedObj *objs, int n, int64_t total) {
    // the split tile's partials: NT rows x 256 lanes x 16 bytes at most (G x S2 <= 256)
    __shared__ uint4 red[kRaggedPermRows * kThreads];
    const int64_t w = xcd_work_index(total);
    const int o = ragged_find(objs, n, w, false);
    const RaggedObj &d = objs[o];
    const int64_t l = w - d.wg0;
    const int rt = int(l % d.row_tiles), cb = int(l / d.row_tiles);
    const MatmulParams q = ragged_params(d);
    const bool partial = q.width - int64_t(cb) * kColBlock < kColBlock;  // workgroup-uniform
    if (partial) {
        if (d.aligned)
            perm_ragged_split_tile<true>(q, rt, cb, red);
        else
            perm_ragged_split_tile<false>(q, rt, cb, red);
    } else if (d.aligned) {
        perm_ragged_tile<true>(q, rt, cb);
    } else {
        perm_ragged_tile<false>(q, rt, cb);
    }
}

// strided row copy (the coded pieces' coefficient headers, encoder.rs:246-248): one byte per thread
__global__ __launch_bounds__(256) void copy_rows_kernel(uint8_t *dst, int64_t dst_stride, const uint8_t *src,
                                                        int64_t src_stride, int64_t width, int64_t total) {
    const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (e >= total) return;
    const int64_t r = e / width, c = e % width;
    dst[r * dst_stride + c] = src[r * src_stride + c];
}

// ---------------------------------------------------------------------------------------------------
// element-wise primitives (simd/mod.rs:18-119); the scalar early-outs are taken on the host
// ---------------------------------------------------------------------------------------------------
template <int OP, bool ALIGNED>  // OP 0: v = c·v   1: d ^= s   2: d ^= c·s
__global__ __launch_bounds__(kThreads) void gf_vec_kernel(uint8_t *dst, const uint8_t *src, int64_t len, uint32_t t0lo,
                                                          uint32_t t0hi, uint32_t t1lo, uint32_t t1hi, uint32_t t2) {
    const int64_t stride = int64_t(gridDim.x) * kThreads * kBytesPerThread;
    for (int64_t off = (int64_t(blockIdx.x) * kThreads + threadIdx.x) * kBytesPerThread; off < len; off += stride) {
        const int nb = int(min<int64_t>(kBytesPerThread, len - off));
        const uint4 x = load16<ALIGNED>((OP == 0 ? dst : src) + off, nb);
        uint4 r;
        if (OP == 1) {
            r = x;
        } else {
            const Sel s = selectors(x);
            uint32_t o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = xor3(vperm(t0hi, t0lo, s.s0[q]), vperm(t1hi, t1lo, s.s1[q]), vperm(t2, t2, s.s2[q]));
            r = make_uint4(o[0], o[1], o[2], o[3]);
        }
        if (OP != 0) {
            const uint4 d = load16<ALIGNED>(dst + off, nb);
            r = make_uint4(r.x ^ d.x, r.y ^ d.y, r.z ^ d.z, r.w ^ d.w);
        }
        store16<ALIGNED>(dst + off, r, nb);
    }
}

template <int OP>
hipError_t launch_vec(uint8_t *dst, const uint8_t *src, int64_t len, uint8_t c, hipStream_t s) {
    if (len <= 0) return hipSuccess;
    const PermTable t = make_perm_table(c);
    const int64_t chunks = (len + kBytesPerThread - 1) / kBytesPerThread;
    const int blocks = int(std::min<int64_t>((chunks + kThreads - 1) / kThreads, 2048));
    const bool aligned = unaligned_vector_ok() || (al16(dst) && (OP == 0 || al16(src)));
    if (aligned)
        hipLaunchKernelGGL((gf_vec_kernel<OP, true>), dim3(blocks), dim3(kThreads), 0, s, dst, src, len, t.t0lo, t.t0hi,
                           t.t1lo, t.t1hi, t.t2);
    else
        hipLaunchKernelGGL((gf_vec_kernel<OP, false>), dim3(blocks), dim3(kThreads), 0, s, dst, src, len, t.t0lo, t.t0hi,
                           t.t1lo, t.t1hi, t.t2);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------
// get_final_data_len on device (decoder.rs:162-177).  Equivalent formulation: the last nonzero byte of
// the padded payload must be the boundary marker and must not sit at index 0.
// ---------------------------------------------------------------------------------------------------
// 16 lanes per object (one DPP row, 64 B a lane) scan 1 KiB chunks from the END of the payload: for any padded object the last
// nonzero byte lies in the final k bytes (Encoder::new pads with < k zeros after the marker,
// encoder.rs:95-99), so the scan normally stops after one chunk — O(1) instead of a full re-read.  The same wave
// then checks the marker and writes the object's status and length (one launch; the round-3 form wrote the index
// to scratch for a second kernel: 5.5 us more per decode of configs[0]'s 4,096 objects).
// rank != nullptr: objects of rank < k are NotAllPiecesReceivedYet (decoder.rs:137-139); the rank is loaded beside
// the first chunk (their latencies overlap) and decides the outcome; invalid_code: the status of a payload without a
// valid marker.  The row maximum is a DPP ladder (row16_max), not __shfl_xor; 16 objects per workgroup: a quarter of
// the waves of the round-4 one-wave-per-object form.
// max over one 16-lane DPP row of a 32-bit key (every lane of the row ends with it): VALU row rotations only
__device__ __forceinline__ uint32_t row16_max(uint32_t a) {
    a = max(a, uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x121, 0xf, 0xf, false)));  // row_ror:1
    a = max(a, uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x122, 0xf, 0xf, false)));  // row_ror:2
    a = max(a, uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x124, 0xf, 0xf, false)));  // row_ror:4
    a = max(a, uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x128, 0xf, 0xf, false)));  // row_ror:8
    return a;
}

constexpr int kScanObjPerWg = 16;  // 16 lanes (one DPP row) per object, 16 objects per 256-thread workgroup

template <bool ALIGNED>
__global__ __launch_bounds__(256) void final_len_scan_kernel(const uint8_t *data, int64_t obj_stride, int64_t len,
                                                             int n_obj, const int32_t *rank, int k, int32_t *status,
                                                             int64_t *final_len, int32_t invalid_code) {
    const int tid = threadIdx.x, l = tid & 15;
    const int obj = blockIdx.x * kScanObjPerWg + (tid >> 4);
    const bool valid = obj < n_obj;
    const int32_t rk = (valid && rank != nullptr) ? rank[obj] : k;
    const uint8_t *d = data + int64_t(valid ? obj : 0) * obj_stride;
    int64_t c = (len + 1023) / 1024 - 1;  // this object's chunk, from the end
    bool done = !valid;
    int64_t hit = -1;  // index of the payload's last nonzero byte
    uint32_t byte = 0;
    for (;;) {
        // (index in the chunk + 1) << 8 | byte of the last nonzero byte of this lane's 64 B, 0 = none: the maximum
        // over the object's 16 lanes is the chunk's last nonzero byte with its value
        uint32_t mine = 0;
        if (!done) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t off = c * 1024 + l * 64 + u * kBytesPerThread;
                if (off < len) {
                    const int nb = int(min<int64_t>(kBytesPerThread, len - off));
                    const uint4 x = load16<ALIGNED>(d + off, nb);
                    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (w[q]) {
                            const int b = (31 - __builtin_clz(w[q])) / 8;
                            mine = (uint32_t(l * 64 + u * kBytesPerThread + 4 * q + b + 1) << 8) |
                                   ((w[q] >> (8 * b)) & 0xFFu);
                        }
                }
            }
        }
        const uint32_t best = row16_max(mine);
        if (!done) {
            if (best) {
                hit = c * 1024 + int64_t(best >> 8) - 1;
                byte = best & 0xFFu;
                done = true;
            } else if (rk < k || c == 0) {
                done = true;  // not decoded (nothing to scan), or an all-zero payload
            } else {
                --c;
            }
        }
        if (__ballot(!done) == 0) break;
    }
    if (valid && l == 0) {
        if (rk < k) {
            status[obj] = RLNC_ERR_NOT_ALL_PIECES_RECEIVED_YET;
            final_len[obj] = 0;
        } else {
            const bool ok = hit > 0 && byte == kBoundaryMarker;  // decoder.rs:162-177
            status[obj] = ok ? RLNC_OK : invalid_code;
            final_len[obj] = ok ? hit : 0;
        }
    }
}

}  // namespace

hipError_t launch_copy_rows(uint8_t *dst, int64_t dst_stride, const uint8_t *src, int64_t src_stride, int64_t width,
                            int64_t rows, hipStream_t s) {
    const int64_t total = width * rows;
    if (total <= 0) return hipSuccess;
    if ((total + 255) / 256 > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(copy_rows_kernel, dim3(unsigned((total + 255) / 256)), dim3(256), 0, s, dst, dst_stride, src,
                       src_stride, width, total);
    return hipGetLastError();
}

hipError_t launch_final_data_len_ranked(const uint8_t *data, int64_t obj_stride, int64_t len, int n_obj, int k,
                                        const int32_t *rank, int32_t *status, int64_t *final_len, hipStream_t s) {
    if (n_obj <= 0) return hipSuccess;
    if (unaligned_vector_ok() || (al16(data) && (n_obj == 1 || al16(obj_stride))))
        hipLaunchKernelGGL(final_len_scan_kernel<true>, dim3((n_obj + kScanObjPerWg - 1) / kScanObjPerWg), dim3(256), 0,
                           s, data, obj_stride, len, n_obj, rank, k, status, final_len,
                           int32_t(RLNC_ERR_INVALID_DECODED_DATA_FORMAT));
    else
        hipLaunchKernelGGL(final_len_scan_kernel<false>, dim3((n_obj + kScanObjPerWg - 1) / kScanObjPerWg), dim3(256), 0,
                           s, data, obj_stride, len, n_obj, rank, k, status, final_len,
                           int32_t(RLNC_ERR_INVALID_DECODED_DATA_FORMAT));
    return hipGetLastError();
}

// 16-byte alignment of an operand: its base, and the strides of the dimensions that have more than one element (a
// single row's stride is never used).  On a device that executes 16-byte vector memory instructions at any byte
// address (unaligned_vector_ok) every operand counts as aligned.
static bool in_aligned(const MatmulParams &p) {
    return unaligned_vector_ok() ||
           (al16(p.in) && (p.n_in == 1 || al16(p.in_row)) && (p.n_obj == 1 || al16(p.in_obj)));
}
static bool out_aligned(const MatmulParams &p) {
    return unaligned_vector_ok() ||
           (al16(p.out) && (p.n_out == 1 || al16(p.out_row)) && (p.n_obj == 1 || al16(p.out_obj)));
}
static bool matmul_aligned(const MatmulParams &p) { return in_aligned(p) && out_aligned(p); }

// ---------------------------------------------------------------------------------------------------
// Byte-misaligned vector memory access.  gfx9 executes global_load/store_dwordx4 and global_load_lds_dwordx4 at any
// byte address when the queue's SH_MEM_CONFIG alignment mode is "unaligned" (the ROCm driver's default for compute
// queues; in "dword" mode the low address bits are dropped).  Measured on the MI355X boxes
// (scripts/ubench_unaligned.hip, profiles/r03_ubench_unaligned.jsonl): exact bytes at every offset, and a 1 GiB copy
// at 4.3-5.2 TB/s misaligned against 4.8 aligned.  A probe kernel checks it once per device; where it holds, rows at
// any alignment take the vector kernels directly, else the realigned path (realign_plan) copies them through
// 16-byte scratch rows.  RLNC_ASSUME_ALIGNED_ONLY=1 forces the realigned path (its tests).
// ---------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void unaligned_probe_kernel(const uint8_t *src, uint8_t *dst, uint8_t *dst_lds) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[64 * 4];
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const int l = threadIdx.x;
    const int off = 1 + l % 15;  // every misalignment 1..15
    const uint8_t *s = src + 32 * l + off;
    uint8_t *d = dst + 32 * l + (16 - off);
    u4 x;
    asm volatile("global_load_dwordx4 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(x) : "v"(s) : "memory");
    asm volatile("global_store_dwordx4 %0, %1, off\n s_waitcnt vmcnt(0)" ::"v"(d), "v"(x) : "memory");
    __builtin_amdgcn_global_load_lds(s, (__attribute__((address_space(3))) void *)buf, 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    reinterpret_cast<u4 *>(dst_lds)[l] = reinterpret_cast<const u4 *>(buf)[l];
}

static std::atomic<int> g_unaligned[64];  // per device: 0 not probed, 1 any byte address works, 2 not (or forced)

static bool run_unaligned_probe() {
    constexpr int kB = 4096;
    uint8_t *src = nullptr, *dst = nullptr, *dl = nullptr;
    hipStream_t st = nullptr;
    bool ok = hipMalloc(&src, kB) == hipSuccess && hipMalloc(&dst, kB) == hipSuccess && hipMalloc(&dl, kB) == hipSuccess &&
              hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess;
    std::vector<uint8_t> h(kB), g(kB), gl(kB);
    for (int i = 0; i < kB; ++i) h[i] = uint8_t(i * 73 + (i >> 8) + 1);
    if (ok) {
        ok = hipMemcpyAsync(src, h.data(), kB, hipMemcpyHostToDevice, st) == hipSuccess &&
             hipMemsetAsync(dst, 0, kB, st) == hipSuccess;
        if (ok) {
            hipLaunchKernelGGL(unaligned_probe_kernel, dim3(1), dim3(64), 0, st, src, dst, dl);
            ok = hipGetLastError() == hipSuccess &&
                 hipMemcpyAsync(g.data(), dst, kB, hipMemcpyDeviceToHost, st) == hipSuccess &&
                 hipMemcpyAsync(gl.data(), dl, kB, hipMemcpyDeviceToHost, st) == hipSuccess &&
                 hipStreamSynchronize(st) == hipSuccess;
        }
    }
    for (int l = 0; ok && l < 64; ++l) {
        const int off = 1 + l % 15;
        for (int b = 0; b < 16; ++b)
            ok = ok && g[32 * l + 16 - off + b] == h[32 * l + off + b] && gl[16 * l + b] == h[32 * l + off + b];
    }
    if (st) (void)hipStreamDestroy(st);
    for (uint8_t *x : {src, dst, dl})
        if (x) (void)hipFree(x);
    (void)hipGetLastError();  // a failed probe leaves no sticky error behind
    return ok;
}

int probe_unaligned_vector_access(int device) {
    if (device < 0 || device >= 64) return 0;
    int v = g_unaligned[device].load();
    if (v != 0) return v == 1;
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    if ((v = g_unaligned[device].load()) != 0) return v == 1;
    const char *e = getenv("RLNC_ASSUME_ALIGNED_ONLY");
    // relaxed capture mode on this thread while probing, so a context created while another stream of the process
    // is being captured neither fails nor invalidates that capture (the probe's allocations are not stream work)
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    const bool swapped = hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess;
    const bool ok = !(e != nullptr && atoi(e) != 0) && run_unaligned_probe();
    if (swapped) (void)hipThreadExchangeStreamCaptureMode(&mode);
    g_unaligned[device].store(ok ? 1 : 2);
    return ok;
}

int unaligned_vector_access(int device) {
    if (device < 0 || device >= 64) return -1;
    const int v = g_unaligned[device].load();
    return v == 0 ? -1 : v == 1;
}

bool unaligned_vector_ok() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    return g_unaligned[dev].load(std::memory_order_relaxed) == 1;
}

// ---------------------------------------------------------------------------------------------------
// Realigned products.  A piece row is rarely 16-byte aligned: Encoder::new pads to L = ceil((len + 1) / k)
// (encoder.rs:93-95), so the reference's own bench shapes (2^20..2^25 bytes over k = 16..256) give odd L, and a
// coded piece's data starts at byte k of a (k + L)-byte row.  The vector kernels need 16-byte rows; the byte-granular
// kernels run 5-7x slower.  So a misaligned operand of a product the bit-sliced or stream kernels take is copied
// into 16-byte-aligned scratch rows (input) or out of them (output) around the aligned product, in chunks of objects
// and column blocks of at most kRealignBudget bytes of scratch.
// ---------------------------------------------------------------------------------------------------
constexpr size_t kRealignBudget = size_t(512) << 20;
constexpr int kRealignDwords = 4;  // destination dwords per thread

// dst[o][r][0:w) = src[o][r][0:w) at any byte alignment of either side: thread t writes dwords of the destination's
// 4-byte grid (a dword the row covers only in part is written byte by byte, so the neighbouring bytes -- e.g. the
// coded piece's coefficient header -- are never touched), reading the source as aligned dwords joined by v_alignbyte;
// every dword read holds at least one byte of the row, so no read leaves the row's pages
__global__ __launch_bounds__(256) void realign_rows_kernel(uint8_t *dst, int64_t dst_row, int64_t dst_obj,
                                                           const uint8_t *src, int64_t src_row, int64_t src_obj,
                                                           int rows, int64_t width, int chunks) {
    const int64_t wg = blockIdx.x;
    const int64_t rr = wg / chunks;
    const int64_t ch = wg % chunks;
    const int64_t o = rr / rows, r = rr % rows;
    uint8_t *d = dst + o * dst_obj + r * dst_row;
    const uint8_t *sp = src + o * src_obj + r * src_row;
    const int dmis = int(reinterpret_cast<uintptr_t>(d) & 3);
    uint32_t *dw = reinterpret_cast<uint32_t *>(d - dmis);
    const int64_t ndw = (dmis + width + 3) >> 2;  // dword t covers row bytes [4t - dmis, 4t - dmis + 4)
#pragma unroll
    for (int u = 0; u < kRealignDwords; ++u) {
        const int64_t t = ch * (256 * kRealignDwords) + u * 256 + threadIdx.x;
        if (t >= ndw) break;
        const int64_t x0 = 4 * t - dmis;
        if (x0 >= 0 && x0 + 4 <= width) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(sp + x0);
            const uint32_t *A = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
            const uint32_t sh = uint32_t(a & 3);
            const uint32_t lo = A[0];
            const uint32_t hi = sh ? A[1] : 0u;
            dw[t] = __builtin_amdgcn_alignbyte(hi, lo, sh);  // ({hi, lo} >> 8 sh)[31:0]
        } else {
            for (int b = 0; b < 4; ++b) {
                const int64_t x = x0 + b;
                if (x >= 0 && x < width) d[x] = sp[x];
            }
        }
    }
}

static hipError_t launch_realign(uint8_t *dst, int64_t dst_row, int64_t dst_obj, const uint8_t *src, int64_t src_row,
                                 int64_t src_obj, int rows, int64_t width, int n_obj, hipStream_t s) {
    const int64_t per_wg = 256 * kRealignDwords * 4;
    const int64_t chunks = (width + 3 + per_wg) / per_wg;  // dwords of the destination grid, + 1 for its offset
    const int64_t total = int64_t(n_obj) * rows * chunks;
    if (total <= 0) return hipSuccess;
    if (total > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(realign_rows_kernel, dim3(unsigned(total)), dim3(256), 0, s, dst, dst_row, dst_obj, src, src_row,
                       src_obj, rows, width, int(chunks));
    return hipGetLastError();
}

static bool jump_variant(MatmulVariant v) {
    return v == MatmulVariant::BitSlicedJump || v == MatmulVariant::BitSlicedJumpShared ||
           v == MatmulVariant::BitSlicedJumpShared8;
}

// the shipped variants; the others (2-5, 9) are the A/B history of kernels_ab.hip (make ab)
static bool shipped_variant(MatmulVariant v) {
    return v == MatmulVariant::Perm || v == MatmulVariant::NibbleLds || jump_variant(v);
}

struct RealignPlan {
    bool in_mis = false, out_mis = false;
    int objs = 0;                           // objects per chunk
    int64_t cw = 0;                         // columns per chunk (a multiple of 4 KiB, or the whole width)
    int64_t lr = 0;                         // scratch row stride (cw rounded up to 16)
    size_t prod_bytes = 0, in_bytes = 0, out_bytes = 0;
};

size_t matmul_scratch_bytes_aligned(const MatmulParams &p, MatmulVariant v);

// The realigned form of a misaligned product that the bit-sliced or stream kernels would take if it were aligned
static bool realign_plan(const MatmulParams &p, MatmulVariant v, RealignPlan &r) {
    if (!jump_variant(v) || p.width < kColBlock || p.n_out <= 0 || p.n_in <= 0 || p.n_obj <= 0 || matmul_aligned(p))
        return false;
    r.in_mis = !in_aligned(p);
    r.out_mis = !out_aligned(p);
    const int64_t rows = (r.in_mis ? p.n_in : 0) + (r.out_mis ? p.n_out : 0);
    const int64_t whole = (p.width + 15) & ~int64_t(15);
    int64_t objs = p.n_obj, cw = whole;
    if (objs * rows * cw > int64_t(kRealignBudget)) {
        cw = std::max<int64_t>(kColBlock, int64_t(kRealignBudget) / (objs * rows) / kColBlock * kColBlock);
        if (cw >= whole) cw = whole;
        if (objs * rows * cw > int64_t(kRealignBudget)) objs = std::max<int64_t>(1, int64_t(kRealignBudget) / (rows * cw));
    }
    r.objs = int(objs);
    r.cw = cw;
    r.lr = (cw + 15) & ~int64_t(15);
    MatmulParams q = p;  // one chunk, aligned
    q.n_obj = r.objs;
    q.width = std::min<int64_t>(cw, p.width);
    q.in = q.out = nullptr;
    q.in_row = q.out_row = r.lr;
    q.in_obj = int64_t(p.n_in) * r.lr;
    q.out_obj = int64_t(p.n_out) * r.lr;
    r.prod_bytes = (matmul_scratch_bytes_aligned(q, v) + 255) & ~size_t(255);
    r.in_bytes = r.in_mis ? size_t(objs) * p.n_in * r.lr : 0;
    r.out_bytes = r.out_mis ? size_t(objs) * p.n_out * r.lr : 0;
    return true;
}

size_t bsj_stream_bytes_bound(int n_obj, int n_out, int n_in) {
    // tiles x tile_rows < n_out + 64 rows, 8 bytes an entry, + the main loop's one-source overrun
    return size_t(n_obj) * size_t(n_out + 64) * size_t(n_in) * 8 + 512;
}

hipError_t launch_bsj_stream(const MatmulParams &p, MatmulVariant v, hipStream_t s, void *buf, size_t bytes,
                             BsjStreamPlan &plan) {
    plan = BsjStreamPlan{};
    if (p.n_out <= 0 || p.width <= 0 || p.n_obj <= 0 || p.n_in <= 0 || !shipped_variant(v) || !jump_variant(v))
        return hipSuccess;
    RealignPlan r;
    if (realign_plan(p, v, r)) return hipSuccess;  // the realigned chunks write their own streams
    const bool aligned = matmul_aligned(p);
    if (aligned && p.n_out <= 3 && p.width >= kColBlock) return hipSuccess;  // the single-pass stream kernel
    if (!bsj_eligible(p, aligned)) return hipSuccess;
    const bool share = v == MatmulVariant::BitSlicedJumpShared || v == MatmulVariant::BitSlicedJumpShared8;
    const bool wide = v == MatmulVariant::BitSlicedJumpShared8;
    MatmulParams q = p;
    q.bsj_stream = nullptr;
    BsjPlan b;
    if (hipError_t e = bsj_prepare(q, s, buf, bytes, share, wide, b); e != hipSuccess) return e;
    plan.tile_rows = kBsjWaveRows * b.waves;
    plan.abs = (b.share && b.waves >= 4) ? 1 : 0;  // the shared programs (4 and 8 waves) call absolute addresses
    return hipSuccess;
}

size_t matmul_scratch_bytes(const MatmulParams &p, MatmulVariant v) {
    if (!shipped_variant(v)) return matmul_scratch_bytes_ab(p, v);
    RealignPlan r;
    if (realign_plan(p, v, r)) return r.prod_bytes + r.in_bytes + r.out_bytes;
    return matmul_scratch_bytes_aligned(p, v);
}

size_t matmul_scratch_bytes_aligned(const MatmulParams &p, MatmulVariant v) {
    if (!jump_variant(v) || p.n_out <= 0 || p.n_in <= 0 || p.n_obj <= 0) return 0;
    return bsj_eligible(p, matmul_aligned(p)) ? bsj_scratch_bytes(p, v == MatmulVariant::BitSlicedJumpShared8) : 0;
}

hipError_t launch_matmul(const MatmulParams &p, hipStream_t s, MatmulVariant v, void *scratch, size_t scratch_bytes) {
    if (p.n_out <= 0 || p.width <= 0 || p.n_obj <= 0) return hipSuccess;
    const bool aligned = matmul_aligned(p);
    if (p.n_in <= 0) return hipErrorInvalidValue;
    if (!shipped_variant(v)) {  // the A/B variants never take the in-tile marker scan
        MatmulParams q = p;
        q.scan_status = nullptr;
        return launch_matmul_ab(q, s, v, scratch, scratch_bytes);
    }
    RealignPlan r;
    if (realign_plan(p, v, r)) {  // misaligned rows: realign copies around the aligned product
        if (scratch == nullptr || scratch_bytes < r.prod_bytes + r.in_bytes + r.out_bytes) return hipErrorInvalidValue;
        uint8_t *ib = static_cast<uint8_t *>(scratch) + r.prod_bytes;
        uint8_t *ob = ib + r.in_bytes;
        for (int o0 = 0; o0 < p.n_obj; o0 += r.objs) {
            const int c = std::min(r.objs, p.n_obj - o0);
            for (int64_t c0 = 0; c0 < p.width; c0 += r.cw) {
                const int64_t w = std::min(r.cw, p.width - c0);
                MatmulParams q = p;
                q.bsj_stream = nullptr;   // laid out for the whole batch
                q.scan_status = nullptr;  // chunks of columns: no workgroup holds a whole object
                q.n_obj = c;
                q.width = w;
                q.in = p.in + int64_t(o0) * p.in_obj + c0;
                q.coef = p.coef + int64_t(o0) * p.coef_obj;
                q.out = p.out + int64_t(o0) * p.out_obj + c0;
                q.hdr = (p.hdr != nullptr && c0 == 0) ? p.hdr + int64_t(o0) * p.hdr_obj : nullptr;
                hipError_t e;
                if (r.in_mis) {
                    if ((e = launch_realign(ib, r.lr, int64_t(p.n_in) * r.lr, q.in, p.in_row, p.in_obj, p.n_in, w, c, s)) !=
                        hipSuccess)
                        return e;
                    q.in = ib;
                    q.in_row = r.lr;
                    q.in_obj = int64_t(p.n_in) * r.lr;
                }
                if (r.out_mis) {
                    q.out = ob;
                    q.out_row = r.lr;
                    q.out_obj = int64_t(p.n_out) * r.lr;
                }
                if ((e = launch_matmul(q, s, v, scratch, r.prod_bytes)) != hipSuccess) return e;
                if (r.out_mis &&
                    (e = launch_realign(p.out + int64_t(o0) * p.out_obj + c0, p.out_row, p.out_obj, ob, r.lr,
                                        int64_t(p.n_out) * r.lr, p.n_out, w, c, s)) != hipSuccess)
                    return e;
            }
        }
        return hipSuccess;
    }
    const bool jump = jump_variant(v);
    if (jump && aligned && p.n_out <= 3 && p.width >= kColBlock) {
        // one to three coded pieces per source pass: HBM-bound, streamed with deep prefetch
        const int64_t full = (p.width / kColBlock) * kColBlock;
        bool tail_done = false;
        hipError_t e = p.n_out == 1   ? launch_stream<1>(p, full, s, tail_done)
                       : p.n_out == 2 ? launch_stream<2>(p, full, s, tail_done)
                                      : launch_stream<3>(p, full, s, tail_done);
        if (e != hipSuccess || full == p.width || tail_done) return e;
        MatmulParams t = p;
        t.in = p.in + full;
        t.out = p.out + full;
        t.width = p.width - full;
        t.hdr = nullptr;
        return launch_matmul(t, s, MatmulVariant::Perm);
    }
    if (jump) {
        const bool share = v == MatmulVariant::BitSlicedJumpShared || v == MatmulVariant::BitSlicedJumpShared8;
        const bool wide = v == MatmulVariant::BitSlicedJumpShared8;
        v = MatmulVariant::Perm;  // whatever the bit-sliced kernels do not cover
        if (bsj_eligible(p, aligned)) {
            int64_t full = 0;
            hipError_t e = launch_bsj(p, s, scratch, scratch_bytes, full, share, wide);
            if (e != hipSuccess || full == p.width) return e;
            MatmulParams t = p;
            t.in = p.in + full;
            t.out = p.out + full;
            t.width = p.width - full;
            t.hdr = nullptr;
            return launch_matmul(t, s, v);
        }
    }
    // narrow (< one 4 KiB column block, e.g. the ragged tail of a recode over k + L bytes): the work is the
    // sources x rows chain of one block, so split the rows over many workgroups (2 rows each)
    // (1-2 rows too while the sources are few, e.g. the short tail of one recoded piece: 107 -> 80 us per
    // Recoder::recode_with_buf call at 16 MiB / k = 64 over 32 pieces with the small-launch stream form below; over 128+
    // sources the perm kernel's chunked tables were faster: profiles/r03_object_api_rates.jsonl)
    if (p.width < kColBlock && (p.n_out > 2 || p.n_in <= kKC)) {
        if (v == MatmulVariant::Perm && narrow_lds_bytes(p.n_in) <= kNarrowMaxLds && narrow_form() == 1)
            return launch_narrow(p, aligned, s);
        if (p.n_out > 2) return launch_nt<2>(p, s, v, aligned);
    }
    if (p.n_out <= 1) return launch_nt<1>(p, s, v, aligned);
    if (p.n_out <= 2) return launch_nt<2>(p, s, v, aligned);
    if (p.n_out <= 4) return launch_nt<4>(p, s, v, aligned);
    if (p.n_out <= 8) return launch_nt<8>(p, s, v, aligned);
    if (p.n_out <= 16) return launch_nt<16>(p, s, v, aligned);
    return launch_nt<32>(p, s, v, aligned);
}

bool bsj_eligible_public(const MatmulParams &p) { return bsj_eligible(p, matmul_aligned(p)); }
uint32_t bsj_block_bytes_public() { return uint32_t(RLNC_BSJ_BLOCK_BYTES); }
int bsj_unshared_tile_rows(int n_out) { return bsj_waves(n_out) <= 2 ? kBsjWaveRows * bsj_waves(n_out) : 0; }
size_t bsj_scratch_bytes_public(const MatmulParams &p, bool wide) { return bsj_scratch_bytes(p, wide); }

// The A/B build (make ab) links kernels_ab.hip, whose definitions replace these
__attribute__((weak)) bool ab_build() { return false; }
__attribute__((weak)) hipError_t launch_matmul_ab(const MatmulParams &, hipStream_t, MatmulVariant, void *, size_t) {
    return hipErrorInvalidValue;  // the A/B variants exist in the diagnostic build only
}
__attribute__((weak)) size_t matmul_scratch_bytes_ab(const MatmulParams &, MatmulVariant) { return 0; }

bool ragged_bsj_eligible(const uint8_t *in, const uint8_t *out, int64_t in_row, int64_t out_row, int64_t width,
                         int n_out, bool unaligned_ok) {
    return (unaligned_ok || (al16(in) && al16(out) && al16(in_row) && al16(out_row))) && width >= kBsjColBlock &&
           n_out >= 4 &&
           in_row < (int64_t(1) << 32) && out_row < (int64_t(1) << 32);
}

int ragged_bsj_waves(int n_out) { return n_out > 32 ? 8 : bsj_waves(n_out); }

hipError_t ragged_bsj_base(hipStream_t s, void *probe_scratch, uint64_t &base) {
    return bsj_shared_base(s, probe_scratch, base);
}

hipError_t launch_ragged_offsets(const RaggedObj *objs, int n, int64_t entries, void *stream, uint64_t base,
                                 hipStream_t s) {
    if (entries <= 0) return hipSuccess;
    if ((entries + 255) / 256 > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(ragged_offset_kernel, dim3(unsigned((entries + 255) / 256)), dim3(256), 0, s, objs, n, entries,
                       static_cast<uint64_t *>(stream), base);
    return hipGetLastError();
}

hipError_t launch_ragged_bsj(int W, const RaggedObj *objs, int n, int64_t wgs, const void *stream, hipStream_t s) {
    if (wgs <= 0) return hipSuccess;
    if (wgs > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    const uint64_t *st = static_cast<const uint64_t *>(stream);
    if (W == 8)
        hipLaunchKernelGGL(gf_matmul_bsj_ragged_kernel<8>, dim3(unsigned(wgs)), dim3(512), 0, s, objs, n, wgs, st);
    else if (W == 4)
        hipLaunchKernelGGL(gf_matmul_bsj_ragged_kernel<4>, dim3(unsigned(wgs)), dim3(256), 0, s, objs, n, wgs, st);
    else if (W == 2)
        hipLaunchKernelGGL(gf_matmul_bsj_ragged_kernel<2>, dim3(unsigned(wgs)), dim3(128), 0, s, objs, n, wgs, st);
    else if (W == 1)
        hipLaunchKernelGGL(gf_matmul_bsj_ragged_kernel<1>, dim3(unsigned(wgs)), dim3(64), 0, s, objs, n, wgs, st);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_ragged_perm(const RaggedObj *objs, int n, int64_t wgs, hipStream_t s) {
    if (wgs <= 0) return hipSuccess;
    if (wgs > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gf_matmul_perm_ragged_kernel, dim3(unsigned(wgs)), dim3(kThreads), 0, s, objs, n, wgs);
    return hipGetLastError();
}

hipError_t launch_mul_vec_by_scalar(uint8_t *vec, int64_t len, uint8_t scalar, hipStream_t s) {
    return launch_vec<0>(vec, nullptr, len, scalar, s);
}
hipError_t launch_add_vectors(uint8_t *dst, const uint8_t *src, int64_t len, hipStream_t s) {
    return launch_vec<1>(dst, src, len, 1, s);
}
hipError_t launch_mul_add(uint8_t *dst, const uint8_t *src, int64_t len, uint8_t scalar, hipStream_t s) {
    return launch_vec<2>(dst, src, len, scalar, s);
}

hipError_t launch_final_data_len(const uint8_t *data, int64_t obj_stride, int64_t len, int n_obj, int32_t *status,
                                 int64_t *final_len, int32_t invalid_code, hipStream_t s) {
    if (n_obj <= 0) return hipSuccess;
    if (unaligned_vector_ok() || (al16(data) && (n_obj == 1 || al16(obj_stride))))
        hipLaunchKernelGGL(final_len_scan_kernel<true>, dim3((n_obj + kScanObjPerWg - 1) / kScanObjPerWg), dim3(256), 0,
                           s, data, obj_stride, len, n_obj, nullptr, 0, status, final_len, invalid_code);
    else
        hipLaunchKernelGGL(final_len_scan_kernel<false>, dim3((n_obj + kScanObjPerWg - 1) / kScanObjPerWg), dim3(256), 0,
                           s, data, obj_stride, len, n_obj, nullptr, 0, status, final_len, invalid_code);
    return hipGetLastError();
}

}  // namespace rlnc
