// kernels_ab.hip — the A/B history of the GF(2^8) product (diagnostic build only: make -C rlnc_amd/csrc ab ->
// librlnc_hip_ab.so, loaded through RLNC_LIB_PATH by the A/B scripts and the variant tests).  Variants 2-5 and 9 of
// rlnc_set_kernel_variant, each measured against the shipped kernels in its round (DESIGN.md §4.1 "Variant history",
// profiles/r01_sweep_*.jsonl, r02_run_ab.txt) and kept so those comparisons can be re-run:
//   2 perm3 (three sources per table lookup), 3 / 4 wide (2 or 4 column slots per lane), 5 bit-sliced with
//   GPR-index-relative XORs (bitslice_asm.inc), 9 the 8-wave shared program walking runs of column blocks.
// Every variant is bit-identical to the shipped path; the dispatcher of kernels.hip hands these variants here
// (launch_matmul_ab), and this file's strong definitions replace its weak stand-ins.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "bsj_tile.hpp"
#include "gf256.hpp"
#include "kernels.hpp"
#include "kernels_common.hpp"

namespace rlnc {

namespace {

// Wide variant: each lane owns VW 16-byte slots per source row (slot v at column v·4 KiB inside an
// (VW·4 KiB) block), so every table read from LDS — the measured bottleneck of the VW = 1 kernel (a build
// that reads one table set per source row ran 2.2× faster) — feeds VW× more multiply-adds.  Full aligned
// blocks only; ragged tails go to the VW = 1 kernels.
template <int NT, int VW>
__global__ __launch_bounds__(kThreads) void gf_matmul_wide_kernel(MatmulParams p, int row_tiles, int col_blocks) {
    __shared__ uint4 s_t01[kKC][NT];
    __shared__ uint32_t s_t2[kKC][NT];
    constexpr int64_t kSlot = int64_t(kThreads) * kBytesPerThread;  // 4 KiB between a lane's slots

    int rt, cb, obj;
    decode_block(p.n_obj * row_tiles * col_blocks, row_tiles, col_blocks, rt, cb, obj);
    const int row0 = rt * NT;
    const int rows_here = min(NT, p.n_out - row0);
    const int64_t col = int64_t(cb) * kSlot * VW + int64_t(threadIdx.x) * kBytesPerThread;
    const uint8_t *in_base = p.in + int64_t(obj) * p.in_obj + col;
    const uint8_t *coef_base = p.coef + int64_t(obj) * p.coef_obj + int64_t(row0) * p.coef_row;

    uint32_t acc[NT][VW][4];
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int v = 0; v < VW; ++v) acc[i][v][0] = acc[i][v][1] = acc[i][v][2] = acc[i][v][3] = 0u;

    for (int j0 = 0; j0 < p.n_in; j0 += kKC) {
        const int kc = min(kKC, p.n_in - j0);
        if (j0) __syncthreads();
        for (int e = threadIdx.x; e < kKC * NT; e += kThreads) {
            const int i = e % NT, j = e / NT;
            const uint8_t c = (i < rows_here && j < kc) ? coef_base[int64_t(i) * p.coef_row + j0 + j] : uint8_t(0);
            const PermTable pt = make_perm_table(c);
            s_t01[j][i] = make_uint4(pt.t0lo, pt.t0hi, pt.t1lo, pt.t1hi);
            s_t2[j][i] = pt.t2;
        }
        __syncthreads();
        const uint8_t *rowp = in_base + int64_t(j0) * p.in_row;
        const uint4 zero = make_uint4(0, 0, 0, 0);
        uint4 na[VW], nb[VW];
#pragma unroll
        for (int v = 0; v < VW; ++v) {
            na[v] = *reinterpret_cast<const uint4 *>(rowp + v * kSlot);
            nb[v] = kc > 1 ? *reinterpret_cast<const uint4 *>(rowp + p.in_row + v * kSlot) : zero;
        }
        for (int j = 0; j < kc; j += 2) {
            Sel a[VW], b[VW];
#pragma unroll
            for (int v = 0; v < VW; ++v) {
                a[v] = selectors(na[v]);
                b[v] = selectors(nb[v]);
            }
            // prefetch the next row pair while this pair is multiplied
#pragma unroll
            for (int v = 0; v < VW; ++v) {
                if (j + 2 < kc) na[v] = *reinterpret_cast<const uint4 *>(rowp + int64_t(j + 2) * p.in_row + v * kSlot);
                nb[v] = (j + 3 < kc) ? *reinterpret_cast<const uint4 *>(rowp + int64_t(j + 3) * p.in_row + v * kSlot) : zero;
            }
#pragma unroll
            for (int i = 0; i < NT; ++i) {
                const uint4 ta = s_t01[j][i];
                const uint32_t ta2 = s_t2[j][i];
                const uint4 tb = s_t01[j + 1][i];
                const uint32_t tb2 = s_t2[j + 1][i];
#pragma unroll
                for (int v = 0; v < VW; ++v)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        uint32_t r = xor3(acc[i][v][q], vperm(ta.y, ta.x, a[v].s0[q]), vperm(ta.w, ta.z, a[v].s1[q]));
                        r = xor3(r, vperm(ta2, ta2, a[v].s2[q]), vperm(tb.y, tb.x, b[v].s0[q]));
                        acc[i][v][q] = xor3(r, vperm(tb.w, tb.z, b[v].s1[q]), vperm(tb2, tb2, b[v].s2[q]));
                    }
            }
        }
    }
    uint8_t *out_base = p.out + int64_t(obj) * p.out_obj + int64_t(row0) * p.out_row + col;
#pragma unroll
    for (int i = 0; i < NT; ++i)
        if (i < rows_here)
#pragma unroll
            for (int v = 0; v < VW; ++v)
                *reinterpret_cast<uint4 *>(out_base + int64_t(i) * p.out_row + v * kSlot) =
                    make_uint4(acc[i][v][0], acc[i][v][1], acc[i][v][2], acc[i][v][3]);
    if (p.hdr != nullptr && cb == 0) {
        uint8_t *h = p.hdr + int64_t(obj) * p.hdr_obj + int64_t(row0) * p.hdr_row;
        for (int e = threadIdx.x; e < rows_here * p.n_in; e += kThreads) {
            const int i = e / p.n_in, j = e % p.n_in;
            h[int64_t(i) * p.hdr_row + j] = coef_base[int64_t(i) * p.coef_row + j];
        }
    }
}

// Three-source variant: the 24 bits of three source bytes (x, y, z) are cut into eight 3-bit chunks
//   x0-2 | x3-5 | x6,x7,y0 | y1-3 | y4-6 | y7,z0,z1 | z2-4 | z5-7
// and each chunk indexes an 8-entry table that already sums the contributions of the coefficients it
// straddles, so three multiply-accumulates of a word cost 8 v_perm_b32 + 4 v_bitop3_b32 (4.0 VALU ops per
// word-multiply-add instead of 4.5).  XOR is associative and GF(2^8) products are exact, so the result is
// byte-identical to the reference's sequential dst ^= c_j · src_j loop.
constexpr int kKC3 = 33;  // coefficient chunk: 11 triples

__device__ __forceinline__ void triple_tables(uint8_t cx, uint8_t cy, uint8_t cz, uint4 out[4]) {
    uint8_t b[24];  // basis: b[t] = contribution of bit t of the 24-bit chunk stream
    uint8_t mx = cx, my = cy, mz = cz;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        b[t] = mx;
        b[8 + t] = my;
        b[16 + t] = mz;
        mx = gf_xtime(mx);
        my = gf_xtime(my);
        mz = gf_xtime(mz);
    }
    uint32_t w[16];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            uint8_t e = 0;
#pragma unroll
            for (int t = 0; t < 3; ++t)
                if (v & (1 << t)) e ^= b[3 * c + t];
            if (v < 4)
                lo |= uint32_t(e) << (8 * v);
            else
                hi |= uint32_t(e) << (8 * (v - 4));
        }
        w[2 * c] = lo;
        w[2 * c + 1] = hi;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) out[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

struct Sel3 {
    uint32_t s[8][4];
};

__device__ __forceinline__ Sel3 selectors3(uint4 X, uint4 Y, uint4 Z) {
    Sel3 r;
    const uint32_t xs[4] = {X.x, X.y, X.z, X.w}, ys[4] = {Y.x, Y.y, Y.z, Y.w}, zs[4] = {Z.x, Z.y, Z.z, Z.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t x = xs[q], y = ys[q], z = zs[q];
        r.s[0][q] = x & 0x07070707u;
        r.s[1][q] = (x >> 3) & 0x07070707u;
        r.s[2][q] = ((x >> 6) & 0x03030303u) | ((y << 2) & 0x04040404u);
        r.s[3][q] = (y >> 1) & 0x07070707u;
        r.s[4][q] = (y >> 4) & 0x07070707u;
        r.s[5][q] = ((y >> 7) & 0x01010101u) | ((z << 1) & 0x06060606u);
        r.s[6][q] = (z >> 2) & 0x07070707u;
        r.s[7][q] = (z >> 5) & 0x07070707u;
    }
    return r;
}

template <int NT, bool VEC>
__device__ __forceinline__ void perm3_chunk(const MatmulParams &p, const uint8_t *rowp, int kc, int nbytes,
                                            const uint4 (*s_tab)[NT][4], uint32_t (&acc)[NT][4]) {
    const uint4 zero = make_uint4(0, 0, 0, 0);
    const int kt = (kc + 2) / 3;
    auto ld = [&](int j) { return j < kc ? ld16<VEC>(rowp + int64_t(j) * p.in_row, nbytes) : zero; };
    uint4 nx = ld(0), ny = ld(1), nz = ld(2);
    for (int t = 0; t < kt; ++t) {
        const Sel3 s = selectors3(nx, ny, nz);
        // prefetch the next triple of source rows while this one is multiplied
        nx = ld(3 * t + 3);
        ny = ld(3 * t + 4);
        nz = ld(3 * t + 5);
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            const uint4 a = s_tab[t][i][0], b = s_tab[t][i][1], c = s_tab[t][i][2], d = s_tab[t][i][3];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t u0 = xor3(vperm(a.y, a.x, s.s[0][q]), vperm(a.w, a.z, s.s[1][q]), vperm(b.y, b.x, s.s[2][q]));
                const uint32_t u1 = xor3(vperm(b.w, b.z, s.s[3][q]), vperm(c.y, c.x, s.s[4][q]), vperm(c.w, c.z, s.s[5][q]));
                const uint32_t u2 = xor3(vperm(d.y, d.x, s.s[6][q]), vperm(d.w, d.z, s.s[7][q]), acc[i][q]);
                acc[i][q] = xor3(u0, u1, u2);
            }
        }
    }
}

// VEC: every lane owns a full, aligned 16-byte slot (all blocks but a ragged/unaligned tail)
template <int NT, bool VEC>
__global__ __launch_bounds__(kThreads) void gf_matmul_perm3_kernel(MatmulParams p, int row_tiles, int col_blocks) {
    constexpr int KT = kKC3 / 3;
    __shared__ uint4 s_tab[KT][NT][4];

    const Tile t = make_tile<NT>(p, row_tiles, col_blocks);
    const uint8_t *in_base = p.in + int64_t(t.obj) * p.in_obj + t.col;
    const uint8_t *coef_base = p.coef + int64_t(t.obj) * p.coef_obj + int64_t(t.row0) * p.coef_row;

    uint32_t acc[NT][4];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0u;

    for (int j0 = 0; j0 < p.n_in; j0 += kKC3) {
        const int kc = min(kKC3, p.n_in - j0);
        if (j0) __syncthreads();
        for (int e = threadIdx.x; e < KT * NT; e += kThreads) {
            const int i = e % NT, tt = e / NT;
            uint8_t c3[3] = {0, 0, 0};
            if (i < t.rows_here)
                for (int u = 0; u < 3; ++u)
                    if (3 * tt + u < kc) c3[u] = coef_base[int64_t(i) * p.coef_row + j0 + 3 * tt + u];
            triple_tables(c3[0], c3[1], c3[2], s_tab[tt][i]);
        }
        __syncthreads();
        if (VEC || t.nbytes > 0)
            perm3_chunk<NT, VEC>(p, in_base + int64_t(j0) * p.in_row, kc, t.nbytes, s_tab, acc);
    }
    store_tile<NT, VEC>(p, t, acc);
    copy_header(p, t);
}


// the perm kernels' column split (kernels.hip launch_one / launch_nt) with the three-source kernel
template <int NT, bool VEC>
hipError_t launch_perm3_one(const MatmulParams &p, int64_t width, hipStream_t s) {
    const int row_tiles = (p.n_out + NT - 1) / NT;
    const int col_blocks = int((width + kColBlock - 1) / kColBlock);
    const int64_t total = int64_t(p.n_obj) * row_tiles * col_blocks;
    if (total <= 0) return hipSuccess;
    if (total > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    MatmulParams q = p;
    q.width = width;
    hipLaunchKernelGGL((gf_matmul_perm3_kernel<NT, VEC>), dim3(unsigned(total)), dim3(kThreads), 0, s, q, row_tiles,
                       col_blocks);
    return hipGetLastError();
}

template <int NT>
hipError_t launch_perm3(const MatmulParams &p, hipStream_t s, bool aligned) {
    if (!aligned) return launch_perm3_one<NT, false>(p, p.width, s);
    const int64_t full = (p.width / kColBlock) * kColBlock;
    if (full > 0)
        if (hipError_t e = launch_perm3_one<NT, true>(p, full, s); e != hipSuccess) return e;
    if (full == p.width) return hipSuccess;
    MatmulParams t = p;
    t.in = p.in + full;
    t.out = p.out + full;
    if (full > 0) t.hdr = nullptr;
    return launch_perm3_one<NT, false>(t, p.width - full, s);
}

template <int NT, int VW>
hipError_t launch_wide(const MatmulParams &p, int64_t full, hipStream_t s) {
    const int row_tiles = (p.n_out + NT - 1) / NT;
    const int col_blocks = int(full / (int64_t(kColBlock) * VW));
    const int64_t total = int64_t(p.n_obj) * row_tiles * col_blocks;
    if (total <= 0) return hipSuccess;
    if (total > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((gf_matmul_wide_kernel<NT, VW>), dim3(unsigned(total)), dim3(kThreads), 0, s, p, row_tiles,
                       col_blocks);
    return hipGetLastError();
}

// Wide variant: whole (VW·4 KiB) blocks through gf_matmul_wide_kernel, the rest through the VW = 1 path.
template <int NT, int VW>
hipError_t launch_wide_split(const MatmulParams &p, hipStream_t s) {
    const int64_t blk = int64_t(kColBlock) * VW;
    const int64_t full = (p.width / blk) * blk;
    if (full > 0) {
        hipError_t e = launch_wide<NT, VW>(p, full, s);
        if (e != hipSuccess) return e;
    }
    if (full == p.width) return hipSuccess;
    MatmulParams t = p;
    t.in = p.in + full;
    t.out = p.out + full;
    t.width = p.width - full;
    if (full > 0) t.hdr = nullptr;
    return launch_matmul(t, s, MatmulVariant::Perm);
}


// ---------------------------------------------------------------------------------------------------
// Bit-sliced variant (gen_bitslice.py has the full derivation).  Measured on gfx950: v_perm_b32 issues at
// ~4.1 cycles/wave64, so the 3-perm lookup costs ~19 cycles per 32-bit multiply-add; GF(2^8) multiply by
// c is instead a GF(2)-linear map on bit-planes, applied with 16 register-indexed XORs per 32 bytes per
// group, the index pair shared by two groups (s_set_gpr_idx_idx + 2 v_xor_b32, ~2 cycles per XOR), i.e.
// ~8 cycles of issue per 32 bytes·source·row plus the amortised transposes.
// ---------------------------------------------------------------------------------------------------
#include "bitslice_asm.inc"  // scripts/bs_diag.sh builds substitute a generated variant (scripts/diag_build.sh)

constexpr int kBsRows = RLNC_BS_NT;           // output rows per workgroup
constexpr int kBsColBlock = 16384;            // 256 lanes × 64 B
constexpr int kBsRowDwords = RLNC_BS_ROW_DWORDS;  // packed indices per (row, source)

// Index n = 2·o + h of (row, source) says which of the source's planes 4h..4h+3 feed output plane o: bit b
// of idx = bit o of (c · 2^(4h+b)).  Packed three per dword as bytes 0x10 | idx, byte 3 = 0x10 (see
// gen_bitslice.py: the byte above each index supplies M0[15:12], the relative-SRC0 enable).  Stream order
// [obj][row tile][j][row in tile][6 dwords] is the order the main kernel consumes it; rows past n_out get
// c = 0 (all indices 0: XOR of the zero register).
__global__ __launch_bounds__(64) void bs_index_kernel(const uint8_t *coef, int64_t coef_obj, int64_t coef_row,
                                                      int n_out, int n_in, int row_tiles, uint32_t *stream) {
    const int j = blockIdx.x, rt = blockIdx.y, obj = blockIdx.z;
    const int i = threadIdx.x / kBsRowDwords, d = threadIdx.x % kBsRowDwords;
    if (i >= kBsRows) return;
    const int row = rt * kBsRows + i;
    const uint32_t c = row < n_out ? coef[int64_t(obj) * coef_obj + int64_t(row) * coef_row + j] : 0u;
    uint32_t m[8];  // c · 2^e
    m[0] = c;
    for (int e = 1; e < 8; ++e) m[e] = ((m[e - 1] << 1) ^ ((m[e - 1] & 0x80u) ? 0x11Bu : 0u)) & 0xFFu;
    uint32_t word = 0x10u << 24;
    for (int b3 = 0; b3 < 3; ++b3) {
        const int n = 3 * d + b3;
        uint32_t idx = 0;
        if (n < 16) {
            const int o = n >> 1, h = n & 1;
            for (int b = 0; b < 4; ++b) idx |= ((m[4 * h + b] >> o) & 1u) << b;
        }
        word |= (0x10u | idx) << (8 * b3);
    }
    stream[((int64_t(obj) * row_tiles + rt) * n_in + j) * (kBsRows * kBsRowDwords) + threadIdx.x] = word;
}

__global__ __launch_bounds__(kThreads) void gf_matmul_bs_kernel(MatmulParams p, const uint32_t *stream,
                                                                int row_tiles, int col_blocks) {
    int rt, cb, obj;
    decode_block(p.n_obj * row_tiles * col_blocks, row_tiles, col_blocks, rt, cb, obj);
    const int row0 = rt * kBsRows;
    const int rows = min(kBsRows, p.n_out - row0);
    if (p.hdr != nullptr && cb == 0) {
        Tile t;
        t.obj = obj;
        t.cb = 0;
        t.row0 = row0;
        t.rows_here = rows;
        copy_header(p, t);
    }
    const uint8_t *src = p.in + int64_t(obj) * p.in_obj + int64_t(cb) * kBsColBlock;
    uint8_t *dst = p.out + int64_t(obj) * p.out_obj + int64_t(row0) * p.out_row + int64_t(cb) * kBsColBlock;
    const uint32_t *idx = stream + (int64_t(obj) * row_tiles + rt) * p.n_in * (kBsRows * kBsRowDwords);
    const uint32_t off = (threadIdx.x >> 6) * 4096u + (threadIdx.x & 63u) * 16u;
    // M0 is clobbered on purpose (it carries the XOR index); nothing else in this kernel uses it
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
    asm volatile(RLNC_BS_ASM
                 :
                 : [src] "s"(src), [idx] "s"(idx), [dst] "s"(dst), [in_row] "s"(uint32_t(p.in_row)),
                   [out_row] "s"(uint32_t(p.out_row)), [n_in] "s"(p.n_in), [rows] "s"(rows), [off] "v"(off)
                 : RLNC_BS_CLOBBER_V, RLNC_BS_CLOBBER_S);
#pragma clang diagnostic pop
}

// Full 16 KiB column blocks of aligned operands; the caller sends the rest elsewhere.
bool bs_eligible(const MatmulParams &p, bool aligned) {
    return aligned && p.width >= kBsColBlock && p.n_out >= 4 && p.in_row < (int64_t(1) << 32) &&
           p.out_row < (int64_t(1) << 32);
}

size_t bs_scratch_bytes(const MatmulParams &p) {
    const int64_t tiles = (p.n_out + kBsRows - 1) / kBsRows;
    // + one step: the main loop prefetches one index step past the end of the last tile
    return size_t(int64_t(p.n_obj) * tiles * p.n_in * kBsRows * kBsRowDwords * 4 + 256);
}

hipError_t launch_bs(const MatmulParams &p, hipStream_t s, void *scratch, size_t scratch_bytes, int64_t &full) {
    full = (p.width / kBsColBlock) * kBsColBlock;
    const int row_tiles = (p.n_out + kBsRows - 1) / kBsRows;
    const int col_blocks = int(full / kBsColBlock);
    const int64_t total = int64_t(p.n_obj) * row_tiles * col_blocks;
    if (scratch == nullptr || scratch_bytes < bs_scratch_bytes(p)) return hipErrorInvalidValue;
    if (total > 0x7FFFFFFFLL || p.n_in > 65535 || row_tiles > 65535 || p.n_obj > 65535) return hipErrorInvalidValue;
    uint32_t *stream = static_cast<uint32_t *>(scratch);
    hipLaunchKernelGGL(bs_index_kernel, dim3(unsigned(p.n_in), unsigned(row_tiles), unsigned(p.n_obj)),
                       dim3(64), 0, s, p.coef, p.coef_obj, p.coef_row, p.n_out, p.n_in, row_tiles,
                       stream);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    MatmulParams q = p;
    q.width = full;
    hipLaunchKernelGGL(gf_matmul_bs_kernel, dim3(unsigned(total)), dim3(kThreads), 0, s, q, stream, row_tiles,
                       col_blocks);
    return hipGetLastError();
}


// ---------------------------------------------------------------------------------------------------
// Variant 9: the 8-wave shared program over runs of column blocks (RLNC_BSJ_ASM_W8R): a workgroup walks `run`
// consecutive column blocks of one (object, row tile), the source-row stream unbroken across them (one prologue per
// run).  Measured -4.8 % for an isolated encode launch and 0 % in the pipelined bench step (profiles/r02_run_ab.txt).
// ---------------------------------------------------------------------------------------------------
// Column blocks per workgroup of the column-run program: enough runs for >= 4 workgroups per CU, at most 8
// blocks each (RLNC_BSJ_RUN = n forces n; A/B knob, read once)
static int bsj_run_length(int64_t tiles, int col_blocks, int requested) {
    static const int forced = [] {
        const char *e = getenv("RLNC_BSJ_RUN");
        return e ? atoi(e) : 0;
    }();
    static std::mutex mu;
    static int cus[64] = {};
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
        std::lock_guard<std::mutex> lock(mu);
        if (cus[dev] == 0 && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus[dev] = 256;
        n = cus[dev] > 0 ? cus[dev] : 256;
    }
    int r = requested > 0 ? requested
            : forced > 0  ? forced
                          : int(std::min<int64_t>(8, std::max<int64_t>(1, tiles / (int64_t(n) * 4))));
    return std::max(1, std::min(r, col_blocks));
}

// Guided column runs (variant 9): percentage of each XCD's run units walked as whole runs, the rest as single
// column blocks dispatched last (RLNC_BSJ_GUIDED; -1 = plain runs).  A/B knob, read once.
static int bsj_guided_pct() {
    static const int pct = [] {
        const char *e = getenv("RLNC_BSJ_GUIDED");
        return e ? std::max(-1, std::min(100, atoi(e))) : -1;
    }();
    return pct;
}


__global__ __launch_bounds__(512) void gf_matmul_bsj_run_kernel(MatmulParams p, const void *stream, int row_tiles,
                                                               int col_blocks, int run, int guided_nl) {
    const int runs = (col_blocks + run - 1) / run;
    int rt, cb, obj, r;
    uint32_t tiles;
    if (guided_nl < 0) {
        decode_block(p.n_obj * row_tiles * runs, row_tiles, runs, rt, r, obj);
        cb = r * run;
        tiles = uint32_t(__builtin_amdgcn_readfirstlane(min(run, col_blocks - cb)));
    } else {
        // guided runs (run | col_blocks, 8 | the run units): XCD x = b & 7 owns run units [x·per, (x+1)·per) (rt
        // fastest, as decode_block), its first guided_nl dispatched workgroups walk one unit each, the later ones one
        // column block of the remaining units -- short workgroups last
        const int per = (p.n_obj * row_tiles * runs) >> 3;
        const int b = blockIdx.x, x = b & 7, i = b >> 3;
        int u, c = 0;
        tiles = 1;
        if (i < guided_nl) {
            u = x * per + i;
            tiles = uint32_t(run);
        } else {
            const int j = i - guided_nl;
            u = x * per + guided_nl + j / run;
            c = j % run;
        }
        rt = u % row_tiles;
        const int rest = u / row_tiles;
        r = rest % runs;
        obj = rest / runs;
        cb = r * run + c;
    }
    bsj_tile<8, true, true>(p, stream, row_tiles, rt, cb, obj, tiles, nullptr);
}

bool operands_aligned(const MatmulParams &p) {
    if (unaligned_vector_ok()) return true;
    return al16(p.in) && (p.n_in == 1 || al16(p.in_row)) && (p.n_obj == 1 || al16(p.in_obj)) && al16(p.out) &&
           (p.n_out == 1 || al16(p.out_row)) && (p.n_obj == 1 || al16(p.out_obj));
}

// the columns [full, width) of a product, through the shipped perm path
hipError_t tail_perm(const MatmulParams &p, int64_t full, hipStream_t s) {
    if (full >= p.width) return hipSuccess;
    MatmulParams t = p;
    t.in = p.in + full;
    t.out = p.out + full;
    t.width = p.width - full;
    t.hdr = nullptr;
    return launch_matmul(t, s, MatmulVariant::Perm);
}

hipError_t launch_run(const MatmulParams &p, hipStream_t s, void *scratch, size_t scratch_bytes) {
    // shapes the run program does not take are variant 8's (stream kernel, realigned copies, <= 32-row tiles)
    if (p.n_out <= 32 || !operands_aligned(p) || !bsj_eligible_public(p))
        return launch_matmul(p, s, MatmulVariant::BitSlicedJumpShared8, scratch, scratch_bytes);
    BsjPlan b;
    if (hipError_t e = bsj_prepare(p, s, scratch, scratch_bytes, true, true, b); e != hipSuccess) return e;
    if (b.waves != 8) return hipErrorInvalidValue;  // first use inside a stream capture: not for this variant
    MatmulParams q = p;
    q.width = b.full;
    const int rl = bsj_run_length(b.total, b.col_blocks, p.col_run);
    const int64_t units = int64_t(p.n_obj) * b.row_tiles * ((b.col_blocks + rl - 1) / rl);
    const int pct = bsj_guided_pct();
    if (pct >= 0 && rl > 1 && b.col_blocks % rl == 0 && units % 8 == 0) {
        // guided: per XCD, pct % of the run units as whole runs (dispatched first), the rest one block each
        const int64_t per = units / 8;
        const int64_t nl = per * pct / 100;
        const int64_t wgs = 8 * (nl + (per - nl) * rl);
        hipLaunchKernelGGL(gf_matmul_bsj_run_kernel, dim3(unsigned(wgs)), dim3(512), 0, s, q, b.stream, b.row_tiles,
                           b.col_blocks, rl, int(nl));
    } else {
        hipLaunchKernelGGL(gf_matmul_bsj_run_kernel, dim3(unsigned(units)), dim3(512), 0, s, q, b.stream, b.row_tiles,
                           b.col_blocks, rl, -1);
    }
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    return tail_perm(p, b.full, s);
}

}  // namespace

bool ab_build() { return true; }

size_t matmul_scratch_bytes_ab(const MatmulParams &p, MatmulVariant v) {
    if (p.n_out <= 0 || p.n_in <= 0 || p.n_obj <= 0) return 0;
    if (v == MatmulVariant::BitSliced) return bs_eligible(p, operands_aligned(p)) ? bs_scratch_bytes(p) : 0;
    if (v == MatmulVariant::BitSlicedJumpRun)
        return std::max(matmul_scratch_bytes(p, MatmulVariant::BitSlicedJumpShared8), bsj_scratch_bytes_public(p, true));
    return 0;
}

hipError_t launch_matmul_ab(const MatmulParams &p, hipStream_t s, MatmulVariant v, void *scratch, size_t scratch_bytes) {
    const bool aligned = operands_aligned(p);
    switch (v) {
        case MatmulVariant::Perm3:
            if (p.width < kColBlock && p.n_out > 2) return launch_perm3<2>(p, s, aligned);
            if (p.n_out <= 1) return launch_perm3<1>(p, s, aligned);
            if (p.n_out <= 2) return launch_perm3<2>(p, s, aligned);
            if (p.n_out <= 4) return launch_perm3<4>(p, s, aligned);
            if (p.n_out <= 8) return launch_perm3<8>(p, s, aligned);
            if (p.n_out <= 16) return launch_perm3<16>(p, s, aligned);
            return launch_perm3<32>(p, s, aligned);
        case MatmulVariant::Wide:
        case MatmulVariant::Wide4:
            if (!aligned) return launch_matmul(p, s, MatmulVariant::Perm);
            if (v == MatmulVariant::Wide4) return p.n_out <= 4 ? launch_wide_split<4, 4>(p, s) : launch_wide_split<8, 4>(p, s);
            if (p.n_out <= 4) return launch_wide_split<4, 2>(p, s);
            if (p.n_out <= 8) return launch_wide_split<8, 2>(p, s);
            return launch_wide_split<16, 2>(p, s);
        case MatmulVariant::BitSliced: {
            if (!bs_eligible(p, aligned)) return launch_matmul(p, s, MatmulVariant::Perm);
            int64_t full = 0;
            if (hipError_t e = launch_bs(p, s, scratch, scratch_bytes, full); e != hipSuccess) return e;
            return tail_perm(p, full, s);
        }
        case MatmulVariant::BitSlicedJumpRun:
            return launch_run(p, s, scratch, scratch_bytes);
        default:
            return hipErrorInvalidValue;
    }
}

}  // namespace rlnc
