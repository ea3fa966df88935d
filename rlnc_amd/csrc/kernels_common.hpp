// kernels_common.hpp — device helpers shared by the matmul kernels of kernels.hip and the A/B variants of
// kernels_ab.hip (internal to librlnc_hip): launch constants, the 3-bit-split v_perm multiply, 16-byte row access, the
// XCD-aware work decode and the perm kernels' tile.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gf256.hpp"
#include "kernels.hpp"

namespace rlnc {
namespace {

constexpr int kThreads = 256;          // 4 waves
constexpr int kBytesPerThread = 16;    // one dwordx4 per source row per lane
constexpr int kColBlock = kThreads * kBytesPerThread;  // 4 KiB of columns per workgroup
constexpr int kKC = 32;                // coefficient chunk (tables per chunk staged in LDS)

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t vperm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// make_perm_table (gf256.hpp) in registers: T0[v] = c·v is linear in the bits of v, so with m_b = c·2^b the
// low dword's bytes are {0, m0, m1, m0^m1} and the high dword's are the low ones XOR m2 (likewise T1 from m3..m5,
// T2 = {0, m6, m7, m6^m7})
__device__ __forceinline__ void perm_table_regs(uint32_t c, uint32_t &t0lo, uint32_t &t0hi, uint32_t &t1lo,
                                                uint32_t &t1hi, uint32_t &t2) {
    uint32_t m[8];
    m[0] = c;
#pragma unroll
    for (int b = 1; b < 8; ++b) m[b] = ((m[b - 1] << 1) ^ ((m[b - 1] & 0x80u) ? 0x1Bu : 0u)) & 0xFFu;
    t0lo = (m[0] << 8) | (m[1] << 16) | ((m[0] ^ m[1]) << 24);
    t0hi = t0lo ^ (m[2] * 0x01010101u);
    t1lo = (m[3] << 8) | (m[4] << 16) | ((m[3] ^ m[4]) << 24);
    t1hi = t1lo ^ (m[5] * 0x01010101u);
    t2 = (m[6] << 8) | (m[7] << 16) | ((m[6] ^ m[7]) << 24);
}

template <bool ALIGNED>
__device__ __forceinline__ uint4 load16(const uint8_t *p, int nbytes) {
    if (ALIGNED && nbytes == 16) return *reinterpret_cast<const uint4 *>(p);
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 16; ++b)
        if (b < nbytes) w[b >> 2] |= uint32_t(p[b]) << (8 * (b & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

template <bool ALIGNED>
__device__ __forceinline__ void store16(uint8_t *p, uint4 v, int nbytes) {
    if (ALIGNED && nbytes == 16) {
        *reinterpret_cast<uint4 *>(p) = v;
        return;
    }
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int b = 0; b < 16; ++b)
        if (b < nbytes) p[b] = uint8_t(w[b >> 2] >> (8 * (b & 3)));
}

struct Sel {
    uint32_t s0[4], s1[4], s2[4];
};

__device__ __forceinline__ Sel selectors(uint4 x) {
    Sel s;
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        s.s0[q] = w[q] & 0x07070707u;
        s.s1[q] = (w[q] >> 3) & 0x07070707u;
        s.s2[q] = (w[q] >> 6) & 0x03030303u;
    }
    return s;
}

// XCD-aware work decode (cdna_hip_programming.md §5.5 T1): blocks b and b+8 share an XCD, so give every
// XCD a contiguous range of work items, ordered row-tile-fastest: the row tiles of one column block then
// run on one XCD and re-read that block's source rows from its L2 instead of HBM.
__device__ __forceinline__ void decode_block(int total, int row_tiles, int col_blocks, int &rt, int &cb, int &obj) {
    int b = blockIdx.x;
    int w = b;
    if ((total & 7) == 0) {
        const int per = total >> 3;
        w = (b & 7) * per + (b >> 3);
    }
    rt = w % row_tiles;
    const int rest = w / row_tiles;
    cb = rest % col_blocks;
    obj = rest / col_blocks;
}

// Per-workgroup tile: column block cb of object obj, output rows [row0, row0 + rows_here).
struct Tile {
    int row0, rows_here, obj, cb;
    int64_t col;
    int nbytes;  // bytes of this lane's 16-byte column slot inside [0, width)
};

template <int NT>
__device__ __forceinline__ Tile make_tile(const MatmulParams &p, int row_tiles, int col_blocks) {
    Tile t;
    int rt;
    decode_block(p.n_obj * row_tiles * col_blocks, row_tiles, col_blocks, rt, t.cb, t.obj);
    t.row0 = rt * NT;
    t.rows_here = min(NT, p.n_out - t.row0);
    t.col = int64_t(t.cb) * kColBlock + int64_t(threadIdx.x) * kBytesPerThread;
    t.nbytes = t.col < p.width ? int(min<int64_t>(kBytesPerThread, p.width - t.col)) : 0;
    return t;
}

// VEC: plain 16-byte vector access (no per-lane branches in the hot loop, so the prefetched loads stay in
// flight); otherwise byte-granular access bounded by nbytes (ragged tail / unaligned rows).
template <bool VEC>
__device__ __forceinline__ uint4 ld16(const uint8_t *p, int nbytes) {
    if (VEC) return *reinterpret_cast<const uint4 *>(p);
    return load16<false>(p, nbytes);
}
template <bool VEC>
__device__ __forceinline__ void st16(uint8_t *p, uint4 v, int nbytes) {
    if (VEC)
        *reinterpret_cast<uint4 *>(p) = v;
    else
        store16<false>(p, v, nbytes);
}

template <int NT, bool VEC>
__device__ __forceinline__ void store_tile(const MatmulParams &p, const Tile &t, const uint32_t (&acc)[NT][4]) {
    if (!VEC && t.nbytes <= 0) return;
    uint8_t *out_base = p.out + int64_t(t.obj) * p.out_obj + int64_t(t.row0) * p.out_row + t.col;
#pragma unroll
    for (int i = 0; i < NT; ++i)
        if (i < t.rows_here)
            st16<VEC>(out_base + int64_t(i) * p.out_row, make_uint4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]),
                      t.nbytes);
}

__device__ __forceinline__ void copy_header(const MatmulParams &p, const Tile &t) {
    if (p.hdr == nullptr || t.cb != 0) return;
    const uint8_t *coef_base = p.coef + int64_t(t.obj) * p.coef_obj + int64_t(t.row0) * p.coef_row;
    uint8_t *h = p.hdr + int64_t(t.obj) * p.hdr_obj + int64_t(t.row0) * p.hdr_row;
    for (int e = threadIdx.x; e < t.rows_here * p.n_in; e += kThreads) {
        const int i = e / p.n_in, j = e % p.n_in;
        h[int64_t(i) * p.hdr_row + j] = coef_base[int64_t(i) * p.coef_row + j];
    }
}

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld16_nt(const uint8_t *ptr) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(ptr));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Selectors from 64-bit shifts: one v_lshrrev_b64 shifts two dwords; the bits that cross the dword boundary land
// in bits 29-31 (>> 3) or 26-31 (>> 6) of the low dword's top byte, which the masks clear.
__device__ __forceinline__ Sel selectors64(uint4 x) {
    Sel s;
    const uint64_t a = (uint64_t(x.y) << 32) | x.x, b = (uint64_t(x.w) << 32) | x.z;
    uint64_t a3, b3, a6, b6;  // the compiler splits a C++ 64-bit shift into 32-bit ones: ask for the pair form
    asm("v_lshrrev_b64 %0, 3, %1" : "=v"(a3) : "v"(a));
    asm("v_lshrrev_b64 %0, 3, %1" : "=v"(b3) : "v"(b));
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(a6) : "v"(a));
    asm("v_lshrrev_b64 %0, 6, %1" : "=v"(b6) : "v"(b));
    s.s0[0] = x.x & 0x07070707u;
    s.s0[1] = x.y & 0x07070707u;
    s.s0[2] = x.z & 0x07070707u;
    s.s0[3] = x.w & 0x07070707u;
    s.s1[0] = uint32_t(a3) & 0x07070707u;
    s.s1[1] = uint32_t(a3 >> 32) & 0x07070707u;
    s.s1[2] = uint32_t(b3) & 0x07070707u;
    s.s1[3] = uint32_t(b3 >> 32) & 0x07070707u;
    s.s2[0] = uint32_t(a6) & 0x03030303u;
    s.s2[1] = uint32_t(a6 >> 32) & 0x03030303u;
    s.s2[2] = uint32_t(b6) & 0x03030303u;
    s.s2[3] = uint32_t(b6 >> 32) & 0x03030303u;
    return s;
}

inline bool al16(const void *ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }
inline bool al16(int64_t v) { return (v & 15) == 0; }

}  // namespace
}  // namespace rlnc
