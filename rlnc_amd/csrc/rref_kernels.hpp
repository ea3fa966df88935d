// rref_kernels.hpp — the device elimination's kernels (see rref.hip for the algorithm), shared by the shipped
// dispatch of rref.hip and the A/B dispatch of rref_ab.hip (internal to librlnc_hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "../../include/rlnc_hip.h"
#include "gf256.hpp"
#include "kernels.hpp"

namespace rlnc {

// dwords per matrix row: a power of two below 64 (the lane-group XOR reduction of clean_append needs
// groups of D lanes that tile the wave), any count from 64 up
__host__ __device__ inline int rref_row_dwords(int k, int m) {
    const int d = (k + m + 3) / 4;
    if (d >= 64) return d;
    int p = 1;
    while (p < d) p <<= 1;
    return p;
}

namespace {

constexpr int kTabDw = 8;  // dwords per multiplier: t0lo t0hi t1lo t1hi t2 inv - -

// The 512 × kTabDw table, built at compile time: entry c < 256 = make_perm_table's layout of multiplier c plus
// c^-1 = c^254 in dword 5; entry 256 + c = the layout of c^-1 (0 for c = 0), so that "multiply by the
// inverse of the pivot" is one table read (the register path's normalisation).
constexpr int kTabEntries = 512;
struct RrefTable {
    uint32_t v[kTabEntries * kTabDw];
};
constexpr void fill_perm_entry(uint32_t *e, uint8_t c) {
    uint8_t m[8] = {};
    m[0] = c;
    for (int b = 1; b < 8; ++b) m[b] = gf_xtime(m[b - 1]);
    uint32_t t0lo = 0, t0hi = 0, t1lo = 0, t1hi = 0, t2 = 0;
    for (int x = 0; x < 8; ++x) {
        uint8_t a = 0, h = 0;
        for (int b = 0; b < 3; ++b)
            if (x & (1 << b)) {
                a = uint8_t(a ^ m[b]);
                h = uint8_t(h ^ m[b + 3]);
            }
        if (x < 4) {
            t0lo |= uint32_t(a) << (8 * x);
            t1lo |= uint32_t(h) << (8 * x);
        } else {
            t0hi |= uint32_t(a) << (8 * (x - 4));
            t1hi |= uint32_t(h) << (8 * (x - 4));
        }
    }
    for (int x = 0; x < 4; ++x) {
        uint8_t a = 0;
        for (int b = 0; b < 2; ++b)
            if (x & (1 << b)) a = uint8_t(a ^ m[b + 6]);
        t2 |= uint32_t(a) << (8 * x);
    }
    e[0] = t0lo;
    e[1] = t0hi;
    e[2] = t1lo;
    e[3] = t1hi;
    e[4] = t2;
}
constexpr RrefTable build_rref_table() {
    RrefTable t{};
    // inverses by the generator-3 logarithm (gf256.rs:16-44, 88-108): c^-1 = 3^(255 - log3 c)
    uint8_t ex[256] = {}, lg[256] = {};
    uint8_t x = 1;
    for (int i = 0; i < 255; ++i) {
        ex[i] = x;
        lg[x] = uint8_t(i);
        x = uint8_t(x ^ gf_xtime(x));  // x·3
    }
    for (int c = 0; c < 256; ++c) {
        const uint8_t inv = c ? ex[(255 - lg[c]) % 255] : uint8_t(0);
        fill_perm_entry(t.v + c * kTabDw, uint8_t(c));
        t.v[c * kTabDw + 5] = inv;
        fill_perm_entry(t.v + (256 + c) * kTabDw, inv);
    }
    return t;
}
__device__ const RrefTable kRrefTable = build_rref_table();
// spot checks against the field (gf256.rs:16-44): identity tables of c = 1, 2^-1 = 0x8D, 3^-1 = 0xF6
static_assert(build_rref_table().v[1 * kTabDw + 0] == 0x03020100u && build_rref_table().v[1 * kTabDw + 1] == 0x07060504u,
              "c = 1 low table");
static_assert(build_rref_table().v[2 * kTabDw + 5] == 0x8Du && build_rref_table().v[3 * kTabDw + 5] == 0xF6u,
              "inverses");
static_assert(build_rref_table().v[(256 + 1) * kTabDw + 0] == 0x03020100u, "1^-1 = 1");

__device__ __forceinline__ uint32_t mul4(const uint32_t *tab, uint32_t q, uint32_t x) {
    const uint4 t = *reinterpret_cast<const uint4 *>(tab + q * kTabDw);
    const uint32_t t2 = tab[q * kTabDw + 4];
    return __builtin_amdgcn_perm(t.y, t.x, x & 0x07070707u) ^ __builtin_amdgcn_perm(t.w, t.z, (x >> 3) & 0x07070707u) ^
           __builtin_amdgcn_perm(t2, t2, (x >> 6) & 0x03030303u);
}
__device__ __forceinline__ uint32_t mul4t(uint4 t, uint32_t t2, uint32_t x) {
    return __builtin_amdgcn_perm(t.y, t.x, x & 0x07070707u) ^ __builtin_amdgcn_perm(t.w, t.z, (x >> 3) & 0x07070707u) ^
           __builtin_amdgcn_perm(t2, t2, (x >> 6) & 0x03030303u);
}
__device__ __forceinline__ uint32_t gfmul(const uint32_t *tab, uint32_t a, uint32_t b) {
    return mul4(tab, a, b) & 0xFFu;
}
__device__ __forceinline__ uint32_t gfinv(const uint32_t *tab, uint32_t a) { return tab[a * kTabDw + 5]; }

// bytes of dword w at columns >= c0
__device__ __forceinline__ uint32_t from_mask(int w, int c0) {
    const int b0 = 4 * w;
    if (b0 >= c0) return 0xFFFFFFFFu;
    if (b0 + 4 <= c0) return 0u;
    return 0xFFFFFFFFu << (8 * (c0 - b0));
}

struct Mat {
    uint8_t *b;     // bytes
    uint32_t *w;    // same storage as dwords
    int S, D;       // row stride in bytes / dwords
    __device__ uint32_t at(int r, int c) const { return b[r * S + c]; }
};

// lane within the wave: the single-wave helpers below also run in one wave of a multi-object workgroup
__device__ __forceinline__ int lane_id() { return int(threadIdx.x & 63u); }

// row_t[c >= c0] ^= q · row_s[c >= c0]   (simd/mod.rs:89-119 on the byte range of decoder_matrix.rs:158-161)
__device__ __forceinline__ void row_muladd(const Mat &M, const uint32_t *tab, int t, int s, uint32_t q, int c0) {
    for (int w = lane_id(); w < M.D; w += 64) {
        const uint32_t mask = from_mask(w, c0);
        if (mask) M.w[t * M.D + w] ^= mul4(tab, q, M.w[s * M.D + w]) & mask;
    }
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }


// WG: a workgroup barrier; else the code runs in one wave only (the other waves of the workgroup are elsewhere and
// must not be waited for): a compiler fence suffices, a wave's LDS operations execute in issue order
template <bool WG>
__device__ __forceinline__ void rsync() {
    if constexpr (WG) {
        __syncthreads();
    } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// Rows j in [j_lo, j_hi) with M[j][i] != 0: row_j[c >= i] ^= (M[j][i] / M[i][i])·row_i[c >= i] -- the bodies of the
// reference's per-row loops (decoder_matrix.rs:143-162 forward, :179-198 backward).  They are independent across j
// (each reads row i, which the step leaves unchanged, and writes its own row), so rows under 64 dwords go 64 / D rows
// per pass, lane = (row, dword), with the quotient byte read before the same instruction stream rewrites it; wider
// rows one at a time over the lanes, the nonzero rows found by ballot.
__device__ __forceinline__ void eliminate_rows(const Mat &M, const uint32_t *tab, int i, uint32_t inv, int j_lo,
                                               int j_hi) {
    const int lane = lane_id();
    const int D = M.D;
    if (D < 64) {
        const int RP = 64 / D, w = lane % D, jr = lane / D;
        const uint32_t mask = from_mask(w, i);
        const uint32_t xi = M.w[i * D + w];
        const uint4 ti4 = *reinterpret_cast<const uint4 *>(tab + inv * kTabDw);  // the quotient = c · inv
        const uint32_t ti2 = tab[inv * kTabDw + 4];
        if (j_hi - j_lo <= 2 * RP) {  // at most two passes over the range: no compaction (one LDS round trip less)
            for (int j0 = j_lo; j0 < j_hi; j0 += RP) {
                const int j = j0 + jr;
                if (j < j_hi) {
                    const uint32_t c = M.at(j, i);
                    if (c != 0u) M.w[j * D + w] ^= mul4(tab, mul4t(ti4, ti2, c) & 0xFFu, xi) & mask;  // :148 / :184
                }
            }
            return;
        }
        for (int g = j_lo; g < j_hi; g += 64) {
            const int jl = g + lane;
            uint64_t b = ballot(jl < j_hi && M.at(jl, i) != 0);  // the rows with work, 64 at a time
            while (b) {  // RP of them per pass: lane group jr takes the jr-th remaining set bit
                uint64_t bb = b;
                for (int t = 0; t < RP - 1; ++t)
                    if (t < jr) bb &= bb - 1;
                if (bb) {
                    const int j = g + __ffsll((unsigned long long)bb) - 1;
                    const uint32_t q = mul4t(ti4, ti2, M.at(j, i)) & 0xFFu;  // :148 / :184
                    M.w[j * D + w] ^= mul4(tab, q, xi) & mask;
                }
                for (int t = 0; t < RP && b; ++t) b &= b - 1;
            }
        }
        return;
    }
    for (int g = j_lo; g < j_hi; g += 64) {
        const int j = g + lane;
        uint64_t b = ballot(j < j_hi && M.at(j, i) != 0);
        while (b) {
            const int jj = g + __ffsll((unsigned long long)b) - 1;
            b &= b - 1;
            const uint32_t q = gfmul(tab, M.at(jj, i), inv);  // :148 / :184
            row_muladd(M, tab, jj, i, q, i);
        }
    }
}

// DecoderMatrix::rref — decoder_matrix.rs:99-244, verbatim.  Returns the new row count.
template <bool WG = true>
__device__ int generic_rref(const Mat &M, const uint32_t *tab, int R, int k) {
    const int lane = lane_id();
    // clean_forward :120-166 (boundary = min(rows, cols) = rows, since rows <= k < cols)
    for (int i = 0; i < R; ++i) {
        uint32_t piv = M.at(i, i);
        if (piv == 0) {
            int found = -1;
            for (int g = i + 1; g < R && found < 0; g += 64) {
                const int j = g + lane;
                const uint64_t b = ballot(j < R && M.at(j, i) != 0);
                if (b) found = g + __ffsll((unsigned long long)b) - 1;
            }
            if (found < 0) continue;
            for (int w = lane; w < M.D; w += 64) {  // swap_rows :69-90
                const uint32_t a = M.w[i * M.D + w];
                M.w[i * M.D + w] = M.w[found * M.D + w];
                M.w[found * M.D + w] = a;
            }
            rsync<WG>();
            piv = M.at(i, i);
        }
        const uint32_t inv = gfinv(tab, piv);
        eliminate_rows(M, tab, i, inv, i + 1, R);
        rsync<WG>();
    }
    // clean_backward :171-215
    for (int i = R - 1; i >= 0; --i) {
        const uint32_t piv = M.at(i, i);
        if (piv == 0) continue;
        const uint32_t inv = gfinv(tab, piv);
        eliminate_rows(M, tab, i, inv, 0, i);
        rsync<WG>();
        if (piv != 1) {  // :200-211
            for (int w = lane; w < M.D; w += 64) {
                const uint32_t mask = from_mask(w, i + 1);
                if (mask) {
                    const uint32_t x = M.w[i * M.D + w];
                    M.w[i * M.D + w] = (x & ~mask) | (mul4(tab, inv, x) & mask);
                }
            }
            rsync<WG>();
            if (lane == 0) M.b[i * M.S + i] = 1;
            rsync<WG>();
        }
    }
    // remove_zero_rows :222-244 (zero test on the first k columns), order preserved
    int dst = 0;
    for (int g = 0; g < R; g += 64) {
        const int r = g + lane;
        bool nz = false;
        if (r < R)
            for (int c4 = 0; 4 * c4 < k && !nz; ++c4) {
                const uint32_t x = M.w[r * M.D + c4];
                nz = (4 * c4 + 4 <= k ? x : (x & (0xFFFFFFFFu >> (8 * (4 * c4 + 4 - k))))) != 0;
            }
        const uint64_t keep = ballot(nz);
        for (int q = 0; q < 64 && g + q < R; ++q) {
            if (!((keep >> q) & 1ull)) continue;
            const int src = g + q;
            if (src != dst) {
                for (int w = lane; w < M.D; w += 64) M.w[dst * M.D + w] = M.w[src * M.D + w];
                rsync<WG>();
            }
            ++dst;
        }
    }
    rsync<WG>();
    return dst;
}

// XOR over the G lane groups (lane blocks of DP = 64 / G): a DPP row rotation below 16 lanes, then the gfx950
// permlane swaps across rows and half-waves -- VALU only (__shfl_xor costs one dependent ds_bpermute per step)
template <int DP>
__device__ __forceinline__ uint32_t group_xor(uint32_t a) {
    // inside a 16-lane row: rotations by 8, 4, 2, 1 down to DP (each lane ends with the XOR of its residue class)
    if constexpr (DP <= 1) a ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x121, 0xf, 0xf, false));  // row_ror:1
    if constexpr (DP <= 2) a ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x122, 0xf, 0xf, false));  // row_ror:2
    if constexpr (DP <= 4) a ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x124, 0xf, 0xf, false));  // row_ror:4
    if constexpr (DP <= 8) a ^= uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x128, 0xf, 0xf, false));  // row_ror:8
    if constexpr (DP <= 16) {  // odd rows of one operand swap with even rows of the other: x ^ x[lane ^ 16]
        const auto s = __builtin_amdgcn_permlane16_swap(a, a, false, false);
        a = s[0] ^ s[1];
    }
    if constexpr (DP <= 32) {  // upper half-wave of one operand swaps with the lower of the other: x ^ x[lane ^ 32]
        const auto s = __builtin_amdgcn_permlane32_swap(a, a, false, false);
        a = s[0] ^ s[1];
    }
    return a;
}

// the same for a run-time group width D (a power of two; D >= 64: one group, nothing to reduce)
__device__ __forceinline__ uint32_t group_xor_rt(uint32_t a, int D) {
    switch (D) {
        case 1: return group_xor<1>(a);
        case 2: return group_xor<2>(a);
        case 4: return group_xor<4>(a);
        case 8: return group_xor<8>(a);
        case 16: return group_xor<16>(a);
        case 32: return group_xor<32>(a);
        default: return a;
    }
}

// rows 0..R-1 a clean RREF: M[i][i] = 1 and column i zero in every other row (i < R)
__device__ bool is_clean(const Mat &M, int R) {
    const int lane = lane_id();
    bool ok = true;
    for (int g = 0; g < R; g += 64) {
        const int j = g + lane;
        if (j < R)
            for (int c4 = 0; 4 * c4 < R; ++c4) {  // bytes 0..R-1 of row j a dword at a time (no early exit: the
                // reads issue together)
                const uint32_t x = M.w[j * M.D + c4];
                const uint32_t want = (j >> 2) == c4 ? 1u << (8 * (j & 3)) : 0u;
                const uint32_t mask = 4 * c4 + 4 <= R ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (8 * (4 * c4 + 4 - R)));
                ok = ok && ((x ^ want) & mask) == 0u;
            }
    }
    return ballot(!ok) == 0;
}

// Clean-state append of row r (see file header).  Returns the new row count; *stays_clean.

__device__ int clean_append(const Mat &M, const uint32_t *tab, int r, int k, bool *stays_clean) {
    const int lane = threadIdx.x;
    const int D = M.D;
    const int G = D >= 64 ? 1 : 64 / D;  // lane groups splitting the pivot rows
    const int w = D >= 64 ? lane : lane % D;
    const int g = D >= 64 ? 0 : lane / D;
    // the original coefficients of row r, kept in the spare row k while row r is rewritten
    for (int ww = lane; ww < D; ww += 64) M.w[k * D + ww] = M.w[r * D + ww];
    __syncthreads();
    // forward (decoder_matrix.rs:143-162 restricted to the new row): row_r ^= Σ_i M[r][i]·row_i.
    // Batches of kU rows per lane group: all quotient, table and data loads of a batch are issued before
    // any product, so the LDS latencies overlap instead of forming one chain per row.
    constexpr int kU = 8;
    for (int w0 = 0; w0 < D; w0 += 64) {
        const int ww = w0 + w;
        const bool act = g < G && ww < D;
        uint32_t acc = 0;
        for (int i0 = g; i0 < r; i0 += kU * G) {
            uint32_t q[kU], x[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int i = i0 + u * G;
                const bool in = act && i < r;
                q[u] = in ? M.at(k, i) : 0u;
                x[u] = in ? M.w[i * D + ww] : 0u;
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) acc ^= mul4(tab, q[u], x[u]);
        }
        if (D < 64) {  // reduce the G partial sums (groups are lane blocks of D)
            acc = group_xor_rt(acc, D);
        }
        if (g == 0 && ww < D) M.w[r * D + ww] ^= acc;
        __syncthreads();
    }
    const uint32_t piv = M.at(r, r);
    if (piv == 0) {
        // the step i = r finds no pivot (no rows below), backward does nothing; the row survives iff a
        // coefficient byte is nonzero (remove_zero_rows).  A kept row breaks the clean state.
        bool nz = false;
        for (int c = lane; c < k; c += 64) nz |= M.at(r, c) != 0;
        const bool keep = ballot(nz) != 0;
        __syncthreads();
        *stays_clean = !keep;
        return keep ? r + 1 : r;
    }
    // normalise row r from column r+1 (:200-211), then eliminate column r above it (:179-198)
    const uint32_t inv = gfinv(tab, piv);
    for (int ww = lane; ww < D; ww += 64) {
        const uint32_t mask = from_mask(ww, r + 1);
        if (mask) {
            const uint32_t x = M.w[r * D + ww];
            M.w[r * D + ww] = (x & ~mask) | (mul4(tab, inv, x) & mask);
        }
    }
    __syncthreads();
    if (lane == 0) M.b[r * M.S + r] = 1;
    __syncthreads();
    // eliminate column r above row r: the quotient M[j][r] of every row of a batch is read before any
    // column block of those rows is rewritten (the block holding column r zeroes it); row r's data is
    // loaded once per column block and shared by all rows
    for (int j0 = g; j0 < r; j0 += kU * G) {
        uint32_t q[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int j = j0 + u * G;
            q[u] = j < r ? M.at(j, r) : 0u;
        }
        // (one wave: its LDS reads complete in issue order, so these quotients precede the writes below)
        for (int w0 = 0; w0 < D; w0 += 64) {
            const int ww = w0 + w;
            if (g >= G || ww >= D) continue;
            const uint32_t xr = M.w[r * D + ww] & from_mask(ww, r);
            uint32_t y[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int j = j0 + u * G;
                y[u] = j < r ? M.w[j * D + ww] : 0u;
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int j = j0 + u * G;
                if (j < r) M.w[j * D + ww] = y[u] ^ mul4(tab, q[u], xr);
            }
        }
    }
    __syncthreads();
    *stays_clean = true;
    return r + 1;
}

// ---------------------------------------------------------------------------------------------------
// Register-resident clean path (same products as clean_append, without LDS round trips on the matrix).
// Lane (w, g) = (lane % DP, lane / DP), DP = 64 / G dword slots per row; register t of lane (w, g) holds
// dword w of row G·t + g.  Rows not yet appended are zero in registers, so products with them are no-ops.
//   forward  (decoder_matrix.rs:143-162 for the new row r): every lane multiplies its rows i < r by the
//            ORIGINAL coefficient M[r][i] (read from the LDS copy of the new row) and the G partial sums are
//            XOR-reduced across lane groups: new row = init ^ Σ_i M[r][i]·row_i;
//   pivot    M[r][r] == 0: not useful (all k coefficient bytes zero) or kept and the clean state ends
//            (registers are written back to LDS for the generic path);
//   normalise from column r+1 (:200-211), byte r := 1;
//   backward (:179-198) every row j < r ^= M[j][r]·row_r, M[j][r] broadcast from lane (r/4, g).
// ---------------------------------------------------------------------------------------------------
template <int G, int RT, bool WG = true>
__device__ void regs_to_lds(const Mat &M, const uint32_t (&v)[RT], int rows) {
    constexpr int DP = 64 / G;
    const int w = lane_id() % DP, g = lane_id() / DP;
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        const int row = G * t + g;
        if (row < rows && w < M.D) M.w[row * M.D + w] = v[t];
    }
    rsync<WG>();
}

template <int G, int RT>
__device__ void lds_to_regs(const Mat &M, uint32_t (&v)[RT], int rows) {
    constexpr int DP = 64 / G;
    const int w = lane_id() % DP, g = lane_id() / DP;
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        const int row = G * t + g;
        v[t] = (row < rows && w < M.D) ? M.w[row * M.D + w] : 0u;
    }
}


// Forward operands of one piece for the current row count r: this lane's dword of the initial row
// [coeffs | unit vector of slot pc] and its quotients M[r][i] = coefficient i (i = G·t + g < r); with few
// rows per lane (RT <= 8) also their tables, so the forward products need no LDS read at all.
template <int G, int RT>
struct FwdOps {
    static constexpr bool kPre = RT <= 8;
    uint32_t init;
    uint32_t q[RT];
    uint4 t4[kPre ? RT : 1];
    uint32_t t2[kPre ? RT : 1];
};

template <int G, int RT>
__device__ __forceinline__ void load_fwd(const Mat &M, const uint32_t *tab, const uint8_t *H, int pc, int r, int k,
                                         FwdOps<G, RT> &f) {
    constexpr int DP = 64 / G;
    const int w = lane_id() % DP, g = lane_id() / DP;
    const uint8_t *h = H + pc * k;
#pragma unroll
    for (int t = 0; t < RT; ++t) {  // unconditional (clamped) reads: all in flight at once, then selected
        const int i = G * t + g;
        const uint32_t x = h[i < k ? i : k - 1];
        f.q[t] = i < r ? x : 0u;
    }
    // this lane's dword of [coeffs | unit vector of slot pc]: with k a multiple of 4 the coefficient dwords are whole
    // dwords of the staged header (4-byte aligned: H is, and pc·k is) -- one clamped load and selects, no per-byte
    // divergent reads (k is uniform: the branch is too)
    uint32_t init = 0;
    const int c0 = 4 * w;
    if ((k & 3) == 0) {
        const uint32_t x = reinterpret_cast<const uint32_t *>(h)[min(w, (k >> 2) - 1)];
        init = c0 < k ? x : 0u;
    } else if (w < M.D) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int c = c0 + b;
            init |= (c < k ? uint32_t(h[c < k ? c : 0]) : 0u) << (8 * b);
        }
    }
    const int u = k + pc - c0;  // the unit vector's byte in this dword
    if (w < M.D && u >= 0 && u < 4) init |= 1u << (8 * u);
    f.init = init;
    if constexpr (FwdOps<G, RT>::kPre) {
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            f.t4[t] = *reinterpret_cast<const uint4 *>(tab + f.q[t] * kTabDw);
            f.t2[t] = tab[f.q[t] * kTabDw + 4];
        }
    }
}

// acc ^= Σ_t q[t]·x[t] over chunks of 8 (table reads of a chunk issued together)
template <int RT>
__device__ __forceinline__ uint32_t dot_chunked(const uint32_t *tab, const uint32_t (&q)[RT], const uint32_t (&x)[RT]) {
    uint32_t acc = 0;
#pragma unroll
    for (int c0 = 0; c0 < RT; c0 += 8) {
        uint4 t4[8];
        uint32_t t2[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            t4[u] = *reinterpret_cast<const uint4 *>(tab + q[c0 + u] * kTabDw);
            t2[u] = tab[q[c0 + u] * kTabDw + 4];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc ^= mul4t(t4[u], t2[u], x[c0 + u]);
    }
    return acc;
}

// Runs pieces pc, pc+1, ... on the registers while the matrix stays a clean RREF (the next piece's forward
// operands are loaded while the current one finishes).  Returns the next piece index; on leaving the clean
// state (a kept row with a zero diagonal) the whole matrix is written back to LDS and *clean = false.
#ifndef RLNC_SMALL_PRIO
#define RLNC_SMALL_PRIO 1
#endif
constexpr bool kSmallPrio = RLNC_SMALL_PRIO != 0;

template <int G, int RT, bool WG = true>
__device__ int reg_run(const Mat &M, const uint32_t *tab, uint32_t (&v)[RT], const uint8_t *H, int pc, int m, int k,
                       int &rows, bool &clean, int32_t *St) {
    constexpr int DP = 64 / G;
    const int lane = lane_id();
    const int w = lane % DP, g = lane / DP;
    const bool wl = w < M.D;
    uint32_t cm = 0;  // coefficient bytes (< k) of this lane's dword
    if (wl && 4 * w < k) cm = 4 * w + 4 <= k ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (8 * (4 * w + 4 - k)));
    FwdOps<G, RT> f;
    pc = __builtin_amdgcn_readfirstlane(pc);  // uniform piece index: scalar loop control
    load_fwd<G, RT>(M, tab, H, pc, rows, k, f);
    for (; pc < m; ++pc) {
        if constexpr (!WG) {
            // one wave per object, several objects per SIMD (the small-object kernel): a wave that has fallen behind
            // wins issue over one ahead of it -- priority 3 for the first quarter of the pieces down to 0 for the last
            // -- so the SIMD's objects finish together instead of one straggler setting the kernel's end
            // (RLNC_SMALL_PRIO diagnostic knob: the A/B build compiles both)
            if (kSmallPrio) {  // s_setprio takes an immediate: step down at the quarter marks
                const int q4 = 4 * pc;
                if (q4 < m) __builtin_amdgcn_s_setprio(3);
                else if (q4 < 2 * m) __builtin_amdgcn_s_setprio(2);
                else if (q4 < 3 * m) __builtin_amdgcn_s_setprio(1);
                else __builtin_amdgcn_s_setprio(0);
            }
        }
        const int r = __builtin_amdgcn_readfirstlane(rows);  // uniform: scalar branches and shift amounts below
        if (r == k) {  // decoder.rs:97-99
            if (lane == 0) St[pc] = RLNC_ERR_RECEIVED_ALL_PIECES;
            continue;
        }
        // forward: new row = init ^ Σ_{i<r} M[r][i]·row_i
        uint32_t acc = 0;
        if constexpr (FwdOps<G, RT>::kPre) {
#pragma unroll
            for (int t = 0; t < RT; ++t) acc ^= mul4t(f.t4[t], f.t2[t], v[t]);
        } else {
            acc = dot_chunked<RT>(tab, f.q, v);
        }
        acc = group_xor<DP>(acc);
        uint32_t nr = f.init ^ acc;
        const int rw = r >> 2, rb = 8 * (r & 3);
        const uint32_t piv = __builtin_amdgcn_readfirstlane((__builtin_amdgcn_readlane(nr, rw) >> rb) & 0xFFu);
        if (piv == 0) {
            const bool keep = ballot((nr & cm) != 0) != 0;  // remove_zero_rows (:222-244)
            if (lane == 0) St[pc] = keep ? RLNC_OK : RLNC_ERR_PIECE_NOT_USEFUL;
            if (keep) {  // the row survives with a zero diagonal: leave the clean state (generic path)
                regs_to_lds<G, RT, WG>(M, v, r);
                if (g == 0 && wl) M.w[r * M.D + w] = nr;
                rsync<WG>();
                rows = r + 1;
                clean = false;
                return pc + 1;
            }
            if (pc + 1 < m) load_fwd<G, RT>(M, tab, H, pc + 1, r, k, f);
            continue;
        }
        // normalise from column r+1 by the inverse of the pivot (:200-211), byte r := 1
        const uint4 ti4 = *reinterpret_cast<const uint4 *>(tab + (256 + piv) * kTabDw);
        const uint32_t ti2 = tab[(256 + piv) * kTabDw + 4];
        const uint32_t mask = from_mask(w, r + 1);
        nr = (nr & ~mask) | (mul4t(ti4, ti2, nr) & mask);
        if (w == rw) nr = (nr & ~(0xFFu << rb)) | (1u << rb);
        // backward (:179-198): rows j < r ^= M[j][r]·row_r (absent rows are zero: q = 0, no-op)
        rows = r + 1;
#pragma unroll
        for (int c0 = 0; c0 < RT; c0 += 8) {
            constexpr int U = RT < 8 ? RT : 8;
            uint4 b4[U];
            uint32_t b2[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t qb = (__shfl(v[c0 + u], rw + DP * g) >> rb) & 0xFFu;
                b4[u] = *reinterpret_cast<const uint4 *>(tab + qb * kTabDw);
                b2[u] = tab[qb * kTabDw + 4];
            }
            if (c0 == 0 && pc + 1 < m) load_fwd<G, RT>(M, tab, H, pc + 1, r + 1, k, f);  // overlaps the products
#pragma unroll
            for (int u = 0; u < U; ++u) v[c0 + u] ^= mul4t(b4[u], b2[u], nr);
        }
#pragma unroll
        for (int t = 0; t < RT; ++t)
            if (G * t + g == r) v[t] = nr;
        if (lane == 0) St[pc] = RLNC_OK;
    }
    return pc;
}

// staged headers: m × k bytes after the matrix (hdr_lds = 1), else read from global memory per piece
// ---------------------------------------------------------------------------------------------------
// Multi-wave clean run (k <= 32, row <= 16 dwords): the same products as reg_run, with the matrix rows spread
// over NW waves (wave s, lane (w, g), register t holds dword w of row 8s + 4t + g).  Per piece: each wave's
// forward partial sum is reduced inside the wave, the NW partials meet in LDS (one barrier per piece, two
// buffers), every wave finishes the new row redundantly, then updates its own rows (backward).  A wave's VALU
// work per piece is 1/NW of the single-wave path's.  Returns the next piece index; on exit (all pieces done,
// or a kept row with a zero diagonal ends the clean state) the whole matrix is in LDS.
// ---------------------------------------------------------------------------------------------------
template <int NW, int MG, int RTW>
__device__ int reg_run_mw(const Mat &M, const uint32_t *tab, const uint8_t *H, uint32_t *P, int m, int k, int &rows,
                          bool &clean, int32_t *St) {
    constexpr int G = MG, DP = 64 / MG;
    constexpr bool kPre = RTW <= 8;  // few rows per lane: the next piece's forward tables are prefetched
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int w = lane % DP, g = lane / DP;
    const bool wl = w < M.D;
    uint32_t cm = 0;  // coefficient bytes (< k) of this lane's dword
    if (wl && 4 * w < k) cm = 4 * w + 4 <= k ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (8 * (4 * w + 4 - k)));
    uint32_t v[RTW];
#pragma unroll
    for (int t = 0; t < RTW; ++t) v[t] = 0;
    auto row_of = [&](int t) { return RTW * G * wave + G * t + g; };
    // forward operands of piece pc for row count r: init dword w, quotients M[r][i] of own rows (and tables)
    uint32_t init = 0, q[RTW], t2[kPre ? RTW : 1];
    uint4 t4[kPre ? RTW : 1];
    auto load_ops = [&](int pc, int r) {
        const uint8_t *h = H + pc * k;
#pragma unroll
        for (int t = 0; t < RTW; ++t) q[t] = row_of(t) < r ? uint32_t(h[row_of(t)]) : 0u;
        uint32_t x = 0;
        if (wl) {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int c = 4 * w + b;
                x |= (c < k ? uint32_t(h[c]) : uint32_t(c == k + pc)) << (8 * b);
            }
        }
        init = x;
        if constexpr (kPre) {
#pragma unroll
            for (int t = 0; t < RTW; ++t) {
                t4[t] = *reinterpret_cast<const uint4 *>(tab + q[t] * kTabDw);
                t2[t] = tab[q[t] * kTabDw + 4];
            }
        }
    };
    auto to_lds = [&](int nrows) {
#pragma unroll
        for (int t = 0; t < RTW; ++t)
            if (row_of(t) < nrows && wl) M.w[row_of(t) * M.D + w] = v[t];
    };
    int buf = 0, pc = 0;
    load_ops(0, 0);
    for (; pc < m; ++pc) {
        const int r = rows;
        if (r == k) {  // decoder.rs:97-99
            if (threadIdx.x == 0) St[pc] = RLNC_ERR_RECEIVED_ALL_PIECES;
            continue;
        }
        uint32_t acc = 0;
        if constexpr (kPre) {
#pragma unroll
            for (int t = 0; t < RTW; ++t) acc ^= mul4t(t4[t], t2[t], v[t]);
        } else {
            acc = dot_chunked<RTW>(tab, q, v);
        }
        acc = group_xor<DP>(acc);
        uint32_t *Pb = P + buf * NW * DP;
        if (lane < DP) Pb[wave * DP + lane] = acc;
        __syncthreads();
        uint32_t nr = init;
#pragma unroll
        for (int s = 0; s < NW; ++s) nr ^= Pb[s * DP + w];
        buf ^= 1;
        const int rw = r >> 2, rb = 8 * (r & 3);
        const uint32_t piv = __builtin_amdgcn_readfirstlane((__builtin_amdgcn_readlane(nr, rw) >> rb) & 0xFFu);
        if (piv == 0) {
            const bool keep = ballot((nr & cm) != 0) != 0;  // remove_zero_rows (:222-244)
            if (threadIdx.x == 0) St[pc] = keep ? RLNC_OK : RLNC_ERR_PIECE_NOT_USEFUL;
            if (keep) {  // leave the clean state: the matrix goes to LDS for the single-wave generic path
                to_lds(r);
                if (wave == 0 && g == 0 && wl) M.w[r * M.D + w] = nr;
                __syncthreads();
                rows = r + 1;
                clean = false;
                return pc + 1;
            }
            if (pc + 1 < m) load_ops(pc + 1, r);
            continue;
        }
        const uint4 ti4 = *reinterpret_cast<const uint4 *>(tab + (256 + piv) * kTabDw);
        const uint32_t ti2 = tab[(256 + piv) * kTabDw + 4];
        const uint32_t mask = from_mask(w, r + 1);
        nr = (nr & ~mask) | (mul4t(ti4, ti2, nr) & mask);
        if (w == rw) nr = (nr & ~(0xFFu << rb)) | (1u << rb);
        rows = r + 1;
#pragma unroll
        for (int c0 = 0; c0 < RTW; c0 += 8) {  // backward in chunks of 8 rows (table reads issued together)
            constexpr int U = RTW < 8 ? RTW : 8;
            uint4 b4[U];
            uint32_t b2[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t qb = (__shfl(v[c0 + u], rw + DP * g) >> rb) & 0xFFu;  // M[row][r], row in this wave
                b4[u] = *reinterpret_cast<const uint4 *>(tab + qb * kTabDw);
                b2[u] = tab[qb * kTabDw + 4];
            }
            if (c0 == 0 && pc + 1 < m) load_ops(pc + 1, r + 1);
#pragma unroll
            for (int u = 0; u < U; ++u) v[c0 + u] ^= mul4t(b4[u], b2[u], nr);
        }
#pragma unroll
        for (int t = 0; t < RTW; ++t)
            if (row_of(t) == r) v[t] = nr;
        if (threadIdx.x == 0) St[pc] = RLNC_OK;
    }
    to_lds(rows);
    __syncthreads();
    return pc;
}

// G > 0: the clean state runs on registers (reg_run<G, RT>); G = 0: on LDS (clean_append).  NW > 1: the
// initial clean run is spread over NW waves (reg_run_mw); then waves 1..NW-1 end and wave 0 continues alone
// (S_BARRIER waits only for the waves that have not terminated).
// ragged batch (p.objs): this workgroup's object replaces the uniform fields, as object 0 of a one-object batch
__device__ __forceinline__ void rref_ragged_object(RrefParams &p, int &o) {
    if (p.objs == nullptr) return;
    const RrefObj &d = p.objs[o];
    p.pieces = d.pieces;
    p.obj_stride = 0;
    p.piece_stride = d.piece_stride;
    p.k = __builtin_amdgcn_readfirstlane(d.k);
    p.m = __builtin_amdgcn_readfirstlane(d.m);
    p.m_stride = 0;
    if (!p.skip_full && d.m_first > 0) {  // the blocked pass over the first pieces only
        p.m = __builtin_amdgcn_readfirstlane(d.m_first);
        p.m_stride = __builtin_amdgcn_readfirstlane(d.m);
    }
    p.skip_full = p.skip_full && d.two_pass;
    p.T = d.T;
    p.T_obj = 0;
    p.status = d.status;
    p.rank = d.rank;
    o = 0;
}

template <int G, int RT, int NW, int MG = 4, int MRTW = 2>
__global__ __launch_bounds__(64 * NW) void gf_rref_batch_kernel(RrefParams p, int hdr_lds) {
    extern __shared__ uint32_t lds[];
    uint32_t *tab = lds;  // kTabEntries × kTabDw dwords
    const int lane = threadIdx.x;  // the single-wave code below runs in wave 0 only (lane < 64)
    const int tid = threadIdx.x;
    int o = blockIdx.x;
    rref_ragged_object(p, o);
    if (p.skip_full && p.rank[o] >= p.k) return;  // two-pass: the blocked pass already full-ranked this object
    const int k = p.k, m = p.m;
    Mat M;
    M.D = rref_row_dwords(k, m);
    M.S = 4 * M.D;
    M.w = lds + kTabEntries * kTabDw;
    M.b = reinterpret_cast<uint8_t *>(M.w);
    // per-piece statuses stay in LDS until the end: a global store before each __syncthreads would make
    // its release fence wait for the store to reach memory, once per piece
    int32_t *St = reinterpret_cast<int32_t *>(M.b + size_t(k + 1) * M.S);
    uint8_t *H = reinterpret_cast<uint8_t *>(St + ((m + 3) & ~3));
    // NW > 1: two buffers of NW × 16 forward partial sums after the staged headers
    uint32_t *P = reinterpret_cast<uint32_t *>(H + ((size_t(m) * k + 15) & ~size_t(15)));

    {  // all loads of the table copy in flight at once (one memory latency, not one per iteration)
        constexpr int kPer = kTabEntries * kTabDw / 4 / (64 * NW);
        const uint4 *src = reinterpret_cast<const uint4 *>(kRrefTable.v);
        uint4 *dst = reinterpret_cast<uint4 *>(tab);
        uint4 t4[kPer];
#pragma unroll
        for (int u = 0; u < kPer; ++u) t4[u] = src[tid + 64 * NW * u];
#pragma unroll
        for (int u = 0; u < kPer; ++u) dst[tid + 64 * NW * u] = t4[u];
    }
    const uint8_t *base = p.pieces + int64_t(o) * p.obj_stride;
    if (hdr_lds) {  // 16 independent byte loads in flight per batch
        for (int e0 = 0; e0 < m * k; e0 += 64 * NW * 16) {
            uint8_t hb[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int e = e0 + tid + 64 * NW * u;
                hb[u] = e < m * k ? base[int64_t(e / k) * p.piece_stride + e % k] : uint8_t(0);
            }
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (e0 + tid + 64 * NW * u < m * k) H[e0 + tid + 64 * NW * u] = hb[u];
        }
    }
    for (int w = tid; w < (k + 1) * M.D; w += 64 * NW) M.w[w] = 0;
    __syncthreads();

    int rows = 0;
    bool clean = true;
    int pc0 = 0;
    if constexpr (NW > 1) {
        pc0 = reg_run_mw<NW, MG, MRTW>(M, tab, H, P, m, k, rows, clean, St);
        if (threadIdx.x >= 64) return;  // wave 0 finishes alone (generic path / output)
    }
    uint32_t v[G > 0 ? RT : 1];
#pragma unroll
    for (int t = 0; t < (G > 0 ? RT : 1); ++t) v[t] = 0;
    if constexpr (NW > 1 && G > 0)
        if (clean && rows > 0 && pc0 < m) lds_to_regs<G, RT>(M, v, rows);
    for (int pc = pc0; pc < m; ++pc) {
        if constexpr (G > 0) {
            if (clean) {
                pc = reg_run<G, RT>(M, tab, v, H, pc, m, k, rows, clean, St);
                __syncthreads();
                if (pc >= m) break;
            }
        }
        if (rows == k) {  // decoder.rs:97-99
            if (lane == 0) St[pc] = RLNC_ERR_RECEIVED_ALL_PIECES;  // ReceivedAllPieces
            continue;
        }
        // add_row (decoder_matrix.rs:53-62): [coeffs | unit vector of this piece's slot]
        // two explicit branches: a run-time choice of pointer would be a flat access (VMEM latency + waits)
        if (hdr_lds) {
            for (int c = lane; c < M.S; c += 64) M.b[rows * M.S + c] = c < k ? H[pc * k + c] : uint8_t(c == k + pc);
        } else {
            const uint8_t *hdr = base + int64_t(pc) * p.piece_stride;
            for (int c = lane; c < M.S; c += 64) M.b[rows * M.S + c] = c < k ? hdr[c] : uint8_t(c == k + pc);
        }
        __syncthreads();
        const int before = rows;
        if (G == 0 && clean) {
            bool sc;
            rows = clean_append(M, tab, rows, k, &sc);
            clean = sc;
        } else {
            rows = generic_rref(M, tab, rows + 1, k);
            clean = is_clean(M, rows);
            if constexpr (G > 0)
                if (clean) lds_to_regs<G, RT>(M, v, rows);
        }
        if (lane == 0) St[pc] = rows == before ? RLNC_ERR_PIECE_NOT_USEFUL : RLNC_OK;  // decoder.rs:112-117
        __syncthreads();
    }
    if constexpr (G > 0)
        if (clean && pc0 < m) regs_to_lds<G, RT>(M, v, rows);
    __syncthreads();
    for (int pc = lane; pc < m; pc += 64) p.status[int64_t(o) * m + pc] = St[pc];
    if (lane == 0) p.rank[o] = rows;
    uint8_t *T = p.T + int64_t(o) * p.T_obj;
    for (int e = lane; e < k * m; e += 64) {
        const int r = e / m, s = e % m;
        T[e] = r < rows ? M.b[r * M.S + k + s] : uint8_t(0);
    }
}


// Many small objects (row <= 16 dwords, k <= 16): NW objects per workgroup, one per wave, over ONE LDS copy of the
// multiplier table.  The one-wave kernel above copies the 16 KiB table per object, which caps a CU at 8 resident
// objects; here a workgroup of 4 holds 4 objects in ~20 KiB, so all 16 objects per CU of a 4,096-object batch are
// resident at once.  Per wave the same steps as gf_rref_batch_kernel<4, 8, 1> (register clean run, the reference's
// rref verbatim when the clean state ends), with wave-local synchronisation only: after the table copy no wave
// waits for another.
// the payload-tail staging of one object (RrefParams::tail_status): the last 64 data bytes of each of its m pieces,
// moved into LDS by DMA at the kernel's start (a valid payload's marker lies in its last k <= 16 bytes)
constexpr int kTailBytes = 64;
__host__ __device__ inline size_t rref_small_tail_bytes(int m) { return size_t(m) * kTailBytes; }
__host__ __device__ inline size_t rref_small_wave_bytes(int k, int m) {
    return size_t(k + 1) * 4 * size_t(rref_row_dwords(k, m)) + 4 * ((size_t(m) + 3) & ~size_t(3)) +
           ((size_t(m) * k + 15) & ~size_t(15));
}
constexpr int kSmallNW = 4;
constexpr int kSmallMinObjects = 2048;

// ---------------------------------------------------------------------------------------------------
// Blocked clean run (path 5, default when k + m <= 256): while rows 0..r-1 are a clean RREF, the next b <= B
// pieces are appended in one block instead of one at a time:
//   1. X_t = init_t ^ Σ_{i<r} P_t[i]·R_i for t < b — the forward pass of every piece of the block against the r
//      clean rows (the quotients are the original coefficients, file header), summed over (wave, lane group)
//      stripes of i and met in LDS by ds_xor;
//   2. the b rows among themselves, exactly as the one-piece clean step would take them in order: y_t ^=
//      Σ_{s<t} X_t[r+s]·y_s, pivot y_t[r+t], normalise from r+t+1 by its inverse, eliminate column r+t from the
//      y_s (s < t) — every wave does this redundantly in registers (lane = dword), so no wave waits for another;
//   3. R_j ^= Σ_{t<c} R_j[r+t]·y_t for every row j < r (rows striped over waves and lane groups), y_t appended as
//      rows r..r+c-1.
// Same state as c one-piece steps: the clean RREF with pivots 0..r+c-1 of span(R, P_0..P_{c-1}) is unique, and y_t
// is the unique vector of P_t + span(committed rows) that is zero in columns 0..r+t-1, which is what the forward
// pass of the one-piece step computes — so pivot tests, normalised rows and statuses are identical.  A zero pivot
// at t ends the block after c = t pieces: piece t's reduced row y_t is then exactly clean_append's row (kept, the
// clean state ends, iff a coefficient byte is nonzero).  Outside the clean state every piece runs the reference
// algorithm verbatim (generic_rref) in wave 0 while the other waves wait at the next workgroup barrier, and the
// blocked run resumes once is_clean holds again.
// ---------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t byte_of(uint32_t v, int lane_dw, int b) {
    return (uint32_t(__builtin_amdgcn_readlane(int(v), lane_dw)) >> (8 * b)) & 0xFFu;
}


// ---- the non-clean step of the blocked kernel (rows 0..cp-1 a clean prefix, rows cp..R-1 dirty) --------------
// Clean prefix: for i < cp, M[i][i] = 1 and column i is zero in every other row < cp.  The reference's rref
// (decoder_matrix.rs:99-244) on such a matrix splits exactly: its forward steps i < cp only reduce the dirty
// rows against the prefix rows (pivot 1, quotient = the dirty row's original byte i, since a prefix row is zero in
// every other prefix column) and never swap; its forward steps i >= cp touch dirty rows only; its backward steps
// i >= cp eliminate column i from every row above (prefix rows included), and its backward steps i < cp do
// nothing (column i is zero above row i, the pivot is 1); remove_zero_rows can only drop dirty rows.

// forward steps i in [r0, R) of clean_forward (:120-166), verbatim, on rows >= r0 (one wave)
__device__ void forward_range(const Mat &M, const uint32_t *tab, int r0, int R) {
    const int lane = threadIdx.x & 63;
    for (int i = r0; i < R; ++i) {
        uint32_t piv = M.at(i, i);
        if (piv == 0) {
            int found = -1;
            for (int g = i + 1; g < R && found < 0; g += 64) {
                const int j = g + lane;
                const uint64_t b = ballot(j < R && M.at(j, i) != 0);
                if (b) found = g + __ffsll((unsigned long long)b) - 1;
            }
            if (found < 0) continue;
            for (int w = lane; w < M.D; w += 64) {  // swap_rows :69-90
                const uint32_t a = M.w[i * M.D + w];
                M.w[i * M.D + w] = M.w[found * M.D + w];
                M.w[found * M.D + w] = a;
            }
            rsync<false>();
            piv = M.at(i, i);
        }
        const uint32_t inv = gfinv(tab, piv);
        for (int g = i + 1; g < R; g += 64) {
            const int j = g + lane;
            uint64_t b = ballot(j < R && M.at(j, i) != 0);
            while (b) {
                const int jj = g + __ffsll((unsigned long long)b) - 1;
                b &= b - 1;
                const uint32_t q = gfmul(tab, M.at(jj, i), inv);  // :148
                for (int w = lane; w < M.D; w += 64) {
                    const uint32_t mask = from_mask(w, i);
                    if (mask) M.w[jj * M.D + w] ^= mul4(tab, q, M.w[i * M.D + w]) & mask;
                }
            }
        }
        rsync<false>();
    }
}

// remove_zero_rows (:222-244) over rows [r0, R) (zero test on the first k columns, order preserved); one wave
__device__ int remove_zero_range(const Mat &M, int r0, int R, int k) {
    const int lane = threadIdx.x & 63;
    int dst = r0;
    for (int g = r0; g < R; g += 64) {
        const int r = g + lane;
        bool nz = false;
        if (r < R)
            for (int c4 = 0; 4 * c4 < k && !nz; ++c4) {
                const uint32_t x = M.w[r * M.D + c4];
                nz = (4 * c4 + 4 <= k ? x : (x & (0xFFFFFFFFu >> (8 * (4 * c4 + 4 - k))))) != 0;
            }
        const uint64_t keep = ballot(nz);
        for (int q = 0; q < 64 && g + q < R; ++q) {
            if (!((keep >> q) & 1ull)) continue;
            const int src = g + q;
            if (src != dst) {
                for (int w = lane; w < M.D; w += 64) M.w[dst * M.D + w] = M.w[src * M.D + w];
                rsync<false>();
            }
            ++dst;
        }
    }
    rsync<false>();
    return dst;
}

// extends the clean prefix from cp while row cp has M[cp][cp] = 1, zeros in columns < cp, and column cp is zero in
// every row above it; one wave
__device__ int extend_prefix(const Mat &M, int cp, int R) {
    const int lane = threadIdx.x & 63;
    while (cp < R) {
        const int c = cp;
        bool bad = false;
        for (int j = lane; j < c; j += 64) bad |= M.at(j, c) != 0;         // column c above row c
        for (int w = lane; 4 * w < c; w += 64) {                            // row c left of column c
            const uint32_t x = M.w[c * M.D + w];
            bad |= (4 * w + 4 <= c ? x : (x & (0xFFFFFFFFu >> (8 * (4 * w + 4 - c))))) != 0;
        }
        if (ballot(bad) != 0 || M.at(c, c) != 1) break;
        ++cp;
    }
    return cp;
}

// One piece outside the clean state, in one wave (the small-object kernel): rows 0..cp-1 are a clean prefix (M[i][i] = 1,
// column i zero in every other prefix row), rows cp..rows-1 dirty; the piece's header becomes row `rows`.  The
// reference's rref on such a matrix splits around the prefix exactly as gf_rref_block_kernel's dirty step relies on
// (comment above forward_range): forward steps i < cp reduce each dirty row by its ORIGINAL byte i times prefix row i,
// forward steps i >= cp run verbatim on the dirty rows, backward steps i >= cp eliminate column i from every row above
// (prefix rows included) and normalise row i, backward steps i < cp change nothing, remove_zero_rows can only drop
// dirty rows.  The generic path it replaces replayed every step of the whole matrix (~7 us a piece on a k = 16
// object, 8x a clean piece: the kernel's tail, profiles/r05_small_elim_timeline.jsonl).  Updates rows and cp.
__device__ void small_dirty_step(const Mat &M, const uint32_t *tab, const uint8_t *hdr, int pc, int k, int &rows,
                                 int &cp) {
    const int lane = lane_id();
    const int D = M.D, G = 64 / D, w = lane % D, g = lane / D;
    const int r0 = cp, R = rows;
    for (int c = lane; c < M.S; c += 64) M.b[R * M.S + c] = c < k ? hdr[c] : uint8_t(c == k + pc);
    rsync<false>();
    // forward steps i < r0: dirty row t ^= Σ_{i<r0} M[t][i]·row_i, lane group g over prefix rows i ≡ g (mod G),
    // the G partial sums met by group_xor; each row's quotients are read before its one write
    if (r0 > 0) {
        for (int t = r0; t <= R; ++t) {
            uint32_t acc = 0;
            for (int i = g; i < r0; i += G) acc ^= mul4(tab, M.at(t, i), M.w[i * D + w]);
            acc = group_xor_rt(acc, D);
            if (g == 0) M.w[t * D + w] ^= acc;
        }
        rsync<false>();
    }
    forward_range(M, tab, r0, R + 1);  // forward steps i >= r0, verbatim on the dirty rows
    // backward steps i = R .. r0 (:171-215): column i out of every row above, then row i normalised from column i+1
    for (int i = R; i >= r0; --i) {
        const uint32_t piv = M.at(i, i);
        if (piv == 0) continue;
        const uint32_t xi = M.w[i * D + w];
        const uint32_t nr = mul4(tab, 256 + piv, xi);  // row i · piv^-1: (q·piv^-1)·x = q·(piv^-1·x)
        const uint32_t mi = from_mask(w, i);
        for (int j = g; j < i; j += G) {
            const uint32_t q = M.at(j, i);  // read by the whole wave before any lane rewrites row j
            if (q) M.w[j * D + w] ^= mul4(tab, q, nr) & mi;
        }
        rsync<false>();
        if (piv != 1) {
            if (g == 0) {
                const uint32_t mask = from_mask(w, i + 1);
                uint32_t v = (xi & ~mask) | (nr & mask);
                if (w == (i >> 2)) v = (v & ~(0xFFu << (8 * (i & 3)))) | (1u << (8 * (i & 3)));
                M.w[i * D + w] = v;
            }
            rsync<false>();
        }
    }
    rows = remove_zero_range(M, r0, R + 1, k);
    cp = extend_prefix(M, r0, rows);
}

template <int NW, int G, int RT, bool PROF = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(G == 8 ? 4 : 1))) void gf_rref_small_kernel(RrefParams p) {
    extern __shared__ uint32_t lds[];
    uint32_t *tab = lds;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    uint64_t ts[6] = {};  // PROF (diagnostic build): wave start, table copied, headers staged, pieces done, end
    if constexpr (PROF) ts[0] = wall_clock64();
    const int o = blockIdx.x * NW + wave;
    const int k = p.k, m = p.m;  // k <= 16 and k + m <= 64 on this path (rref.hip small_many)
    // this object's headers first (lane = piece, its k <= 16 coefficient bytes in flight at once, no index
    // division), then the shared table copy: both global-load latencies overlap
    uint8_t hb[16];
    const bool hl = o < p.n_obj && lane < m;
    const uint8_t *hp = p.pieces + int64_t(o) * p.obj_stride + int64_t(lane) * p.piece_stride;
#pragma unroll
    for (int u = 0; u < 16; ++u) hb[u] = (hl && u < k) ? hp[u] : uint8_t(0);
    {  // the shared table copy, all loads in flight at once
        constexpr int kPer = kTabEntries * kTabDw / 4 / (64 * NW);
        const uint4 *src = reinterpret_cast<const uint4 *>(kRrefTable.v);
        uint4 *dst = reinterpret_cast<uint4 *>(tab);
        uint4 t4[kPer];
#pragma unroll
        for (int u = 0; u < kPer; ++u) t4[u] = src[tid + 64 * NW * u];
#pragma unroll
        for (int u = 0; u < kPer; ++u) dst[tid + 64 * NW * u] = t4[u];
    }
    Mat M;
    M.D = rref_row_dwords(k, m);
    M.S = 4 * M.D;
    M.w = lds + kTabEntries * kTabDw + size_t(wave) * (rref_small_wave_bytes(k, m) / 4);
    M.b = reinterpret_cast<uint8_t *>(M.w);
    int32_t *St = reinterpret_cast<int32_t *>(M.b + size_t(k + 1) * M.S);
    uint8_t *H = reinterpret_cast<uint8_t *>(St + ((m + 3) & ~3));
    if (hl) {
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (u < k) H[lane * k + u] = hb[u];
    }
    for (int w = lane; w < (k + 1) * M.D; w += 64) M.w[w] = 0;
    // RrefParams::tail_status: the pieces' last 64 data bytes on their way into this wave's LDS (DMA, no registers;
    // lanes 0-15, a dword each), used once the elimination is done
    uint32_t *tailb = lds + kTabEntries * kTabDw + NW * (rref_small_wave_bytes(k, m) / 4) +
                      size_t(wave) * (rref_small_tail_bytes(m) / 4);
    if (p.tail_status != nullptr && o < p.n_obj && lane < kTailBytes / 4) {
        typedef __attribute__((address_space(1))) void gvoid;
        typedef __attribute__((address_space(3))) void lvoid;
        const uint8_t *tb = p.pieces + int64_t(o) * p.obj_stride + k + (p.tail_L - kTailBytes) + 4 * lane;
        for (int j = 0; j < m; ++j)
            __builtin_amdgcn_global_load_lds((gvoid *)(tb + int64_t(j) * p.piece_stride), (lvoid *)(tailb + (kTailBytes / 4) * j), 4, 0,
                                             0);
    }
    __syncthreads();  // the only workgroup barrier: the table, and this wave's headers and zeroed matrix
    if constexpr (PROF) ts[1] = ts[2] = wall_clock64();
    if (o >= p.n_obj) return;

    int rows = 0, cp = -1;  // cp: the clean prefix while outside the clean state (-1 inside it)
    bool clean = true;
    uint32_t v[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) v[t] = 0;
    for (int pc = 0; pc < m; ++pc) {
        if (clean) {
            pc = reg_run<G, RT, false>(M, tab, v, H, pc, m, k, rows, clean, St);
            rsync<false>();
            if (pc >= m) break;
        }
        if (rows == k) {  // decoder.rs:97-99
            if (lane == 0) St[pc] = RLNC_ERR_RECEIVED_ALL_PIECES;
            continue;
        }
        // add_row (decoder_matrix.rs:53-62) and the reference's rref (decoder_matrix.rs:99-244) on a clean prefix
        // (rows < cp) + dirty rows, decomposed around the prefix (small_dirty_step)
        if (cp < 0) cp = rows - 1;  // reg_run left the clean state: its last kept row is the first dirty one
        const int before = rows;
        if constexpr (PROF) ++ts[5];  // pieces outside the clean state
        small_dirty_step(M, tab, H + pc * k, pc, k, rows, cp);
        clean = cp == rows;
        if (clean) {
            lds_to_regs<G, RT>(M, v, rows);
            cp = -1;
        }
        if (lane == 0) St[pc] = rows == before ? RLNC_ERR_PIECE_NOT_USEFUL : RLNC_OK;  // decoder.rs:112-117
        rsync<false>();
    }
    if (clean) regs_to_lds<G, RT, false>(M, v, rows);
    rsync<false>();
    // RrefParams::tail_status: the marker scan's answer from the payload tail -- before this wave's stores below, so
    // that the wait for the staging DMAs does not wait for them too
    int32_t tail_st = RLNC_ERR_NOT_ALL_PIECES_RECEIVED_YET;
    int64_t tail_len = 0;
    int32_t tail_need = 0;
    if (p.tail_status != nullptr) {
        if (rows == k) {
            // lane l < 16: dword l of decoded row k - 1's last 64 bytes = Σ_j T[k-1][j] · (piece j's data dword
            // there, staged in LDS at the start)
            const int64_t L = p.tail_L;
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the staging DMAs (long landed)
            uint32_t acc = 0;
            for (int j0 = 0; j0 < m; j0 += 8) {
                uint32_t c[8], x[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int j = j0 + u;
                    c[u] = j < m ? uint32_t(M.b[(k - 1) * M.S + k + j]) : 0u;
                    x[u] = j < m && lane < kTailBytes / 4 ? tailb[(kTailBytes / 4) * j + lane] : 0u;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) acc ^= mul4(tab, c[u], x[u]);
            }
            const uint64_t nz = __ballot(acc != 0);
            if (nz != 0) {
                const int h = __builtin_amdgcn_readfirstlane(63 - __builtin_clzll(nz));  // the last lane with a byte
                const uint32_t a = __builtin_amdgcn_readlane(acc, h);
                const int b = (31 - __builtin_clz(a)) / 8;
                const int64_t pos = int64_t(k - 1) * L + (L - kTailBytes) + 4 * h + b;
                const bool ok = ((a >> (8 * b)) & 0xFFu) == kBoundaryMarker && pos > 0;
                tail_st = ok ? RLNC_OK : RLNC_ERR_INVALID_DECODED_DATA_FORMAT;
                tail_len = ok ? pos : 0;
            } else {
                tail_st = RLNC_OK;  // decided by the product's workgroup (scan_need)
                tail_need = 1;
            }
        }
    }
    if constexpr (PROF) ts[3] = wall_clock64();
    for (int pc = lane; pc < m; pc += 64) p.status[int64_t(o) * m + pc] = St[pc];
    if (lane == 0) p.rank[o] = rows;
    if (p.tail_status != nullptr && lane == 0) {
        p.tail_status[o] = tail_st;
        p.tail_len[o] = tail_len;
        p.tail_need[o] = tail_need;
    }
    // T row by row, lane = column (m <= 64 here): no per-element index division
    uint8_t *T = p.T + int64_t(o) * p.T_obj;
    for (int r = 0; r < k; ++r)
        if (lane < m) T[r * m + lane] = r < rows ? M.b[r * M.S + k + lane] : uint8_t(0);
    if (p.bsj_stream != nullptr) {  // T again, as the product's block-offset stream ([j][i], i < tile rows)
        const int tr = p.bsj_tile_rows;  // 8 or 16 (the 1- / 2-wave programs): lane = (column group, row)
        uint32_t *st = p.bsj_stream + int64_t(o) * m * tr;
        const int r = lane & (tr - 1), step = 64 / tr;
        for (int s = lane / tr; s < m; s += step)
            st[s * tr + r] = (r < rows ? uint32_t(M.b[r * M.S + k + s]) : 0u) * p.bsj_block_bytes;
    }
    if constexpr (PROF) {
        ts[4] = wall_clock64();
        ts[5] |= uint64_t(__smid()) << 32;
        if (lane < 6) p.prof[int64_t(o) * 8 + lane] = ts[lane];
        if (lane == 6) p.prof[int64_t(o) * 8 + 6] = uint64_t(rows);
    }
}

struct Sel1 {  // v_perm selectors of one dword: bits 0-2, 3-5, 6-7 of every byte
    uint32_t s0, s1, s2;
};

template <int NW, int B>
__global__ __launch_bounds__(64 * NW) void gf_rref_block_kernel(RrefParams p) {
    extern __shared__ uint32_t lds[];
    uint32_t *tab = lds;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    int o = blockIdx.x;
    rref_ragged_object(p, o);
    const int k = p.k, m = p.m;
    const int kH = (k + 3) & ~3;  // staged header stride (dword-aligned coefficient groups, zero padded)
    Mat M;
    M.D = rref_row_dwords(k, m);  // <= 64 here
    M.S = 4 * M.D;
    M.w = lds + kTabEntries * kTabDw;
    M.b = reinterpret_cast<uint8_t *>(M.w);
    const int D = M.D;
    const int G = 64 / D;                     // lane groups per wave (one matrix row each)
    const int w = lane % D, g = lane / D;     // this lane's dword and group
    const int NS = NW * G, sid = wave * G + g;  // stripes
    int32_t *St = reinterpret_cast<int32_t *>(M.b + size_t(k + 1) * M.S);
    uint8_t *H = reinterpret_cast<uint8_t *>(St + ((m + 3) & ~3));
    uint32_t *X = reinterpret_cast<uint32_t *>(H + ((size_t(m) * kH + 15) & ~size_t(15)));  // B x D dwords
    int *flag = reinterpret_cast<int *>(X + B * D);

    {  // the multiplier tables: all loads in flight at once
        constexpr int kPer = kTabEntries * kTabDw / 4 / (64 * NW);
        const uint4 *src = reinterpret_cast<const uint4 *>(kRrefTable.v);
        uint4 *dst = reinterpret_cast<uint4 *>(tab);
        uint4 t4[kPer];
#pragma unroll
        for (int u = 0; u < kPer; ++u) t4[u] = src[tid + 64 * NW * u];
#pragma unroll
        for (int u = 0; u < kPer; ++u) dst[tid + 64 * NW * u] = t4[u];
    }
    const uint8_t *base = p.pieces + int64_t(o) * p.obj_stride;
    for (int e0 = 0; e0 < m * kH; e0 += 64 * NW * 16) {  // headers, 16 byte loads in flight per thread
        uint8_t hb[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int e = e0 + tid + 64 * NW * u;
            const int pc = e / kH, c = e % kH;
            hb[u] = (e < m * kH && c < k) ? base[int64_t(pc) * p.piece_stride + c] : uint8_t(0);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u)
            if (e0 + tid + 64 * NW * u < m * kH) H[e0 + tid + 64 * NW * u] = hb[u];
    }
    for (int e = tid; e < (k + 1) * D; e += 64 * NW) M.w[e] = 0;
    __syncthreads();

  // setup: tables, headers, zeroed matrix
    uint32_t cm = 0;  // coefficient bytes (< k) of this lane's dword
    if (4 * w < k) cm = 4 * w + 4 <= k ? 0xFFFFFFFFu : (0xFFFFFFFFu >> (8 * (4 * w + 4 - k)));
    int rows = 0, pc = 0, cp = 0;  // cp: clean prefix (== rows in the clean state)
    bool clean = true;
    while (pc < m) {
        if (rows == k) {  // decoder.rs:97-99
            for (int q = pc + tid; q < m; q += 64 * NW) St[q] = RLNC_ERR_RECEIVED_ALL_PIECES;
            break;
        }
        if (!clean) {
            const int r0 = cp, R = rows;  // rows r0..R-1 dirty; this piece becomes row R
            if (R + 1 - r0 > B) {  // many dirty rows: the reference verbatim, wave 0
                if (wave == 0) {
                    for (int c = lane; c < M.S; c += 64)
                        M.b[R * M.S + c] = c < k ? H[pc * kH + c] : uint8_t(c == k + pc);
                    rsync<false>();
                    const int r2 = generic_rref<false>(M, tab, R + 1, k);
                    const int cp2 = extend_prefix(M, r0, r2);
                    if (lane == 0) {
                        St[pc] = r2 == R ? RLNC_ERR_PIECE_NOT_USEFUL : RLNC_OK;  // decoder.rs:112-117
                        flag[0] = r2;
                        flag[1] = cp2;
                    }
                }
            } else {
                const int nb = R + 1 - r0;  // dirty rows including the new one
                for (int c = tid; c < M.S; c += 64 * NW) M.b[R * M.S + c] = c < k ? H[pc * kH + c] : uint8_t(c == k + pc);
                for (int e = tid; e < B * D; e += 64 * NW) X[e] = 0;
                __syncthreads();
                // forward steps i < r0: the dirty rows reduced against the prefix (stripes of i, met by ds_xor)
                {
                    uint32_t acc[B];
#pragma unroll
                    for (int t = 0; t < B; ++t) acc[t] = 0;
                    for (int i0 = 4 * sid; i0 < r0; i0 += 4 * NS) {
                        uint32_t x[4];
#pragma unroll
                        for (int ii = 0; ii < 4; ++ii) x[ii] = i0 + ii < r0 ? M.w[(i0 + ii) * D + w] : 0u;
                        uint32_t q4[B];
#pragma unroll
                        for (int t = 0; t < B; ++t) {
                            const uint32_t v = M.w[min(r0 + t, R) * D + (i0 >> 2)];
                            q4[t] = t < nb ? v : 0u;
                        }
#pragma unroll
                        for (int t = 0; t < B; ++t)
#pragma unroll
                            for (int ii = 0; ii < 4; ++ii) acc[t] ^= mul4(tab, (q4[t] >> (8 * ii)) & 0xFFu, x[ii]);
                    }
#pragma unroll
                    for (int t = 0; t < B; ++t) {
                        if (t < nb) {
                            uint32_t a = acc[t];
                            a = group_xor_rt(a, D);
                            if (g == 0 && a) atomicXor(&X[t * D + w], a);
                        }
                    }
                }
                __syncthreads();
                for (int e = tid; e < nb * D; e += 64 * NW) M.w[r0 * D + e] ^= X[e];
                __syncthreads();
                // forward steps i >= r0, verbatim on the dirty rows
                if (wave == 0) forward_range(M, tab, r0, R + 1);
                __syncthreads();
                // backward steps i = R .. r0 (:171-215): column i out of every row above (stripes), then row i
                // normalised from column i+1
                for (int i = R; i >= r0; --i) {
                    const uint32_t piv = M.at(i, i);
                    if (piv == 0) continue;  // every wave reads the same byte (no write since the last barrier)
                    const uint32_t xi = M.w[i * D + w];
                    const uint32_t nr = mul4(tab, 256 + piv, xi);  // row i · piv^-1: (q·piv^-1)·x = q·(piv^-1·x)
                    const uint32_t mi = from_mask(w, i);
                    for (int j = sid; j < i; j += NS) {
                        const uint32_t q = M.at(j, i);
                        if (q) M.w[j * D + w] ^= mul4(tab, q, nr) & mi;
                    }
                    __syncthreads();
                    if (piv != 1) {
                        if (tid < D) {
                            const uint32_t mask = from_mask(w, i + 1);
                            uint32_t v = (xi & ~mask) | (nr & mask);
                            if (w == (i >> 2)) v = (v & ~(0xFFu << (8 * (i & 3)))) | (1u << (8 * (i & 3)));
                            M.w[i * D + w] = v;
                        }
                        __syncthreads();
                    }
                }
                if (wave == 0) {
                    const int r2 = remove_zero_range(M, r0, R + 1, k);
                    const int cp2 = extend_prefix(M, r0, r2);
                    if (lane == 0) {
                        St[pc] = r2 == R ? RLNC_ERR_PIECE_NOT_USEFUL : RLNC_OK;  // decoder.rs:112-117
                        flag[0] = r2;
                        flag[1] = cp2;
                    }
                }
            }
            __syncthreads();
            rows = flag[0];
            cp = flag[1];
            clean = cp == rows;
            ++pc;
            __syncthreads();
  // one piece outside the clean state
            continue;
        }
        const int r = rows;
        const int b = min(B, min(m - pc, k - r));
        // 1. X_t = init_t ^ Σ_{i<r} P_t[i]·R_i
        for (int e = tid; e < B * D; e += 64 * NW) {
            const int t = e / D, ww = e % D;
            uint32_t x = 0;
            if (t < b) {
#pragma unroll
                for (int bb = 0; bb < 4; ++bb) {
                    const int c = 4 * ww + bb;
                    x |= (c < k ? uint32_t(H[(pc + t) * kH + c]) : uint32_t(c == k + pc + t)) << (8 * bb);
                }
            }
            X[e] = x;
        }
        __syncthreads();
        if (r > 0) {
            uint32_t acc[B];
#pragma unroll
            for (int t = 0; t < B; ++t) acc[t] = 0;
            const uint32_t *H32 = reinterpret_cast<const uint32_t *>(H);
            for (int i0 = 4 * sid; i0 < r; i0 += 4 * NS) {
                uint32_t x[4];
#pragma unroll
                for (int ii = 0; ii < 4; ++ii) x[ii] = i0 + ii < r ? M.w[(i0 + ii) * D + w] : 0u;  // rows >= r: 0
                // the 4 coefficients P_t[i0..i0+3] of every piece of the block (0 past the block: zero products),
                // all read before any table read, and no branch on t: the reads of a chunk overlap
                uint32_t q4[B];
#pragma unroll
                for (int t = 0; t < B; ++t) {
                    const uint32_t v = H32[(min(pc + t, m - 1) * kH + i0) >> 2];
                    q4[t] = t < b ? v : 0u;
                }
                Sel1 sl[4];
#pragma unroll
                for (int ii = 0; ii < 4; ++ii) {
                    sl[ii].s0 = x[ii] & 0x07070707u;
                    sl[ii].s1 = (x[ii] >> 3) & 0x07070707u;
                    sl[ii].s2 = (x[ii] >> 6) & 0x03030303u;
                }
                // the tables of piece t (its 4 coefficients), double-buffered: piece t+1's 8 LDS reads are in
                // flight while piece t's products run
                uint4 ta[2][4];
                uint32_t tb[2][4];
#pragma unroll
                for (int ii = 0; ii < 4; ++ii) {
                    const uint32_t q = (q4[0] >> (8 * ii)) & 0xFFu;
                    ta[0][ii] = *reinterpret_cast<const uint4 *>(tab + q * kTabDw);
                    tb[0][ii] = tab[q * kTabDw + 4];
                }
#pragma unroll
                for (int t = 0; t < B; ++t) {
                    if (t + 1 < B) {
#pragma unroll
                        for (int ii = 0; ii < 4; ++ii) {
                            const uint32_t q = (q4[t + 1] >> (8 * ii)) & 0xFFu;
                            ta[(t + 1) & 1][ii] = *reinterpret_cast<const uint4 *>(tab + q * kTabDw);
                            tb[(t + 1) & 1][ii] = tab[q * kTabDw + 4];
                        }
                    }
#pragma unroll
                    for (int ii = 0; ii < 4; ++ii) {
                        const uint4 t4 = ta[t & 1][ii];
                        const uint32_t t2 = tb[t & 1][ii];
                        acc[t] = xor3(acc[t], __builtin_amdgcn_perm(t4.y, t4.x, sl[ii].s0),
                                      xor3(__builtin_amdgcn_perm(t4.w, t4.z, sl[ii].s1), __builtin_amdgcn_perm(t2, t2, sl[ii].s2), 0u));
                    }
                }
            }
#pragma unroll
            for (int t = 0; t < B; ++t) {
                if (t < b) {
                    uint32_t a = acc[t];
                    a = group_xor_rt(a, D);
                    if (g == 0 && a) atomicXor(&X[t * D + w], a);
                }
            }
            __syncthreads();
        }
  // step 1 (with the block's initial rows)
        // 2. the block's rows among themselves (every wave redundantly, registers, lane = dword; lane groups hold identical copies: wave 0 alone with the
        // rows passed through LDS measured equal, profiles/r02_elim_ab.txt).  No
        // branch inside a piece's forward or backward products: their table reads are issued together.
        uint32_t y[B];
        int c = b;
        {
#pragma unroll
        for (int t = 0; t < B; ++t) y[t] = t < b ? X[t * D + w] : 0u;
#pragma unroll
        for (int t = 0; t < B; ++t) {
            if (t < c) {
                // forward: quotients are the block-reduced row's bytes r+s (s < t), read before any update.  The
                // backward step's quotients y_s[r+t] (s < t) do not change during this piece's forward pass either,
                // so their table reads are issued here too: one dependent LDS round trip less per piece
                uint32_t acc = y[t];
                uint4 b4[B];
                uint32_t b2[B];
                {
                    uint4 f4[B];
                    uint32_t f2[B];
#pragma unroll
                    for (int s2 = 0; s2 < t; ++s2) {
                        const uint32_t q = byte_of(y[t], (r + s2) >> 2, (r + s2) & 3);
                        f4[s2] = *reinterpret_cast<const uint4 *>(tab + q * kTabDw);
                        f2[s2] = tab[q * kTabDw + 4];
                    }
#pragma unroll
                    for (int s2 = 0; s2 < t; ++s2) {
                        const uint32_t qb = byte_of(y[s2], (r + t) >> 2, (r + t) & 3);
                        b4[s2] = *reinterpret_cast<const uint4 *>(tab + qb * kTabDw);
                        b2[s2] = tab[qb * kTabDw + 4];
                    }
#pragma unroll
                    for (int s2 = 0; s2 < t; ++s2) acc ^= mul4t(f4[s2], f2[s2], y[s2]);
                }
                y[t] = acc;
                const uint32_t piv = byte_of(y[t], (r + t) >> 2, (r + t) & 3);
                if (piv == 0) {
                    c = t;
                } else {
                    const uint32_t mask = from_mask(w, r + t + 1);  // normalise from column r+t+1 (:200-211)
                    y[t] = (y[t] & ~mask) | (mul4(tab, 256 + piv, y[t]) & mask);
                    if (w == ((r + t) >> 2)) y[t] = (y[t] & ~(0xFFu << (8 * ((r + t) & 3)))) | (1u << (8 * ((r + t) & 3)));
                    // backward inside the block: y_s ^= y_s[r+t]·y_t (s < t), y_t's selectors shared
                    const uint32_t e0 = y[t] & 0x07070707u, e1 = (y[t] >> 3) & 0x07070707u, e2 = (y[t] >> 6) & 0x03030303u;
#pragma unroll
                    for (int s2 = 0; s2 < t; ++s2)
                        y[s2] = xor3(y[s2], __builtin_amdgcn_perm(b4[s2].y, b4[s2].x, e0),
                                     xor3(__builtin_amdgcn_perm(b4[s2].w, b4[s2].z, e1), __builtin_amdgcn_perm(b2[s2], b2[s2], e2), 0u));
                }
            }
        }
        }
        // 3. rows j < r: R_j ^= Σ_{t<c} R_j[r+t]·y_t; then y_t become rows r..r+c-1
        if (c > 0) {
            Sel1 ys[B];
#pragma unroll
            for (int t = 0; t < B; ++t) {
                ys[t].s0 = y[t] & 0x07070707u;
                ys[t].s1 = (y[t] >> 3) & 0x07070707u;
                ys[t].s2 = (y[t] >> 6) & 0x03030303u;
            }
            const int d0 = r >> 2, sh = r & 3;
            constexpr int NC = (B + 3) / 4 + 1;  // the dwords holding bytes r .. r+B-1 of a row
            // software-pipelined over this stripe's rows: row j+NS's words are read while row j's products run
            uint32_t cw[NC], xj = 0;
            int j = sid;
#pragma unroll
            for (int u = 0; u < NC; ++u) cw[u] = (j < r && d0 + u < D) ? M.w[j * D + d0 + u] : 0u;
            if (j < r) xj = M.w[j * D + w];
            for (; j < r; j += NS) {
                uint32_t qw[NC - 1];  // bytes r.. aligned to dword boundaries
#pragma unroll
                for (int u = 0; u < NC - 1; ++u) qw[u] = __builtin_amdgcn_alignbyte(cw[u + 1], cw[u], sh);
                uint4 t4[B];
                uint32_t t2[B];
#pragma unroll
                for (int t = 0; t < B; ++t) {  // no branch: pieces past c multiply by 0
                    const uint32_t qq = t < c ? (qw[t >> 2] >> (8 * (t & 3))) & 0xFFu : 0u;
                    t4[t] = *reinterpret_cast<const uint4 *>(tab + qq * kTabDw);
                    t2[t] = tab[qq * kTabDw + 4];
                }
                const int jn = j + NS;
                uint32_t cwn[NC], xjn = 0;
#pragma unroll
                for (int u = 0; u < NC; ++u) cwn[u] = (jn < r && d0 + u < D) ? M.w[jn * D + d0 + u] : 0u;
                if (jn < r) xjn = M.w[jn * D + w];
#pragma unroll
                for (int t = 0; t < B; ++t)
                    xj = xor3(xj, __builtin_amdgcn_perm(t4[t].y, t4[t].x, ys[t].s0),
                              xor3(__builtin_amdgcn_perm(t4[t].w, t4[t].z, ys[t].s1), __builtin_amdgcn_perm(t2[t], t2[t], ys[t].s2), 0u));
                M.w[j * D + w] = xj;
#pragma unroll
                for (int u = 0; u < NC; ++u) cw[u] = cwn[u];
                xj = xjn;
            }
            if (wave == 0 && g == 0) {
#pragma unroll
                for (int t = 0; t < B; ++t)
                    if (t < c) M.w[(r + t) * D + w] = y[t];
            }
            if (tid < c) St[pc + tid] = RLNC_OK;
        }
        rows = r + c;
        pc += c;
        if (c < b) {  // piece pc: zero pivot after its forward pass; its reduced row is y[c]
            uint32_t yc = 0;
#pragma unroll
            for (int t = 0; t < B; ++t)
                if (t == c) yc = y[t];
            const bool keep = __ballot(g == 0 && (yc & cm) != 0) != 0;  // remove_zero_rows (:222-244)
            if (keep && wave == 0 && g == 0) M.w[rows * D + w] = yc;
            if (tid == 0) St[pc] = keep ? RLNC_OK : RLNC_ERR_PIECE_NOT_USEFUL;
            if (keep) {
                cp = rows;
                ++rows;
                clean = false;
            }
            ++pc;
        }
        __syncthreads();
  // zero-pivot piece + the block's closing barrier
    }
    __syncthreads();
    // two-pass (m_stride > m): the pieces after the first m are ReceivedAllPieces when they full-ranked the object
    // (decoder.rs:97-99, no state change), else the general pass rewrites this object; their T columns are zero
    const int ms = p.m_stride > m ? p.m_stride : m;
    for (int q = tid; q < ms; q += 64 * NW)
        p.status[int64_t(o) * ms + q] = q < m ? St[q] : (rows == k ? RLNC_ERR_RECEIVED_ALL_PIECES : -1);
    if (tid == 0) p.rank[o] = rows;
    uint8_t *T = p.T + int64_t(o) * p.T_obj;
    for (int e = tid; e < k * ms; e += 64 * NW) {
        const int rr = e / ms, s2 = e % ms;
        T[e] = rr < rows && s2 < m ? M.b[rr * M.S + k + s2] : uint8_t(0);
    }
}

constexpr int kBlkNW = 4, kBlkB = 16, kBlkDefault = 8;

size_t rref_block_lds_bytes(int k, int m) {
    const int D = rref_row_dwords(k, m);
    return size_t(kTabEntries) * kTabDw * 4 + size_t(k + 1) * 4 * D + 4 * ((size_t(m) + 3) & ~size_t(3)) +
           ((size_t(m) * ((k + 3) & ~3) + 15) & ~size_t(15)) + size_t(kBlkB) * D * 4 + 16;
}

inline size_t rref_lds_bytes_staged(int k, int m) {  // + the staged headers, + 2 × 4 × 64 dwords of partial sums
    return rref_lds_bytes(k, m) + ((size_t(k) * m + 15) & ~size_t(15)) + 2 * 4 * 64 * 4;
}

}  // namespace
}  // namespace rlnc
