// rref.hip — the decoder's coefficient-side elimination on the device, one wave per object.
//
// Replays Decoder::decode (src/full/decoder.rs:96-118) for pieces 0..m-1 of every object, exactly like
// the host engine (elimination.hpp): the diagonal-pivot RREF of DecoderMatrix
// (src/full/decoder_matrix.rs:99-244) is run on [coeffs | E] where E (m columns) tracks every row as a
// combination of the received pieces.  Outputs per object: the status of every decode() call, the rank,
// and T = E (k × m, rows >= rank zero) so that decoded rows = T × received data rows (one matmul).
//
// Two paths, both exact:
//   * generic — the reference algorithm verbatim (pivot test, swap with the first nonzero row below,
//     eliminate every row below/above with q = M[j][i] / M[i][i] from column i on, normalise from column
//     i+1, drop rows whose k coefficient bytes are zero), with the independent row operations of one step
//     done in parallel across the wave;
//   * clean  — used while rows 0..r-1 are a clean RREF (M[i][i] = 1 and every pivot column zero in the
//     other rows).  Then the reference's forward pass only touches the new row r and all its quotients are
//     the ORIGINAL coefficients M[r][i] (row i is zero in every other pivot column), so the whole forward
//     pass is one vector-matrix product; its backward pass only eliminates column r from the rows above
//     and normalises row r.  Same products, same XORs, same bytes — computed with all lanes at once.
//     Leaving the clean state (a zero diagonal after the forward pass: SURVEY.md §0.5) switches to the
//     generic path, which re-checks cleanliness after every piece.
// GF products use v_perm_b32 with the 3-bit split tables of all 256 multipliers staged in LDS (copied from a
// compile-time table), and all m piece headers are staged in LDS up front when they fit: the per-piece loop
// then never waits on HBM.
#include <hip/hip_runtime.h>

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

// The 256 × kTabDw table, built at compile time (make_perm_table's layout plus c^-1 = c^254).
struct RrefTable {
    uint32_t v[256 * kTabDw];
};
constexpr RrefTable build_rref_table() {
    RrefTable t{};
    for (int c = 0; c < 256; ++c) {
        uint8_t m[8] = {};
        m[0] = uint8_t(c);
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
        uint8_t inv = 1, sq = uint8_t(c);  // c^254 (0 for c = 0)
        for (int e = 254; e; e >>= 1) {
            if (e & 1) inv = gf_mul_slow(inv, sq);
            sq = gf_mul_slow(sq, sq);
        }
        uint32_t *e = t.v + c * kTabDw;
        e[0] = t0lo;
        e[1] = t0hi;
        e[2] = t1lo;
        e[3] = t1hi;
        e[4] = t2;
        e[5] = c ? inv : 0u;
    }
    return t;
}
__device__ const RrefTable kRrefTable = build_rref_table();
// spot checks against the field (gf256.rs:16-44): identity tables of c = 1, 2^-1 = 0x8D, 3^-1 = 0xF6
static_assert(build_rref_table().v[1 * kTabDw + 0] == 0x03020100u && build_rref_table().v[1 * kTabDw + 1] == 0x07060504u,
              "c = 1 low table");
static_assert(build_rref_table().v[2 * kTabDw + 5] == 0x8Du && build_rref_table().v[3 * kTabDw + 5] == 0xF6u,
              "inverses");

__device__ __forceinline__ uint32_t mul4(const uint32_t *tab, uint32_t q, uint32_t x) {
    const uint4 t = *reinterpret_cast<const uint4 *>(tab + q * kTabDw);
    const uint32_t t2 = tab[q * kTabDw + 4];
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

// row_t[c >= c0] ^= q · row_s[c >= c0]   (simd/mod.rs:89-119 on the byte range of decoder_matrix.rs:158-161)
__device__ __forceinline__ void row_muladd(const Mat &M, const uint32_t *tab, int t, int s, uint32_t q, int c0) {
    for (int w = threadIdx.x; w < M.D; w += 64) {
        const uint32_t mask = from_mask(w, c0);
        if (mask) M.w[t * M.D + w] ^= mul4(tab, q, M.w[s * M.D + w]) & mask;
    }
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// DecoderMatrix::rref — decoder_matrix.rs:99-244, verbatim.  Returns the new row count.
__device__ int generic_rref(const Mat &M, const uint32_t *tab, int R, int k) {
    const int lane = threadIdx.x;
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
            __syncthreads();
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
                row_muladd(M, tab, jj, i, q, i);
            }
        }
        __syncthreads();
    }
    // clean_backward :171-215
    for (int i = R - 1; i >= 0; --i) {
        const uint32_t piv = M.at(i, i);
        if (piv == 0) continue;
        const uint32_t inv = gfinv(tab, piv);
        for (int g = 0; g < i; g += 64) {
            const int j = g + lane;
            uint64_t b = ballot(j < i && M.at(j, i) != 0);
            while (b) {
                const int jj = g + __ffsll((unsigned long long)b) - 1;
                b &= b - 1;
                const uint32_t q = gfmul(tab, M.at(jj, i), inv);  // :184
                row_muladd(M, tab, jj, i, q, i);
            }
        }
        __syncthreads();
        if (piv != 1) {  // :200-211
            for (int w = lane; w < M.D; w += 64) {
                const uint32_t mask = from_mask(w, i + 1);
                if (mask) {
                    const uint32_t x = M.w[i * M.D + w];
                    M.w[i * M.D + w] = (x & ~mask) | (mul4(tab, inv, x) & mask);
                }
            }
            __syncthreads();
            if (lane == 0) M.b[i * M.S + i] = 1;
            __syncthreads();
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
                __syncthreads();
            }
            ++dst;
        }
    }
    __syncthreads();
    return dst;
}

// rows 0..R-1 a clean RREF: M[i][i] = 1 and column i zero in every other row (i < R)
__device__ bool is_clean(const Mat &M, int R) {
    const int lane = threadIdx.x;
    bool ok = true;
    for (int g = 0; g < R; g += 64) {
        const int j = g + lane;
        if (j < R)
            for (int i = 0; i < R && ok; ++i) ok = M.at(j, i) == (i == j ? 1u : 0u);
    }
    return ballot(!ok) == 0;
}

// Clean-state append of row r (see file header).  Returns the new row count; *stays_clean.
#ifdef RLNC_RREF_PROFILE
#define PROF_MARK(i)                                      \
    do {                                                  \
        const uint64_t _t = __builtin_amdgcn_s_memtime(); \
        prof[i] += _t - prof_t;                           \
        prof_t = _t;                                      \
    } while (0)
#define PROF_ARGS , uint64_t *prof, uint64_t &prof_t
#define PROF_PASS , prof, prof_t
#else
#define PROF_MARK(i) \
    do {             \
    } while (0)
#define PROF_ARGS
#define PROF_PASS
#endif

__device__ int clean_append(const Mat &M, const uint32_t *tab, int r, int k, bool *stays_clean PROF_ARGS) {
    const int lane = threadIdx.x;
    const int D = M.D;
    const int G = D >= 64 ? 1 : 64 / D;  // lane groups splitting the pivot rows
    const int w = D >= 64 ? lane : lane % D;
    const int g = D >= 64 ? 0 : lane / D;
    // the original coefficients of row r, kept in the spare row k while row r is rewritten
    for (int ww = lane; ww < D; ww += 64) M.w[k * D + ww] = M.w[r * D + ww];
    __syncthreads();
    PROF_MARK(1);
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
            for (int sh = D; sh < 64; sh <<= 1) acc ^= __shfl_xor(acc, sh);
        }
        if (g == 0 && ww < D) M.w[r * D + ww] ^= acc;
        __syncthreads();
    }
    PROF_MARK(2);
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
    PROF_MARK(3);
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
    PROF_MARK(4);
    *stays_clean = true;
    return r + 1;
}

// staged headers: m × k bytes after the matrix (hdr_lds = 1), else read from global memory per piece
__global__ __launch_bounds__(64) void gf_rref_batch_kernel(RrefParams p, int hdr_lds) {
    extern __shared__ uint32_t lds[];
    uint32_t *tab = lds;  // 256 × kTabDw dwords
    const int lane = threadIdx.x;
    const int o = blockIdx.x;
    const int k = p.k, m = p.m;
#ifdef RLNC_RREF_PROFILE  // diagnostic build: statuses become per-piece cycle counts, rank the setup cycles
    const uint64_t t_start = __builtin_amdgcn_s_memtime();
#endif
    Mat M;
    M.D = rref_row_dwords(k, m);
    M.S = 4 * M.D;
    M.w = lds + 256 * kTabDw;
    M.b = reinterpret_cast<uint8_t *>(M.w);
    // per-piece statuses stay in LDS until the end: a global store before each __syncthreads would make
    // its release fence wait for the store to reach memory, once per piece
    int32_t *St = reinterpret_cast<int32_t *>(M.b + size_t(k + 1) * M.S);
    uint8_t *H = reinterpret_cast<uint8_t *>(St + ((m + 3) & ~3));

    {
        const uint4 *src = reinterpret_cast<const uint4 *>(kRrefTable.v);
        uint4 *dst = reinterpret_cast<uint4 *>(tab);
        for (int q = lane; q < 256 * kTabDw / 4; q += 64) dst[q] = src[q];
    }
    const uint8_t *base = p.pieces + int64_t(o) * p.obj_stride;
    if (hdr_lds)
        for (int e = lane; e < m * k; e += 64) H[e] = base[int64_t(e / k) * p.piece_stride + e % k];
    for (int w = lane; w < (k + 1) * M.D; w += 64) M.w[w] = 0;
    __syncthreads();

    int rows = 0;
    bool clean = true;
#ifdef RLNC_RREF_PROFILE
    const uint64_t t_setup = __builtin_amdgcn_s_memtime();
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t prof_t = t_setup;
#endif
    for (int pc = 0; pc < m; ++pc) {
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
        PROF_MARK(0);
        if (clean) {
            bool sc;
            rows = clean_append(M, tab, rows, k, &sc PROF_PASS);
            clean = sc;
        } else {
            rows = generic_rref(M, tab, rows + 1, k);
            PROF_MARK(5);
            clean = is_clean(M, rows);
            PROF_MARK(6);
        }
        if (lane == 0) St[pc] = rows == before ? RLNC_ERR_PIECE_NOT_USEFUL : RLNC_OK;  // decoder.rs:112-117
        __syncthreads();
        PROF_MARK(7);
    }
    __syncthreads();
#ifdef RLNC_RREF_PROFILE  // phases: 0 row init, 1 spare copy, 2 forward, 3 normalise, 4 backward, 5 generic, 6 is_clean, 7 status
    if (lane == 0)
        for (int i = 0; i < 8 && i < m; ++i) St[i] = int32_t(prof[i]);
    __syncthreads();
#endif
    for (int pc = lane; pc < m; pc += 64) p.status[int64_t(o) * m + pc] = St[pc];
#ifdef RLNC_RREF_PROFILE
    if (lane == 0) p.rank[o] = int32_t(t_setup - t_start);
#else
    if (lane == 0) p.rank[o] = rows;
#endif
    uint8_t *T = p.T + int64_t(o) * p.T_obj;
    for (int e = lane; e < k * m; e += 64) {
        const int r = e / m, s = e % m;
        T[e] = r < rows ? M.b[r * M.S + k + s] : uint8_t(0);
    }
}

}  // namespace

size_t rref_lds_bytes(int k, int m) {
    return 256 * kTabDw * 4 + size_t(k + 1) * 4 * size_t(rref_row_dwords(k, m)) + 4 * ((size_t(m) + 3) & ~size_t(3));
}
static size_t rref_lds_bytes_staged(int k, int m) { return rref_lds_bytes(k, m) + ((size_t(k) * m + 15) & ~size_t(15)); }

hipError_t launch_rref_batch(const RrefParams &p, hipStream_t s) {
    if (p.n_obj <= 0) return hipSuccess;
    size_t lds = rref_lds_bytes(p.k, p.m);
    if (lds > kRrefMaxLds) return hipErrorInvalidValue;
    const int hdr_lds = rref_lds_bytes_staged(p.k, p.m) <= kRrefMaxLds ? 1 : 0;
    if (hdr_lds) lds = rref_lds_bytes_staged(p.k, p.m);
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&gf_rref_batch_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, int(kRrefMaxLds));
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    hipLaunchKernelGGL(gf_rref_batch_kernel, dim3(p.n_obj), dim3(64), lds, s, p, hdr_lds);
    return hipGetLastError();
}

}  // namespace rlnc
