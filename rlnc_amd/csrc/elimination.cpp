// elimination.cpp — exact replica of DecoderMatrix::rref on [coeffs | E] (see elimination.hpp).
#include "elimination.hpp"

#include <algorithm>
#include <cstring>

#include "../../include/rlnc_hip.h"
#include "gf256.hpp"

#if !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>
#endif

namespace rlnc {

#if !defined(__HIP_DEVICE_COMPILE__)
namespace {
// 4-bit split product tables of every multiplier: lo[q][v] = q·v, hi[q][v] = q·(v << 4) (simd_mul_table.rs:36-80)
struct NibbleTables {
    alignas(16) uint8_t lo[256][16];
    alignas(16) uint8_t hi[256][16];
    NibbleTables() {
        for (int q = 0; q < 256; ++q)
            for (int v = 0; v < 16; ++v) {
                lo[q][v] = gf_mul_slow(uint8_t(q), uint8_t(v));
                hi[q][v] = gf_mul_slow(uint8_t(q), uint8_t(v << 4));
            }
    }
};
const NibbleTables kNib;

// d[0..n) ^= q·s[0..n) (or d = q·d when s == nullptr) 32 bytes at a time: the product of a byte is
// lo[x & 15] ^ hi[x >> 4], one vpshufb each.  The host runs this for every pivot step of every Decoder::decode call
// (k = 128: ≈ 90 K products per call), so the tables are precomputed, not rebuilt per row.
__attribute__((target("avx2"))) void muladd_avx2(uint8_t *d, const uint8_t *s, size_t n, uint8_t q, const uint8_t *mt) {
    const __m256i tl = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i *>(kNib.lo[q])));
    const __m256i th = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i *>(kNib.hi[q])));
    const __m256i m = _mm256_set1_epi8(0x0f);
    size_t c = 0;
    for (; c + 32 <= n; c += 32) {
        const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i *>((s ? s : d) + c));
        const __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(tl, _mm256_and_si256(x, m)),
                                           _mm256_shuffle_epi8(th, _mm256_and_si256(_mm256_srli_epi16(x, 4), m)));
        __m256i *dp = reinterpret_cast<__m256i *>(d + c);
        _mm256_storeu_si256(dp, s ? _mm256_xor_si256(_mm256_loadu_si256(dp), p) : p);
    }
    if (c + 16 <= n) {
        const __m128i m16 = _mm_set1_epi8(0x0f);
        const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i *>((s ? s : d) + c));
        const __m128i p = _mm_xor_si128(_mm_shuffle_epi8(_mm256_castsi256_si128(tl), _mm_and_si128(x, m16)),
                                        _mm_shuffle_epi8(_mm256_castsi256_si128(th), _mm_and_si128(_mm_srli_epi16(x, 4), m16)));
        __m128i *dp = reinterpret_cast<__m128i *>(d + c);
        _mm_storeu_si128(dp, s ? _mm_xor_si128(_mm_loadu_si128(dp), p) : p);
        c += 16;
    }
    for (; c < n; ++c) d[c] = s ? uint8_t(d[c] ^ mt[s[c]]) : mt[d[c]];
}
const bool kHostAvx2 = __builtin_cpu_supports("avx2");
}  // namespace
#endif

// u[0..n) |= rows[r][0..n) for r < nrows (row pitch `pitch`), vectorised: u never aliases the rows
static void or_rows(uint8_t *__restrict u, const uint8_t *__restrict rows, size_t pitch, size_t nrows, size_t n) {
    for (size_t r = 0; r < nrows; ++r) {
        const uint8_t *__restrict e = rows + r * pitch;
        for (size_t c = 0; c < n; ++c) u[c] |= e[c];
    }
}

static bool all_zero(const uint8_t *p, size_t n) {
    uint64_t acc = 0;
    size_t c = 0;
    for (; c + 8 <= n; c += 8) {
        uint64_t v;
        std::memcpy(&v, p + c, 8);
        acc |= v;
    }
    for (; c < n; ++c) acc |= p[c];
    return acc == 0;
}

// d[0..n) ^= s[0..n) (distinct rows)
static void xor_row(uint8_t *__restrict d, const uint8_t *__restrict s, size_t n) {
    for (size_t c = 0; c < n; ++c) d[c] ^= s[c];
}

// d[0..n) ^= q·s[0..n), or d = q·d when s == nullptr (mt = the product table of q)
static void gf_muladd(uint8_t *d, const uint8_t *s, size_t n, uint8_t q) {
    const uint8_t *mt = host_field().mul[q];
#if !defined(__HIP_DEVICE_COMPILE__)
    if (kHostAvx2 && n >= 16) return muladd_avx2(d, s, n, q, mt);
#endif
    for (size_t c = 0; c < n; ++c) d[c] = s ? uint8_t(d[c] ^ mt[s[c]]) : mt[d[c]];
}

const HostField &host_field() {
    static const HostField f;
    return f;
}

Elimination::Elimination(size_t k, size_t fixed_slots) : k_(k), fixed_(fixed_slots > 0) {
    cap_ = fixed_ ? fixed_slots : std::max<size_t>(k, 1) + 1;
    m_.assign((k_ + 1) * stride(), 0);
    live_.assign(cap_, 0);
}

void Elimination::grow(size_t new_cap) {
    std::vector<uint8_t> n((k_ + 1) * (k_ + new_cap), 0);
    for (size_t r = 0; r < rows_; ++r) std::memcpy(&n[r * (k_ + new_cap)], &m_[r * stride()], stride());
    m_.swap(n);
    cap_ = new_cap;
    live_.resize(new_cap, 0);
}

// row_j[from..] ^= q · row_i[from..]  (gf256_mul_vec_by_scalar_then_add_into_vec, simd/mod.rs:89-119)
void Elimination::row_muladd(size_t dst, size_t src, size_t from, uint8_t q) {
    if (q == 0) return;
    uint8_t *d = &m_[dst * stride()];
    const uint8_t *s = &m_[src * stride()];
    const size_t n = stride();
    if (q == 1) return xor_row(d + from, s + from, n - from);
    gf_muladd(d + from, s + from, n - from, q);
}

// clean_forward — decoder_matrix.rs:120-166.  The reference scans every column i for a pivot row and for rows
// below it to eliminate.  Between pushes the matrix is the output of the previous rref, whose rows are all zero below
// the diagonal (this pass zeroes column i below row i and later steps only touch columns > i; the backward pass and
// the removal of zero rows keep it), so of the rows below i only the last one -- the piece just appended, or the row
// a swap moved there -- can hold a nonzero in column i.  The scans therefore find exactly what the reference's would
// by looking at the last row alone: the same swaps and row operations in the same order, O(rows) instead of O(rows^2)
// strided reads.
void Elimination::clean_forward() {
    const size_t cols = stride();
    if (rows_ < 2) return;
    const size_t last = rows_ - 1;
    const HostField &f = host_field();
    uint8_t *rl = &m_[last * cols];
    for (size_t i = 0; i < last; ++i) {
        const uint8_t v = rl[i];
        if (v == 0) continue;  // no pivot to find below row i, nothing to eliminate
        uint8_t *ri = &m_[i * cols];
        if (ri[i] == 0) {
            // swap_rows :69-90 (the last row is the first below i with a nonzero in column i); the row that lands
            // last has a zero there (its old diagonal), so column i needs no elimination
            std::swap_ranges(ri, ri + cols, rl);
            continue;
        }
        row_muladd(last, i, i, f.mul[v][f.inv[ri[i]]]);  // quotient = M[j][i] / M[i][i], :148
    }
}

#if !defined(__HIP_DEVICE_COMPILE__)
namespace {
// bit c of the result: r[c] != 0 && piv[c] != 0, for the 64 columns [c0, c0 + 64)
__attribute__((target("avx2"))) uint64_t pivot_nonzero_mask(const uint8_t *r, const uint8_t *piv) {
    const __m256i z = _mm256_setzero_si256();
    const __m256i a = _mm256_and_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i *>(r)),
                                       _mm256_loadu_si256(reinterpret_cast<const __m256i *>(piv)));
    const __m256i b = _mm256_and_si256(_mm256_loadu_si256(reinterpret_cast<const __m256i *>(r + 32)),
                                       _mm256_loadu_si256(reinterpret_cast<const __m256i *>(piv + 32)));
    const uint32_t za = uint32_t(_mm256_movemask_epi8(_mm256_cmpeq_epi8(a, z)));
    const uint32_t zb = uint32_t(_mm256_movemask_epi8(_mm256_cmpeq_epi8(b, z)));
    return ~(uint64_t(za) | (uint64_t(zb) << 32));
}
}  // namespace
#endif

// clean_backward — decoder_matrix.rs:171-215, row by row.  The reference walks the pivots i from the bottom up and,
// at each, clears column i in every row above with row i (reduced by the pivots below it, not yet normalised), then
// normalises row i.  Row j's own sequence of operations is therefore: for each pivot i > j, from the highest down,
// if M[j][i] != 0 (its value at that point) subtract (M[j][i] / M[i][i]) · row i from column i on; then normalise.
// Running the rows from the bottom up and giving each row that sequence, with every row i it uses already finished
// (normalised: M[j][i] · (row i / M[i][i]) equals (M[j][i] / M[i][i]) · row i byte for byte), performs the same
// operations with the same results, and the column test becomes a scan along row j (64 columns per step) instead of
// a strided walk down column i.  The pivots do not move in this pass (an operation from pivot i touches columns
// >= i > j only), and a pivot row i has zeros in the pivot columns above i once finished, so a scan's nonzero bits
// below the column just processed stay valid.
void Elimination::clean_backward() {
    const size_t cols = stride();
    const size_t n = rows_;  // boundary = min(rows, cols) = rows (rows <= k + 1 <= cols)
    const HostField &f = host_field();
    piv_.assign(((n + 63) & ~size_t(63)) + 64, 0);
    for (size_t i = 0; i < n; ++i) piv_[i] = m_[i * cols + i] ? 0xFF : 0;
    row_pad_.resize(piv_.size());
    for (size_t jj = n; jj-- > 0;) {
        const size_t j = jj;
        uint8_t *rj = &m_[j * cols];
        // pivot columns c in (j, n) with rj[c] != 0, from the highest down
#if !defined(__HIP_DEVICE_COMPILE__)
        if (kHostAvx2) {
            // the row's columns [0, n) copied to a padded buffer so 64-byte loads stay in bounds
            std::memcpy(row_pad_.data(), rj, n);
            for (size_t b = (n - 1) / 64 + 1; b-- > (j + 1) / 64;) {
                const size_t c0 = b * 64;
                uint64_t mask = pivot_nonzero_mask(row_pad_.data() + c0, piv_.data() + c0);
                if (c0 + 64 > n) mask &= (n - c0 >= 64) ? ~0ull : ((1ull << (n - c0)) - 1);
                if (c0 <= j) mask &= ~((2ull << (j - c0)) - 1);  // columns > j only
                while (mask) {
                    const size_t c = c0 + 63 - size_t(__builtin_clzll(mask));
                    mask &= ~(1ull << (c - c0));
                    row_muladd(j, c, c, rj[c]);  // pivot row c is finished: M[c][c] = 1
                }
            }
        } else
#endif
        {
            for (size_t c = n; c-- > j + 1;)
                if (piv_[c] && rj[c]) row_muladd(j, c, c, rj[c]);
        }
        const uint8_t p = rj[j];
        if (p == 0 || p == 1) continue;  // :200-202
        rj[j] = 1;                       // :205
        gf_muladd(rj + j + 1, nullptr, cols - j - 1, f.inv[p]);  // :207-211
    }
}

// remove_zero_rows — decoder_matrix.rs:222-244 (zero test on the k coefficient columns only)
void Elimination::remove_zero_rows() {
    const size_t cols = stride();
    const size_t before = rows_;
    size_t i = 0;
    while (i < rows_) {
        const uint8_t *r = &m_[i * cols];
        // after the backward pass a row's first nonzero is its pivot, at its diagonal: test that byte first
        bool nz = i < k_ && r[i] != 0;
        if (!nz) nz = !all_zero(r, k_);
        if (nz) {
            ++i;
            continue;
        }
        if (i + 1 < rows_) std::memmove(&m_[i * cols], &m_[(i + 1) * cols], (rows_ - i - 1) * cols);
        --rows_;
    }
    // rows beyond rows_ read as zero (the rows removed here; the ones past them already are)
    if (rows_ < before) std::memset(&m_[rows_ * cols], 0, (before - rows_) * cols);
}

void Elimination::rref() {
    clean_forward();
    clean_backward();
    remove_zero_rows();
}

int Elimination::push(const uint8_t *coeffs, int *slot, bool *keep) {
    if (rows_ == k_) return RLNC_ERR_RECEIVED_ALL_PIECES;  // decoder.rs:97-99
    size_t s;
    if (fixed_) {
        if (pushed_ >= cap_) grow(std::max<size_t>(cap_ * 2, 1));
        s = pushed_;
    } else {
        s = cap_;
        for (size_t c = 0; c < cap_; ++c)
            if (!live_[c]) {
                s = c;
                break;
            }
        if (s == cap_) grow(cap_ * 2);
    }
    ++pushed_;
    live_[s] = 1;
    const size_t before = rows_;
    uint8_t *r = &m_[rows_ * stride()];  // add_row, decoder_matrix.rs:53-62
    std::memcpy(r, coeffs, k_);
    std::memset(r + k_, 0, cap_);
    r[k_ + s] = 1;
    ++rows_;
    rref();  // decoder.rs:106
    // a slot stays live while some row still references its piece (the rows' E parts OR-ed, row by row)
    used_.assign(cap_, 0);
    or_rows(used_.data(), &m_[k_], stride(), rows_, cap_);
    for (size_t c = 0; c < cap_; ++c) {
        if (!live_[c]) continue;
        const bool used = used_[c] != 0;
        if (!used && !fixed_) live_[c] = 0;
        if (c == s) *keep = used;
    }
    *slot = int(s);
    return rows_ == before ? RLNC_ERR_PIECE_NOT_USEFUL : RLNC_OK;  // decoder.rs:112-117
}

void Elimination::transform(uint8_t *T, size_t ld) const {
    for (size_t r = 0; r < rows_; ++r) {
        std::memcpy(T + r * ld, &m_[r * stride() + k_], cap_);
        if (ld > cap_) std::memset(T + r * ld + cap_, 0, ld - cap_);
    }
}

}  // namespace rlnc
