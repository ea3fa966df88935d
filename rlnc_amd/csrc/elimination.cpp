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
// d[0..n) ^= q·s[0..n) (or d = q·d when s == nullptr) 32 bytes at a time: the product of a byte is
// lo[x & 15] ^ hi[x >> 4] (16-entry tables of q·v and q·(v << 4)), one vpshufb each.  The host runs this for every
// pivot step of every Decoder::decode call (k = 128: ≈ 90 K products per call).
__attribute__((target("avx2"))) void muladd_avx2(uint8_t *d, const uint8_t *s, size_t n, const uint8_t *mt) {
    alignas(16) uint8_t lo[16], hi[16];
    for (int v = 0; v < 16; ++v) {
        lo[v] = mt[v];
        hi[v] = mt[v << 4];
    }
    const __m256i tl = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i *>(lo)));
    const __m256i th = _mm256_broadcastsi128_si256(_mm_load_si128(reinterpret_cast<const __m128i *>(hi)));
    const __m256i m = _mm256_set1_epi8(0x0f);
    size_t c = 0;
    for (; c + 32 <= n; c += 32) {
        const __m256i x = _mm256_loadu_si256(reinterpret_cast<const __m256i *>((s ? s : d) + c));
        const __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(tl, _mm256_and_si256(x, m)),
                                           _mm256_shuffle_epi8(th, _mm256_and_si256(_mm256_srli_epi16(x, 4), m)));
        __m256i *dp = reinterpret_cast<__m256i *>(d + c);
        _mm256_storeu_si256(dp, s ? _mm256_xor_si256(_mm256_loadu_si256(dp), p) : p);
    }
    for (; c < n; ++c) d[c] = s ? uint8_t(d[c] ^ mt[s[c]]) : mt[d[c]];
}
const bool kHostAvx2 = __builtin_cpu_supports("avx2");
}  // namespace
#endif

// d[0..n) ^= q·s[0..n), or d = q·d when s == nullptr (mt = the product table of q)
static void gf_muladd(uint8_t *d, const uint8_t *s, size_t n, const uint8_t *mt) {
#if !defined(__HIP_DEVICE_COMPILE__)
    if (kHostAvx2 && n >= 32) return muladd_avx2(d, s, n, mt);
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
    if (q == 1) {
        for (size_t c = from; c < n; ++c) d[c] ^= s[c];
        return;
    }
    gf_muladd(d + from, s + from, n - from, host_field().mul[q]);
}

// clean_forward — decoder_matrix.rs:120-166
void Elimination::clean_forward() {
    const size_t cols = stride();
    const size_t boundary = std::min(rows_, cols);
    const HostField &f = host_field();
    for (size_t i = 0; i < boundary; ++i) {
        if (m_[i * cols + i] == 0) {
            size_t p = i + 1;
            while (p < rows_ && m_[p * cols + i] == 0) ++p;
            if (p == rows_) continue;
            std::swap_ranges(&m_[i * cols], &m_[i * cols] + cols, &m_[p * cols]);  // swap_rows :69-90
        }
        const uint8_t inv_pivot = f.inv[m_[i * cols + i]];
        for (size_t j = i + 1; j < rows_; ++j) {
            const uint8_t v = m_[j * cols + i];
            if (v == 0) continue;
            row_muladd(j, i, i, f.mul[v][inv_pivot]);  // quotient = M[j][i] / M[i][i], :148
        }
    }
}

// clean_backward — decoder_matrix.rs:171-215
void Elimination::clean_backward() {
    const size_t cols = stride();
    const size_t boundary = std::min(rows_, cols);
    const HostField &f = host_field();
    for (size_t ii = boundary; ii-- > 0;) {
        const size_t i = ii;
        const uint8_t piv = m_[i * cols + i];
        if (piv == 0) continue;
        const uint8_t inv_pivot = f.inv[piv];
        for (size_t j = 0; j < i; ++j) {
            const uint8_t v = m_[j * cols + i];
            if (v == 0) continue;
            row_muladd(j, i, i, f.mul[v][inv_pivot]);  // :184-197
        }
        if (piv == 1) continue;  // :200-202
        m_[i * cols + i] = 1;    // :205
        gf_muladd(&m_[i * cols + i + 1], nullptr, cols - i - 1, f.mul[inv_pivot]);  // :207-211
    }
}

// remove_zero_rows — decoder_matrix.rs:222-244 (zero test on the k coefficient columns only)
void Elimination::remove_zero_rows() {
    const size_t cols = stride();
    size_t i = 0;
    while (i < rows_) {
        const uint8_t *r = &m_[i * cols];
        bool nz = false;
        for (size_t c = 0; c < k_; ++c)
            if (r[c]) {
                nz = true;
                break;
            }
        if (nz) {
            ++i;
            continue;
        }
        if (i + 1 < rows_) std::memmove(&m_[i * cols], &m_[(i + 1) * cols], (rows_ - i - 1) * cols);
        --rows_;
    }
    // rows beyond rows_ must read as zero the next time they are appended to
    std::memset(&m_[rows_ * cols], 0, (k_ + 1 - rows_) * cols);
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
    for (size_t q = 0; q < rows_; ++q) {
        const uint8_t *e = &m_[q * stride() + k_];
        for (size_t c = 0; c < cap_; ++c) used_[c] |= e[c];
    }
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
