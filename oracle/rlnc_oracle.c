/*
 * rlnc_oracle.c — CPU restatement of itzmeanjan/rlnc 0.8.5 (see rlnc_oracle.h for the contract).
 *
 * TEST INFRASTRUCTURE: the parity checker for the HIP path and the timed CPU "port" baseline in
 * bench.py.  Never linked into the product.  Every function cites the reference file:line it follows
 * (paths relative to the reference crate root).
 *
 * Build: oracle/Makefile (plain gcc, -O3, runtime ISA dispatch like src/common/simd/x86/mod.rs:59-91 —
 * GFNI+AVX512 → AVX2 nibble pshufb → scalar; no -march=native so the .so built here runs on the GPU
 * box's host CPU too).
 */
#include "rlnc_oracle.h"

#include <immintrin.h>
#include <stdlib.h>
#include <string.h>

enum {
    ST_OK = 0,
    ST_CODING_VECTOR_LENGTH_MISMATCH = 1,
    ST_DATA_LENGTH_MISMATCH = 2,
    ST_PIECE_COUNT_ZERO = 3,
    ST_DATA_LENGTH_ZERO = 4,
    ST_PIECE_LENGTH_ZERO = 5,
    ST_NOT_ENOUGH_PIECES_TO_RECODE = 6,
    ST_PIECE_LENGTH_TOO_SHORT = 7,
    ST_PIECE_NOT_USEFUL = 8,
    ST_RECEIVED_ALL_PIECES = 9,
    ST_NOT_ALL_PIECES_RECEIVED_YET = 10,
    ST_INVALID_DECODED_DATA_FORMAT = 11,
    ST_INVALID_PIECE_LENGTH = 12,
    ST_INVALID_OUTPUT_BUFFER = 13,
};

#define BOUNDARY_MARKER 0x81 /* src/full/consts.rs:5 */

/* ------------------------------------------------------------------------------------------------
 * GF(2^8), AES polynomial x^8+x^4+x^3+x+1 (0x11B), generator 3 — src/common/gf256.rs:16-44,50-51,82-85.
 * The tables are regenerated from the polynomial; tests/test_oracle.py checks them against the
 * reference's literal tables (tests/golden/gf256_tables.json).
 * ---------------------------------------------------------------------------------------------- */
static uint8_t LOG[256];
static uint8_t EXP[510];
static uint8_t LOWT[256][32];  /* simd_mul_table.rs:36-52: LOW[c][i] = c*i, i<16, bytes 16..31 zero */
static uint8_t HIGHT[256][32]; /* simd_mul_table.rs:54-70: HIGH[c][i] = c*(i<<4) */
static int g_init = 0;

static uint8_t xtime_aes(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1B : 0x00)); }

static void init_tables(void) {
    if (g_init) return;
    uint8_t x = 1;
    for (int i = 0; i < 255; i++) {
        EXP[i] = x;
        EXP[i + 255] = x;
        LOG[x] = (uint8_t)i;
        x = (uint8_t)(xtime_aes(x) ^ x); /* multiply by generator 3 = x + 1 */
    }
    LOG[0] = 0; /* gf256.rs:17 — LOG[0] is 0 and is never used for a==0 (mul_const early-outs) */
    for (int c = 0; c < 256; c++) {
        for (int i = 0; i < 32; i++) {
            LOWT[c][i] = 0;
            HIGHT[c][i] = 0;
        }
        for (int i = 0; i < 16; i++) {
            LOWT[c][i] = orc_gf256_mul((uint8_t)c, (uint8_t)i);
            HIGHT[c][i] = orc_gf256_mul((uint8_t)c, (uint8_t)(i << 4));
        }
    }
    g_init = 1;
}

__attribute__((constructor)) static void orc_ctor(void) { init_tables(); }

void orc_gf256_tables(uint8_t log_tbl[256], uint8_t exp_tbl[510]) {
    memcpy(log_tbl, LOG, 256);
    memcpy(exp_tbl, EXP, 510);
}

/* Gf256::mul_const — gf256.rs:88-97 */
uint8_t orc_gf256_mul(uint8_t a, uint8_t b) {
    if (a == 0 || b == 0) return 0;
    return EXP[(size_t)LOG[a] + (size_t)LOG[b]];
}

/* Gf256::inv — gf256.rs:100-108 */
int orc_gf256_inv(uint8_t a) {
    if (a == 0) return -1;
    return EXP[255 - (size_t)LOG[a]];
}

/* Div — gf256.rs:159-167 (callers guarantee b != 0, as the reference's unwrap_unchecked does) */
static inline uint8_t gf_div(uint8_t a, uint8_t b) { return orc_gf256_mul(a, (uint8_t)orc_gf256_inv(b)); }

void orc_gf256_nibble_tables(uint8_t low[256][32], uint8_t high[256][32]) {
    memcpy(low, LOWT, sizeof(LOWT));
    memcpy(high, HIGHT, sizeof(HIGHT));
}

/* ------------------------------------------------------------------------------------------------
 * Vector kernels — src/common/simd/{x86/{gfni/m512i,avx2}.rs, mod.rs}.  Same dispatch order as
 * x86/mod.rs:59-91 (GFNI+AVX512F first, then AVX2 nibble pshufb), scalar mul_const tail/fallback.
 * ---------------------------------------------------------------------------------------------- */
enum { V_SCALAR = 0, V_AVX2 = 1, V_GFNI512 = 2 };
static int g_variant = -1;
static int g_force_scalar = 0;

static int variant(void) {
    if (g_force_scalar) return V_SCALAR;
    if (g_variant < 0) {
        __builtin_cpu_init();
        if (__builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw"))
            g_variant = V_GFNI512;
        else if (__builtin_cpu_supports("avx2"))
            g_variant = V_AVX2;
        else
            g_variant = V_SCALAR;
    }
    return g_variant;
}

const char *orc_simd_variant(void) {
    switch (variant()) {
    case V_GFNI512: return "gfni-avx512";
    case V_AVX2: return "avx2-pshufb";
    default: return "scalar";
    }
}
void orc_force_scalar(int on) { g_force_scalar = on; }

/* scalar fallback — simd/mod.rs:40-46, :113-118 */
static void scalar_mul(uint8_t *v, size_t n, uint8_t c) {
    for (size_t i = 0; i < n; i++) v[i] = orc_gf256_mul(v[i], c);
}
static void scalar_muladd(uint8_t *d, const uint8_t *s, size_t n, uint8_t c) {
    for (size_t i = 0; i < n; i++) d[i] ^= orc_gf256_mul(s[i], c);
}
static void scalar_add(uint8_t *d, const uint8_t *s, size_t n) {
    for (size_t i = 0; i < n; i++) d[i] ^= s[i];
}

/* AVX2 nibble-table kernel — x86/avx2.rs:64-100 */
__attribute__((target("avx2"))) static void avx2_muladd(uint8_t *d, const uint8_t *s, size_t n, uint8_t c) {
    const __m256i lt = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)LOWT[c]));
    const __m256i ht = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)HIGHT[c]));
    const __m256i m = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i *)(s + i));
        __m256i lo = _mm256_shuffle_epi8(lt, _mm256_and_si256(x, m));
        __m256i hi = _mm256_shuffle_epi8(ht, _mm256_and_si256(_mm256_srli_epi64(x, 4), m));
        __m256i acc = _mm256_loadu_si256((const __m256i *)(d + i));
        _mm256_storeu_si256((__m256i *)(d + i), _mm256_xor_si256(acc, _mm256_xor_si256(lo, hi)));
    }
    scalar_muladd(d + i, s + i, n - i, c);
}
__attribute__((target("avx2"))) static void avx2_mul(uint8_t *v, size_t n, uint8_t c) {
    const __m256i lt = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)LOWT[c]));
    const __m256i ht = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)HIGHT[c]));
    const __m256i m = _mm256_set1_epi8(0x0f);
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i *)(v + i));
        __m256i lo = _mm256_shuffle_epi8(lt, _mm256_and_si256(x, m));
        __m256i hi = _mm256_shuffle_epi8(ht, _mm256_and_si256(_mm256_srli_epi64(x, 4), m));
        _mm256_storeu_si256((__m256i *)(v + i), _mm256_xor_si256(lo, hi));
    }
    scalar_mul(v + i, n - i, c);
}
__attribute__((target("avx2"))) static void avx2_add(uint8_t *d, const uint8_t *s, size_t n) {
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        __m256i a = _mm256_loadu_si256((const __m256i *)(d + i));
        __m256i b = _mm256_loadu_si256((const __m256i *)(s + i));
        _mm256_storeu_si256((__m256i *)(d + i), _mm256_xor_si256(a, b));
    }
    scalar_add(d + i, s + i, n - i);
}

/* GFNI zmm kernel — x86/gfni/m512i.rs:10-54 (gf2p8mulb uses the same AES polynomial 0x11B) */
__attribute__((target("avx512f,avx512bw,gfni"))) static void gfni_muladd(uint8_t *d, const uint8_t *s, size_t n, uint8_t c) {
    const __m512i cv = _mm512_set1_epi8((char)c);
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        __m512i x = _mm512_loadu_si512((const void *)(s + i));
        __m512i acc = _mm512_loadu_si512((const void *)(d + i));
        _mm512_storeu_si512((void *)(d + i), _mm512_xor_si512(acc, _mm512_gf2p8mul_epi8(x, cv)));
    }
    scalar_muladd(d + i, s + i, n - i, c);
}
__attribute__((target("avx512f,avx512bw,gfni"))) static void gfni_mul(uint8_t *v, size_t n, uint8_t c) {
    const __m512i cv = _mm512_set1_epi8((char)c);
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        __m512i x = _mm512_loadu_si512((const void *)(v + i));
        _mm512_storeu_si512((void *)(v + i), _mm512_gf2p8mul_epi8(x, cv));
    }
    scalar_mul(v + i, n - i, c);
}
__attribute__((target("avx512f,avx512bw"))) static void avx512_add(uint8_t *d, const uint8_t *s, size_t n) {
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        __m512i a = _mm512_loadu_si512((const void *)(d + i));
        __m512i b = _mm512_loadu_si512((const void *)(s + i));
        _mm512_storeu_si512((void *)(d + i), _mm512_xor_si512(a, b));
    }
    scalar_add(d + i, s + i, n - i);
}

/* gf256_inplace_mul_vec_by_scalar — simd/mod.rs:18-47 */
void orc_mul_vec_by_scalar(uint8_t *vec, size_t len, uint8_t scalar) {
    if (len == 0) return;
    if (scalar == 0) {
        memset(vec, 0, len);
        return;
    }
    if (scalar == 1) return;
    switch (variant()) {
    case V_GFNI512: gfni_mul(vec, len, scalar); return;
    case V_AVX2: avx2_mul(vec, len, scalar); return;
    default: scalar_mul(vec, len, scalar); return;
    }
}

/* gf256_inplace_add_vectors — simd/mod.rs:58-76 */
void orc_add_vectors(uint8_t *dst, const uint8_t *src, size_t len) {
    switch (variant()) {
    case V_GFNI512: avx512_add(dst, src, len); return;
    case V_AVX2: avx2_add(dst, src, len); return;
    default: scalar_add(dst, src, len); return;
    }
}

/* gf256_mul_vec_by_scalar_then_add_into_vec — simd/mod.rs:89-119 */
void orc_mul_vec_by_scalar_then_add_into_vec(uint8_t *dst, const uint8_t *src, size_t len, uint8_t scalar) {
    if (len == 0) return;
    if (scalar == 0) return;
    if (scalar == 1) {
        orc_add_vectors(dst, src, len);
        return;
    }
    switch (variant()) {
    case V_GFNI512: gfni_muladd(dst, src, len, scalar); return;
    case V_AVX2: avx2_muladd(dst, src, len, scalar); return;
    default: scalar_muladd(dst, src, len, scalar); return;
    }
}

/* ------------------------------------------------------------------------------------------------
 * Encoder — src/full/encoder.rs
 * ---------------------------------------------------------------------------------------------- */
/* encoder.rs:93-95: L = ceil((len + 1) / k) */
size_t orc_piece_byte_len(size_t data_len, size_t piece_count) {
    if (piece_count == 0) return 0;
    return (data_len + 1 + piece_count - 1) / piece_count;
}

/* Encoder::new — encoder.rs:85-106.  out must hold k*L bytes. */
int orc_encoder_pad(const uint8_t *data, size_t data_len, size_t piece_count, uint8_t *out) {
    if (data_len == 0) return ST_DATA_LENGTH_ZERO; /* :86-88 */
    if (piece_count == 0) return ST_PIECE_COUNT_ZERO; /* :89-91 */
    size_t L = orc_piece_byte_len(data_len, piece_count);
    size_t padded = piece_count * L;
    memcpy(out, data, data_len);
    memset(out + data_len, 0, padded - data_len); /* :98 resize(padded, 0) */
    out[data_len] = BOUNDARY_MARKER;                 /* :99 */
    return ST_OK;
}

/* Encoder::code_with_coding_vector (serial) — encoder.rs:128-144 */
int orc_code_with_coding_vector(const uint8_t *src, size_t piece_count, size_t piece_len,
                                const uint8_t *coding_vector, size_t cv_len,
                                uint8_t *coded, size_t coded_len) {
    if (cv_len != piece_count) return ST_CODING_VECTOR_LENGTH_MISMATCH; /* :129-131 */
    if (coded_len != piece_len) return ST_INVALID_OUTPUT_BUFFER;       /* :132-134 */
    memset(coded, 0, coded_len);                                        /* :136 */
    for (size_t i = 0; i < piece_count; i++)                           /* :138-141 */
        orc_mul_vec_by_scalar_then_add_into_vec(coded, src + i * piece_len, piece_len, coding_vector[i]);
    return ST_OK;
}

/* n × Encoder::code_with_buf with the coding vectors supplied (encoder.rs:241-250 minus rng.fill_bytes) */
int orc_code_full_batch(const uint8_t *src, size_t piece_count, size_t piece_len,
                        const uint8_t *coeffs, size_t n, uint8_t *out) {
    size_t full = piece_count + piece_len;
    for (size_t r = 0; r < n; r++) {
        uint8_t *piece = out + r * full;
        memcpy(piece, coeffs + r * piece_count, piece_count); /* :246-248 split_at_mut + fill */
        int st = orc_code_with_coding_vector(src, piece_count, piece_len, piece, piece_count, piece + piece_count, piece_len);
        if (st) return st;
    }
    return ST_OK;
}

/* ------------------------------------------------------------------------------------------------
 * Recoder — src/full/recoder.rs:68-153, recoding vector explicit (rng.fill_bytes at :131 removed).
 * ---------------------------------------------------------------------------------------------- */
int orc_recode_with_vector(const uint8_t *pieces, size_t data_len, size_t full_len, size_t k,
                           const uint8_t *r, size_t r_len, uint8_t *out, size_t out_len) {
    if (data_len == 0) return ST_NOT_ENOUGH_PIECES_TO_RECODE; /* :69-71 */
    if (full_len == 0) return ST_PIECE_LENGTH_ZERO;            /* :72-74 */
    if (k == 0) return ST_PIECE_COUNT_ZERO;                    /* :75-77 */
    if (full_len <= k) return ST_PIECE_LENGTH_TOO_SHORT;       /* :78-80 */
    size_t L = full_len - k;                                   /* :82 */
    size_t n = data_len / full_len;                            /* :83 (trailing partial piece ignored, :88) */
    if (n == 0) return ST_NOT_ENOUGH_PIECES_TO_RECODE;         /* reference: UB via unwrap_unchecked (:97) */
    if (out_len != full_len) return ST_INVALID_OUTPUT_BUFFER;  /* :123-125 */
    if (r_len != n) return ST_CODING_VECTOR_LENGTH_MISMATCH;   /* encoder.rs:129-131 via :148 */
    /* :133-144 coefficient composition, fold in index order */
    for (size_t c = 0; c < k; c++) {
        uint8_t acc = 0;
        for (size_t i = 0; i < n; i++) acc ^= orc_gf256_mul(r[i], pieces[i * full_len + c]);
        out[c] = acc;
    }
    /* :146-150 data = Encoder::code_with_coding_vector(r, D) */
    uint8_t *dst = out + k;
    memset(dst, 0, L);
    for (size_t i = 0; i < n; i++) orc_mul_vec_by_scalar_then_add_into_vec(dst, pieces + i * full_len + k, L, r[i]);
    return ST_OK;
}

/* ------------------------------------------------------------------------------------------------
 * DecoderMatrix — src/full/decoder_matrix.rs (row-major bytes, rows × cols, k coefficient columns)
 * ---------------------------------------------------------------------------------------------- */
#define M(m, cols, r, c) ((m)[(size_t)(r) * (cols) + (c)])

/* swap_rows — decoder_matrix.rs:69-90 */
void orc_swap_rows(uint8_t *m, size_t cols, size_t r1, size_t r2) {
    if (r1 == r2) return;
    uint8_t *a = m + r1 * cols, *b = m + r2 * cols;
    for (size_t c = 0; c < cols; c++) {
        uint8_t t = a[c];
        a[c] = b[c];
        b[c] = t;
    }
}

/* clean_forward — decoder_matrix.rs:120-166 (diagonal pivots only) */
static void clean_forward(uint8_t *m, size_t rows, size_t cols) {
    size_t boundary = rows < cols ? rows : cols; /* :121 */
    for (size_t i = 0; i < boundary; i++) {
        if (M(m, cols, i, i) == 0) { /* :124-141 */
            size_t p = i + 1;
            int found = 0;
            while (p < rows) {
                if (M(m, cols, p, i) != 0) {
                    found = 1;
                    break;
                }
                p++;
            }
            if (!found) continue;
            orc_swap_rows(m, cols, i, p);
        }
        for (size_t j = i + 1; j < rows; j++) { /* :143-162 */
            if (M(m, cols, j, i) == 0) continue;
            uint8_t q = gf_div(M(m, cols, j, i), M(m, cols, i, i));
            orc_mul_vec_by_scalar_then_add_into_vec(m + j * cols + i, m + i * cols + i, cols - i, q);
        }
    }
}

/* clean_backward — decoder_matrix.rs:171-215 */
static void clean_backward(uint8_t *m, size_t rows, size_t cols) {
    size_t boundary = rows < cols ? rows : cols; /* :172 */
    for (size_t ii = boundary; ii-- > 0;) {
        size_t i = ii;
        if (M(m, cols, i, i) == 0) continue; /* :175-177 */
        for (size_t j = 0; j < i; j++) {     /* :179-198 */
            if (M(m, cols, j, i) == 0) continue;
            uint8_t q = gf_div(M(m, cols, j, i), M(m, cols, i, i));
            orc_mul_vec_by_scalar_then_add_into_vec(m + j * cols + i, m + i * cols + i, cols - i, q);
        }
        if (M(m, cols, i, i) == 1) continue; /* :200-202 */
        uint8_t inv = (uint8_t)orc_gf256_inv(M(m, cols, i, i));
        M(m, cols, i, i) = 1;                                       /* :205 */
        orc_mul_vec_by_scalar(m + i * cols + i + 1, cols - i - 1, inv); /* :207-211 */
    }
}

/* remove_zero_rows — decoder_matrix.rs:222-244 (zero test on the first k columns only) */
static size_t remove_zero_rows(uint8_t *m, size_t rows, size_t cols, size_t k) {
    size_t i = 0;
    while (i < rows) {
        int nz = 0;
        for (size_t c = 0; c < k; c++)
            if (M(m, cols, i, c) != 0) {
                nz = 1;
                break;
            }
        if (nz) {
            i++;
            continue;
        }
        if (i + 1 < rows) memmove(m + i * cols, m + (i + 1) * cols, (rows - i - 1) * cols);
        rows--;
    }
    return rows;
}

/* rref — decoder_matrix.rs:99-101 */
size_t orc_rref(uint8_t *m, size_t rows, size_t cols, size_t k) {
    clean_forward(m, rows, cols);
    clean_backward(m, rows, cols);
    return remove_zero_rows(m, rows, cols, k);
}

/* ------------------------------------------------------------------------------------------------
 * Decoder — src/full/decoder.rs
 * ---------------------------------------------------------------------------------------------- */
struct orc_decoder {
    size_t L, k, cols;
    size_t rows;
    size_t received, useful;
    uint8_t *m; /* capacity k rows (decode refuses a piece once rows == k, :97-99) */
};

orc_decoder *orc_decoder_new(size_t piece_byte_len, size_t required_piece_count, int *status) {
    if (piece_byte_len == 0) { /* decoder.rs:66-68 */
        if (status) *status = ST_PIECE_LENGTH_ZERO;
        return NULL;
    }
    if (required_piece_count == 0) { /* :69-71 */
        if (status) *status = ST_PIECE_COUNT_ZERO;
        return NULL;
    }
    orc_decoder *d = (orc_decoder *)calloc(1, sizeof(orc_decoder));
    d->L = piece_byte_len;
    d->k = required_piece_count;
    d->cols = d->k + d->L;
    d->m = (uint8_t *)malloc(d->k * d->cols);
    if (!d->m) {
        free(d);
        if (status) *status = -1;
        return NULL;
    }
    if (status) *status = ST_OK;
    return d;
}

void orc_decoder_free(orc_decoder *d) {
    if (!d) return;
    free(d->m);
    free(d);
}

int orc_decoder_is_already_decoded(const orc_decoder *d) { return d->rows == d->k; } /* :121-123 */
size_t orc_decoder_received(const orc_decoder *d) { return d->received; }
size_t orc_decoder_useful(const orc_decoder *d) { return d->useful; }
size_t orc_decoder_rows(const orc_decoder *d) { return d->rows; }
const uint8_t *orc_decoder_matrix(const orc_decoder *d) { return d->m; }

/* Decoder::decode — decoder.rs:96-118 */
int orc_decoder_decode(orc_decoder *d, const uint8_t *piece, size_t len) {
    if (orc_decoder_is_already_decoded(d)) return ST_RECEIVED_ALL_PIECES; /* :97-99 */
    if (len != d->cols) return ST_INVALID_PIECE_LENGTH;                   /* :100-102 */
    size_t before = d->rows;                                               /* :104 */
    memcpy(d->m + d->rows * d->cols, piece, d->cols);                      /* add_row, decoder_matrix.rs:53-62 */
    d->rows = orc_rref(d->m, d->rows + 1, d->cols, d->k);                   /* :106 */
    d->received++;                                                         /* :107 */
    if (d->rows == before) return ST_PIECE_NOT_USEFUL;                     /* :112-113 */
    d->useful = d->rows;                                                   /* :115 */
    return ST_OK;
}

/* get_final_data_len — decoder.rs:162-177 */
int orc_final_data_len(const uint8_t *padded, size_t len, size_t *out_len) {
    size_t last_index = len ? len - 1 : 0; /* saturating_sub(1) */
    size_t rev = last_index;               /* unwrap_or(last_index) */
    for (size_t r = 0; r < len; r++)
        if (padded[len - 1 - r] == BOUNDARY_MARKER) {
            rev = r;
            break;
        }
    size_t idx = last_index - rev;
    if (idx == 0) return ST_INVALID_DECODED_DATA_FORMAT; /* :168-170 */
    for (size_t i = idx + 1; i < len; i++)
        if (padded[i] != 0) return ST_INVALID_DECODED_DATA_FORMAT; /* :171-173 */
    *out_len = idx;
    return ST_OK;
}

/* get_decoded_data — decoder.rs:136-159 (payload rows concatenated in matrix row order) */
int orc_decoder_get_decoded_data(const orc_decoder *d, uint8_t *out, size_t *out_len) {
    if (!orc_decoder_is_already_decoded(d)) return ST_NOT_ALL_PIECES_RECEIVED_YET; /* :137-139 */
    for (size_t r = 0; r < d->rows; r++) memcpy(out + r * d->L, d->m + r * d->cols + d->k, d->L);
    return orc_final_data_len(out, d->L * d->k, out_len);
}
