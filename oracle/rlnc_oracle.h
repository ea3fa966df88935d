/*
 * rlnc_oracle.h — CPU restatement of itzmeanjan/rlnc 0.8.5 (Rust) for the RLNC hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker / the timed CPU "port" baseline.  The product
 * (librlnc_hip.so, rlnc_amd/) never links, loads or calls it.
 *
 * Parity status: field arithmetic is pinned (the reference's literal LOG/EXP tables are committed as
 * tests/golden/gf256_tables.json and compared bit-for-bit; FIPS-197 AES-field KATs).  The reference
 * itself (Rust) cannot be compiled or run here (no cargo/rustc), so coding/decoding outputs are pinned
 * by the reference's own deterministic tests (swap_rows KAT, getter arithmetic, error-order tables) and
 * its property tests (round trips, rref idempotence, useless-recode rejection), plus an independent
 * numpy restatement (oracle/np_oracle.py) that must agree byte-for-byte.  RNG parity (rand 0.9.2
 * fill_bytes) is unpinned by design: coefficients are always explicit inputs.
 *
 * Status codes: 0 = Ok, otherwise (RLNCError discriminant + 1), errors.rs:3-32 order.
 */
#ifndef RLNC_ORACLE_H
#define RLNC_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- field: src/common/gf256.rs ---- */
void orc_gf256_tables(uint8_t log_tbl[256], uint8_t exp_tbl[510]);
uint8_t orc_gf256_mul(uint8_t a, uint8_t b);
int orc_gf256_inv(uint8_t a); /* -1 for a == 0 (Option::None) */
void orc_gf256_nibble_tables(uint8_t low[256][32], uint8_t high[256][32]); /* simd_mul_table.rs:36-80 */

/* ---- vector primitives: src/common/simd/mod.rs ---- */
void orc_mul_vec_by_scalar(uint8_t *vec, size_t len, uint8_t scalar);                         /* :18-47 */
void orc_add_vectors(uint8_t *dst, const uint8_t *src, size_t len);                            /* :58-76 */
void orc_mul_vec_by_scalar_then_add_into_vec(uint8_t *dst, const uint8_t *src, size_t len, uint8_t scalar); /* :89-119 */
const char *orc_simd_variant(void);  /* which CPU kernel the dispatcher picked */
void orc_force_scalar(int on);       /* force the scalar path (for A/B tests) */

/* ---- encoder: src/full/encoder.rs ---- */
size_t orc_piece_byte_len(size_t data_len, size_t piece_count);                       /* :95 */
int orc_encoder_pad(const uint8_t *data, size_t data_len, size_t piece_count, uint8_t *out); /* :85-106 */
int orc_code_with_coding_vector(const uint8_t *src, size_t piece_count, size_t piece_len,
                                const uint8_t *coding_vector, size_t cv_len,
                                uint8_t *coded, size_t coded_len);                      /* :128-144 */
/* n full coded pieces (coeffs ‖ data), coefficient rows given: encoder.rs:241-250 per row */
int orc_code_full_batch(const uint8_t *src, size_t piece_count, size_t piece_len,
                        const uint8_t *coeffs, size_t n, uint8_t *out);

/* ---- recoder: src/full/recoder.rs ---- */
int orc_recode_with_vector(const uint8_t *pieces, size_t data_len, size_t full_len, size_t k,
                           const uint8_t *r, size_t r_len, uint8_t *out, size_t out_len); /* :68-153 */

/* ---- decoder matrix: src/full/decoder_matrix.rs ---- */
/* In-place rref of a row-major rows×cols matrix with k coefficient columns (:99-244). Returns new rows. */
size_t orc_rref(uint8_t *m, size_t rows, size_t cols, size_t k);
void orc_swap_rows(uint8_t *m, size_t cols, size_t r1, size_t r2); /* :69-90 */

/* ---- decoder: src/full/decoder.rs ---- */
typedef struct orc_decoder orc_decoder;
orc_decoder *orc_decoder_new(size_t piece_byte_len, size_t required_piece_count, int *status); /* :65-80 */
void orc_decoder_free(orc_decoder *d);
int orc_decoder_decode(orc_decoder *d, const uint8_t *piece, size_t len);                      /* :96-118 */
int orc_decoder_is_already_decoded(const orc_decoder *d);                                       /* :121 */
size_t orc_decoder_received(const orc_decoder *d);
size_t orc_decoder_useful(const orc_decoder *d);
size_t orc_decoder_rows(const orc_decoder *d);
const uint8_t *orc_decoder_matrix(const orc_decoder *d);
/* get_decoded_data (:136-159): writes up to k*L bytes, *out_len = final length. */
int orc_decoder_get_decoded_data(const orc_decoder *d, uint8_t *out, size_t *out_len);
int orc_final_data_len(const uint8_t *padded, size_t len, size_t *out_len);                      /* :162-177 */

#ifdef __cplusplus
}
#endif
#endif
