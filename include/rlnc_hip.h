/*
 * rlnc_hip.h — C ABI of librlnc_hip.so, the MI355X (gfx950) engine for the RLNC hot path of
 * itzmeanjan/rlnc 0.8.5.
 *
 * Drop-in boundary.  The reference exposes exactly three types plus one error enum
 * (rlnc::full::{Encoder, Decoder, Recoder}, rlnc::RLNCError — src/lib.rs:127-130, src/full/mod.rs:9-11);
 * its internal seam is the three src/common/simd functions (simd/mod.rs:18,58,89).  Every entry point
 * below names the reference item it replaces.  The Rust-side binding a maintainer would add is in
 * INTEGRATION.md.
 *
 * Conventions
 *   - Plain C: pointers + sizes, no exceptions across the ABI, no torch types.
 *   - Return value: RLNC_OK (0) or a status code.  Codes 1..13 are RLNCError discriminant + 1
 *     (src/common/errors.rs:3-32, same order); >= 100 are engine/device errors (rlnc_last_error() has
 *     the message, thread-local).
 *   - Randomness stays with the caller (the reference draws coefficients with rng.fill_bytes,
 *     encoder.rs:248 / recoder.rs:131): functions that the reference feeds from an RNG take those
 *     bytes explicitly, so outputs are bit-exact given the same coefficient bytes.
 *   - "_device" / batch functions take device pointers (hipMalloc'd memory on the context's device) and
 *     are asynchronous on the context's stream; the object API (encoder/decoder/recoder on host buffers)
 *     is synchronous, like the Rust API it mirrors.
 *   - Threading.  The object API (Encoder/Decoder/Recoder on host buffers) is safe to call from many host
 *     threads on one context: every call leases its own stream and buffers from the context's pool, so
 *     rlnc_encoder_code_with_buf on ONE encoder from many threads at once is safe, like the reference's
 *     code(&self) on a Send + Sync Encoder (encoder.rs:264).  A decoder or recoder must not be used by two
 *     threads at the same time (the reference's &mut self).  The stream-ordered batch / _device calls use the
 *     context's own workspaces: one caller thread per context at a time (one context per stream).
 *   - Lifetime.  Objects hold a reference on the context that created them: rlnc_context_destroy drops the
 *     creator's reference and the context is freed when its last object is freed, so an object may outlive
 *     the thread (and thread-local context) that created it.  Freeing an object waits only for its own
 *     stream-ordered uses (its _batch_device / _device launches, on whichever streams the context had then),
 *     not for other work queued on the context's stream; its device memory is reused only after them.
 *   - HIP graphs.  Once a batch call on a context has been captured into a HIP graph, the graph holds that
 *     context's workspace addresses: they are frozen, and a later call that would need a larger workspace
 *     fails with RLNC_ERR_INVALID_ARGUMENT instead of moving them (run the largest shape eagerly before
 *     capturing, or use another context for other shapes).
 */
#ifndef RLNC_HIP_H
#define RLNC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes: errors.rs:3-32 (discriminant + 1) ------------------------------------------- */
#define RLNC_OK 0
#define RLNC_ERR_CODING_VECTOR_LENGTH_MISMATCH 1 /* errors.rs:6  */
#define RLNC_ERR_DATA_LENGTH_MISMATCH 2          /* errors.rs:8  */
#define RLNC_ERR_PIECE_COUNT_ZERO 3              /* errors.rs:10 */
#define RLNC_ERR_DATA_LENGTH_ZERO 4              /* errors.rs:12 */
#define RLNC_ERR_PIECE_LENGTH_ZERO 5             /* errors.rs:14 */
#define RLNC_ERR_NOT_ENOUGH_PIECES_TO_RECODE 6   /* errors.rs:17 */
#define RLNC_ERR_PIECE_LENGTH_TOO_SHORT 7        /* errors.rs:19 */
#define RLNC_ERR_PIECE_NOT_USEFUL 8              /* errors.rs:22 */
#define RLNC_ERR_RECEIVED_ALL_PIECES 9           /* errors.rs:24 */
#define RLNC_ERR_NOT_ALL_PIECES_RECEIVED_YET 10  /* errors.rs:26 */
#define RLNC_ERR_INVALID_DECODED_DATA_FORMAT 11  /* errors.rs:28 */
#define RLNC_ERR_INVALID_PIECE_LENGTH 12         /* errors.rs:30 */
#define RLNC_ERR_INVALID_OUTPUT_BUFFER 13        /* errors.rs:31 */
/* engine errors (no reference counterpart) */
#define RLNC_ERR_INVALID_ARGUMENT 100 /* null handle/pointer, size overflow, misuse of the ABI */
#define RLNC_ERR_DEVICE 101           /* HIP runtime / launch failure */
#define RLNC_ERR_OUT_OF_MEMORY 102    /* device or pinned-host allocation failed */
#define RLNC_ERR_NO_DEVICE 103        /* no usable gfx950 device */

const char *rlnc_status_name(int status); /* "Ok", "PieceNotUseful", ... (errors.rs:34-58 variant names) */
const char *rlnc_status_message(int status); /* Display text, errors.rs:34-58 */
const char *rlnc_last_error(void);        /* detail of the last engine error on this thread */
const char *rlnc_version(void);

/* ---- context: device + HIP stream + workspace ----------------------------------------------------- */
typedef struct rlnc_context rlnc_context;
int rlnc_context_create(int device, rlnc_context **out);
void rlnc_context_destroy(rlnc_context *ctx);
/* Launch on an external hipStream_t, taken literally: NULL is HIP's null (default) stream, which is what
 * torch.cuda.current_stream().cuda_stream returns for torch's default stream.  The caller keeps ownership. */
int rlnc_context_set_stream(rlnc_context *ctx, void *hip_stream);
/* Go back to the context's own non-blocking stream (the initial state). */
int rlnc_context_use_own_stream(rlnc_context *ctx);
void *rlnc_context_get_stream(rlnc_context *ctx);
int rlnc_context_synchronize(rlnc_context *ctx);
int rlnc_context_device(const rlnc_context *ctx);
/* *capturing = 1 when `hip_stream` (NULL: the null stream) is inside a HIP stream capture, else 0, asked of the HIP
 * runtime this library is linked against (the one a host framework such as torch shares).  On any runtime error it
 * returns RLNC_ERR_DEVICE and sets *capturing = 1 (a caller deciding whether it may synchronise assumes the worst). */
int rlnc_stream_is_capturing(void *hip_stream, int *capturing);
/* 1 when 16-byte vector loads/stores (and LDS-DMA) at any byte address return the right bytes on `device` (the
 * queue's unaligned memory mode, checked by a probe kernel when the first context on the device is created):
 * piece rows at any alignment (odd L from Encoder::new, data at byte k of a (k + L)-byte coded piece) then take the
 * vector kernels directly; 0: misaligned rows are copied through 16-byte-aligned scratch around them (same results).
 * -1 before a context exists on the device.  RLNC_ASSUME_ALIGNED_ONLY=1 in the environment forces 0 and skips the
 * probe.  The probe's misaligned accesses return wrong bytes in the "dword" alignment mode (detected: 0) but fault
 * the process under a strict alignment mode: on a queue configured that way (not the ROCm default for compute
 * queues) set RLNC_ASSUME_ALIGNED_ONLY=1 before the first rlnc_context_create. */
int rlnc_device_unaligned_vector_access(int device);

/* ---- L1: vector primitives on device buffers (src/common/simd/mod.rs) --------------------------------
 * Same scalar early-outs as the reference (0 → zero-fill / no-op, 1 → no-op / plain XOR). */
int rlnc_gf256_inplace_mul_vec_by_scalar(rlnc_context *ctx, uint8_t *vec_dev, size_t len, uint8_t scalar); /* :18-47 */
int rlnc_gf256_inplace_add_vectors(rlnc_context *ctx, uint8_t *dst_dev, const uint8_t *src_dev, size_t len); /* :58-76 */
int rlnc_gf256_mul_vec_by_scalar_then_add_into_vec(rlnc_context *ctx, uint8_t *dst_dev, const uint8_t *src_dev,
                                                   size_t len, uint8_t scalar); /* :89-119 */

/* ---- L2: the matrix-level hot operator (device buffers) -----------------------------------------------
 * out[o][i][0:width) = XOR_j coef[o][i][j] · in[o][j][0:width)   (i < n_out, j < n_in, o < n_obj)
 * Replaces the loop of gf256_mul_vec_by_scalar_then_add_into_vec calls in
 * Encoder::code_with_coding_vector (encoder.rs:138-141), batched over n_out coding vectors and n_obj
 * independent objects.  All strides in bytes.  hdr (optional, may be NULL) also receives the coefficient
 * rows, hdr[o][i][0:n_in) — the coeffs‖data framing of a full coded piece (encoder.rs:246-248). */
typedef struct rlnc_matmul_desc {
    const uint8_t *in;
    int64_t in_obj_stride, in_row_stride;
    const uint8_t *coef;
    int64_t coef_obj_stride, coef_row_stride;
    uint8_t *out;
    int64_t out_obj_stride, out_row_stride;
    uint8_t *hdr;
    int64_t hdr_obj_stride, hdr_row_stride;
    int32_t n_out, n_in;
    int64_t width;
    int32_t n_obj;
} rlnc_matmul_desc;
int rlnc_gf256_matmul(rlnc_context *ctx, const rlnc_matmul_desc *desc);
/* Kernel variant of the GF(2^8) matmul (all bit-identical; the switch exists for A/B measurement):
 *   0 = perm       3-bit split tables in LDS consumed by v_perm_b32
 *   1 = nibble     the reference's 4-bit LOW/HIGH tables looked up from LDS byte-wise (ablation)
 *   6 = bitsliced-jump  bit-plane transpose; each (row, source) is one call into a code block specialised for the
 *                  coefficient (16 v_bitop3_b32 XOR3s of plane combinations); full 4 KiB column blocks of 16-byte
 *                  aligned operands with >= 4 output rows, the rest goes to perm
 *   7 = bitsliced-jump-shared  as 6; in 32-row tiles each of the 4 waves builds one quarter of every source
 *                  row's plane combinations and the quarters are exchanged through LDS
 *   8 = bitsliced-jump-shared-8w  as 7; above 32 output rows, 64-row tiles of 8 waves (one workgroup per CU):
 *                  waves 0-3 stage the source and build the combinations three rows ahead, waves 4-7 only
 *                  read them and call; a barrier every third row -- the default
 * Other values fail with RLNC_ERR_INVALID_ARGUMENT, except in the diagnostic A/B build (make -C rlnc_amd/csrc ab:
 * librlnc_hip_ab.so), which keeps the measured history: 2 perm3, 3/4 wide2/wide4, 5 bitsliced with
 * register-indexed XORs, 9 column runs.
 * max_tile_rows caps the output rows per launch/workgroup (0 = automatic, else 1/2/4/8/16/32). */
int rlnc_set_kernel_variant(rlnc_context *ctx, int variant, int max_tile_rows);
/* Column blocks per workgroup of variant 9 (A/B build only; 0 = automatic, else 1..64).  Bit-identical for every
 * value. */
int rlnc_set_column_run(rlnc_context *ctx, int col_run);
/* Where rlnc_decode_batch runs the coefficient elimination: 0 = auto (device when it fits LDS, default),
 * 1 = host threads, 2 = device, 5 = device, blocked clean run (k + m <= 256, else RLNC_ERR_INVALID_ARGUMENT; what 0
 * and 2 use when it applies).  The A/B build adds 3 (clean state on LDS), 4 (one wave's registers) and 6 (the
 * round-1 multi-wave register path).  All are exact replicas; the switch exists for A/B tests. */
int rlnc_set_decode_path(rlnc_context *ctx, int path);

/* ---- Encoder: src/full/encoder.rs ----------------------------------------------------------------- */
typedef struct rlnc_encoder rlnc_encoder;
/* Encoder::new (encoder.rs:85-106): pads with the 0x81 marker + zeros; data is host memory (copied). */
int rlnc_encoder_new(rlnc_context *ctx, const uint8_t *data, size_t data_len, size_t piece_count, rlnc_encoder **out);
/* Encoder::without_padding (encoder.rs:50-71). */
int rlnc_encoder_without_padding(rlnc_context *ctx, const uint8_t *data, size_t data_len, size_t piece_count,
                                 rlnc_encoder **out);
/* Device-resident source: piece_count rows of piece_len bytes at row_stride (borrowed, not copied; must
 * outlive the encoder). */
int rlnc_encoder_from_device(rlnc_context *ctx, const uint8_t *pieces_dev, size_t piece_count, size_t piece_len,
                             size_t row_stride, rlnc_encoder **out);
/* #[derive(Clone)] (encoder.rs:18): an independent copy (an owned source is copied on the device; a borrowed
 * device source stays borrowed). */
int rlnc_encoder_clone(const rlnc_encoder *enc, rlnc_encoder **out);
void rlnc_encoder_free(rlnc_encoder *enc);
size_t rlnc_encoder_get_piece_count(const rlnc_encoder *enc);              /* encoder.rs:27-29 */
size_t rlnc_encoder_get_piece_byte_len(const rlnc_encoder *enc);           /* encoder.rs:32-34 */
size_t rlnc_encoder_get_full_coded_piece_byte_len(const rlnc_encoder *enc); /* encoder.rs:37-39 */
/* Encoder::code_with_coding_vector (encoder.rs:128-144), host buffers. */
int rlnc_encoder_code_with_coding_vector(rlnc_encoder *enc, const uint8_t *coding_vector, size_t cv_len,
                                         uint8_t *coded_data, size_t coded_len);
/* Encoder::code_with_buf (encoder.rs:241-250): random_bytes are the piece_count bytes rng.fill_bytes
 * would have written into the coefficient prefix (n_random must equal piece_count, else
 * CodingVectorLengthMismatch); the output length is checked first, like the reference. */
int rlnc_encoder_code_with_buf(rlnc_encoder *enc, const uint8_t *random_bytes, size_t n_random,
                               uint8_t *full_coded_piece, size_t full_len);
/* n coded pieces in one launch, device buffers: coeffs_dev [n][k] → out_dev [n][k+L] (coeffs‖data,
 * row stride out_row_stride >= k+L; pass 0 for k+L). */
int rlnc_encoder_code_batch_device(rlnc_encoder *enc, const uint8_t *coeffs_dev, size_t n, uint8_t *out_dev,
                                   size_t out_row_stride);

/* ---- Recoder: src/full/recoder.rs ---------------------------------------------------------------- */
typedef struct rlnc_recoder rlnc_recoder;
/* Recoder::new (recoder.rs:68-108); data = concatenated full coded pieces (host, copied). */
int rlnc_recoder_new(rlnc_context *ctx, const uint8_t *data, size_t data_len, size_t full_coded_piece_byte_len,
                     size_t num_pieces_coded_together, rlnc_recoder **out);
int rlnc_recoder_clone(const rlnc_recoder *rec, rlnc_recoder **out); /* #[derive(Clone)], recoder.rs:12 */
void rlnc_recoder_free(rlnc_recoder *rec);
size_t rlnc_recoder_get_original_num_pieces_coded_together(const rlnc_recoder *rec); /* recoder.rs:26-28 */
size_t rlnc_recoder_get_num_pieces_recoded_together(const rlnc_recoder *rec);       /* recoder.rs:31-33 */
size_t rlnc_recoder_get_piece_byte_len(const rlnc_recoder *rec);                    /* recoder.rs:36-38 */
size_t rlnc_recoder_get_full_coded_piece_byte_len(const rlnc_recoder *rec);         /* recoder.rs:41-43 */
/* Recoder::recode_with_buf (recoder.rs:122-153): random_bytes = the n recoding coefficients that
 * rng.fill_bytes would have drawn (n_random must equal n, else CodingVectorLengthMismatch). */
int rlnc_recoder_recode_with_buf(rlnc_recoder *rec, const uint8_t *random_bytes, size_t n_random,
                                 uint8_t *full_recoded_piece, size_t full_len);
/* count recoded pieces in one launch: r_dev [count][n] → out_dev [count][k+L] (device). */
int rlnc_recoder_recode_batch_device(rlnc_recoder *rec, const uint8_t *r_dev, size_t count, uint8_t *out_dev);

/* ---- Decoder: src/full/decoder.rs ----------------------------------------------------------------- */
typedef struct rlnc_decoder rlnc_decoder;
/* Decoder::new(piece_byte_len, required_piece_count) (decoder.rs:65-80; note the argument order). */
int rlnc_decoder_new(rlnc_context *ctx, size_t piece_byte_len, size_t required_piece_count, rlnc_decoder **out);
/* #[derive(Clone)] (decoder.rs:8): elimination state, counters and the received data rows are copied. */
int rlnc_decoder_clone(const rlnc_decoder *dec, rlnc_decoder **out);
void rlnc_decoder_free(rlnc_decoder *dec);
/* Decoder::decode (decoder.rs:96-118): Ok / PieceNotUseful / ReceivedAllPieces / InvalidPieceLength.
 * The accept/reject answer is immediate (exact replica of the diagonal-pivot RREF on the coefficient
 * block); the data rows are combined on the device when the data is requested.  The piece's data bytes are
 * staged in pinned memory before the call returns (the caller may reuse its buffer at once); staged pieces are
 * copied to the device in batches on the context's upload stream, at the latest when the decoder's rows are next
 * used (get_decoded_data, clone, drop), which is ordered after them. */
int rlnc_decoder_decode(rlnc_decoder *dec, const uint8_t *full_coded_piece, size_t len);
/* Same, piece already in HBM (only its k coefficient bytes are read back to the host). */
int rlnc_decoder_decode_device(rlnc_decoder *dec, const uint8_t *piece_dev, size_t len);
int rlnc_decoder_is_already_decoded(const rlnc_decoder *dec);                   /* decoder.rs:121-123 */
size_t rlnc_decoder_get_num_pieces_coded_together(const rlnc_decoder *dec);     /* decoder.rs:25-27 */
size_t rlnc_decoder_get_piece_byte_len(const rlnc_decoder *dec);                /* decoder.rs:30-32 */
size_t rlnc_decoder_get_full_coded_piece_byte_len(const rlnc_decoder *dec);     /* decoder.rs:35-37 */
size_t rlnc_decoder_get_received_piece_count(const rlnc_decoder *dec);          /* decoder.rs:40-42 */
size_t rlnc_decoder_get_useful_piece_count(const rlnc_decoder *dec);            /* decoder.rs:45-47 */
size_t rlnc_decoder_get_remaining_piece_count(const rlnc_decoder *dec);         /* decoder.rs:50-52 */
/* Decoder::get_decoded_data (decoder.rs:136-177) into host memory: out must hold k*L bytes (the padded
 * size); *out_len receives the unpadded length.  Does not consume the decoder (the C caller frees it). */
int rlnc_decoder_get_decoded_data(rlnc_decoder *dec, uint8_t *out, size_t out_cap, size_t *out_len);
/* Same into device memory (out_dev holds k*L bytes). */
int rlnc_decoder_get_decoded_data_device(rlnc_decoder *dec, uint8_t *out_dev, size_t out_cap, size_t *out_len);

/* ---- multi-object batch API (device-resident) -------------------------------
 * Layouts (bytes, contiguous): src [obj][k][L]; coeffs [obj][n][k]; pieces [obj][n][k+L] (coeffs‖data). */
/* n coded pieces for each of num_objects objects (encoder.rs:241-250 × n × objects). */
int rlnc_encode_batch(rlnc_context *ctx, const uint8_t *src_dev, size_t k, size_t L, size_t num_objects,
                      const uint8_t *coeffs_dev, size_t n, uint8_t *pieces_dev);
/* rlnc_encode_batch in two parts, for pipelining a decoder's elimination against the data work (bench.py):
 * the coefficient headers alone (pieces[o][i][0..k) = coeffs[o][i], one strided copy) and the data alone
 * (pieces[o][i][k..k+L)).  Together they write exactly what rlnc_encode_batch writes. */
int rlnc_encode_batch_headers(rlnc_context *ctx, const uint8_t *coeffs_dev, size_t k, size_t L, size_t num_objects,
                              size_t n, uint8_t *pieces_dev);
int rlnc_encode_batch_data(rlnc_context *ctx, const uint8_t *src_dev, size_t k, size_t L, size_t num_objects,
                           const uint8_t *coeffs_dev, size_t n, uint8_t *pieces_dev);
/* rlnc_encode_batch_data with the kernel's per-coefficient code-block address stream written ahead: _prepare runs
 * the (coefficient-only) address launch on ITS context's stream into plan_dev (device memory of at least
 * rlnc_encode_batch_plan_bytes bytes), e.g. on a side stream beside other work; _data_planned, with the same
 * arguments and the same kernel variant, then runs the product without that launch (the caller orders it after the
 * prepare, e.g. with an event).  A plan buffer serves the product it was prepared for.  The library remembers each
 * prepare by the plan buffer's address with its arguments (buffers, shape, device, kernel variant) and
 * _data_planned returns InvalidArgument when those arguments differ.  What it cannot see is the memory itself: the
 * caller keeps the plan buffer alive and unwritten, and the coefficient bytes unchanged, from the prepare to the
 * product.  A plan buffer freed and reallocated at the same address, or coefficients rewritten in place, must be
 * prepared again: the product takes the buffer's entries as code addresses, so a stale plan gives wrong bytes and
 * a plan buffer overwritten with other data is undefined behaviour, like a dangling pointer.  Writes exactly what
 * rlnc_encode_batch_data writes. */
size_t rlnc_encode_batch_plan_bytes(size_t k, size_t num_objects, size_t n);
int rlnc_encode_batch_prepare(rlnc_context *ctx, const uint8_t *src_dev, size_t k, size_t L, size_t num_objects,
                              const uint8_t *coeffs_dev, size_t n, uint8_t *pieces_dev, void *plan_dev,
                              size_t plan_bytes);
int rlnc_encode_batch_data_planned(rlnc_context *ctx, const uint8_t *src_dev, size_t k, size_t L, size_t num_objects,
                                   const uint8_t *coeffs_dev, size_t n, uint8_t *pieces_dev, const void *plan_dev);
/* count recoded pieces per object from n received pieces: r [obj][count][n] → out [obj][count][k+L]
 * (recoder.rs:122-153; coefficient header and data are one linear combination of the full pieces). */
int rlnc_recode_batch(rlnc_context *ctx, const uint8_t *pieces_dev, size_t k, size_t L, size_t n,
                      size_t num_objects, const uint8_t *r_dev, size_t count, uint8_t *out_dev);
/* Feeds pieces 0..m-1 of every object, in order, to a fresh Decoder (decoder.rs:96-118) and extracts the
 * data (decoder.rs:136-177).  decoded_dev [obj][k][L] receives the padded payload rows in the reference's
 * row order.  pieces_obj_stride = bytes between objects' first pieces (0 = m*(k+L), i.e. dense; a larger
 * stride decodes from the first m of more coded pieces in place).  Host outputs (each may be NULL): piece_status [obj][m] (status of each decode() call),
 * object_status [obj] (Ok / NotAllPiecesReceivedYet / InvalidDecodedDataFormat of get_decoded_data),
 * data_len [obj] (unpadded length when Ok).  Synchronous. */
int rlnc_decode_batch(rlnc_context *ctx, const uint8_t *pieces_dev, size_t pieces_obj_stride, size_t k, size_t L,
                      size_t m, size_t num_objects, uint8_t *decoded_dev, int32_t *piece_status,
                      int32_t *object_status, uint64_t *data_len);

/* Fully asynchronous variant: everything stays on the device (statuses int32 [obj][m] and [obj], unpadded
 * lengths int64 [obj], all device pointers).  The exact elimination runs on the device (one wave per
 * object, LDS-resident [coeffs | E]; requires (k+1)·4·ceil_pow2((k+m)/4) + 8 KiB <= 160 KiB). */
int rlnc_decode_batch_device(rlnc_context *ctx, const uint8_t *pieces_dev, size_t pieces_obj_stride, size_t k,
                             size_t L, size_t m, size_t num_objects, uint8_t *decoded_dev, int32_t *piece_status_dev,
                             int32_t *object_status_dev, int64_t *data_len_dev);

/* rlnc_decode_batch_device in two parts (same results): the exact elimination, which reads only the k
 * coefficient bytes of each piece — T_dev [obj][k][m] (decoded rows = T × received data rows; rows >= rank
 * zero), per-piece statuses, ranks int32 [obj] — and the data side (T × data + the marker scan).  The two may
 * run on different contexts/streams; the caller orders them (e.g. a HIP event). */
int rlnc_decode_batch_eliminate(rlnc_context *ctx, const uint8_t *pieces_dev, size_t pieces_obj_stride, size_t k,
                                size_t L, size_t m, size_t num_objects, uint8_t *T_dev, int32_t *piece_status_dev,
                                int32_t *rank_dev);
int rlnc_decode_batch_apply(rlnc_context *ctx, const uint8_t *pieces_dev, size_t pieces_obj_stride, size_t k,
                            size_t L, size_t m, size_t num_objects, const uint8_t *T_dev, const int32_t *rank_dev,
                            uint8_t *decoded_dev, int32_t *object_status_dev, int64_t *data_len_dev);
/* rlnc_decode_batch_apply with the T x data product's code-block address stream written ahead, the decode's form of
 * rlnc_encode_batch_prepare / _data_planned: _prepare runs the (T-only) address launch on ITS context's stream into
 * plan_dev (device memory of at least rlnc_decode_batch_apply_plan_bytes bytes) once T is final -- e.g. on the
 * elimination's stream right behind rlnc_decode_batch_eliminate -- and _planned, with the same arguments and kernel
 * variant, runs the product and the marker scan without it (the caller orders it after the prepare).  The plan
 * contract is the encode plan's: prepares are remembered by the plan buffer's address with their arguments and
 * _planned returns InvalidArgument when those differ; the caller keeps the plan buffer alive and unwritten and T
 * unchanged from the prepare to the product.  Writes exactly what rlnc_decode_batch_apply writes. */
size_t rlnc_decode_batch_apply_plan_bytes(size_t k, size_t m, size_t num_objects);
int rlnc_decode_batch_apply_prepare(rlnc_context *ctx, const uint8_t *pieces_dev, size_t pieces_obj_stride, size_t k,
                                    size_t L, size_t m, size_t num_objects, const uint8_t *T_dev, uint8_t *decoded_dev,
                                    void *plan_dev, size_t plan_bytes);
int rlnc_decode_batch_apply_planned(rlnc_context *ctx, const uint8_t *pieces_dev, size_t pieces_obj_stride, size_t k,
                                    size_t L, size_t m, size_t num_objects, const uint8_t *T_dev,
                                    const int32_t *rank_dev, uint8_t *decoded_dev, int32_t *object_status_dev,
                                    int64_t *data_len_dev, const void *plan_dev);

/* ---- wire formats on the device ------------------------------------------------------------
 * Encoder::new's padded image (encoder.rs:85-106, BOUNDARY_MARKER consts.rs:5) built by a kernel from a byte
 * string already in HBM: out[r][c] (r < k, c < L = ceil((data_len+1)/k), row stride out_row_stride, 0 = L) =
 * data[r·L + c] below data_len, 0x81 at data_len, zeros after.  Errors as Encoder::new (DataLengthZero before
 * PieceCountZero).  Asynchronous on the context stream; data may be unaligned. */
typedef struct rlnc_pad_desc {
    const uint8_t *data;
    size_t data_len;
    size_t k;
    uint8_t *out;
    size_t out_row_stride;
} rlnc_pad_desc;
size_t rlnc_padded_piece_byte_len(size_t data_len, size_t k); /* encoder.rs:93-95 (0 when k == 0) */
int rlnc_pad_device(rlnc_context *ctx, const uint8_t *data_dev, size_t data_len, size_t k, uint8_t *out_dev,
                    size_t out_row_stride);
int rlnc_pad_batch_device(rlnc_context *ctx, const rlnc_pad_desc *descs, size_t count); /* one launch */
/* Encoder::new from a device byte string: the encoder owns its padded image (built on the device). */
int rlnc_encoder_new_device(rlnc_context *ctx, const uint8_t *data_dev, size_t data_len, size_t piece_count,
                            rlnc_encoder **out);
/* Ragged batches: every object with its own shape and buffers (device pointers; strides 0 = dense), as a sender or
 * receiver holding pieces of many objects has them.  Each kernel stage is one launch over a device-side descriptor
 * table, whatever the number of objects and shapes (the matmul stage: <= 6 launches -- block addresses, the
 * bit-sliced program for <= 8, <= 16, <= 32 and > 32 output rows, the perm kernel for < 4 KiB tails -- and for
 * misaligned operands on a device without unaligned vector access, rlnc_device_unaligned_vector_access).
 * Asynchronous on the context stream.  Error checks run over all descriptors before anything is launched.
 * rlnc_encode_ragged: n coded pieces coeffs ‖ data per object (encoder.rs:241-250 × n). */
typedef struct rlnc_object_desc {
    const uint8_t *src;      /* k source pieces of L bytes */
    size_t src_row_stride;   /* >= L, 0 = L */
    const uint8_t *coeffs;   /* n × k coding vectors */
    uint8_t *pieces;         /* n full coded pieces */
    size_t piece_row_stride; /* >= k + L, 0 = k + L */
    size_t k, L, n;
} rlnc_object_desc;
int rlnc_encode_ragged(rlnc_context *ctx, const rlnc_object_desc *objs, size_t count);
/* Recoder::recode_with_buf (recoder.rs:122-153) × n_recoded per object: out[i] = Σ_j r[i][j] · pieces[j] over the
 * full pieces (coefficient header and data are one linear map).  Checks in Recoder::new's order (recoder.rs:69-80):
 * n == 0 NotEnoughPiecesToRecode, k + L == 0 PieceLengthZero, k == 0 PieceCountZero, L == 0 PieceLengthTooShort. */
typedef struct rlnc_recode_object_desc {
    const uint8_t *pieces;   /* n received full pieces of k + L bytes */
    size_t piece_row_stride; /* >= k + L, 0 = k + L */
    const uint8_t *r;        /* n_recoded × n recoding coefficients (rng.fill_bytes draws them, recoder.rs:131) */
    uint8_t *out;            /* n_recoded full recoded pieces */
    size_t out_row_stride;   /* >= k + L, 0 = k + L */
    size_t k, L, n, n_recoded;
} rlnc_recode_object_desc;
int rlnc_recode_ragged(rlnc_context *ctx, const rlnc_recode_object_desc *objs, size_t count);
/* Decoder::decode for pieces 0..m-1 of every object + get_decoded_data (decoder.rs:96-177), like
 * rlnc_decode_batch_device per object: decoded [k][L] (padded payload rows in the reference's row order),
 * piece_status_dev int32 [Σ m] (object order, each object's m statuses of its decode() calls), object_status_dev
 * int32 [count] (Ok / NotAllPiecesReceivedYet / InvalidDecodedDataFormat), data_len_dev int64 [count] (unpadded
 * length when Ok).  The exact elimination runs on the device when an object's [coeffs | E] fits LDS, else on host
 * threads (then the call is not capturable).  L == 0 PieceLengthZero, k == 0 PieceCountZero (decoder.rs:66-71). */
typedef struct rlnc_decode_object_desc {
    const uint8_t *pieces;   /* m received full pieces, coeffs ‖ data */
    size_t piece_row_stride; /* >= k + L, 0 = k + L */
    uint8_t *decoded;        /* k × L bytes */
    size_t k, L, m;
} rlnc_decode_object_desc;
int rlnc_decode_ragged(rlnc_context *ctx, const rlnc_decode_object_desc *objs, size_t count, int32_t *piece_status_dev,
                       int32_t *object_status_dev, int64_t *data_len_dev);

/* ---- host-resident pieces (a socket or a file) ---------------------------------------------
 * The batch API above for host buffers: objects stream through the device in windows of `window` objects (0 =
 * automatic, >= 32 MiB of input per window) as a three-stage pipeline on three streams (host-to-device copies, the
 * encode/decode on the context's stream, device-to-host copies; windows rotate over three slots of device buffers,
 * ordered by events), so that window w+1's copy in, window w's encode/decode and window w-1's copy out overlap.
 * Pinned host buffers (hipHostMalloc / hipHostRegister) are copied by DMA directly; pageable ones are staged through
 * pinned buffers by host threads.  Same results as the device-resident calls (they run them).  Synchronous; like the
 * batch calls, one caller thread per context at a time (the slot buffers and copy streams belong to the context). */
/* src [obj][k][L], coeffs [obj][n][k] → pieces [obj][n][k+L] (rlnc_encode_batch). */
int rlnc_encode_host_stream(rlnc_context *ctx, const uint8_t *src, size_t k, size_t L, size_t num_objects,
                            const uint8_t *coeffs, size_t n, uint8_t *pieces, size_t window);
/* pieces: the first m pieces of each object (object stride in bytes, 0 = m*(k+L)) → decoded [obj][k][L], host
 * statuses as rlnc_decode_batch (each may be NULL). */
int rlnc_decode_host_stream(rlnc_context *ctx, const uint8_t *pieces, size_t pieces_obj_stride, size_t k, size_t L,
                            size_t m, size_t num_objects, uint8_t *decoded, int32_t *piece_status,
                            int32_t *object_status, uint64_t *data_len, size_t window);

/* ---- host-only: the decoder's exact coefficient elimination (no device needed) ---------------------------
 * The diagonal-pivot RREF of DecoderMatrix (decoder_matrix.rs:99-244) replicated on [coeffs | E] where E
 * tracks every row as a combination of received pieces; data rows = E × received data (elimination.hpp).
 * fixed_slots > 0: piece p owns E column p; 0: columns are recycled once unreferenced. */
typedef struct rlnc_elimination rlnc_elimination;
int rlnc_elimination_new(size_t k, size_t fixed_slots, rlnc_elimination **out);
void rlnc_elimination_free(rlnc_elimination *e);
/* Decoder::decode on the k coefficient bytes: Ok / PieceNotUseful / ReceivedAllPieces. */
int rlnc_elimination_push(rlnc_elimination *e, const uint8_t *coeffs, int32_t *slot, int32_t *keep);
size_t rlnc_elimination_rank(const rlnc_elimination *e);
size_t rlnc_elimination_slots(const rlnc_elimination *e);
int rlnc_elimination_transform(const rlnc_elimination *e, uint8_t *T, size_t ld); /* k × ld, zero-filled */
int rlnc_elimination_coefficients(const rlnc_elimination *e, uint8_t *C);        /* rank × k */

#ifdef __cplusplus
}
#endif
#endif /* RLNC_HIP_H */
