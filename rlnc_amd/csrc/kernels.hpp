// kernels.hpp — launch interface of the gfx950 kernels in kernels.hip (internal to librlnc_hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rlnc {

// Out[o][i][0:width) = XOR_j coef[o][i][j] · In[o][j][0:width)  over GF(2^8)  (i < n_out, j < n_in)
//
// This single operator is the whole hot path of the reference:
//   * encode  (encoder.rs:128-144, batched over n coding vectors):  coef = coding vectors, In = source pieces
//   * recode  (recoder.rs:122-153):  coef = recoding vectors, In = received full pieces (coeffs ‖ data)
//   * decode  (decoder_matrix.rs:99-244 applied to the data columns):  coef = transform T from the exact
//     diagonal-pivot elimination of the coefficient block, In = received data rows
// Byte strides everywhere; every row must be readable for `width` bytes.
struct MatmulParams {
    const uint8_t *in;
    int64_t in_obj, in_row;
    const uint8_t *coef;
    int64_t coef_obj, coef_row;
    uint8_t *out;
    int64_t out_obj, out_row;
    uint8_t *hdr;  // optional: coefficient rows are also copied to hdr[o][i][0:n_in) (coded-piece framing)
    int64_t hdr_obj, hdr_row;
    int n_out, n_in;
    int64_t width;
    int n_obj;
    int col_run = 0;  // column blocks per workgroup of the column-run program (variant 9): 0 = chosen per launch
    // optional: the block-offset stream of this product already written (by the small-object elimination, rref.hip):
    // 4-byte offsets laid out as bsj_offset_kernel<false> lays them out for tiles of bsj_stream_rows rows; used when
    // the product takes the 1- or 2-wave bit-sliced program with exactly those tiles, else ignored
    const void *bsj_stream = nullptr;
    int bsj_stream_rows = 0;
    // 1: bsj_stream holds the shared programs' 8-byte absolute block addresses instead (launch_bsj_stream, written
    // ahead on another stream: the encode's block-address stream off the launch stream's critical path)
    int bsj_stream_abs = 0;
    // optional (the small-object decode, RrefParams::tail_need): objects that are ONE workgroup's tile of the 1- / 2-wave
    // bit-sliced program (n_out = scan_k <= 16 rows, width = out_row = one 4 KiB column block) and whose final length
    // the elimination could not decide from the payload tail (scan_need[obj] != 0) are scanned by that workgroup once
    // its stores are done (decoder.rs:162-177) -- the marker scan without a launch of its own; launch_matmul sets
    // *scan_done (a host flag) when it took this form, else the caller runs the scan kernel
    int32_t *scan_status = nullptr;
    const int32_t *scan_need = nullptr;
    int64_t *scan_len = nullptr;
    int scan_k = 0;
    bool *scan_done = nullptr;
};

enum class MatmulVariant : int {
    Perm = 0,
    NibbleLds = 1,
    Perm3 = 2,
    Wide = 3,
    Wide4 = 4,
    BitSliced = 5,
    BitSlicedJump = 6,
    BitSlicedJumpShared = 7,  // 6 with each row's combination sets built once per workgroup (4-wave tiles)
    BitSlicedJumpShared8 = 8,  // 7 with 64-row tiles of 8 waves (n_out > 32): waves 4-7 only read the sets and call,
                               // the builders run three rows ahead, one barrier per three rows
    BitSlicedJumpRun = 9       // 8 with column runs: a workgroup walks up to 8 column blocks of one (object, row
                               // tile), the source-row stream unbroken across them (one prologue per run)
};

// Device scratch the BitSliced variant needs for its coefficient-index stream (0 for the others, and for
// shapes that variant hands to the perm kernel).  launch_matmul fails with hipErrorInvalidValue when a
// BitSliced launch gets less.
size_t matmul_scratch_bytes(const MatmulParams &p, MatmulVariant v);
// Byte-misaligned 16-byte vector memory access (kernels.hip): probe_unaligned_vector_access runs the check on the
// current device once (synchronous; rlnc_context_create) and returns whether it holds; unaligned_vector_access(dev)
// is 1 / 0, or -1 before the probe; unaligned_vector_ok() is the current device's result.
int probe_unaligned_vector_access(int device);
int unaligned_vector_access(int device);
bool unaligned_vector_ok();
hipError_t launch_matmul(const MatmulParams &p, hipStream_t stream, MatmulVariant v = MatmulVariant::Perm,
                         void *scratch = nullptr, size_t scratch_bytes = 0);

struct RrefParams;

// ---- the A/B build (make ab: kernels_ab.hip adds matmul variants 2-5 and 9, rref_ab.hip decode paths 3, 4, 6) ----
// The shipped library defines these weakly (ab_build() false, the launches hipErrorInvalidValue); the A/B build's
// definitions replace them.
bool ab_build();
bool launch_rref_ab(const RrefParams &p, hipStream_t s, hipError_t *result);  // true: launched (*result its status)
hipError_t launch_matmul_ab(const MatmulParams &p, hipStream_t s, MatmulVariant v, void *scratch, size_t scratch_bytes);
size_t matmul_scratch_bytes_ab(const MatmulParams &p, MatmulVariant v);
// what the A/B variants reuse of the shipped bit-sliced jump path (kernels.hip): eligibility (whole 4 KiB column blocks
// of aligned operands, >= 4 output rows), scratch size, and the block-address stream + launch geometry of a product
struct BsjPlan {
    int64_t full = 0;   // columns the bit-sliced program takes (whole 4 KiB blocks)
    int64_t total = 0;  // workgroups of the uniform launch
    int waves = 0, row_tiles = 0, col_blocks = 0;
    bool share = false;
    void *stream = nullptr;  // the block-address stream (in the scratch)
};
bool bsj_eligible_public(const MatmulParams &p);
size_t bsj_scratch_bytes_public(const MatmulParams &p, bool wide);
hipError_t bsj_prepare(const MatmulParams &p, hipStream_t s, void *scratch, size_t scratch_bytes, bool share, bool wide,
                       BsjPlan &b);
// The block-address stream of launch_matmul(p, v)'s bit-sliced product written ahead into buf (one offset launch on s),
// for a later launch_matmul of the same p with bsj_stream = buf, bsj_stream_rows = tile_rows, bsj_stream_abs = abs.
// tile_rows = 0: that product takes no stream (another kernel, or realigned operands) and nothing is launched.
struct BsjStreamPlan {
    int tile_rows = 0;
    int abs = 0;
};
hipError_t launch_bsj_stream(const MatmulParams &p, MatmulVariant v, hipStream_t s, void *buf, size_t bytes,
                             BsjStreamPlan &plan);
// an upper bound of launch_bsj_stream's buffer for n_obj objects of n_out x n_in coefficients
size_t bsj_stream_bytes_bound(int n_obj, int n_out, int n_in);

// ---- ragged batches: one launch per kernel stage over objects of different shapes (wire.hip) -----------------
// One object's part of a ragged matmul launch (device-side descriptor table, 120 bytes).  Objects are ordered by
// wg0 (and, in the block-address stream, by idx0).
struct RaggedObj {
    const uint8_t *in;    // source rows (n_in of them), row stride in_row
    const uint8_t *coef;  // n_out x n_in coefficients, row stride coef_row
    uint8_t *out;         // n_out output rows, row stride out_row
    uint8_t *hdr;         // coefficient rows copied here too (coded-piece header), or nullptr
    int64_t in_row, coef_row, out_row, hdr_row;
    int64_t col0;   // first column (bytes) of this launch's part of the object
    int64_t width;  // columns of this part, from col0
    int64_t wg0;    // the object's first workgroup in its launch
    int64_t idx0;   // the object's first entry in the block-address stream (bit-sliced part)
    int32_t n_out, n_in;
    int32_t row_tiles, col_blocks;
    int32_t tile_rows;  // bit-sliced part: 8 x waves per workgroup
    int32_t aligned;    // perm part: operands 16-byte aligned (vector loads for full slots)
};
static_assert(sizeof(RaggedObj) == 120, "RaggedObj layout");
constexpr int kRaggedPermRows = 8;     // output rows per workgroup of the ragged perm kernel
constexpr int kRaggedColBlock = 4096;  // columns per workgroup (both ragged kernels)
// the bit-sliced program takes whole 4 KiB column blocks of 16-byte-aligned operands with >= 4 output rows
bool ragged_bsj_eligible(const uint8_t *in, const uint8_t *out, int64_t in_row, int64_t out_row, int64_t width,
                         int n_out,
                         bool unaligned_ok);  // unaligned_ok: unaligned_vector_ok(), looked up once per call
int ragged_bsj_waves(int n_out);  // 1, 2, 4 waves (8, 16, 32-row tiles) up to 32 output rows, else 8 (64-row tiles)
// the shared program's block table address (probe_scratch: >= 8 device bytes; synchronous the first time)
hipError_t ragged_bsj_base(hipStream_t s, void *probe_scratch, uint64_t &base);
hipError_t launch_ragged_offsets(const RaggedObj *objs, int n, int64_t entries, void *stream, uint64_t base,
                                 hipStream_t s);
hipError_t launch_ragged_bsj(int W, const RaggedObj *objs, int n, int64_t wgs, const void *stream, hipStream_t s);
hipError_t launch_ragged_perm(const RaggedObj *objs, int n, int64_t wgs, hipStream_t s);

// Element-wise primitives (src/common/simd/mod.rs:18-119) on one device vector.
hipError_t launch_mul_vec_by_scalar(uint8_t *vec, int64_t len, uint8_t scalar, hipStream_t s);
hipError_t launch_add_vectors(uint8_t *dst, const uint8_t *src, int64_t len, hipStream_t s);
// dst[r][0..width) = src[r][0..width) for rows r < rows (strided byte rows, e.g. coded-piece headers)
hipError_t launch_copy_rows(uint8_t *dst, int64_t dst_stride, const uint8_t *src, int64_t src_stride, int64_t width,
                            int64_t rows, hipStream_t s);
hipError_t launch_mul_add(uint8_t *dst, const uint8_t *src, int64_t len, uint8_t scalar, hipStream_t s);

// decoder.rs:162-177 on device, per object: finds the last nonzero byte of the padded payload
// data[o][0:len); status[o] = 0 / invalid_code, final_len[o] = marker index (one launch, one wave per object).
hipError_t launch_final_data_len(const uint8_t *data, int64_t obj_stride, int64_t len, int n_obj, int32_t *status,
                                 int64_t *final_len, int32_t invalid_code, hipStream_t s);

// Device replica of Decoder::decode over pieces 0..m-1 of every object (rref.hip).  Piece p of object o
// starts (coefficient header first) at pieces + o*obj_stride + p*piece_stride.  Outputs: status[o][p]
// (RLNC status of each decode() call), rank[o], T[o] (k × m, row-major, rows >= rank zero).
struct RrefParams {
    const uint8_t *pieces;
    int64_t obj_stride, piece_stride;
    int k, m, n_obj;
    uint8_t *T;
    int64_t T_obj;
    int32_t *status;
    int32_t *rank;
    int lds_only;  // clean-state path (A/B, all exact): 0 auto (blocked clean run when k + m <= 256, else 4);
                   // 1 LDS; 2 registers, one wave; 3 blocked clean run (gf_rref_block_kernel); 4 registers, multi-wave
    const struct RrefObj *objs = nullptr;  // ragged batch: object o's shape and buffers (the fields above unused)
    // two-pass elimination when k + m > 256 (k <= 128): pass 1 (the blocked run) replays only the first m pieces of
    // each object with statuses / T at row stride m_stride (> m): an object full-ranked within them is exact
    // (decode() answers ReceivedAllPieces for every later piece and leaves the state alone, decoder.rs:97-99); pass 2
    // (the general kernel over all pieces) skips the objects pass 1 full-ranked (skip_full) and redoes the others
    int m_stride = 0;   // 0 = m
    int skip_full = 0;
    // optional (the small-object kernel only): also write T as the 1- / 2-wave bit-sliced program's block-offset
    // stream -- bsj_stream[o][j][i] = T[i][j] · bsj_block_bytes for i < bsj_tile_rows (0 past k) -- so the T × data
    // product needs no offset launch (MatmulParams::bsj_stream); launch_rref_batch reports whether it did
    uint32_t *bsj_stream = nullptr;
    uint32_t bsj_block_bytes = 0;
    int bsj_tile_rows = 0;
    // optional, with bsj_stream (same kernel): get_final_data_len (decoder.rs:162-177) decided from the last 64
    // payload bytes -- decoded row k - 1's last 64 bytes computed from T and the pieces' tails (tail_L = L, a multiple
    // of 4, >= 64; k and the object stride multiples of 4): tail_status / tail_len the object's status and final length when its last
    // nonzero byte lies there (or rank < k), else tail_need[o] = 1 (the product's workgroup scans the whole payload,
    // MatmulParams::scan_need)
    int32_t *tail_status = nullptr;
    int64_t *tail_len = nullptr;
    int32_t *tail_need = nullptr;
    int64_t tail_L = 0;
    // diagnostic build only (rref_ab.hip, RLNC_SMALL_PROF): per-wave phase timestamps of the small-object kernel
    uint64_t *prof = nullptr;
};
// One object of a ragged elimination launch (rlnc_decode_ragged): T is k x m row-major, status m entries.
struct RrefObj {
    const uint8_t *pieces;
    int64_t piece_stride;
    uint8_t *T;
    int32_t *status;
    int32_t *rank;
    int32_t k, m;      // m = received pieces (the row stride of T and of the statuses)
    int32_t m_first;   // > 0: the blocked pass replays only the first m_first pieces (see RrefParams::m_stride)
    int32_t two_pass;  // the general pass skips this object when the blocked pass full-ranked it
};
// ragged elimination: one workgroup per object of the device table objs (n objects, k + m <= 256 each when
// block = true -- the blocked clean run -- else the one-wave LDS kernel); lds = the largest object's need
size_t rref_block_lds_bytes_public(int k, int m);
hipError_t launch_rref_ragged(const RrefObj *objs, int n, bool block, size_t lds, int hdr_lds, hipStream_t s);
size_t rref_lds_bytes_staged_public(int k, int m);
constexpr size_t kRrefMaxLds = 160 * 1024;
size_t rref_lds_bytes(int k, int m);
// the blocked clean-run kernel (decode path 5, and what 0 / 2 pick) applies: a row fits one wave (k + m <= 256)
bool rref_block_eligible(int k, int m);
hipError_t launch_rref_batch(const RrefParams &p, hipStream_t s, bool *bsj_written = nullptr);
// block bytes and tile rows of the unshared bit-sliced programs (for RrefParams::bsj_*): tile rows 0 = not one of them
uint32_t bsj_block_bytes_public();
int bsj_unshared_tile_rows(int n_out);

// final_len with the decoder's rank: objects with rank < k report NotAllPiecesReceivedYet
hipError_t launch_final_data_len_ranked(const uint8_t *data, int64_t obj_stride, int64_t len, int n_obj, int k,
                                        const int32_t *rank, int32_t *status, int64_t *final_len, hipStream_t s);

}  // namespace rlnc
