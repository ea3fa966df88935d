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
hipError_t launch_matmul(const MatmulParams &p, hipStream_t stream, MatmulVariant v = MatmulVariant::Perm,
                         void *scratch = nullptr, size_t scratch_bytes = 0);

// Element-wise primitives (src/common/simd/mod.rs:18-119) on one device vector.
hipError_t launch_mul_vec_by_scalar(uint8_t *vec, int64_t len, uint8_t scalar, hipStream_t s);
hipError_t launch_add_vectors(uint8_t *dst, const uint8_t *src, int64_t len, hipStream_t s);
// dst[r][0..width) = src[r][0..width) for rows r < rows (strided byte rows, e.g. coded-piece headers)
hipError_t launch_copy_rows(uint8_t *dst, int64_t dst_stride, const uint8_t *src, int64_t src_stride, int64_t width,
                            int64_t rows, hipStream_t s);
hipError_t launch_mul_add(uint8_t *dst, const uint8_t *src, int64_t len, uint8_t scalar, hipStream_t s);

// decoder.rs:162-177 on device, per object: finds the last nonzero byte of the padded payload
// data[o][0:len); status[o] = 0 / InvalidDecodedDataFormat code, final_len[o] = marker index.
// `scratch` holds n_obj uint64 words.
hipError_t launch_final_data_len(const uint8_t *data, int64_t obj_stride, int64_t len, int n_obj,
                                 unsigned long long *scratch, int32_t *status, int64_t *final_len,
                                 int32_t invalid_code, hipStream_t s);

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
};
constexpr size_t kRrefMaxLds = 160 * 1024;
size_t rref_lds_bytes(int k, int m);
hipError_t launch_rref_batch(const RrefParams &p, hipStream_t s);

// final_len with the decoder's rank: objects with rank < k report NotAllPiecesReceivedYet
hipError_t launch_final_data_len_ranked(const uint8_t *data, int64_t obj_stride, int64_t len, int n_obj, int k,
                                        const int32_t *rank, unsigned long long *scratch, int32_t *status,
                                        int64_t *final_len, hipStream_t s);

}  // namespace rlnc
