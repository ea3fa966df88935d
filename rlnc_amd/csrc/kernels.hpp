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
};

enum class MatmulVariant : int { Perm = 0, NibbleLds = 1 };

hipError_t launch_matmul(const MatmulParams &p, hipStream_t stream, MatmulVariant v = MatmulVariant::Perm);

// Element-wise primitives (src/common/simd/mod.rs:18-119) on one device vector.
hipError_t launch_mul_vec_by_scalar(uint8_t *vec, int64_t len, uint8_t scalar, hipStream_t s);
hipError_t launch_add_vectors(uint8_t *dst, const uint8_t *src, int64_t len, hipStream_t s);
hipError_t launch_mul_add(uint8_t *dst, const uint8_t *src, int64_t len, uint8_t scalar, hipStream_t s);

// decoder.rs:162-177 on device, per object: finds the last nonzero byte of the padded payload
// data[o][0:len); status[o] = 0 / InvalidDecodedDataFormat code, final_len[o] = marker index.
// `scratch` holds n_obj uint64 words.
hipError_t launch_final_data_len(const uint8_t *data, int64_t obj_stride, int64_t len, int n_obj,
                                 unsigned long long *scratch, int32_t *status, int64_t *final_len,
                                 int32_t invalid_code, hipStream_t s);

}  // namespace rlnc
