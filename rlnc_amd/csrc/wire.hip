// wire.hip — the data formats either side of the hot path, on the device:
//   * Encoder::new's padded image (encoder.rs:85-106, marker consts.rs:5) written by a kernel from a byte string
//     already in HBM: rlnc_pad_device / rlnc_pad_batch_device / rlnc_encoder_new_device;
//   * a ragged batch: objects with their own k, L, n and buffers in one call (rlnc_encode_ragged), as socket or
//     file ingestion produces them.
// The coeffs ‖ data framing of a coded piece is written by the matmul kernels themselves (header copy), and the
// decoder's marker scan by last_nonzero_kernel (kernels.hip).
#include <map>
#include <tuple>

#include "context.hpp"
#include "gf256.hpp"

using namespace rlnc::eng;

namespace {

struct PadDesc {
    const uint8_t *data;
    uint8_t *out;
    int64_t len, L, stride;
    int k;
};

// out[r][c] (r < k, c < L, row stride `stride`) = data[r·L + c] below len, the 0x81 marker at len, zeros after
// (encoder.rs:93-99).  One thread per 16 output bytes of a row; blockIdx.y = descriptor.
__global__ __launch_bounds__(256) void pad_kernel(const PadDesc *descs) {
    const PadDesc d = descs[blockIdx.y];
    const int64_t chunks = (d.L + 15) / 16;
    const int64_t e = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (e >= chunks * d.k) return;
    const int64_t r = e / chunks, c0 = (e % chunks) * 16;
    const int64_t i0 = r * d.L + c0;  // logical index of the first byte
    uint8_t *o = d.out + r * d.stride + c0;
    const int nb = int(min<int64_t>(16, d.L - c0));
    uint8_t b[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int64_t i = i0 + q;
        b[q] = i < d.len ? d.data[i] : (i == d.len ? rlnc::kBoundaryMarker : uint8_t(0));
    }
    if (nb == 16 && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
        uint4 v;
        __builtin_memcpy(&v, b, 16);
        *reinterpret_cast<uint4 *>(o) = v;
    } else {
        for (int q = 0; q < nb; ++q) o[q] = b[q];
    }
}

// descriptor upload: pinned staging guarded by an event (the previous call's copy must have run before the
// staging buffer is rewritten), device copy in the context's workspace
int upload_descs(rlnc_context *ctx, const void *host, size_t bytes, void **dev) {
    int st;
    if (ctx->tab_ev) HIP_TRY(hipEventSynchronize(ctx->tab_ev));
    if ((st = ctx->grow(ctx->pin_tab, bytes)) || (st = ctx->grow(ctx->ws_tab, bytes))) return st;
    std::memcpy(ctx->pin_tab.p, host, bytes);
    HIP_TRY(hipMemcpyAsync(ctx->ws_tab.p, ctx->pin_tab.p, bytes, hipMemcpyHostToDevice, ctx->stream));
    if (!ctx->tab_ev) HIP_TRY(hipEventCreateWithFlags(&ctx->tab_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(ctx->tab_ev, ctx->stream));
    *dev = ctx->ws_tab.p;
    return RLNC_OK;
}

int launch_pad(rlnc_context *ctx, const std::vector<PadDesc> &d) {
    int64_t max_blocks = 0;
    for (const auto &x : d) max_blocks = std::max<int64_t>(max_blocks, ((x.L + 15) / 16 * x.k + 255) / 256);
    if (max_blocks == 0) return RLNC_OK;
    if (max_blocks > 0x7FFFFFFF || d.size() > 65535) return set_error(RLNC_ERR_INVALID_ARGUMENT, "pad batch too large");
    void *dd = nullptr;
    int st = upload_descs(ctx, d.data(), d.size() * sizeof(PadDesc), &dd);
    if (st) return st;
    hipLaunchKernelGGL(pad_kernel, dim3(unsigned(max_blocks), unsigned(d.size())), dim3(256), 0, ctx->stream,
                       static_cast<const PadDesc *>(dd));
    HIP_TRY(hipGetLastError());
    return RLNC_OK;
}

int pad_check(const rlnc_pad_desc &d, PadDesc &o) {
    if (d.data_len == 0) return RLNC_ERR_DATA_LENGTH_ZERO;  // encoder.rs:86-88
    if (d.k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;         // :89-91
    CHECK_ARG(d.data != nullptr && d.out != nullptr && d.k <= 0x7FFFFFFF);
    const size_t L = (d.data_len + 1 + d.k - 1) / d.k;  // :93-95
    const size_t stride = d.out_row_stride ? d.out_row_stride : L;
    CHECK_ARG(stride >= L);
    o = PadDesc{d.data, d.out, int64_t(d.data_len), int64_t(L), int64_t(stride), int(d.k)};
    return RLNC_OK;
}

int64_t addr(const void *p) { return int64_t(reinterpret_cast<intptr_t>(p)); }

}  // namespace

extern "C" {

size_t rlnc_padded_piece_byte_len(size_t data_len, size_t k) { return k ? (data_len + 1 + k - 1) / k : 0; }

int rlnc_pad_batch_device(rlnc_context *ctx, const rlnc_pad_desc *descs, size_t count) {
    CHECK_ARG(ctx != nullptr);
    if (count == 0) return RLNC_OK;
    CHECK_ARG(descs != nullptr);
    std::vector<PadDesc> d(count);
    for (size_t i = 0; i < count; ++i)
        if (int st = pad_check(descs[i], d[i])) return st;
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    return launch_pad(ctx, d);
}

int rlnc_pad_device(rlnc_context *ctx, const uint8_t *data_dev, size_t len, size_t k, uint8_t *out_dev,
                    size_t out_row_stride) {
    const rlnc_pad_desc d{data_dev, len, k, out_dev, out_row_stride};
    return rlnc_pad_batch_device(ctx, &d, 1);
}

int rlnc_encode_ragged(rlnc_context *ctx, const rlnc_object_desc *objs, size_t count) {
    CHECK_ARG(ctx != nullptr);
    if (count == 0) return RLNC_OK;
    CHECK_ARG(objs != nullptr);
    for (size_t i = 0; i < count; ++i) {  // every descriptor is checked before anything is launched
        const rlnc_object_desc &o = objs[i];
        if (o.k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
        if (o.L == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;
        if (o.n == 0) continue;
        CHECK_ARG(o.src && o.coeffs && o.pieces && o.n <= 0x7FFFFFFF && o.k <= 0x7FFFFFFF);
        CHECK_ARG(o.src_row_stride == 0 || o.src_row_stride >= o.L);
        CHECK_ARG(o.piece_row_stride == 0 || o.piece_row_stride >= o.k + o.L);
    }
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    // objects of one shape (k, L, n, strides) in input order; each maximal run whose buffers sit at one constant
    // object stride is ONE launch (the kernels' object dimension), others one launch each
    std::map<std::tuple<size_t, size_t, size_t, size_t, size_t>, std::vector<size_t>> groups;
    for (size_t i = 0; i < count; ++i) {
        const rlnc_object_desc &o = objs[i];
        if (o.n == 0) continue;
        const size_t ss = o.src_row_stride ? o.src_row_stride : o.L;
        const size_t ps = o.piece_row_stride ? o.piece_row_stride : o.k + o.L;
        groups[{o.k, o.L, o.n, ss, ps}].push_back(i);
    }
    for (auto &g : groups) {
        const size_t k = std::get<0>(g.first), L = std::get<1>(g.first), n = std::get<2>(g.first);
        const size_t ss = std::get<3>(g.first), ps = std::get<4>(g.first);
        const auto &ix = g.second;
        for (size_t a = 0; a < ix.size();) {
            // extend the run while src / coeffs / pieces advance by the same strides as between the first two
            size_t b = a + 1;
            int64_t ds = 0, dc = 0, dp = 0;
            if (b < ix.size()) {
                ds = addr(objs[ix[b]].src) - addr(objs[ix[a]].src);
                dc = addr(objs[ix[b]].coeffs) - addr(objs[ix[a]].coeffs);
                dp = addr(objs[ix[b]].pieces) - addr(objs[ix[a]].pieces);
                const bool ok = ds >= int64_t(k * ss) && dc >= int64_t(n * k) && dp >= int64_t(n * ps);
                if (ok) {
                    while (b < ix.size() && addr(objs[ix[b]].src) - addr(objs[ix[b - 1]].src) == ds &&
                           addr(objs[ix[b]].coeffs) - addr(objs[ix[b - 1]].coeffs) == dc &&
                           addr(objs[ix[b]].pieces) - addr(objs[ix[b - 1]].pieces) == dp && b - a < 0xFFFF)
                        ++b;
                } else {
                    b = a + 1;
                }
            }
            const rlnc_object_desc &o = objs[ix[a]];
            rlnc::MatmulParams p{};
            p.in = o.src;
            p.in_obj = ds;
            p.in_row = int64_t(ss);
            p.coef = o.coeffs;
            p.coef_obj = dc;
            p.coef_row = int64_t(k);
            p.out = o.pieces + k;
            p.out_obj = dp;
            p.out_row = int64_t(ps);
            p.hdr = o.pieces;
            p.hdr_obj = dp;
            p.hdr_row = int64_t(ps);
            p.n_out = int(n);
            p.n_in = int(k);
            p.width = int64_t(L);
            p.n_obj = int(b - a);
            if ((st = ctx->matmul(p))) return st;
            a = b;
        }
    }
    return RLNC_OK;
}

// Encoder::new (encoder.rs:85-106) from a byte string already in HBM: the padded image is built on the device
int rlnc_encoder_new_device(rlnc_context *ctx, const uint8_t *data_dev, size_t len, size_t k, rlnc_encoder **out) {
    CHECK_ARG(ctx != nullptr && out != nullptr);
    *out = nullptr;
    if (len == 0) return RLNC_ERR_DATA_LENGTH_ZERO;
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
    CHECK_ARG(data_dev != nullptr);
    const size_t L = rlnc_padded_piece_byte_len(len, k), stride = round16(L);
    int st = ctx->activate();
    if (st) return st;
    uint8_t *img = nullptr;
    HIP_TRY(hipMalloc(&img, k * stride));
    rlnc_pad_desc d{data_dev, len, k, img, stride};
    if ((st = rlnc_pad_batch_device(ctx, &d, 1)) || (st = encoder_adopt_device(ctx, img, k, L, stride, out))) {
        (void)hipFree(img);
        return st;
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));  // the image is complete when Encoder::new returns
    return RLNC_OK;
}

}  // extern "C"
