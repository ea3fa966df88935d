// host_stream.cpp — pieces that start and end in host memory (a socket or a file), SURVEY.md §8(f1).
//
// rlnc_encode_host_stream / rlnc_decode_host_stream stream a batch of objects through the device in windows of
// objects.  Three pipeline slots, each with its own stream, device buffers and (for pageable host memory) pinned
// staging: window w's host→device copy, its encode/decode and its device→host copy run on slot w % 3's stream,
// so the copy engines (both PCIe directions) and the compute of consecutive windows overlap.  Host buffers that
// are already pinned (hipHostMalloc / hipHostRegister) are copied by DMA directly; pageable ones are staged
// through the slot's pinned buffers by host threads (a multi-threaded memcpy runs while the device works on the
// other two slots).  The device work is the batch API itself (rlnc_encode_batch, rlnc_decode_batch_device) on
// one sub-context per slot, so results are bit-identical to the device-resident path.
#include <thread>

#include "context.hpp"

using namespace rlnc::eng;

namespace {

constexpr int kSlots = 3;

bool is_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // clear the sticky "invalid value" of an unregistered pointer
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// memcpy of `rows` rows of `width` bytes (strides in bytes) on up to 16 host threads
void copy_rows(uint8_t *dst, size_t dst_stride, const uint8_t *src, size_t src_stride, size_t width, size_t rows) {
    const size_t total = width * rows;
    const size_t nth = std::min<size_t>(16, std::max<size_t>(1, total >> 23));  // >= 8 MiB per thread
    auto part = [&](size_t r0, size_t r1) {
        if (dst_stride == width && src_stride == width) {
            std::memcpy(dst + r0 * width, src + r0 * width, (r1 - r0) * width);
        } else {
            for (size_t r = r0; r < r1; ++r) std::memcpy(dst + r * dst_stride, src + r * src_stride, width);
        }
    };
    if (nth <= 1 || rows < nth) {
        if (rows == 1 && nth > 1) {  // one long row: split the bytes
            std::vector<std::thread> th;
            const size_t per = (width + nth - 1) / nth;
            for (size_t t = 0; t < nth; ++t) {
                const size_t a = t * per, b = std::min(width, a + per);
                if (a < b) th.emplace_back([=] { std::memcpy(dst + a, src + a, b - a); });
            }
            for (auto &t : th) t.join();
            return;
        }
        part(0, rows);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (rows + nth - 1) / nth;
    for (size_t t = 0; t < nth; ++t) {
        const size_t a = t * per, b = std::min(rows, a + per);
        if (a < b) th.emplace_back(part, a, b);
    }
    for (auto &t : th) t.join();
}

struct Slot {
    rlnc_context *ctx = nullptr;  // sub-context: own stream and workspaces; its hs_* buffers are this slot's
    hipEvent_t done = nullptr;
    size_t w0 = 0, w1 = 0;  // objects of the window in flight
    bool busy = false;
};

struct Pipeline {
    rlnc_context *parent;
    Slot slot[kSlots];
    explicit Pipeline(rlnc_context *p) : parent(p) {}
    int init() {
        for (auto &s : slot) {
            int st = parent->sub_context(&s - slot, &s.ctx);
            if (st) return st;
            HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
        }
        return RLNC_OK;
    }
    ~Pipeline() {
        for (auto &s : slot) {
            if (s.done) {
                (void)hipEventSynchronize(s.done);
                (void)hipEventDestroy(s.done);
            }
        }
    }
};

size_t auto_window(size_t bytes_per_object, size_t nobj) {
    // >= 64 MiB of input per window (PCIe copies of that size run at full rate), at most a third of the batch
    // so that the three slots overlap
    size_t w = std::max<size_t>(1, (size_t(64) << 20) / std::max<size_t>(1, bytes_per_object));
    w = std::min(w, std::max<size_t>(1, (nobj + 2) / 3));
    return std::min(w, nobj);
}

}  // namespace

// sub-context `i` of a context (created on first use, owned by the parent, same device and kernel settings)
int rlnc_context::sub_context(size_t i, rlnc_context **out) {
    std::lock_guard<std::mutex> lock(pool_mu);
    if (subs.size() <= i) subs.resize(i + 1, nullptr);
    if (!subs[i]) {
        int st = rlnc_context_create(device, &subs[i]);
        if (st) return st;
    }
    subs[i]->variant = variant;
    subs[i]->max_tile_rows = max_tile_rows;
    subs[i]->decode_path = decode_path;
    *out = subs[i];
    return RLNC_OK;
}

extern "C" {

int rlnc_encode_host_stream(rlnc_context *ctx, const uint8_t *src, size_t k, size_t L, size_t nobj,
                            const uint8_t *coeffs, size_t n, uint8_t *pieces, size_t window) {
    CHECK_ARG(ctx != nullptr);
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
    if (L == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;
    if (n == 0 || nobj == 0) return RLNC_OK;
    CHECK_ARG(src && coeffs && pieces);
    int st = ctx->activate();
    if (st) return st;
    HIP_TRY(hipStreamSynchronize(ctx->stream));  // earlier work on the context is done (synchronous call)
    const size_t full = k + L, in_b = k * L, co_b = n * k, out_b = n * full;
    const size_t W = window ? std::min(window, nobj) : auto_window(in_b, nobj);
    const bool pin_in = is_pinned(src) && is_pinned(coeffs), pin_out = is_pinned(pieces);
    Pipeline pl(ctx);
    if ((st = pl.init())) return st;
    for (auto &s : pl.slot) {
        if ((st = s.ctx->hs_din.ensure(W * in_b)) || (st = s.ctx->hs_dcoef.ensure(W * co_b)) || (st = s.ctx->hs_dout.ensure(W * out_b)))
            return st;
        if (!pin_in && ((st = s.ctx->hs_hin.ensure(W * (in_b + co_b))))) return st;
        if (!pin_out && (st = s.ctx->hs_hout.ensure(W * out_b))) return st;
    }
    auto retire = [&](Slot &s) -> int {  // the slot's window is done; pageable output copied out
        if (!s.busy) return RLNC_OK;
        HIP_TRY(hipEventSynchronize(s.done));
        if (!pin_out) copy_rows(pieces + s.w0 * out_b, 0, s.ctx->hs_hout.as<uint8_t>(), 0, (s.w1 - s.w0) * out_b, 1);
        s.busy = false;
        return RLNC_OK;
    };
    size_t w = 0;
    for (size_t o0 = 0; o0 < nobj; o0 += W, ++w) {
        Slot &s = pl.slot[w % kSlots];
        if ((st = retire(s))) return st;
        const size_t o1 = std::min(nobj, o0 + W), b = o1 - o0;
        hipStream_t hs = s.ctx->stream;
        const uint8_t *hin = src + o0 * in_b, *hco = coeffs + o0 * co_b;
        if (!pin_in) {  // stage through the slot's pinned buffer (host threads), then DMA
            uint8_t *h = s.ctx->hs_hin.as<uint8_t>();
            copy_rows(h, 0, hin, 0, b * in_b, 1);
            std::memcpy(h + b * in_b, hco, b * co_b);
            hin = h;
            hco = h + b * in_b;
        }
        HIP_TRY(hipMemcpyAsync(s.ctx->hs_din.p, hin, b * in_b, hipMemcpyHostToDevice, hs));
        HIP_TRY(hipMemcpyAsync(s.ctx->hs_dcoef.p, hco, b * co_b, hipMemcpyHostToDevice, hs));
        if ((st = rlnc_encode_batch(s.ctx, s.ctx->hs_din.as<uint8_t>(), k, L, b, s.ctx->hs_dcoef.as<uint8_t>(), n,
                                    s.ctx->hs_dout.as<uint8_t>())))
            return st;
        HIP_TRY(hipMemcpyAsync(pin_out ? pieces + o0 * out_b : s.ctx->hs_hout.as<uint8_t>(), s.ctx->hs_dout.p, b * out_b,
                               hipMemcpyDeviceToHost, hs));
        HIP_TRY(hipEventRecord(s.done, hs));
        s.w0 = o0;
        s.w1 = o1;
        s.busy = true;
    }
    for (size_t i = 0; i < kSlots; ++i)  // drain in window order
        if ((st = retire(pl.slot[(w + i) % kSlots]))) return st;
    return RLNC_OK;
}

int rlnc_decode_host_stream(rlnc_context *ctx, const uint8_t *pieces, size_t obj_stride, size_t k, size_t L, size_t m,
                            size_t nobj, uint8_t *decoded, int32_t *piece_status, int32_t *object_status,
                            uint64_t *data_len, size_t window) {
    CHECK_ARG(ctx != nullptr);
    if (L == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
    if (nobj == 0) return RLNC_OK;
    CHECK_ARG(pieces && decoded && m > 0);
    const size_t full = k + L, in_b = m * full, out_b = k * L;
    if (obj_stride == 0) obj_stride = in_b;
    CHECK_ARG(obj_stride >= in_b);
    const bool dev_elim = rlnc::rref_lds_bytes(int(k), int(m)) <= rlnc::kRrefMaxLds && ctx->decode_path != 1;
    int st = ctx->activate();
    if (st) return st;
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    const size_t W = window ? std::min(window, nobj) : auto_window(in_b, nobj);
    const bool pin_in = is_pinned(pieces), pin_out = is_pinned(decoded);
    const size_t st_b = 8 + m * 4 + 4;  // per object: length (int64, first: aligned), piece statuses, object status
    Pipeline pl(ctx);
    if ((st = pl.init())) return st;
    for (auto &s : pl.slot) {
        if ((st = s.ctx->hs_din.ensure(W * in_b)) || (st = s.ctx->hs_dout.ensure(W * out_b)) || (st = s.ctx->hs_dst.ensure(W * st_b)) ||
            (st = s.ctx->hs_hst.ensure(W * st_b)))
            return st;
        if (!pin_in && (st = s.ctx->hs_hin.ensure(W * in_b))) return st;
        if (!pin_out && (st = s.ctx->hs_hout.ensure(W * out_b))) return st;
    }
    auto retire = [&](Slot &s) -> int {
        if (!s.busy) return RLNC_OK;
        HIP_TRY(hipEventSynchronize(s.done));
        const size_t b = s.w1 - s.w0;
        if (!pin_out) copy_rows(decoded + s.w0 * out_b, 0, s.ctx->hs_hout.as<uint8_t>(), 0, b * out_b, 1);
        if (dev_elim) {
            const uint8_t *h = s.ctx->hs_hst.as<uint8_t>();
            const int64_t *dl = reinterpret_cast<const int64_t *>(h);
            const int32_t *ps = reinterpret_cast<const int32_t *>(h + b * 8);
            const int32_t *os = reinterpret_cast<const int32_t *>(h + b * 8 + b * m * 4);
            for (size_t o = 0; o < b; ++o) {
                if (object_status) object_status[s.w0 + o] = os[o];
                if (data_len) data_len[s.w0 + o] = uint64_t(os[o] == 0 ? dl[o] : 0);
            }
            if (piece_status) std::memcpy(piece_status + s.w0 * m, ps, b * m * 4);
        }
        s.busy = false;
        return RLNC_OK;
    };
    size_t w = 0;
    for (size_t o0 = 0; o0 < nobj; o0 += W, ++w) {
        Slot &s = pl.slot[w % kSlots];
        if ((st = retire(s))) return st;
        const size_t o1 = std::min(nobj, o0 + W), b = o1 - o0;
        hipStream_t hs = s.ctx->stream;
        uint8_t *dout = s.ctx->hs_dout.as<uint8_t>();
        if (pin_in) {  // the first m pieces of each object, strided by obj_stride, straight from pinned memory
            HIP_TRY(hipMemcpy2DAsync(s.ctx->hs_din.p, in_b, pieces + o0 * obj_stride, obj_stride, in_b, b,
                                     hipMemcpyHostToDevice, hs));
        } else {
            copy_rows(s.ctx->hs_hin.as<uint8_t>(), in_b, pieces + o0 * obj_stride, obj_stride, in_b, b);
            HIP_TRY(hipMemcpyAsync(s.ctx->hs_din.p, s.ctx->hs_hin.p, b * in_b, hipMemcpyHostToDevice, hs));
        }
        if (dev_elim) {
            uint8_t *dst = s.ctx->hs_dst.as<uint8_t>();
            int64_t *dl = reinterpret_cast<int64_t *>(dst);
            int32_t *ps = reinterpret_cast<int32_t *>(dst + b * 8);
            int32_t *os = reinterpret_cast<int32_t *>(dst + b * 8 + b * m * 4);
            if ((st = rlnc_decode_batch_device(s.ctx, s.ctx->hs_din.as<uint8_t>(), in_b, k, L, m, b, dout, ps, os, dl)))
                return st;
            HIP_TRY(hipMemcpyAsync(s.ctx->hs_hst.p, dst, b * st_b, hipMemcpyDeviceToHost, hs));
        } else {  // elimination too large for LDS: the host-elimination batch path (synchronous per window)
            if ((st = rlnc_decode_batch(s.ctx, s.ctx->hs_din.as<uint8_t>(), in_b, k, L, m, b, dout,
                                        piece_status ? piece_status + o0 * m : nullptr,
                                        object_status ? object_status + o0 : nullptr,
                                        data_len ? data_len + o0 : nullptr)))
                return st;
        }
        HIP_TRY(hipMemcpyAsync(pin_out ? decoded + o0 * out_b : s.ctx->hs_hout.as<uint8_t>(), dout, b * out_b,
                               hipMemcpyDeviceToHost, hs));
        HIP_TRY(hipEventRecord(s.done, hs));
        s.w0 = o0;
        s.w1 = o1;
        s.busy = true;
    }
    for (size_t i = 0; i < kSlots; ++i)
        if ((st = retire(pl.slot[(w + i) % kSlots]))) return st;
    return RLNC_OK;
}

}  // extern "C"
