// host_stream.cpp — pieces that start and end in host memory (a socket or a file), SURVEY.md §8(f1).
//
// rlnc_encode_host_stream / rlnc_decode_host_stream stream a batch of objects through the device in windows of
// objects, as a three-stage pipeline on three streams: every host→device copy on one stream, every encode/decode
// on a compute stream, every device→host copy on a third, ordered per window by events.  Each direction's DMA
// engine is fed back to back (copies of consecutive windows are adjacent on their stream), and the compute of
// window w overlaps the copies of its neighbours.  Windows rotate over `n` slots of device buffers (and, for
// pageable host memory, pinned staging); a slot is refilled only after the kernel that read its input and the copy
// that read its output have run (event waits on the device, no host round trip).  Three streams in all (the
// context's own for the compute, one per copy direction): HIP multiplexes streams over GPU_MAX_HW_QUEUES (4)
// hardware queues, and a copy stream sharing a queue with another stage serialises behind it (measured: a
// sub-context and stream per slot made the decode call's copies erratic, 44-89 GB/s).  Host buffers that are already
// pinned (hipHostMalloc / hipHostRegister) are copied by DMA directly and the host thread never blocks until the
// end; pageable ones are staged through the slot's pinned buffers by host threads (a multi-threaded memcpy runs
// while the device works on the other slots).  The device work is the batch API itself (rlnc_encode_batch,
// rlnc_decode_batch_device) on the context, so results are bit-identical to the device-resident path.
#include <cstdlib>
#include <thread>

#include "context.hpp"

using namespace rlnc::eng;

namespace {

constexpr int kDefaultSlots = 3;  // profiles/r02_host_stream_ab.txt
constexpr int kMaxSlots = 8;
// pipeline slots (windows in flight); RLNC_HS_SLOTS (A/B knob, read once) overrides the default
int num_slots() {
    static const int n = [] {
        const char *e = getenv("RLNC_HS_SLOTS");
        const int v = e ? atoi(e) : kDefaultSlots;
        return v >= 2 && v <= kMaxSlots ? v : kDefaultSlots;
    }();
    return n;
}

// What a host-stream buffer [p, p + bytes) is: 1 = pinned over the whole range (hipHostMalloc, or hipHostRegister
// covering it: copied by DMA directly), 0 = pageable (staged through pinned buffers by host threads), -1 = device
// memory (a misuse: the host threads would fault on it).  A registration that covers only the start of the range, or
// whose extent cannot be read, counts as pageable: the staged copy is always correct for host memory.
int host_kind(const void *p, size_t bytes) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // clear the sticky "invalid value" of an unregistered pointer
        return 0;
    }
    if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeArray) return -1;
    if (a.type != hipMemoryTypeHost) return 0;
    // the registered allocation must cover the whole range
    void *base = nullptr;
    size_t size = 0;
    const void *dp = a.devicePointer ? a.devicePointer : p;
    if (hipMemGetAddressRange(&base, &size, const_cast<void *>(dp)) != hipSuccess || base == nullptr) {
        (void)hipGetLastError();
        return 0;
    }
    const uintptr_t off = reinterpret_cast<uintptr_t>(dp) - reinterpret_cast<uintptr_t>(base);
    return off <= size && bytes <= size - off ? 1 : 0;
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

using HsSlot = rlnc_context::HsSlot;

struct Slot {
    HsSlot *buf = nullptr;                                          // the context's window buffers of this slot
    hipEvent_t hdone = nullptr, kdone = nullptr, ddone = nullptr;  // its last H2D / kernel / D2H
    size_t w0 = 0, w1 = 0;                                          // objects of the window it holds
    bool busy = false;
};

struct Pipeline {
    rlnc_context *comp;  // compute stage: the context itself (its stream, its batch workspaces)
    hipStream_t h2d = nullptr, d2h = nullptr;
    Slot slot[kMaxSlots];
    const int n = num_slots();
    explicit Pipeline(rlnc_context *c) : comp(c) {}
    int init() {
        {
            std::lock_guard<std::mutex> lock(comp->pool_mu);
            if (!comp->hs_h2d) HIP_TRY(hipStreamCreateWithFlags(&comp->hs_h2d, hipStreamNonBlocking));
            if (!comp->hs_d2h) HIP_TRY(hipStreamCreateWithFlags(&comp->hs_d2h, hipStreamNonBlocking));
            while (comp->hs_slots.size() < size_t(n)) comp->hs_slots.emplace_back(new HsSlot);
        }
        h2d = comp->hs_h2d;
        d2h = comp->hs_d2h;
        // the copy stages start after the work already enqueued on the context stream
        hipEvent_t start;
        HIP_TRY(hipEventCreateWithFlags(&start, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(start, comp->stream));
        HIP_TRY(hipStreamWaitEvent(h2d, start, 0));
        HIP_TRY(hipStreamWaitEvent(d2h, start, 0));
        (void)hipEventDestroy(start);
        for (int i = 0; i < n; ++i) {
            Slot &s = slot[i];
            s.buf = comp->hs_slots[size_t(i)].get();
            HIP_TRY(hipEventCreateWithFlags(&s.hdone, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&s.kdone, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&s.ddone, hipEventDisableTiming));
        }
        return RLNC_OK;
    }
    // slot s may take window w: its previous window's kernel has read the input buffers (H2D waits on kdone) and
    // its D2H has read the output buffers (the kernel waits on ddone)
    int before_h2d(Slot &s) {
        if (s.busy) HIP_TRY(hipStreamWaitEvent(h2d, s.kdone, 0));
        return RLNC_OK;
    }
    int before_kernel(Slot &s) {
        HIP_TRY(hipStreamWaitEvent(comp->stream, s.hdone, 0));
        if (s.busy) HIP_TRY(hipStreamWaitEvent(comp->stream, s.ddone, 0));
        return RLNC_OK;
    }
    int before_d2h(Slot &s) {
        HIP_TRY(hipStreamWaitEvent(d2h, s.kdone, 0));
        return RLNC_OK;
    }
    ~Pipeline() {
        if (d2h) (void)hipStreamSynchronize(d2h);
        (void)hipStreamSynchronize(comp->stream);
        if (h2d) (void)hipStreamSynchronize(h2d);
        for (auto &s : slot)
            for (hipEvent_t e : {s.hdone, s.kdone, s.ddone})
                if (e) (void)hipEventDestroy(e);
    }
};

size_t auto_window(size_t bytes_per_object, size_t nobj, int slots) {
    // >= 32 MiB of input per window (PCIe copies of that size run at full rate), at most 1/slots of the batch
    // so that the slots overlap (profiles/r02_host_stream_ab.txt)
    size_t w = std::max<size_t>(1, (size_t(32) << 20) / std::max<size_t>(1, bytes_per_object));
    w = std::min(w, std::max<size_t>(1, (nobj + slots - 1) / slots));
    return std::min(w, nobj);
}

}  // namespace

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
    const size_t full = k + L, in_b = k * L, co_b = n * k, out_b = n * full;
    const int ks = host_kind(src, nobj * in_b), kc = host_kind(coeffs, nobj * co_b), kp = host_kind(pieces, nobj * out_b);
    if (ks < 0 || kc < 0 || kp < 0)
        return set_error(RLNC_ERR_INVALID_ARGUMENT, "host-stream buffers must be host memory (got a device pointer)");
    const bool pin_in = ks == 1 && kc == 1, pin_out = kp == 1;
    Pipeline pl(ctx);
    if ((st = pl.init())) return st;
    const size_t W = window ? std::min(window, nobj) : auto_window(in_b, nobj, pl.n);
    for (int i = 0; i < pl.n; ++i) {
        HsSlot *b = pl.slot[i].buf;
        if ((st = b->din.ensure(W * in_b)) || (st = b->dcoef.ensure(W * co_b)) || (st = b->dout.ensure(W * out_b)))
            return st;
        if (!pin_in && ((st = b->hin.ensure(W * (in_b + co_b))))) return st;
        if (!pin_out && (st = b->hout.ensure(W * out_b))) return st;
    }
    auto retire = [&](Slot &s) -> int {  // pageable output: the slot's coded pieces copied out of its staging
        if (!s.busy || pin_out) return RLNC_OK;
        HIP_TRY(hipEventSynchronize(s.ddone));
        copy_rows(pieces + s.w0 * out_b, 0, s.buf->hout.as<uint8_t>(), 0, (s.w1 - s.w0) * out_b, 1);
        return RLNC_OK;
    };
    size_t w = 0;
    for (size_t o0 = 0; o0 < nobj; o0 += W, ++w) {
        Slot &s = pl.slot[w % pl.n];
        HsSlot *b = s.buf;
        if ((st = retire(s))) return st;
        const size_t o1 = std::min(nobj, o0 + W), cnt = o1 - o0;
        const uint8_t *hin = src + o0 * in_b, *hco = coeffs + o0 * co_b;
        if (!pin_in) {  // stage through the slot's pinned buffer once its previous H2D has read it
            if (s.busy) HIP_TRY(hipEventSynchronize(s.hdone));
            uint8_t *h = b->hin.as<uint8_t>();
            copy_rows(h, 0, hin, 0, cnt * in_b, 1);
            std::memcpy(h + cnt * in_b, hco, cnt * co_b);
            hin = h;
            hco = h + cnt * in_b;
        }
        if ((st = pl.before_h2d(s))) return st;
        HIP_TRY(hipMemcpyAsync(b->din.p, hin, cnt * in_b, hipMemcpyHostToDevice, pl.h2d));
        HIP_TRY(hipMemcpyAsync(b->dcoef.p, hco, cnt * co_b, hipMemcpyHostToDevice, pl.h2d));
        HIP_TRY(hipEventRecord(s.hdone, pl.h2d));
        if ((st = pl.before_kernel(s))) return st;
        if ((st = rlnc_encode_batch(pl.comp, b->din.as<uint8_t>(), k, L, cnt, b->dcoef.as<uint8_t>(), n,
                                    b->dout.as<uint8_t>())))
            return st;
        HIP_TRY(hipEventRecord(s.kdone, pl.comp->stream));
        if ((st = pl.before_d2h(s))) return st;
        HIP_TRY(hipMemcpyAsync(pin_out ? pieces + o0 * out_b : b->hout.as<uint8_t>(), b->dout.p, cnt * out_b,
                               hipMemcpyDeviceToHost, pl.d2h));
        HIP_TRY(hipEventRecord(s.ddone, pl.d2h));
        s.w0 = o0;
        s.w1 = o1;
        s.busy = true;
    }
    for (size_t i = 0; i < size_t(pl.n); ++i)  // drain in window order
        if ((st = retire(pl.slot[(w + i) % pl.n]))) return st;
    HIP_TRY(hipStreamSynchronize(pl.d2h));
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
    const int kin = host_kind(pieces, (nobj - 1) * obj_stride + in_b), kout = host_kind(decoded, nobj * out_b);
    if (kin < 0 || kout < 0)
        return set_error(RLNC_ERR_INVALID_ARGUMENT, "host-stream buffers must be host memory (got a device pointer)");
    const bool pin_in = kin == 1, pin_out = kout == 1;
    const size_t st_b = 8 + m * 4 + 4;  // per object: length (int64, first: aligned), piece statuses, object status
    Pipeline pl(ctx);
    if ((st = pl.init())) return st;
    const size_t W = window ? std::min(window, nobj) : auto_window(in_b, nobj, pl.n);
    for (int i = 0; i < pl.n; ++i) {
        HsSlot *b = pl.slot[i].buf;
        if ((st = b->din.ensure(W * in_b)) || (st = b->dout.ensure(W * out_b)) || (st = b->dst.ensure(W * st_b)) ||
            (st = b->hst.ensure(W * st_b)))
            return st;
        if (!pin_in && (st = b->hin.ensure(W * in_b))) return st;
        if (!pin_out && (st = b->hout.ensure(W * out_b))) return st;
    }
    auto retire = [&](Slot &s) -> int {  // the slot's window is out: statuses (and pageable payload) copied out
        if (!s.busy) return RLNC_OK;
        HIP_TRY(hipEventSynchronize(s.ddone));
        const size_t cnt = s.w1 - s.w0;
        if (!pin_out) copy_rows(decoded + s.w0 * out_b, 0, s.buf->hout.as<uint8_t>(), 0, cnt * out_b, 1);
        if (dev_elim) {
            const uint8_t *h = s.buf->hst.as<uint8_t>();
            const int64_t *dl = reinterpret_cast<const int64_t *>(h);
            const int32_t *ps = reinterpret_cast<const int32_t *>(h + cnt * 8);
            const int32_t *os = reinterpret_cast<const int32_t *>(h + cnt * 8 + cnt * m * 4);
            for (size_t o = 0; o < cnt; ++o) {
                if (object_status) object_status[s.w0 + o] = os[o];
                if (data_len) data_len[s.w0 + o] = uint64_t(os[o] == 0 ? dl[o] : 0);
            }
            if (piece_status) std::memcpy(piece_status + s.w0 * m, ps, cnt * m * 4);
        }
        return RLNC_OK;
    };
    size_t w = 0;
    for (size_t o0 = 0; o0 < nobj; o0 += W, ++w) {
        Slot &s = pl.slot[w % pl.n];
        HsSlot *b = s.buf;
        if ((st = retire(s))) return st;
        const size_t o1 = std::min(nobj, o0 + W), cnt = o1 - o0;
        uint8_t *dout = b->dout.as<uint8_t>();
        if (!pin_in) {  // the first m pieces of each object into the slot's staging (its previous H2D is done)
            if (s.busy) HIP_TRY(hipEventSynchronize(s.hdone));
            copy_rows(b->hin.as<uint8_t>(), in_b, pieces + o0 * obj_stride, obj_stride, in_b, cnt);
        }
        if ((st = pl.before_h2d(s))) return st;
        if (pin_in) {  // strided by obj_stride, straight from pinned memory: one linear copy per object (the 2D
                       // copy measured erratic, 44-89 GB/s)
            for (size_t o = 0; o < cnt; ++o)
                HIP_TRY(hipMemcpyAsync(b->din.as<uint8_t>() + o * in_b, pieces + (o0 + o) * obj_stride, in_b,
                                       hipMemcpyHostToDevice, pl.h2d));
        } else {
            HIP_TRY(hipMemcpyAsync(b->din.p, b->hin.p, cnt * in_b, hipMemcpyHostToDevice, pl.h2d));
        }
        HIP_TRY(hipEventRecord(s.hdone, pl.h2d));
        if ((st = pl.before_kernel(s))) return st;
        if (dev_elim) {
            uint8_t *dst = b->dst.as<uint8_t>();
            int64_t *dl = reinterpret_cast<int64_t *>(dst);
            int32_t *ps = reinterpret_cast<int32_t *>(dst + cnt * 8);
            int32_t *os = reinterpret_cast<int32_t *>(dst + cnt * 8 + cnt * m * 4);
            if ((st = rlnc_decode_batch_device(pl.comp, b->din.as<uint8_t>(), in_b, k, L, m, cnt, dout, ps, os, dl)))
                return st;
        } else {  // elimination too large for LDS: the host-elimination batch path (synchronous per window)
            if ((st = rlnc_decode_batch(pl.comp, b->din.as<uint8_t>(), in_b, k, L, m, cnt, dout,
                                        piece_status ? piece_status + o0 * m : nullptr,
                                        object_status ? object_status + o0 : nullptr,
                                        data_len ? data_len + o0 : nullptr)))
                return st;
        }
        HIP_TRY(hipEventRecord(s.kdone, pl.comp->stream));
        if ((st = pl.before_d2h(s))) return st;
        if (dev_elim) HIP_TRY(hipMemcpyAsync(b->hst.p, b->dst.p, cnt * st_b, hipMemcpyDeviceToHost, pl.d2h));
        HIP_TRY(hipMemcpyAsync(pin_out ? decoded + o0 * out_b : b->hout.as<uint8_t>(), dout, cnt * out_b,
                               hipMemcpyDeviceToHost, pl.d2h));
        HIP_TRY(hipEventRecord(s.ddone, pl.d2h));
        s.w0 = o0;
        s.w1 = o1;
        s.busy = true;
    }
    for (size_t i = 0; i < size_t(pl.n); ++i)
        if ((st = retire(pl.slot[(w + i) % pl.n]))) return st;
    HIP_TRY(hipStreamSynchronize(pl.d2h));
    return RLNC_OK;
}

}  // extern "C"
