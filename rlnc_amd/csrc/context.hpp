// context.hpp — librlnc_hip internals shared by engine.cpp, host_stream.cpp and wire.cpp: error reporting, the
// grow-only device / pinned buffers, the per-call workspace pool and struct rlnc_context (include/rlnc_hip.h).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/rlnc_hip.h"
#include "kernels.hpp"

namespace rlnc::eng {

extern thread_local std::string g_last_error;

inline int set_error(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                                    \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess) {                                                                          \
            return ::rlnc::eng::set_error(e_ == hipErrorOutOfMemory ? RLNC_ERR_OUT_OF_MEMORY : RLNC_ERR_DEVICE, \
                                          "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                                          __LINE__);                                                     \
        }                                                                                                \
    } while (0)

#define CHECK_ARG(cond)                                                                                     \
    do {                                                                                                    \
        if (!(cond)) return ::rlnc::eng::set_error(RLNC_ERR_INVALID_ARGUMENT, "invalid argument: %s", #cond); \
    } while (0)

inline size_t round16(size_t v) { return (v + 15) & ~size_t(15); }

// grow-only device buffer
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return RLNC_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        HIP_TRY(hipMalloc(&p, std::max<size_t>(bytes, 256)));
        cap = std::max<size_t>(bytes, 256);
        return RLNC_OK;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    template <class T>
    T *as() const {
        return static_cast<T *>(p);
    }
};

// grow-only pinned host buffer
struct PinBuf {
    void *p = nullptr;
    size_t cap = 0;
    unsigned flags = hipHostMallocDefault;  // hipHostMallocCoherent: read / written by a running kernel
    int ensure(size_t bytes) {
        if (bytes <= cap) return RLNC_OK;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        HIP_TRY(hipHostMalloc(&p, std::max<size_t>(bytes, 256), flags));
        cap = std::max<size_t>(bytes, 256);
        return RLNC_OK;
    }
    ~PinBuf() {
        if (p) (void)hipHostFree(p);
    }
    template <class T>
    T *as() const {
        return static_cast<T *>(p);
    }
};


// Workspace of one object-API call (Encoder/Recoder/Decoder on host buffers): its own stream, scratch and
// staging buffers, leased from the context's pool for the duration of the call.  Concurrent calls on one
// context (e.g. Encoder::code(&self) from many threads, encoder.rs:264 -- the reference type is Send + Sync)
// therefore never share a buffer.
struct CallWs {
    hipStream_t stream = nullptr;
    hipEvent_t ev = nullptr;
    DevBuf coef, out, idx, status, len;
    PinBuf pin_a, pin_b, pin_c;
    // the call-latency kernel (piece.hip): coefficients read and output rows written by the kernel in host memory,
    // per-chunk completion flags raised to the call's epoch, and the chunks' workgroup counters on the device
    PinBuf pc_coef, pc_out, pc_flag;
    DevBuf pc_count;
    size_t pc_count_words = 0;  // zeroed words of pc_count
    DevBuf pc_part, pc_pcount;  // split products (piece.hpp): partial slabs and per-block counters
    size_t pc_pcount_words = 0;  // zeroed words of pc_pcount
    uint32_t epoch = 0;
    // large copy-outs to host (Decoder::get_decoded_data): a ring of pinned chunks the DMA fills while host threads
    // copy the previous chunks into the caller's buffer (engine.cpp copy_out)
    static constexpr int kOutRing = 4;
    PinBuf pin_out;
    hipEvent_t out_ev[kOutRing] = {};
    CallWs() { pc_coef.flags = pc_out.flags = pc_flag.flags = hipHostMallocCoherent; }
    ~CallWs() {
        for (hipEvent_t e : out_ev)
            if (e) (void)hipEventDestroy(e);
        if (ev) (void)hipEventDestroy(ev);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

// Staging ring of the object API's host -> device piece uploads (Decoder::decode): a call copies its piece into the
// open pinned slot and returns.  A slot collects pieces until it is full or one of its decoders needs its rows on the
// device; then it is flushed -- one DMA per run of consecutive store rows, queued on the context's one upload stream
// -- and its event recorded.  All DMAs run on that one stream, so a slot's event, whenever it was last recorded,
// follows every upload flushed before it.  Pieces larger than a slot take several.
struct UpRun {
    uint8_t *dst;
    size_t off, len;  // bytes [off, off + len) of the slot go to dst
};
struct UpSlot {
    PinBuf buf;
    hipEvent_t ev = nullptr;  // the slot's last flush (the slot may be rewritten once it has run)
    std::vector<UpRun> runs;  // staged, not yet flushed
    size_t used = 0;
    unsigned gen = 0;  // bumped each time the slot is reopened
    bool open = false;
    ~UpSlot() {
        if (ev) (void)hipEventDestroy(ev);
    }
};
// The stream-ordered uses of an object's device block (the *_batch_device calls, queued on whatever stream the
// context had then): the block may be reused by another object only after the last of them.  Synchronous uses (the
// object API on host buffers, the decoder's uploads) are complete when their call returns and need no record.
struct ObjUse {
    hipEvent_t ev = nullptr;  // recorded after the latest stream-ordered use, and after every earlier one
    hipStream_t last = nullptr;
    bool used = false;
    bool captured = false;  // a use inside a HIP graph capture: the graph may replay it at any time
    ~ObjUse() {
        if (ev) (void)hipEventDestroy(ev);
    }
    int note(hipStream_t s) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        HIP_TRY(hipStreamIsCapturing(s, &cs));
        if (cs != hipStreamCaptureStatusNone) {
            captured = true;
            return RLNC_OK;
        }
        if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        // a use on another stream than the previous one: the event re-recorded on s must still follow that earlier
        // use (it may run after this one), so s waits for the event's previous recording first
        if (used && s != last) HIP_TRY(hipStreamWaitEvent(s, ev, 0));
        HIP_TRY(hipEventRecord(ev, s));
        last = s;
        used = true;
        return RLNC_OK;
    }
};

constexpr int kUpSlots = 8;
constexpr size_t kUpChunk = size_t(4) << 20;
constexpr size_t kUpRuns = 256;  // runs per slot before it is flushed
// where a decoder's last piece was staged: ring slot and its generation then
struct UpTicket {
    int slot = -1;
    unsigned gen = 0;
};

}  // namespace rlnc::eng

using rlnc::eng::set_error;

struct rlnc_context {
    using DevBuf = rlnc::eng::DevBuf;
    using PinBuf = rlnc::eng::PinBuf;
    using CallWs = rlnc::eng::CallWs;
    std::atomic<int> refs{1};  // the creator's reference + one per Encoder/Decoder/Recoder bound to it
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    // variant 9 (column runs) is 5 % faster for an isolated encode launch but not in the bench's pipelined step,
    // whose encode and decode launches share the CUs better with short workgroups (profiles/r02_run_ab.txt)
    rlnc::MatmulVariant variant = rlnc::MatmulVariant::BitSlicedJumpShared8;
    int max_tile_rows = 0;
    int col_run = 0;  // column blocks per workgroup of variant 9 (0 = chosen per launch; rlnc_set_column_run)
    int decode_path = 0;  // 0 auto (device when it fits LDS), 1 host elimination, 2 device elimination,
                          // 3 device elimination with the clean state on LDS, 4 ... on one wave's
                          // registers, 5 blocked clean run, 6 round-1 multi-wave registers (A/B)
    // workspaces of the stream-ordered batch / _device API (one caller thread per context at a time)
    DevBuf ws_bsj;   // the small-object decode's block-offset stream, written by its elimination
    DevBuf ws_need;  // ... and its per-object "payload tail all zero" flags (RrefParams::tail_need)
    DevBuf ws_coef, ws_out, ws_status, ws_len, ws_pstat, ws_rank, ws_idx;
    PinBuf pin_a, pin_b, pin_c;
    // set once a batch call ran inside a HIP stream capture: the graph holds the workspace addresses, so
    // they must never move again (grow() refuses instead of reallocating)
    std::atomic<bool> graph_bound{false};
    std::mutex pool_mu;
    std::vector<std::unique_ptr<CallWs>> pool;
    // host-stream pipeline (host_stream.cpp): per-slot window buffers and the two copy streams, kept between calls.
    // Few streams on purpose: HIP multiplexes streams over GPU_MAX_HW_QUEUES (4) hardware queues, and a copy
    // stream sharing a queue with another stage serialises behind it.
    struct HsSlot {
        DevBuf din, dcoef, dout, dst;
        PinBuf hin, hout, hst;
    };
    std::vector<std::unique_ptr<HsSlot>> hs_slots;
    hipStream_t hs_h2d = nullptr, hs_d2h = nullptr;
    DevBuf ws_tab;  // descriptor tables of the wire-format / ragged calls (wire.hip), uploaded from pin_tab
    // a ring of pinned staging buffers, each with the event of its last upload (it may be rewritten once that has
    // run): a ragged decode stages three tables per call, and with one buffer its third upload waited on the host for
    // the second's copy, queued behind the whole elimination
    static constexpr int kTabRing = 4;
    PinBuf pin_tab[kTabRing];
    hipEvent_t tab_ev[kTabRing] = {};
    int tab_next = 0;
    // descriptor tables of calls captured into HIP graphs: bump-allocated, never reused or moved (a replay rewrites
    // exactly its captured bytes); reserved by eager calls, since nothing may be allocated inside a capture
    std::vector<std::unique_ptr<DevBuf>> cap_arenas;
    size_t cap_used = 0;
    rlnc::eng::UpSlot up[rlnc::eng::kUpSlots];
    int up_cur = 0;       // the slot being filled
    std::mutex up_mu;     // guards the ring and the upload stream
    hipStream_t up_stream = nullptr;
    // device blocks of dropped encoders / recoders / decoders, reused by the next object of a similar size: a
    // hipMalloc + hipFree pair costs 0.1-0.6 ms per object, as much as a small object's whole decode
    std::mutex blk_mu;
    std::vector<std::pair<size_t, void *>> blk;  // (bytes, block), oldest first
    size_t blk_bytes = 0;
    static constexpr size_t kBlkCacheBytes = size_t(1) << 30;
    static constexpr size_t kBlkCacheCount = 32;

    void retain() { refs.fetch_add(1, std::memory_order_relaxed); }
    void release() {
        if (refs.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
        (void)hipSetDevice(device);
        (void)hipStreamSynchronize(stream);
        for (hipStream_t x : {hs_h2d, hs_d2h})
            if (x) {
                (void)hipStreamSynchronize(x);
                (void)hipStreamDestroy(x);
            }
        hs_slots.clear();
        if (up_stream) {
            (void)hipStreamSynchronize(up_stream);
            (void)hipStreamDestroy(up_stream);
        }
        for (auto &b : blk) (void)hipFree(b.second);
        for (hipEvent_t e : tab_ev)
            if (e) (void)hipEventDestroy(e);
        if (own) (void)hipStreamDestroy(own);
        delete this;  // the buffers' destructors free on this device
    }
    int activate() const {
        HIP_TRY(hipSetDevice(device));
        return RLNC_OK;
    }
    // batch API: note a stream capture in progress (freezes the workspaces)
    int note_capture() {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        HIP_TRY(hipStreamIsCapturing(stream, &cs));
        if (cs != hipStreamCaptureStatusNone) graph_bound = true;
        return RLNC_OK;
    }
    int grow(DevBuf &b, size_t bytes) {
        if (bytes <= b.cap) return RLNC_OK;
        if (graph_bound)
            return set_error(RLNC_ERR_INVALID_ARGUMENT,
                             "this context's workspaces are bound to a captured HIP graph and cannot grow to %zu "
                             "bytes: capture the largest shape first, or use another context",
                             bytes);
        return b.ensure(bytes);
    }
    int grow(PinBuf &b, size_t bytes) {
        if (bytes <= b.cap) return RLNC_OK;
        if (graph_bound)
            return set_error(RLNC_ERR_INVALID_ARGUMENT,
                             "this context's workspaces are bound to a captured HIP graph and cannot grow");
        return b.ensure(bytes);
    }
    // an object's device block of at least n bytes (*cap = its size): a cached one when one fits (at most twice n
    // plus 1 MiB), else hipMalloc -- after emptying the cache into the device if that fails
    int obj_alloc(size_t n, uint8_t **p, size_t *cap) {
        {
            std::lock_guard<std::mutex> lock(blk_mu);
            int best = -1;
            for (int i = 0; i < int(blk.size()); ++i)
                if (blk[i].first >= n && blk[i].first <= 2 * n + (size_t(1) << 20) &&
                    (best < 0 || blk[i].first < blk[best].first))
                    best = i;
            if (best >= 0) {
                *p = static_cast<uint8_t *>(blk[best].second);
                *cap = blk[best].first;
                blk_bytes -= *cap;
                blk.erase(blk.begin() + best);
                return RLNC_OK;
            }
        }
        const size_t bytes = std::max<size_t>(n, 256);
        if (hipMalloc(reinterpret_cast<void **>(p), bytes) != hipSuccess) {
            (void)hipGetLastError();
            {
                std::lock_guard<std::mutex> lock(blk_mu);
                for (auto &b : blk) (void)hipFree(b.second);
                blk.clear();
                blk_bytes = 0;
            }
            HIP_TRY(hipMalloc(reinterpret_cast<void **>(p), bytes));
        }
        *cap = bytes;
        return RLNC_OK;
    }
    // return an object's block: once its stream-ordered uses (u; nullptr = none) have run it joins the cache; a block
    // a captured graph may still use is freed (hipFree waits for the device), as is a large one
    void obj_free(void *p, size_t cap, const rlnc::eng::ObjUse *u) {
        if (!p) return;
        if (cap > kBlkCacheBytes / 4 || (u && u->captured) || (u && u->used && hipEventSynchronize(u->ev) != hipSuccess)) {
            (void)hipFree(p);
            return;
        }
        std::lock_guard<std::mutex> lock(blk_mu);
        blk.emplace_back(cap, p);
        blk_bytes += cap;
        while (blk_bytes > kBlkCacheBytes || blk.size() > kBlkCacheCount) {
            (void)hipFree(blk.front().second);
            blk_bytes -= blk.front().first;
            blk.erase(blk.begin());
        }
    }
    int upload_stream_locked() {
        if (!up_stream) HIP_TRY(hipStreamCreateWithFlags(&up_stream, hipStreamNonBlocking));
        return RLNC_OK;
    }
    int upload_stream(hipStream_t &s) {
        std::lock_guard<std::mutex> lock(up_mu);
        if (int st = upload_stream_locked()) return st;
        s = up_stream;
        return RLNC_OK;
    }
    int upload_flush_locked(rlnc::eng::UpSlot &u) {
        if (!u.open) return RLNC_OK;
        u.open = false;
        for (const auto &r : u.runs)
            HIP_TRY(hipMemcpyAsync(r.dst, u.buf.as<uint8_t>() + r.off, r.len, hipMemcpyHostToDevice, up_stream));
        u.runs.clear();
        HIP_TRY(hipEventRecord(u.ev, up_stream));
        return RLNC_OK;
    }
    // host -> device copy of n bytes to dst through the staging ring: returns once the bytes are staged (src may then
    // be reused).  pitch >= n: the destination row's size -- a piece landing right after the previous one's row
    // joins its DMA (the pad bytes between rows are copied too).  *t = where the last byte was staged.
    int upload(uint8_t *dst, const uint8_t *src, size_t n, size_t pitch, rlnc::eng::UpTicket *t) {
        using namespace rlnc::eng;
        std::lock_guard<std::mutex> lock(up_mu);
        if (int st = upload_stream_locked()) return st;
        for (size_t o = 0; o < n; o += kUpChunk) {
            const size_t c = std::min(kUpChunk, n - o);
            const size_t span = (c == n && pitch <= kUpChunk) ? pitch : c;  // staged bytes incl. the row's pad
            UpSlot *u = &up[up_cur];
            if (!u->open || u->used + span > kUpChunk || u->runs.size() >= kUpRuns) {
                if (int st = upload_flush_locked(*u)) return st;
                up_cur = (up_cur + 1) % kUpSlots;
                u = &up[up_cur];
                if (!u->ev)
                    HIP_TRY(hipEventCreateWithFlags(&u->ev, hipEventDisableTiming));
                else
                    HIP_TRY(hipEventSynchronize(u->ev));  // the slot's last flush has read it
                if (int st = u->buf.ensure(kUpChunk)) return st;
                u->used = 0;
                u->gen += 1;
                u->open = true;
            }
            std::memcpy(u->buf.as<uint8_t>() + u->used, src + o, c);
            UpRun *last = u->runs.empty() ? nullptr : &u->runs.back();
            if (last && last->dst + last->len == dst + o && last->off + last->len == u->used)
                last->len += span;
            else
                u->runs.push_back(UpRun{dst + o, u->used, span});
            u->used += span;
            t->slot = up_cur;
            t->gen = u->gen;
        }
        return RLNC_OK;
    }
    // flush the ticket's slot if it still holds the staged piece; *ev = nullptr when nothing was ever staged
    int upload_flush(const rlnc::eng::UpTicket &t, hipEvent_t *ev) {
        *ev = nullptr;
        if (t.slot < 0) return RLNC_OK;
        std::lock_guard<std::mutex> lock(up_mu);
        rlnc::eng::UpSlot &u = up[t.slot];
        if (u.gen == t.gen)
            if (int st = upload_flush_locked(u)) return st;
        *ev = u.ev;  // this flush, or a later one of the same slot (after it on the upload stream)
        return RLNC_OK;
    }
    // order stream s after every upload up to the ticket's
    int upload_wait(const rlnc::eng::UpTicket &t, hipStream_t s) {
        hipEvent_t ev = nullptr;
        if (int st = upload_flush(t, &ev)) return st;
        if (!ev) return RLNC_OK;
        std::lock_guard<std::mutex> lock(up_mu);  // the event is not re-recorded while waited on
        HIP_TRY(hipStreamWaitEvent(s, ev, 0));
        return RLNC_OK;
    }
    int upload_sync(const rlnc::eng::UpTicket &t) {
        hipEvent_t ev = nullptr;
        if (int st = upload_flush(t, &ev)) return st;
        if (!ev) return RLNC_OK;
        HIP_TRY(hipEventSynchronize(ev));
        return RLNC_OK;
    }
    // a call workspace; ordered: after the work already enqueued on the context stream (a call that reads
    // memory the caller's stream-ordered work may still write, e.g. a borrowed device source)
    int lease(std::unique_ptr<CallWs> &ws, bool ordered = true) {
        {
            std::lock_guard<std::mutex> lock(pool_mu);
            if (!pool.empty()) {
                ws = std::move(pool.back());
                pool.pop_back();
            }
        }
        if (!ws) {
            ws.reset(new (std::nothrow) CallWs);
            if (!ws) return set_error(RLNC_ERR_OUT_OF_MEMORY, "call workspace allocation");
            HIP_TRY(hipStreamCreateWithFlags(&ws->stream, hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&ws->ev, hipEventDisableTiming));
        }
        if (!ordered) return RLNC_OK;
        HIP_TRY(hipEventRecord(ws->ev, stream));
        HIP_TRY(hipStreamWaitEvent(ws->stream, ws->ev, 0));
        return RLNC_OK;
    }
    void unlease(std::unique_ptr<CallWs> ws) {
        if (!ws) return;
        std::lock_guard<std::mutex> lock(pool_mu);
        pool.push_back(std::move(ws));
    }
    // the GF(2^8) matmul on stream s with index scratch idx (batch API: the context's; object API: the lease's)
    int matmul(rlnc::MatmulParams p, hipStream_t s, DevBuf &idx, bool batch) {
        if (max_tile_rows > 0 && p.n_out > max_tile_rows) {
            // split the output rows into launches of at most max_tile_rows rows (tuning knob)
            const int total = p.n_out;
            for (int r0 = 0; r0 < total; r0 += max_tile_rows) {
                rlnc::MatmulParams q = p;
                q.bsj_stream = nullptr;   // laid out for all the rows
                q.scan_status = nullptr;  // rows split over launches: no workgroup holds a whole object
                q.n_out = std::min(max_tile_rows, total - r0);
                q.coef = p.coef + int64_t(r0) * p.coef_row;
                q.out = p.out + int64_t(r0) * p.out_row;
                if (p.hdr) q.hdr = p.hdr + int64_t(r0) * p.hdr_row;
                if (int st = launch(q, s, idx, batch)) return st;
            }
            return RLNC_OK;
        }
        return launch(p, s, idx, batch);
    }
    int matmul(const rlnc::MatmulParams &p) { return matmul(p, stream, ws_idx, true); }
    int launch(rlnc::MatmulParams p, hipStream_t s, DevBuf &idx, bool batch) {
        const rlnc::MatmulVariant v = variant;
        p.col_run = col_run;
        const size_t need = rlnc::matmul_scratch_bytes(p, v);
        if (need)
            if (int st = batch ? grow(idx, need) : idx.ensure(need)) return st;
        HIP_TRY(rlnc::launch_matmul(p, s, v, idx.p, idx.cap));
        return RLNC_OK;
    }
};

namespace rlnc::eng {
// RAII lease of a call workspace
struct Lease {
    rlnc_context *ctx;
    std::unique_ptr<CallWs> ws;
    explicit Lease(rlnc_context *c) : ctx(c) {}
    int acquire(bool ordered = true) { return ctx->lease(ws, ordered); }
    CallWs *operator->() const { return ws.get(); }
    ~Lease() { ctx->unlease(std::move(ws)); }
};
}  // namespace rlnc::eng

struct rlnc_encoder;
namespace rlnc::eng {
// an Encoder owning the padded image img (k rows of L bytes at `stride`, hipMalloc'd; freed with the encoder)
int encoder_adopt_device(rlnc_context *ctx, uint8_t *img, size_t k, size_t L, size_t stride, rlnc_encoder **out);
}  // namespace rlnc::eng
