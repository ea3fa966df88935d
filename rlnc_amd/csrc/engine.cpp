// engine.cpp — librlnc_hip: context, Encoder / Recoder / Decoder objects and the batch API behind the
// C ABI of include/rlnc_hip.h.  Mirrors rlnc::full::{Encoder, Recoder, Decoder} (src/full/*.rs):
// same constructor validation order, same status for every error, same getters.  All GF(2^8) byte work on
// pieces runs on the device through the kernels of kernels.hip; the host only runs the k×(k+slots)
// coefficient elimination of the decoder (elimination.hpp).
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../include/rlnc_hip.h"
#include "context.hpp"
#include "elimination.hpp"
#include "gf256.hpp"
#include "host_copy.hpp"
#include "kernels.hpp"
#include "piece.hpp"

using rlnc::Elimination;
using namespace rlnc::eng;

namespace rlnc::eng {
thread_local std::string g_last_error;
}  // namespace rlnc::eng


// Encoder / Recoder / Decoder hold a reference on their context (released when the object is freed), so an
// object outlives the handle its creator held -- e.g. one built on a worker thread whose thread-local context
// has since been destroyed.
struct rlnc_encoder {
    rlnc_context *ctx = nullptr;
    size_t k = 0, L = 0, stride = 0;
    uint8_t *src = nullptr;  // k rows × stride
    size_t src_cap = 0;      // bytes of the owned block
    bool owned = false;
    rlnc::eng::ObjUse use;   // code_batch_device launches reading src
    void bind(rlnc_context *c) {
        ctx = c;
        c->retain();
    }
    ~rlnc_encoder() {
        if (owned && src) ctx->obj_free(src, src_cap, &use);
        if (ctx) ctx->release();
    }
};

struct rlnc_recoder {
    rlnc_context *ctx = nullptr;
    size_t k = 0, n = 0, full = 0, stride = 0;
    uint8_t *pieces = nullptr;  // n rows × stride (coeffs ‖ data)
    size_t pieces_cap = 0;
    rlnc::eng::ObjUse use;      // recode_batch_device launches reading pieces
    void bind(rlnc_context *c) {
        ctx = c;
        c->retain();
    }
    ~rlnc_recoder() {
        if (pieces) ctx->obj_free(pieces, pieces_cap, &use);
        if (ctx) ctx->release();
    }
};

struct rlnc_decoder {
    rlnc_context *ctx = nullptr;
    size_t k = 0, L = 0, stride = 0;
    size_t received = 0, useful = 0;
    std::unique_ptr<Elimination> elim;
    uint8_t *store = nullptr;  // slot rows × stride (received data rows still referenced by E)
    size_t store_slots = 0, store_cap = 0;
    // the context's upload-ring slot of the last upload into store (Decoder::decode returns once its piece is staged,
    // before the DMA): every later use of store, on whichever stream, is ordered after it
    rlnc::eng::UpTicket up;
    void bind(rlnc_context *c) {
        ctx = c;
        c->retain();
    }
    int order(hipStream_t s) const { return ctx->upload_wait(up, s); }
    ~rlnc_decoder() {
        // every other use of the store is synchronous (decode_device, get_decoded_data*, clone): the uploads only
        (void)ctx->upload_sync(up);
        if (store) ctx->obj_free(store, store_cap, nullptr);
        if (ctx) ctx->release();
    }
};

namespace {

int matmul_desc_to_params(const rlnc_matmul_desc *d, rlnc::MatmulParams &p) {
    p.in = d->in;
    p.in_obj = d->in_obj_stride;
    p.in_row = d->in_row_stride;
    p.coef = d->coef;
    p.coef_obj = d->coef_obj_stride;
    p.coef_row = d->coef_row_stride;
    p.out = d->out;
    p.out_obj = d->out_obj_stride;
    p.out_row = d->out_row_stride;
    p.hdr = d->hdr;
    p.hdr_obj = d->hdr_obj_stride;
    p.hdr_row = d->hdr_row_stride;
    p.n_out = d->n_out;
    p.n_in = d->n_in;
    p.width = d->width;
    p.n_obj = d->n_obj;
    return RLNC_OK;
}

// n coded pieces of one encoder: out[i][0:L) = Σ_j cv[i][j] · src_j  (cv already on the device)
rlnc::MatmulParams encoder_params(const rlnc_encoder *e, const uint8_t *cv_dev, int64_t cv_row, int n,
                                  uint8_t *out_dev, int64_t out_row, uint8_t *hdr_dev, int64_t hdr_row) {
    rlnc::MatmulParams p{};
    p.in = e->src;
    p.in_row = int64_t(e->stride);
    p.coef = cv_dev;
    p.coef_row = cv_row;
    p.out = out_dev;
    p.out_row = out_row;
    p.hdr = hdr_dev;
    p.hdr_row = hdr_row;
    p.n_out = n;
    p.n_in = int(e->k);
    p.width = int64_t(e->L);
    p.n_obj = 1;
    return p;
}

// ---- the call-latency path of the object API (piece.hip) ----------------------------------------------------------
// Encoder::code_with_buf / Recoder::recode_with_buf / Decoder::get_decoded_data take it up to this much output (a
// pooled workspace keeps a coherent pinned output buffer as large as the largest piece it produced), the decoder up to
// this many multiply-adds too (the kernel reads every
// source chunk once per output row, so larger products go to the batch kernels instead; its 16-byte write-through
// stores across PCIe run at ~10 GB/s, so outputs of many MiB come back faster as one DMA: 16 MiB objects 0.63 ms that
// way against 0.92 through the kernel, 1 MiB objects 0.11 ms against 0.22 -- profiles/r04_object_api_bench_full_v1)
constexpr size_t kPieceMaxBytes = size_t(4) << 20;
constexpr size_t kPieceDecodeMaxMacs = size_t(1) << 31;

// rows of `width` bytes at a 16-byte-aligned stride with room for the last slot's whole 16 bytes
bool piece_eligible(const uint8_t *in, size_t in_row, size_t width) {
    static const bool off = [] {
        const char *e = getenv("RLNC_PIECE");  // A/B knob, read once: RLNC_PIECE=0 keeps the round-3 path
        return e && atoi(e) == 0;
    }();
    return !off && (reinterpret_cast<uintptr_t>(in) & 15) == 0 && (in_row & 15) == 0 && in_row >= round16(width);
}

int piece_waves_for(int n_in) {
    static const int forced = [] {
        const char *e = getenv("RLNC_PIECE_WAVES");  // A/B knob, read once
        return e ? atoi(e) : 0;
    }();
    return forced ? forced : rlnc::piece_waves(n_in);
}

// Spin until the kernel raises *f to epoch.  The stream is queried only once the wait is long (a faulted kernel never
// raises its flag: hipStreamQuery then reports the error).
int piece_wait(const uint32_t *f, uint32_t epoch, hipStream_t s) {
    if (__atomic_load_n(f, __ATOMIC_ACQUIRE) == epoch) return RLNC_OK;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1;; ++i) {
        if (__atomic_load_n(f, __ATOMIC_ACQUIRE) == epoch) return RLNC_OK;
        __builtin_ia32_pause();
        if ((i & 4095) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipErrorNotReady) continue;
            if (__atomic_load_n(f, __ATOMIC_ACQUIRE) == epoch) return RLNC_OK;
            if (q == hipSuccess) return set_error(RLNC_ERR_DEVICE, "piece kernel finished without raising its flag");
            return set_error(RLNC_ERR_DEVICE, "piece kernel: %s", hipGetErrorString(q));
        }
    }
}

// RLNC_PIECE_TRACE=1 (diagnostic, read once): per-phase host time of the piece calls, averaged, on stderr at exit
struct PieceTrace {
    bool on = [] {
        const char *e = getenv("RLNC_PIECE_TRACE");
        return e && atoi(e) != 0;
    }();
    std::mutex mu;
    std::vector<float> pre, launch, first, rest;  // per call, us
    void add(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
        std::lock_guard<std::mutex> lock(mu);
        pre.push_back(a / 1e3f);
        launch.push_back(b / 1e3f);
        first.push_back(c / 1e3f);
        rest.push_back(d / 1e3f);
    }
    static float med(std::vector<float> v) {
        if (v.empty()) return 0.f;
        std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
        return v[v.size() / 2];
    }
    ~PieceTrace() {
        if (on && !pre.empty())
            std::fprintf(stderr, "{\"piece_trace\": {\"calls\": %zu, \"median_pre_us\": %.2f, \"median_launch_us\": %.2f, "
                                 "\"median_to_first_flag_us\": %.2f, \"median_copies_and_rest_us\": %.2f}}\n",
                         pre.size(), med(pre), med(launch), med(first), med(rest));
    }
};
PieceTrace g_piece_trace;
inline uint64_t now_ns() {
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now().time_since_epoch()).count());
}

bool piece_inline() {
    static const bool on = [] {
        const char *e = getenv("RLNC_PIECE_INLINE");  // A/B knob, read once: 0 = coefficients always from pinned memory
        return !e || atoi(e) != 0;
    }();
    return on;
}

constexpr size_t kGridUploadMax = size_t(8) << 20;  // Recoder::new uploads up to this many bytes by the grid kernel

bool grid_upload() {
    static const bool on = [] {
        const char *e = getenv("RLNC_GRID_UPLOAD");  // A/B knob, read once: 0 = the DMA upload for every object
        return !e || atoi(e) != 0;
    }();
    return on;
}

bool obj_warm() {
    static const bool on = [] {
        const char *e = getenv("RLNC_OBJ_WARM");
        return e && atoi(e) != 0;
    }();
    return on;
}

int piece_chunk_blocks() {
    static const int c = [] {
        const char *e = getenv("RLNC_PIECE_CHUNK");  // A/B knob, read once: workgroups per completion flag
        return e ? std::max(1, atoi(e)) : 64;
    }();
    return c;
}

bool piece_chunk_forced() {
    static const bool f = getenv("RLNC_PIECE_CHUNK") != nullptr;
    return f;
}

// Waves of a column-split workgroup (piece.hpp col_waves: each wave owns 1 KiB of columns and walks every source), or
// 0 for the source-split form.  RLNC_PIECE_COLW (A/B knob, read once): W = column-split with W waves for every call
// that does not split its sources over workgroups, 0 / unset = the source-split form
int piece_col_waves() {
    static const int forced = [] {
        const char *e = getenv("RLNC_PIECE_COLW");
        const int w = e ? atoi(e) : 0;
        return (w == 1 || w == 2 || w == 4 || w == 8 || w == 16) ? w : 0;
    }();
    return forced;
}

// out rows r < n_out: dst[r·dst_row + 0 : width) = XOR_j coef[r·coef_row + j] · in[j·in_row + 0 : width), j < n_in.
// coef: host memory; one row of at most kPieceInline bytes travels in the kernel arguments, more are read by the kernel
// from ws->pc_coef (coef may already point there).  Synchronous: returns once dst holds every row.
// workgroups per (row, column block) of the call-latency kernel: rlnc::piece_split, or RLNC_PIECE_SPLIT (A/B knob,
// read once: 1 = never split, n = n workgroups whenever n_in > 64; 0 / unset = rlnc::piece_split)
int piece_split_for(int n_in, int64_t blocks) {
    static const int forced = [] {
        const char *e = getenv("RLNC_PIECE_SPLIT");
        return e ? std::max(0, atoi(e)) : 0;
    }();
    if (forced == 1) return 1;
    if (forced > 1) return n_in > 64 ? std::min(forced, 32) : 1;
    return rlnc::piece_split(n_in, blocks);
}

int piece_call(CallWs *ws, const uint8_t *in, size_t in_row, size_t n_in, size_t width, const uint8_t *coef,
               size_t coef_row, size_t n_out, uint8_t *dst, size_t dst_row) {
    const uint64_t t0 = g_piece_trace.on ? now_ns() : 0;
    rlnc::PieceParams p{};
    p.in = in;
    p.in_row = int64_t(in_row);
    p.coef_row = int64_t(coef_row);
    if (n_out == 1 && n_in <= size_t(rlnc::kPieceInline) && piece_inline()) {
        p.coef = nullptr;
        std::memcpy(p.coef_inline, coef, n_in);
    } else {
        if (int st = ws->pc_coef.ensure(n_out * coef_row)) return st;
        if (coef != ws->pc_coef.as<uint8_t>()) std::memcpy(ws->pc_coef.p, coef, n_out * coef_row);
        p.coef = ws->pc_coef.as<uint8_t>();
    }
    p.out_row = int64_t(round16(width));
    p.width = int64_t(width);
    p.n_in = int(n_in);
    p.n_out = int(n_out);
    const int64_t gx = (p.width + rlnc::kPieceCols - 1) / rlnc::kPieceCols;
    p.split = piece_split_for(p.n_in, gx * int64_t(n_out));
    const int colw = p.split == 1 ? piece_col_waves() : 0;  // measured slower: off unless forced
    p.col_waves = colw ? 1 : 0;
    const int waves = colw ? colw : piece_waves_for((p.n_in + p.split - 1) / p.split);
    p.chunk_blocks = piece_chunk_blocks();  // 64 KiB of a row per flag: the host copies one while the device writes on
    if (colw && !piece_chunk_forced()) p.chunk_blocks = std::max(1, p.chunk_blocks / colw);
    const size_t chunks = size_t(rlnc::piece_chunks(p, waves));
    if (int st = ws->pc_out.ensure(n_out * size_t(p.out_row))) return st;
    if (chunks * 4 > ws->pc_flag.cap) {
        // completion is "flag == epoch" and every workspace counts its epochs from 1: a freshly allocated pinned
        // buffer may hold another (freed) workspace's flag values, so it starts zeroed (epochs are never 0)
        if (int st = ws->pc_flag.ensure(chunks * 4)) return st;
        std::memset(ws->pc_flag.p, 0, ws->pc_flag.cap);
    }
    if (chunks > ws->pc_count_words) {
        if (int st = ws->pc_count.ensure(chunks * 4)) return st;
        HIP_TRY(hipMemsetAsync(ws->pc_count.p, 0, chunks * 4, ws->stream));
        ws->pc_count_words = chunks;
    }
    if (p.split > 1) {
        const size_t blocks = size_t(gx) * n_out;
        if (int st = ws->pc_part.ensure(blocks * size_t(p.split) * 64 * 16)) return st;
        if (blocks > ws->pc_pcount_words) {
            if (int st = ws->pc_pcount.ensure(blocks * 4)) return st;
            HIP_TRY(hipMemsetAsync(ws->pc_pcount.p, 0, blocks * 4, ws->stream));
            ws->pc_pcount_words = blocks;
        }
        p.part = ws->pc_part.as<uint4>();
        p.pcount = ws->pc_pcount.as<uint32_t>();
    }
    p.out = ws->pc_out.as<uint8_t>();
    p.count = ws->pc_count.as<uint32_t>();
    p.flag = ws->pc_flag.as<uint32_t>();
    if (++ws->epoch == 0) ws->epoch = 1;
    p.epoch = ws->epoch;
    const uint64_t t1 = g_piece_trace.on ? now_ns() : 0;
    HIP_TRY(rlnc::launch_piece(p, waves, ws->stream));
    const uint64_t t2 = g_piece_trace.on ? now_ns() : 0;
    uint64_t t3 = 0;
    const size_t chunk_bytes = size_t(p.chunk_blocks) * size_t(rlnc::piece_cols_per_wg(p, waves));
    const size_t cpr = chunks / n_out;
    for (size_t c = 0; c < chunks; ++c) {
        if (int st = piece_wait(p.flag + c, p.epoch, ws->stream)) {
            // a failed launch may leave counters part-way: wait for the stream and re-arm them
            (void)hipStreamSynchronize(ws->stream);
            ws->pc_count_words = 0;
            ws->pc_pcount_words = 0;
            return st;
        }
        if (c == 0 && g_piece_trace.on) t3 = now_ns();
        const size_t r = c / cpr, c0 = (c % cpr) * chunk_bytes, c1 = std::min(width, c0 + chunk_bytes);
        std::memcpy(dst + r * dst_row + c0, p.out + r * size_t(p.out_row) + c0, c1 - c0);
    }
    if (g_piece_trace.on) g_piece_trace.add(t1 - t0, t2 - t1, t3 - t2, now_ns() - t3);
    return RLNC_OK;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------------------------------------------------
// status text — errors.rs:3-58
// ------------------------------------------------------------------------------------------------------
const char *rlnc_status_name(int s) {
    static const char *names[] = {"Ok",
                                  "CodingVectorLengthMismatch",
                                  "DataLengthMismatch",
                                  "PieceCountZero",
                                  "DataLengthZero",
                                  "PieceLengthZero",
                                  "NotEnoughPiecesToRecode",
                                  "PieceLengthTooShort",
                                  "PieceNotUseful",
                                  "ReceivedAllPieces",
                                  "NotAllPiecesReceivedYet",
                                  "InvalidDecodedDataFormat",
                                  "InvalidPieceLength",
                                  "InvalidOutputBuffer"};
    if (s >= 0 && s <= 13) return names[s];
    switch (s) {
    case RLNC_ERR_INVALID_ARGUMENT: return "InvalidArgument";
    case RLNC_ERR_DEVICE: return "DeviceError";
    case RLNC_ERR_OUT_OF_MEMORY: return "OutOfMemory";
    case RLNC_ERR_NO_DEVICE: return "NoDevice";
    default: return "Unknown";
    }
}

const char *rlnc_status_message(int s) {
    static const char *msgs[] = {"Ok",
                                 "Coding vector length mismatch",
                                 "Data length mismatch",
                                 "Piece count is zero",
                                 "Data length is zero",
                                 "Piece length is zero",
                                 "Not enough pieces received to recode",
                                 "Piece length is too short",
                                 "Received piece is not useful",
                                 "Received all pieces",
                                 "Not all pieces are received yet",
                                 "Invalid decoded data format",
                                 "Invalid piece length",
                                 "Invalid output buffer"};
    if (s >= 0 && s <= 13) return msgs[s];
    return rlnc_status_name(s);
}

const char *rlnc_last_error(void) { return g_last_error.c_str(); }
const char *rlnc_version(void) { return "rlnc_hip 0.1.0 (gfx950; reference itzmeanjan/rlnc 0.8.5)"; }

// ------------------------------------------------------------------------------------------------------
// context
// ------------------------------------------------------------------------------------------------------
int rlnc_context_create(int device, rlnc_context **out) {
    CHECK_ARG(out != nullptr);
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return set_error(RLNC_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= count) return set_error(RLNC_ERR_NO_DEVICE, "device %d out of range (%d)", device, count);
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_error(RLNC_ERR_NO_DEVICE, "device %d is %s, librlnc_hip is built for gfx950 only", device,
                         prop.gcnArchName);
    (void)rlnc::probe_unaligned_vector_access(device);  // once per device: rows at any byte alignment on the vector path
    auto *c = new (std::nothrow) rlnc_context;
    if (!c) return set_error(RLNC_ERR_OUT_OF_MEMORY, "context allocation");
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return set_error(RLNC_ERR_DEVICE, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    c->stream = c->own;
    *out = c;
    return RLNC_OK;
}

// Drops the creator's reference; the context lives on while objects bound to it exist.
void rlnc_context_destroy(rlnc_context *ctx) {
    if (ctx) ctx->release();
}

int rlnc_context_set_stream(rlnc_context *ctx, void *s) {
    CHECK_ARG(ctx != nullptr);
    ctx->stream = static_cast<hipStream_t>(s);
    return RLNC_OK;
}

int rlnc_context_use_own_stream(rlnc_context *ctx) {
    CHECK_ARG(ctx != nullptr);
    ctx->stream = ctx->own;
    return RLNC_OK;
}

void *rlnc_context_get_stream(rlnc_context *ctx) { return ctx ? ctx->stream : nullptr; }
int rlnc_context_device(const rlnc_context *ctx) { return ctx ? ctx->device : -1; }
int rlnc_device_unaligned_vector_access(int device) { return rlnc::unaligned_vector_access(device); }

int rlnc_stream_is_capturing(void *hip_stream, int *capturing) {
    CHECK_ARG(capturing != nullptr);
    *capturing = 1;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const hipError_t e = hipStreamIsCapturing(static_cast<hipStream_t>(hip_stream), &cs);
    if (e != hipSuccess)
        return set_error(RLNC_ERR_DEVICE, "hipStreamIsCapturing: %s", hipGetErrorString(e));
    *capturing = cs != hipStreamCaptureStatusNone;
    return RLNC_OK;
}

int rlnc_context_synchronize(rlnc_context *ctx) {
    CHECK_ARG(ctx != nullptr);
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return RLNC_OK;
}

// Shipped decode paths: 0 auto, 1 host, 2 device, 5 device blocked run; 3, 4 and 6 (the round-1 LDS / register
// forms) exist in the diagnostic build only (make -C rlnc_amd/csrc ab: rref_ab.hip).
int rlnc_set_decode_path(rlnc_context *ctx, int path) {
    CHECK_ARG(ctx != nullptr && (path == 0 || path == 1 || path == 2 || path == 5 ||
                                 (rlnc::ab_build() && (path == 3 || path == 4 || path == 6))));
    ctx->decode_path = path;
    return RLNC_OK;
}

int rlnc_set_kernel_variant(rlnc_context *ctx, int variant, int max_tile_rows) {
    CHECK_ARG(ctx != nullptr);
    // shipped: 0 perm, 1 nibble (the reference's tables, ablation), 6 (the unshared bit-sliced program, which also
    // serves <= 16-row products and a first use inside a graph capture), 7 and 8 (the bit-sliced default); 2-5 and 9
    // are the A/B history, in the diagnostic build only (kernels_ab.hip)
    CHECK_ARG(variant == 0 || variant == 1 || variant == 6 || variant == 7 || variant == 8 ||
              (rlnc::ab_build() && variant >= 2 && variant <= 9));
    CHECK_ARG(max_tile_rows == 0 || max_tile_rows == 1 || max_tile_rows == 2 || max_tile_rows == 4 ||
              max_tile_rows == 8 || max_tile_rows == 16 || max_tile_rows == 32);
    ctx->variant = static_cast<rlnc::MatmulVariant>(variant);
    ctx->max_tile_rows = max_tile_rows;
    return RLNC_OK;
}

int rlnc_set_column_run(rlnc_context *ctx, int col_run) {
    CHECK_ARG(ctx != nullptr);
    CHECK_ARG(col_run >= 0 && col_run <= 64);
    ctx->col_run = col_run;
    return RLNC_OK;
}

// ------------------------------------------------------------------------------------------------------
// L1 primitives — simd/mod.rs:18-119 (early-outs on the host, exactly as the reference)
// ------------------------------------------------------------------------------------------------------
int rlnc_gf256_inplace_mul_vec_by_scalar(rlnc_context *ctx, uint8_t *vec, size_t len, uint8_t scalar) {
    CHECK_ARG(ctx != nullptr);
    if (len == 0) return RLNC_OK;  // :19-21
    CHECK_ARG(vec != nullptr);
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    if (scalar == 0) {  // :22-25
        HIP_TRY(hipMemsetAsync(vec, 0, len, ctx->stream));
        return RLNC_OK;
    }
    if (scalar == 1) return RLNC_OK;  // :26-28
    HIP_TRY(rlnc::launch_mul_vec_by_scalar(vec, int64_t(len), scalar, ctx->stream));
    return RLNC_OK;
}

int rlnc_gf256_inplace_add_vectors(rlnc_context *ctx, uint8_t *dst, const uint8_t *src, size_t len) {
    CHECK_ARG(ctx != nullptr);
    if (len == 0) return RLNC_OK;
    CHECK_ARG(dst != nullptr && src != nullptr);
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    HIP_TRY(rlnc::launch_add_vectors(dst, src, int64_t(len), ctx->stream));
    return RLNC_OK;
}

int rlnc_gf256_mul_vec_by_scalar_then_add_into_vec(rlnc_context *ctx, uint8_t *dst, const uint8_t *src, size_t len,
                                                   uint8_t scalar) {
    CHECK_ARG(ctx != nullptr);
    if (len == 0) return RLNC_OK;  // :90-92
    if (scalar == 0) return RLNC_OK;  // :93-95
    CHECK_ARG(dst != nullptr && src != nullptr);
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    if (scalar == 1) {  // :96-99
        HIP_TRY(rlnc::launch_add_vectors(dst, src, int64_t(len), ctx->stream));
        return RLNC_OK;
    }
    HIP_TRY(rlnc::launch_mul_add(dst, src, int64_t(len), scalar, ctx->stream));
    return RLNC_OK;
}

int rlnc_gf256_matmul(rlnc_context *ctx, const rlnc_matmul_desc *desc) {
    CHECK_ARG(ctx != nullptr && desc != nullptr);
    CHECK_ARG(desc->n_out >= 0 && desc->n_in >= 0 && desc->width >= 0 && desc->n_obj >= 0);
    if (desc->n_out == 0 || desc->width == 0 || desc->n_obj == 0) return RLNC_OK;
    CHECK_ARG(desc->n_in > 0 && desc->in && desc->coef && desc->out);
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    rlnc::MatmulParams p;
    matmul_desc_to_params(desc, p);
    return ctx->matmul(p);
}

// ------------------------------------------------------------------------------------------------------
// Encoder — encoder.rs
// ------------------------------------------------------------------------------------------------------
static int encoder_from_host(rlnc_context *ctx, const uint8_t *data, size_t len, size_t k, bool pad, rlnc_encoder **out) {
    CHECK_ARG(ctx != nullptr && out != nullptr);
    *out = nullptr;
    if (len == 0) return RLNC_ERR_DATA_LENGTH_ZERO;  // encoder.rs:86-88 / :51-53
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;    // :89-91 / :54-56
    CHECK_ARG(data != nullptr);
    size_t L;
    if (pad) {
        L = (len + 1 + k - 1) / k;  // :93-95
    } else {
        L = len / k;
        if (L * k != len) return RLNC_ERR_DATA_LENGTH_MISMATCH;  // :58-64
    }
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    std::unique_ptr<rlnc_encoder> e(new (std::nothrow) rlnc_encoder);
    if (!e) return set_error(RLNC_ERR_OUT_OF_MEMORY, "encoder allocation");
    e->bind(ctx);
    e->k = k;
    e->L = L;
    e->stride = round16(L);
    e->owned = true;
    if ((st = ctx->obj_alloc(k * e->stride, &e->src, &e->src_cap))) return st;
    Lease ws(ctx);
    if ((st = ws.acquire())) return st;
    // padded image: data, 0x81 marker, zeros (encoder.rs:98-99), laid out at a 16-B row stride
    if ((st = ws->pin_a.ensure(k * e->stride))) return st;
    uint8_t *h = ws->pin_a.as<uint8_t>();
    std::memset(h, 0, k * e->stride);
    for (size_t r = 0; r < k; ++r) {
        const size_t off = r * L;
        if (off < len) std::memcpy(h + r * e->stride, data + off, std::min(L, len - off));
    }
    if (pad) h[(len / L) * e->stride + (len % L)] = rlnc::kBoundaryMarker;
    HIP_TRY(hipMemcpyAsync(e->src, h, k * e->stride, hipMemcpyHostToDevice, ws->stream));
    HIP_TRY(hipStreamSynchronize(ws->stream));
    *out = e.release();
    return RLNC_OK;
}

int rlnc_encoder_new(rlnc_context *ctx, const uint8_t *data, size_t len, size_t k, rlnc_encoder **out) {
    return encoder_from_host(ctx, data, len, k, true, out);
}

int rlnc_encoder_without_padding(rlnc_context *ctx, const uint8_t *data, size_t len, size_t k, rlnc_encoder **out) {
    return encoder_from_host(ctx, data, len, k, false, out);
}

int rlnc_encoder_from_device(rlnc_context *ctx, const uint8_t *pieces, size_t k, size_t L, size_t row_stride,
                             rlnc_encoder **out) {
    CHECK_ARG(ctx != nullptr && out != nullptr);
    *out = nullptr;
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
    if (L == 0) return RLNC_ERR_DATA_LENGTH_ZERO;
    CHECK_ARG(pieces != nullptr && row_stride >= L);
    auto *e = new (std::nothrow) rlnc_encoder;
    if (!e) return set_error(RLNC_ERR_OUT_OF_MEMORY, "encoder allocation");
    e->bind(ctx);
    e->k = k;
    e->L = L;
    e->stride = row_stride;
    e->src = const_cast<uint8_t *>(pieces);
    e->owned = false;
    *out = e;
    return RLNC_OK;
}

}  // extern "C"

int rlnc::eng::encoder_adopt_device(rlnc_context *ctx, uint8_t *img, size_t k, size_t L, size_t stride,
                                    rlnc_encoder **out) {
    auto *e = new (std::nothrow) rlnc_encoder;
    if (!e) return set_error(RLNC_ERR_OUT_OF_MEMORY, "encoder allocation");
    e->bind(ctx);
    e->k = k;
    e->L = L;
    e->stride = stride;
    e->src = img;
    e->src_cap = k * stride;
    e->owned = true;
    *out = e;
    return RLNC_OK;
}

extern "C" {

// #[derive(Clone)] (encoder.rs:18): an owned source is copied; a borrowed device source stays borrowed
int rlnc_encoder_clone(const rlnc_encoder *e, rlnc_encoder **out) {
    CHECK_ARG(e != nullptr && out != nullptr);
    *out = nullptr;
    int st = e->ctx->activate();
    if (st) return st;
    std::unique_ptr<rlnc_encoder> c(new (std::nothrow) rlnc_encoder);
    if (!c) return set_error(RLNC_ERR_OUT_OF_MEMORY, "encoder allocation");
    c->bind(e->ctx);
    c->k = e->k;
    c->L = e->L;
    c->stride = e->stride;
    c->owned = e->owned;
    if (e->owned) {
        if ((st = e->ctx->obj_alloc(e->k * e->stride, &c->src, &c->src_cap))) return st;
        Lease ws(e->ctx);
        if ((st = ws.acquire())) return st;
        HIP_TRY(hipMemcpyAsync(c->src, e->src, e->k * e->stride, hipMemcpyDeviceToDevice, ws->stream));
        HIP_TRY(hipStreamSynchronize(ws->stream));
    } else {
        c->src = e->src;
    }
    *out = c.release();
    return RLNC_OK;
}

void rlnc_encoder_free(rlnc_encoder *e) { delete e; }
size_t rlnc_encoder_get_piece_count(const rlnc_encoder *e) { return e ? e->k : 0; }
size_t rlnc_encoder_get_piece_byte_len(const rlnc_encoder *e) { return e ? e->L : 0; }
size_t rlnc_encoder_get_full_coded_piece_byte_len(const rlnc_encoder *e) { return e ? e->k + e->L : 0; }

// Thread-safe on one encoder (the reference's code(&self) on a Send + Sync Encoder): each call leases its own
// stream and buffers.
int rlnc_encoder_code_with_coding_vector(rlnc_encoder *e, const uint8_t *cv, size_t cv_len, uint8_t *coded,
                                         size_t coded_len) {
    CHECK_ARG(e != nullptr);
    if (cv_len != e->k) return RLNC_ERR_CODING_VECTOR_LENGTH_MISMATCH;  // encoder.rs:129-131
    if (coded_len != e->L) return RLNC_ERR_INVALID_OUTPUT_BUFFER;       // :132-134
    CHECK_ARG(cv != nullptr && coded != nullptr);
    rlnc_context *ctx = e->ctx;
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    Lease ws(ctx);
    if (e->L <= kPieceMaxBytes && piece_eligible(e->src, e->stride, e->L)) {
        // an owned source is immutable after Encoder::new (its upload synchronised); a borrowed one is ordered after
        // the context stream's work
        if ((st = ws.acquire(!e->owned))) return st;
        return piece_call(ws.ws.get(), e->src, e->stride, e->k, e->L, cv, e->k, 1, coded, e->L);
    }
    if ((st = ws.acquire())) return st;
    if ((st = ws->coef.ensure(e->k)) || (st = ws->out.ensure(e->L))) return st;
    HIP_TRY(hipMemcpyAsync(ws->coef.p, cv, e->k, hipMemcpyHostToDevice, ws->stream));
    const auto p = encoder_params(e, ws->coef.as<uint8_t>(), int64_t(e->k), 1, ws->out.as<uint8_t>(), int64_t(e->L),
                                  nullptr, 0);
    if ((st = ctx->matmul(p, ws->stream, ws->idx, false))) return st;
    HIP_TRY(hipMemcpyAsync(coded, ws->out.p, e->L, hipMemcpyDeviceToHost, ws->stream));
    HIP_TRY(hipStreamSynchronize(ws->stream));
    return RLNC_OK;
}

int rlnc_encoder_code_with_buf(rlnc_encoder *e, const uint8_t *rnd, size_t n_rnd, uint8_t *full, size_t full_len) {
    CHECK_ARG(e != nullptr);
    if (full_len != e->k + e->L) return RLNC_ERR_INVALID_OUTPUT_BUFFER;  // encoder.rs:242-244
    if (n_rnd != e->k) return RLNC_ERR_CODING_VECTOR_LENGTH_MISMATCH;    // fill_bytes fills exactly k bytes
    CHECK_ARG(rnd != nullptr && full != nullptr);
    std::memmove(full, rnd, e->k);  // :246-248
    return rlnc_encoder_code_with_coding_vector(e, full, e->k, full + e->k, e->L);
}

int rlnc_encoder_code_batch_device(rlnc_encoder *e, const uint8_t *coeffs_dev, size_t n, uint8_t *out_dev,
                                   size_t out_row_stride) {
    CHECK_ARG(e != nullptr);
    if (n == 0) return RLNC_OK;
    CHECK_ARG(coeffs_dev != nullptr && out_dev != nullptr && n <= 0x7FFFFFFF);
    const size_t row = out_row_stride ? out_row_stride : e->k + e->L;
    CHECK_ARG(row >= e->k + e->L);
    int st = e->ctx->activate();
    if (st || (st = e->ctx->note_capture())) return st;
    if ((st = e->ctx->matmul(encoder_params(e, coeffs_dev, int64_t(e->k), int(n), out_dev + e->k, int64_t(row), out_dev,
                                            int64_t(row)))))
        return st;
    return e->owned ? e->use.note(e->ctx->stream) : RLNC_OK;
}

// ------------------------------------------------------------------------------------------------------
// Recoder — recoder.rs
// ------------------------------------------------------------------------------------------------------
int rlnc_recoder_new(rlnc_context *ctx, const uint8_t *data, size_t len, size_t full, size_t k, rlnc_recoder **out) {
    CHECK_ARG(ctx != nullptr && out != nullptr);
    *out = nullptr;
    if (len == 0) return RLNC_ERR_NOT_ENOUGH_PIECES_TO_RECODE;  // recoder.rs:69-71
    if (full == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;            // :72-74
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;                // :75-77
    if (full <= k) return RLNC_ERR_PIECE_LENGTH_TOO_SHORT;       // :78-80
    const size_t n = len / full;                                 // :83 (trailing bytes ignored, :88)
    if (n == 0) return RLNC_ERR_NOT_ENOUGH_PIECES_TO_RECODE;     // reference: UB (unwrap_unchecked, :97)
    CHECK_ARG(data != nullptr && n <= 0x7FFFFFFF);
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    std::unique_ptr<rlnc_recoder> r(new (std::nothrow) rlnc_recoder);
    if (!r) return set_error(RLNC_ERR_OUT_OF_MEMORY, "recoder allocation");
    r->bind(ctx);
    r->k = k;
    r->n = n;
    r->full = full;
    r->stride = round16(full);
    if ((st = ctx->obj_alloc(n * r->stride, &r->pieces, &r->pieces_cap))) return st;
    Lease ws(ctx);
    if ((st = ws.acquire())) return st;
    if (full % 16 == 0 && full <= kPieceMaxBytes && n * full <= kGridUploadMax && grid_upload() &&
        piece_eligible(r->pieces, r->stride, full)) {
        // small objects: staged through the lease's pinned buffer and copied by a kernel on the recode call's grid, so
        // the recode calls that follow find the pieces in the reading XCDs' L2 (piece.hip piece_upload_kernel)
        if ((st = ws->pc_coef.ensure(n * full))) return st;
        std::memcpy(ws->pc_coef.p, data, n * full);
        HIP_TRY(rlnc::launch_piece_upload(ws->pc_coef.as<uint8_t>(), int64_t(full), r->pieces, int64_t(r->stride),
                                          int64_t(full), int(n), ws->stream));
    } else {
        HIP_TRY(hipMemcpy2DAsync(r->pieces, r->stride, data, full, full, n, hipMemcpyHostToDevice, ws->stream));
    }
    HIP_TRY(hipStreamSynchronize(ws->stream));
    if (obj_warm() && full <= kPieceMaxBytes && piece_eligible(r->pieces, r->stride, full)) {
        // A/B knob RLNC_OBJ_WARM=1: one throwaway call-kernel pass over the fresh pieces (zero coefficients, the recode
        // call's grid, so each workgroup's lines land in the L2 of the XCD that will read them)
        std::vector<uint8_t> zc(n, 0), scratch(full);
        if ((st = piece_call(ws.ws.get(), r->pieces, r->stride, n, full, zc.data(), n, 1, scratch.data(), full))) return st;
    }
    *out = r.release();
    return RLNC_OK;
}

// #[derive(Clone)] (recoder.rs:12)
int rlnc_recoder_clone(const rlnc_recoder *r, rlnc_recoder **out) {
    CHECK_ARG(r != nullptr && out != nullptr);
    *out = nullptr;
    int st = r->ctx->activate();
    if (st) return st;
    std::unique_ptr<rlnc_recoder> c(new (std::nothrow) rlnc_recoder);
    if (!c) return set_error(RLNC_ERR_OUT_OF_MEMORY, "recoder allocation");
    c->bind(r->ctx);
    c->k = r->k;
    c->n = r->n;
    c->full = r->full;
    c->stride = r->stride;
    if ((st = r->ctx->obj_alloc(r->n * r->stride, &c->pieces, &c->pieces_cap))) return st;
    Lease ws(r->ctx);
    if ((st = ws.acquire())) return st;
    HIP_TRY(hipMemcpyAsync(c->pieces, r->pieces, r->n * r->stride, hipMemcpyDeviceToDevice, ws->stream));
    HIP_TRY(hipStreamSynchronize(ws->stream));
    *out = c.release();
    return RLNC_OK;
}

void rlnc_recoder_free(rlnc_recoder *r) { delete r; }
size_t rlnc_recoder_get_original_num_pieces_coded_together(const rlnc_recoder *r) { return r ? r->k : 0; }
size_t rlnc_recoder_get_num_pieces_recoded_together(const rlnc_recoder *r) { return r ? r->n : 0; }
size_t rlnc_recoder_get_piece_byte_len(const rlnc_recoder *r) { return r ? r->full - r->k : 0; }
size_t rlnc_recoder_get_full_coded_piece_byte_len(const rlnc_recoder *r) { return r ? r->full : 0; }

static rlnc::MatmulParams recoder_params(const rlnc_recoder *r, const uint8_t *r_dev, int count, uint8_t *out_dev,
                                         int64_t out_row) {
    // recoded piece = Σ_i r_i · (coeffs_i ‖ data_i): the coefficient fold of recoder.rs:133-144 and the
    // data combination of :146-150 are the same linear map applied to different columns
    rlnc::MatmulParams p{};
    p.in = r->pieces;
    p.in_row = int64_t(r->stride);
    p.coef = r_dev;
    p.coef_row = int64_t(r->n);
    p.out = out_dev;
    p.out_row = out_row;
    p.n_out = count;
    p.n_in = int(r->n);
    p.width = int64_t(r->full);
    p.n_obj = 1;
    return p;
}

int rlnc_recoder_recode_with_buf(rlnc_recoder *r, const uint8_t *rnd, size_t n_rnd, uint8_t *full, size_t full_len) {
    CHECK_ARG(r != nullptr);
    if (full_len != r->full) return RLNC_ERR_INVALID_OUTPUT_BUFFER;  // recoder.rs:123-125
    if (n_rnd != r->n) return RLNC_ERR_CODING_VECTOR_LENGTH_MISMATCH;  // fill_bytes fills exactly n bytes
    CHECK_ARG(rnd != nullptr && full != nullptr);
    rlnc_context *ctx = r->ctx;
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    Lease ws(ctx);
    if (r->full <= kPieceMaxBytes && piece_eligible(r->pieces, r->stride, r->full)) {
        // the received pieces are immutable after Recoder::new (its upload synchronised): no ordering
        if ((st = ws.acquire(false))) return st;
        return piece_call(ws.ws.get(), r->pieces, r->stride, r->n, r->full, rnd, r->n, 1, full, r->full);
    }
    if ((st = ws.acquire())) return st;
    if ((st = ws->coef.ensure(r->n)) || (st = ws->out.ensure(r->full))) return st;
    HIP_TRY(hipMemcpyAsync(ws->coef.p, rnd, r->n, hipMemcpyHostToDevice, ws->stream));
    const auto p = recoder_params(r, ws->coef.as<uint8_t>(), 1, ws->out.as<uint8_t>(), int64_t(r->full));
    if ((st = ctx->matmul(p, ws->stream, ws->idx, false))) return st;
    HIP_TRY(hipMemcpyAsync(full, ws->out.p, r->full, hipMemcpyDeviceToHost, ws->stream));
    HIP_TRY(hipStreamSynchronize(ws->stream));
    return RLNC_OK;
}

int rlnc_recoder_recode_batch_device(rlnc_recoder *r, const uint8_t *r_dev, size_t count, uint8_t *out_dev) {
    CHECK_ARG(r != nullptr);
    if (count == 0) return RLNC_OK;
    CHECK_ARG(r_dev != nullptr && out_dev != nullptr && count <= 0x7FFFFFFF);
    int st = r->ctx->activate();
    if (st || (st = r->ctx->note_capture())) return st;
    if ((st = r->ctx->matmul(recoder_params(r, r_dev, int(count), out_dev, int64_t(r->full))))) return st;
    return r->use.note(r->ctx->stream);
}

// ------------------------------------------------------------------------------------------------------
// Decoder — decoder.rs
// ------------------------------------------------------------------------------------------------------
int rlnc_decoder_new(rlnc_context *ctx, size_t L, size_t k, rlnc_decoder **out) {
    CHECK_ARG(ctx != nullptr && out != nullptr);
    *out = nullptr;
    if (L == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;  // decoder.rs:66-68
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;   // :69-71
    CHECK_ARG(k <= 0x7FFFFFFF);
    std::unique_ptr<rlnc_decoder> d(new (std::nothrow) rlnc_decoder);
    if (!d) return set_error(RLNC_ERR_OUT_OF_MEMORY, "decoder allocation");
    d->bind(ctx);
    d->k = k;
    d->L = L;
    d->stride = round16(L);
    d->elim.reset(new (std::nothrow) Elimination(k));
    if (!d->elim) return set_error(RLNC_ERR_OUT_OF_MEMORY, "decoder allocation");
    *out = d.release();
    return RLNC_OK;
}

// #[derive(Clone)] (decoder.rs:8): elimination state, counters and the stored data rows
int rlnc_decoder_clone(const rlnc_decoder *d, rlnc_decoder **out) {
    CHECK_ARG(d != nullptr && out != nullptr);
    *out = nullptr;
    int st = d->ctx->activate();
    if (st) return st;
    std::unique_ptr<rlnc_decoder> c(new (std::nothrow) rlnc_decoder);
    if (!c) return set_error(RLNC_ERR_OUT_OF_MEMORY, "decoder allocation");
    c->bind(d->ctx);
    c->k = d->k;
    c->L = d->L;
    c->stride = d->stride;
    c->received = d->received;
    c->useful = d->useful;
    c->elim.reset(new (std::nothrow) Elimination(*d->elim));
    if (!c->elim) return set_error(RLNC_ERR_OUT_OF_MEMORY, "decoder allocation");
    if (d->store_slots) {
        if ((st = d->ctx->obj_alloc(d->store_slots * d->stride, &c->store, &c->store_cap))) return st;
        c->store_slots = d->store_slots;
        Lease ws(d->ctx);
        if ((st = ws.acquire()) || (st = d->order(ws->stream))) return st;
        HIP_TRY(hipMemcpyAsync(c->store, d->store, d->store_slots * d->stride, hipMemcpyDeviceToDevice, ws->stream));
        HIP_TRY(hipStreamSynchronize(ws->stream));
    }
    *out = c.release();
    return RLNC_OK;
}

void rlnc_decoder_free(rlnc_decoder *d) { delete d; }

// s: the stream of the row copy (host pieces: the context's upload stream, where a store reallocation then also runs)
static int decoder_store_slot(rlnc_decoder *d, hipStream_t s, int slot, const uint8_t *src, hipMemcpyKind kind) {
    // device pieces: the row copy on s follows the decoder's staged host uploads (a host piece's upload runs on the
    // upload stream itself, behind every earlier one: no flush of the open ring slot per call)
    if (kind != hipMemcpyHostToDevice)
        if (int st = d->order(s)) return st;
    if (size_t(slot) >= d->store_slots) {
        const size_t ns = std::max(d->elim->slots(), size_t(slot) + 1);
        if (ns * d->stride > d->store_cap) {
            uint8_t *n = nullptr;
            size_t cap = 0;
            if (int st = d->ctx->obj_alloc(ns * d->stride, &n, &cap)) return st;
            // staged rows still target the old store: flush them ahead of the copy
            if (kind == hipMemcpyHostToDevice)
                if (int st = d->order(s)) return st;
            if (d->store) {
                HIP_TRY(hipMemcpyAsync(n, d->store, d->store_slots * d->stride, hipMemcpyDeviceToDevice, s));
                HIP_TRY(hipStreamSynchronize(s));
                d->ctx->obj_free(d->store, d->store_cap, nullptr);
            }
            d->store = n;
            d->store_cap = cap;
        }
        d->store_slots = ns;
    }
    uint8_t *row = d->store + size_t(slot) * d->stride;
    if (kind == hipMemcpyHostToDevice)
        // staged through pinned memory: the caller may reuse the piece when the call returns, no synchronisation
        // (a pageable copy's cost 30 us per call for small pieces)
        return d->ctx->upload(row, src, d->L, d->stride, &d->up);
    HIP_TRY(hipMemcpyAsync(row, src, d->L, kind, s));
    HIP_TRY(hipStreamSynchronize(s));  // the caller may reuse the piece; the call is synchronous
    return RLNC_OK;
}

static int decoder_decode_impl(rlnc_decoder *d, hipStream_t s, const uint8_t *coeffs_host, const uint8_t *data,
                               hipMemcpyKind kind) {
    int slot = -1;
    bool keep = false;
    const int st = d->elim->push(coeffs_host, &slot, &keep);
    if (st == RLNC_ERR_RECEIVED_ALL_PIECES) return st;
    d->received += 1;                                     // decoder.rs:107
    if (st == RLNC_OK) d->useful = d->elim->rank();       // :115
    if (keep)
        if (int s2 = decoder_store_slot(d, s, slot, data, kind)) return s2;
    return st;
}

int rlnc_decoder_decode(rlnc_decoder *d, const uint8_t *piece, size_t len) {
    CHECK_ARG(d != nullptr);
    if (d->elim->decoded()) return RLNC_ERR_RECEIVED_ALL_PIECES;  // decoder.rs:97-99
    if (len != d->k + d->L) return RLNC_ERR_INVALID_PIECE_LENGTH; // :100-102
    CHECK_ARG(piece != nullptr);
    int st = d->ctx->activate();
    if (st) return st;
    hipStream_t s = nullptr;  // no call workspace: the piece goes through the context's upload ring
    if ((st = d->ctx->upload_stream(s))) return st;
    return decoder_decode_impl(d, s, piece, piece + d->k, hipMemcpyHostToDevice);
}

int rlnc_decoder_decode_device(rlnc_decoder *d, const uint8_t *piece_dev, size_t len) {
    CHECK_ARG(d != nullptr);
    if (d->elim->decoded()) return RLNC_ERR_RECEIVED_ALL_PIECES;
    if (len != d->k + d->L) return RLNC_ERR_INVALID_PIECE_LENGTH;
    CHECK_ARG(piece_dev != nullptr);
    int st = d->ctx->activate();
    if (st) return st;
    Lease ws(d->ctx);
    if ((st = ws.acquire()) || (st = ws->pin_c.ensure(d->k))) return st;
    HIP_TRY(hipMemcpyAsync(ws->pin_c.p, piece_dev, d->k, hipMemcpyDeviceToHost, ws->stream));
    HIP_TRY(hipStreamSynchronize(ws->stream));
    std::vector<uint8_t> coeffs(ws->pin_c.as<uint8_t>(), ws->pin_c.as<uint8_t>() + d->k);
    return decoder_decode_impl(d, ws->stream, coeffs.data(), piece_dev + d->k, hipMemcpyDeviceToDevice);
}

int rlnc_decoder_is_already_decoded(const rlnc_decoder *d) { return d && d->elim->decoded() ? 1 : 0; }
size_t rlnc_decoder_get_num_pieces_coded_together(const rlnc_decoder *d) { return d ? d->k : 0; }
size_t rlnc_decoder_get_piece_byte_len(const rlnc_decoder *d) { return d ? d->L : 0; }
size_t rlnc_decoder_get_full_coded_piece_byte_len(const rlnc_decoder *d) { return d ? d->k + d->L : 0; }
size_t rlnc_decoder_get_received_piece_count(const rlnc_decoder *d) { return d ? d->received : 0; }
size_t rlnc_decoder_get_useful_piece_count(const rlnc_decoder *d) { return d ? d->useful : 0; }
size_t rlnc_decoder_get_remaining_piece_count(const rlnc_decoder *d) { return d ? d->k - d->useful : 0; }

// the store holds (at least) `slots` rows, on stream s (after the decoder's uploads); rows never stored are zeroed
// when `clear`
static int decoder_store_rows(rlnc_decoder *d, hipStream_t s, size_t slots, bool clear) {
    if (d->store_slots >= slots) return RLNC_OK;
    if (slots * d->stride > d->store_cap) {
        uint8_t *n = nullptr;
        size_t cap = 0;
        if (int st = d->ctx->obj_alloc(slots * d->stride, &n, &cap)) return st;
        if (d->store) HIP_TRY(hipMemcpyAsync(n, d->store, d->store_slots * d->stride, hipMemcpyDeviceToDevice, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (d->store) d->ctx->obj_free(d->store, d->store_cap, nullptr);
        d->store = n;
        d->store_cap = cap;
    }
    if (clear) HIP_TRY(hipMemsetAsync(d->store + d->store_slots * d->stride, 0, (slots - d->store_slots) * d->stride, s));
    d->store_slots = slots;
    return RLNC_OK;
}

// decoded rows = T × stored data rows, written to out_dev [k][L] on the lease's stream
static int decoder_apply(rlnc_decoder *d, CallWs *ws, uint8_t *out_dev) {
    const size_t slots = d->elim->slots();
    int st;
    if ((st = d->order(ws->stream))) return st;
    if ((st = ws->pin_b.ensure(d->k * slots)) || (st = ws->coef.ensure(d->k * slots))) return st;
    d->elim->transform(ws->pin_b.as<uint8_t>(), slots);
    HIP_TRY(hipMemcpyAsync(ws->coef.p, ws->pin_b.p, d->k * slots, hipMemcpyHostToDevice, ws->stream));
    // slots never stored were never referenced; give them zero rows so T × D is well defined
    if ((st = decoder_store_rows(d, ws->stream, slots, true))) return st;
    rlnc::MatmulParams p{};
    p.in = d->store;
    p.in_row = int64_t(d->stride);
    p.coef = ws->coef.as<uint8_t>();
    p.coef_row = int64_t(slots);
    p.out = out_dev;
    p.out_row = int64_t(d->L);
    p.n_out = int(d->k);
    p.n_in = int(slots);
    p.width = int64_t(d->L);
    p.n_obj = 1;
    return d->ctx->matmul(p, ws->stream, ws->idx, false);
}

namespace {
// Device -> caller host memory for large outputs: chunks DMA'd into a ring of pinned buffers (ws->pin_out), each
// copied into dst by the host copy pool (host_copy.hpp) while the next chunks are in flight.  The caller's buffer is
// typically fresh (the reference returns a new vec![0u8; k·L], decoder.rs:141-142): the pool's threads also share its
// page faults, which one thread paid alone in the runtime's pageable copy (round 4: 5.8 ms for 32 MiB).
constexpr size_t kOutChunk = size_t(4) << 20;
constexpr size_t kOutParallelMin = size_t(8) << 20;  // below this one pageable DMA is as fast (profiles/r05_copyout*)

// RLNC_COPY_TRACE=1 (diagnostic, read once): per-call host time of copy_out's phases, medians on stderr at exit
struct CopyTrace {
    bool on = [] {
        const char *e = getenv("RLNC_COPY_TRACE");
        return e && atoi(e) != 0;
    }();
    std::mutex mu;
    std::vector<float> total, wait, copy, first;  // us per call
    void add(float t, float w, float c, float f) {
        std::lock_guard<std::mutex> lock(mu);
        total.push_back(t);
        wait.push_back(w);
        copy.push_back(c);
        first.push_back(f);
    }
    ~CopyTrace() {
        if (on && !total.empty())
            std::fprintf(stderr, "{\"copy_trace\": {\"calls\": %zu, \"median_total_us\": %.1f, \"median_event_wait_us\": %.1f, "
                                 "\"median_host_copy_us\": %.1f, \"median_first_chunk_wait_us\": %.1f}}\n",
                         total.size(), PieceTrace::med(total), PieceTrace::med(wait), PieceTrace::med(copy),
                         PieceTrace::med(first));
    }
};
CopyTrace g_copy_trace;

// The whole 2 MiB-aligned pages inside dst[0, n) may be backed by transparent huge pages (a hint, where the host's
// THP mode is "madvise"): a fresh buffer then faults in 2 MiB at a time instead of 4 KiB.  The advice changes the
// flags of the caller's mapping (they outlive the buffer in its allocator's arena), so the library gives it only when
// the caller opts in with RLNC_COPY_HUGEPAGE=1 (read once).  A caller that owns a fresh result buffer advises it
// itself: the C++ mirror's get_decoded_data does (include/rlnc/full.hpp), which is where the 32 MB rows' huge-page
// gain is measured.
void advise_huge(uint8_t *dst, size_t n) {
    static const bool on = [] {
        const char *e = getenv("RLNC_COPY_HUGEPAGE");
        return e && atoi(e) != 0;
    }();
    constexpr uintptr_t kHuge = uintptr_t(2) << 20;
    const uintptr_t a = (reinterpret_cast<uintptr_t>(dst) + kHuge - 1) & ~(kHuge - 1);
    const uintptr_t b = (reinterpret_cast<uintptr_t>(dst) + n) & ~(kHuge - 1);
    if (on && b > a) (void)madvise(reinterpret_cast<void *>(a), b - a, MADV_HUGEPAGE);
}

// whether dst's pages are already mapped (a heap block the caller's allocator reused, zeroed on the caller's thread):
// mincore on its first, middle and last pages -- a fresh mapping has none of them
bool pages_resident(const uint8_t *dst, size_t n) {
    const uintptr_t pg = 4096;
    for (size_t off : {size_t(0), n / 2, n - 1}) {
        unsigned char v = 0;
        void *a = reinterpret_cast<void *>(reinterpret_cast<uintptr_t>(dst + off) & ~(pg - 1));
        if (mincore(a, pg, &v) != 0 || !(v & 1)) return false;
    }
    return true;
}

bool touch_first() {
    static const bool on = [] {
        const char *e = getenv("RLNC_COPY_TOUCH");  // A/B knob, read once: 0 = no pre-faulting
        return !e || atoi(e) != 0;
    }();
    return on;
}

int copy_out(CallWs *ws, uint8_t *dst, const uint8_t *src_dev, size_t n) {
    const int threads = copy_threads();
    if (n < kOutParallelMin || threads <= 1) {
        HIP_TRY(hipMemcpyAsync(dst, src_dev, n, hipMemcpyDeviceToHost, ws->stream));
        HIP_TRY(hipStreamSynchronize(ws->stream));
        return RLNC_OK;
    }
    constexpr int R = CallWs::kOutRing;
    if (int st = ws->pin_out.ensure(size_t(R) * kOutChunk)) return st;
    for (hipEvent_t &e : ws->out_ev)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    uint8_t *stage = ws->pin_out.as<uint8_t>();
    advise_huge(dst, n);
    const size_t chunks = (n + kOutChunk - 1) / kOutChunk;
    auto issue = [&](size_t c) -> int {
        const size_t off = c * kOutChunk, len = std::min(kOutChunk, n - off);
        HIP_TRY(hipMemcpyAsync(stage + (c % R) * kOutChunk, src_dev + off, len, hipMemcpyDeviceToHost, ws->stream));
        HIP_TRY(hipEventRecord(ws->out_ev[c % R], ws->stream));
        return RLNC_OK;
    };
    for (size_t c = 0; c < std::min<size_t>(R, chunks); ++c)
        if (int st = issue(c)) return st;
    // while the device runs the product and the first chunks' DMAs: fault the caller's pages in, in parallel (a fresh
    // buffer's page faults were most of the host copies' time: profiles/r05_copyout_trace*)
    if (touch_first() && !pages_resident(dst, n)) par_touch(dst, n, threads);
    const bool tr = g_copy_trace.on;
    const uint64_t t0 = tr ? now_ns() : 0;
    uint64_t tw = 0, tc = 0, tf = 0;
    for (size_t c = 0; c < chunks; ++c) {
        const uint64_t a = tr ? now_ns() : 0;
        HIP_TRY(hipEventSynchronize(ws->out_ev[c % R]));
        const uint64_t b = tr ? now_ns() : 0;
        const size_t off = c * kOutChunk, len = std::min(kOutChunk, n - off);
        par_copy(dst + off, stage + (c % R) * kOutChunk, len, threads);
        if (tr) {
            tw += b - a;
            tc += now_ns() - b;
            if (c == 0) tf = b - a;
        }
        if (c + R < chunks)
            if (int st = issue(c + R)) return st;
    }
    if (tr) g_copy_trace.add((now_ns() - t0) / 1e3f, tw / 1e3f, tc / 1e3f, tf / 1e3f);
    return RLNC_OK;
}
}  // namespace

int rlnc_decoder_get_decoded_data(rlnc_decoder *d, uint8_t *out, size_t cap, size_t *out_len) {
    CHECK_ARG(d != nullptr);
    if (!d->elim->decoded()) return RLNC_ERR_NOT_ALL_PIECES_RECEIVED_YET;  // decoder.rs:137-139
    CHECK_ARG(out != nullptr && out_len != nullptr && cap >= d->k * d->L);
    int st = d->ctx->activate();
    if (st) return st;
    Lease ws(d->ctx);
    const size_t slots = d->elim->slots();
    if (d->k * round16(d->L) <= kPieceMaxBytes && d->k * slots * d->L <= kPieceDecodeMaxMacs &&
        piece_eligible(d->store, d->stride, d->L)) {
        // T (k x slots) is read by the kernel from pinned memory and the rows land in pinned memory, copied into out
        // chunk by chunk as the device finishes them.  Store rows never stored are referenced by zero columns of T
        // only (0 · x = 0 for whatever they hold), so they need to exist, not to be cleared.
        if ((st = ws.acquire(false)) || (st = d->order(ws->stream))) return st;
        if ((st = decoder_store_rows(d, ws->stream, slots, false))) return st;
        if ((st = ws->pc_coef.ensure(d->k * slots))) return st;
        d->elim->transform(ws->pc_coef.as<uint8_t>(), slots);
        if ((st = piece_call(ws.ws.get(), d->store, d->stride, slots, d->L, ws->pc_coef.as<uint8_t>(), slots, d->k, out,
                             d->L)))
            return st;
    } else {
        if ((st = ws.acquire()) || (st = ws->out.ensure(d->k * d->L))) return st;
        if ((st = decoder_apply(d, ws.ws.get(), ws->out.as<uint8_t>()))) return st;
        if ((st = copy_out(ws.ws.get(), out, ws->out.as<uint8_t>(), d->k * d->L))) return st;
    }
    // get_final_data_len — decoder.rs:162-177: last nonzero byte must be the 0x81 marker, not at 0
    size_t n = d->k * d->L;
    while (n > 0 && out[n - 1] == 0) --n;
    if (n == 0 || out[n - 1] != rlnc::kBoundaryMarker || n - 1 == 0) return RLNC_ERR_INVALID_DECODED_DATA_FORMAT;
    *out_len = n - 1;
    return RLNC_OK;
}

int rlnc_decoder_get_decoded_data_device(rlnc_decoder *d, uint8_t *out_dev, size_t cap, size_t *out_len) {
    CHECK_ARG(d != nullptr);
    if (!d->elim->decoded()) return RLNC_ERR_NOT_ALL_PIECES_RECEIVED_YET;
    CHECK_ARG(out_dev != nullptr && out_len != nullptr && cap >= d->k * d->L);
    int st = d->ctx->activate();
    if (st) return st;
    Lease ws(d->ctx);
    if ((st = ws.acquire())) return st;
    if ((st = decoder_apply(d, ws.ws.get(), out_dev))) return st;
    if ((st = ws->status.ensure(4)) || (st = ws->len.ensure(8)) ||
        (st = ws->pin_c.ensure(16)))
        return st;
    HIP_TRY(rlnc::launch_final_data_len(out_dev, 0, int64_t(d->k * d->L), 1, ws->status.as<int32_t>(),
                                        ws->len.as<int64_t>(), RLNC_ERR_INVALID_DECODED_DATA_FORMAT, ws->stream));
    HIP_TRY(hipMemcpyAsync(ws->pin_c.p, ws->status.p, 4, hipMemcpyDeviceToHost, ws->stream));
    HIP_TRY(hipMemcpyAsync(ws->pin_c.as<uint8_t>() + 8, ws->len.p, 8, hipMemcpyDeviceToHost, ws->stream));
    HIP_TRY(hipStreamSynchronize(ws->stream));
    const int32_t status = *ws->pin_c.as<int32_t>();
    if (status) return status;
    std::memcpy(out_len, ws->pin_c.as<uint8_t>() + 8, 8);
    return RLNC_OK;
}

// ------------------------------------------------------------------------------------------------------
// batch API
// ------------------------------------------------------------------------------------------------------
static rlnc::MatmulParams encode_batch_params(const uint8_t *src, size_t k, size_t L, size_t nobj,
                                              const uint8_t *coeffs, size_t n, uint8_t *pieces, bool headers) {
    const int64_t full = int64_t(k + L);
    rlnc::MatmulParams p{};
    p.in = src;
    p.in_obj = int64_t(k * L);
    p.in_row = int64_t(L);
    p.coef = coeffs;
    p.coef_obj = int64_t(n * k);
    p.coef_row = int64_t(k);
    p.out = pieces + k;
    p.out_obj = int64_t(n) * full;
    p.out_row = full;
    p.hdr = headers ? pieces : nullptr;
    p.hdr_obj = int64_t(n) * full;
    p.hdr_row = full;
    p.n_out = int(n);
    p.n_in = int(k);
    p.width = int64_t(L);
    p.n_obj = int(nobj);
    return p;
}

// Block-address streams written ahead by rlnc_encode_batch_prepare (any context, any stream), by buffer: the product
// they were written for and their layout.  rlnc_encode_batch_data_planned uses one only for exactly that product.
// The decode's data side has the same pair (rlnc_decode_batch_apply_prepare / _planned): kind 1, with src = the
// received pieces, coeffs = T, pieces = the decoded output, n = m and the pieces' object stride.
struct EncodePlanRec {
    int device;
    const uint8_t *src, *coeffs;
    uint8_t *pieces;
    size_t k, L, nobj, n;
    int variant;
    rlnc::BsjStreamPlan plan;
    int kind = 0;  // 0 encode, 1 decode apply
    size_t obj_stride = 0;
};
static std::mutex g_plan_mu;
static std::vector<std::pair<const void *, EncodePlanRec>> g_plans;  // (buffer, record), most recent last
constexpr size_t kPlanRecs = 64;

static void remember_plan(const void *buf, const EncodePlanRec &rec) {
    std::lock_guard<std::mutex> lock(g_plan_mu);
    for (auto it = g_plans.begin(); it != g_plans.end(); ++it)
        if (it->first == buf) {
            g_plans.erase(it);
            break;
        }
    if (g_plans.size() >= kPlanRecs) g_plans.erase(g_plans.begin());
    g_plans.emplace_back(buf, rec);
}

static bool find_plan(const void *buf, EncodePlanRec *rec) {
    std::lock_guard<std::mutex> lock(g_plan_mu);
    for (auto it = g_plans.rbegin(); it != g_plans.rend(); ++it)
        if (it->first == buf) {
            *rec = it->second;
            return true;
        }
    return false;
}

static int encode_batch_impl(rlnc_context *ctx, const uint8_t *src, size_t k, size_t L, size_t nobj,
                             const uint8_t *coeffs, size_t n, uint8_t *pieces, bool headers,
                             const void *plan_buf = nullptr) {
    CHECK_ARG(ctx != nullptr);
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
    if (L == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;
    if (n == 0 || nobj == 0) return RLNC_OK;
    CHECK_ARG(src && coeffs && pieces && n <= 0x7FFFFFFF && k <= 0x7FFFFFFF && nobj <= 0x7FFFFFFF);
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    rlnc::MatmulParams p = encode_batch_params(src, k, L, nobj, coeffs, n, pieces, headers);
    if (plan_buf) {
        EncodePlanRec rec{};
        const bool found = find_plan(plan_buf, &rec);
        if (!found || rec.kind != 0 || rec.device != ctx->device || rec.src != src || rec.coeffs != coeffs ||
            rec.pieces != pieces ||
            rec.k != k || rec.L != L || rec.nobj != nobj || rec.n != n || rec.variant != int(ctx->variant))
            return set_error(RLNC_ERR_INVALID_ARGUMENT,
                             "encode plan %p was not prepared for this product (same buffers, shape, device and kernel "
                             "variant): call rlnc_encode_batch_prepare with the arguments of this call",
                             plan_buf);
        if (rec.plan.tile_rows > 0) {
            p.bsj_stream = plan_buf;
            p.bsj_stream_rows = rec.plan.tile_rows;
            p.bsj_stream_abs = rec.plan.abs;
        }
    }
    return ctx->matmul(p);
}

int rlnc_encode_batch(rlnc_context *ctx, const uint8_t *src, size_t k, size_t L, size_t nobj, const uint8_t *coeffs,
                      size_t n, uint8_t *pieces) {
    return encode_batch_impl(ctx, src, k, L, nobj, coeffs, n, pieces, true);
}

int rlnc_encode_batch_data(rlnc_context *ctx, const uint8_t *src, size_t k, size_t L, size_t nobj,
                           const uint8_t *coeffs, size_t n, uint8_t *pieces) {
    return encode_batch_impl(ctx, src, k, L, nobj, coeffs, n, pieces, false);
}

size_t rlnc_encode_batch_plan_bytes(size_t k, size_t nobj, size_t n) {
    if (k == 0 || n == 0 || nobj == 0 || k > 0x7FFFFFFF || n > 0x7FFFFFFF || nobj > 0x7FFFFFFF) return 0;
    return rlnc::bsj_stream_bytes_bound(int(nobj), int(n), int(k));
}

int rlnc_encode_batch_prepare(rlnc_context *ctx, const uint8_t *src, size_t k, size_t L, size_t nobj,
                              const uint8_t *coeffs, size_t n, uint8_t *pieces, void *plan_buf, size_t plan_bytes) {
    CHECK_ARG(ctx != nullptr);
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
    if (L == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;
    if (n == 0 || nobj == 0) return RLNC_OK;
    CHECK_ARG(src && coeffs && pieces && plan_buf && n <= 0x7FFFFFFF && k <= 0x7FFFFFFF && nobj <= 0x7FFFFFFF);
    CHECK_ARG(plan_bytes >= rlnc_encode_batch_plan_bytes(k, nobj, n));
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    const rlnc::MatmulParams p = encode_batch_params(src, k, L, nobj, coeffs, n, pieces, false);
    rlnc::BsjStreamPlan plan;
    // the row-split tuning knob launches per row range, each with its own stream: nothing to write ahead
    if (!(ctx->max_tile_rows > 0 && p.n_out > ctx->max_tile_rows))
        HIP_TRY(rlnc::launch_bsj_stream(p, ctx->variant, ctx->stream, plan_buf, plan_bytes, plan));
    EncodePlanRec rec{ctx->device, src, coeffs, pieces, k, L, nobj, n, int(ctx->variant), plan};
    remember_plan(plan_buf, rec);
    return RLNC_OK;
}

int rlnc_encode_batch_data_planned(rlnc_context *ctx, const uint8_t *src, size_t k, size_t L, size_t nobj,
                                   const uint8_t *coeffs, size_t n, uint8_t *pieces, const void *plan_buf) {
    CHECK_ARG(plan_buf != nullptr);
    return encode_batch_impl(ctx, src, k, L, nobj, coeffs, n, pieces, false, plan_buf);
}

int rlnc_encode_batch_headers(rlnc_context *ctx, const uint8_t *coeffs, size_t k, size_t L, size_t nobj, size_t n,
                              uint8_t *pieces) {
    CHECK_ARG(ctx != nullptr);
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
    if (L == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;
    if (n == 0 || nobj == 0) return RLNC_OK;
    CHECK_ARG(coeffs && pieces);
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    // pieces[o][i][0..k) = coeffs[o][i] (encoder.rs:246-248): one strided copy (a kernel: the runtime's 2D
    // blit took 36 µs for 1,024 rows of 32 B)
    HIP_TRY(rlnc::launch_copy_rows(pieces, int64_t(k + L), coeffs, int64_t(k), int64_t(k), int64_t(n * nobj),
                                   ctx->stream));
    return RLNC_OK;
}

int rlnc_recode_batch(rlnc_context *ctx, const uint8_t *pieces, size_t k, size_t L, size_t n, size_t nobj,
                      const uint8_t *r, size_t count, uint8_t *out) {
    CHECK_ARG(ctx != nullptr);
    if (n == 0) return RLNC_ERR_NOT_ENOUGH_PIECES_TO_RECODE;
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
    if (L == 0) return RLNC_ERR_PIECE_LENGTH_TOO_SHORT;
    if (count == 0 || nobj == 0) return RLNC_OK;
    CHECK_ARG(pieces && r && out && n <= 0x7FFFFFFF && count <= 0x7FFFFFFF && nobj <= 0x7FFFFFFF);
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    const int64_t full = int64_t(k + L);
    rlnc::MatmulParams p{};
    p.in = pieces;
    p.in_obj = int64_t(n) * full;
    p.in_row = full;
    p.coef = r;
    p.coef_obj = int64_t(count * n);
    p.coef_row = int64_t(n);
    p.out = out;
    p.out_obj = int64_t(count) * full;
    p.out_row = full;
    p.n_out = int(count);
    p.n_in = int(n);
    p.width = full;
    p.n_obj = int(nobj);
    return ctx->matmul(p);
}

// Device path: exact elimination on the device (rref.hip) → T × data (one matmul) → marker scan.
// Everything is enqueued on the context stream; outputs stay on the device.
// The elimination alone: reads only the k coefficient bytes of each piece; writes T [obj][k][m], the per-piece
// statuses and the ranks.
// tail (optional, with bsj): the small-object elimination also answers get_final_data_len from the payload tail
// (RrefParams::tail_status): {status, length, need-scan flags} device arrays
struct TailOut {
    int32_t *status = nullptr;
    int64_t *len = nullptr;
    int32_t *need = nullptr;
};

static int decode_eliminate_impl(rlnc_context *ctx, const uint8_t *pieces, size_t obj_stride, size_t k, size_t L,
                                 size_t m, size_t nobj, uint8_t *T, int32_t *pstat_dev, int32_t *rank_dev,
                                 uint32_t *bsj = nullptr, int bsj_rows = 0, bool *bsj_written = nullptr,
                                 const TailOut *tail = nullptr) {
    const size_t full = k + L;
    rlnc::RrefParams rp{};
    rp.pieces = pieces;
    rp.obj_stride = int64_t(obj_stride);
    rp.piece_stride = int64_t(full);
    rp.k = int(k);
    rp.m = int(m);
    rp.n_obj = int(nobj);
    rp.T = T;
    rp.T_obj = int64_t(k * m);
    rp.status = pstat_dev;
    rp.rank = rank_dev;
    rp.lds_only = ctx->decode_path == 3 ? 1 : ctx->decode_path == 4 ? 2 : ctx->decode_path == 5 ? 3 : ctx->decode_path == 6 ? 4 : 0;
    if (ctx->decode_path == 5 && !rlnc::rref_block_eligible(int(k), int(m)))  // no silent fallback to another kernel
        return set_error(RLNC_ERR_INVALID_ARGUMENT, "decode path 5 (blocked run) needs k + m <= 256 (k=%zu, m=%zu)", k, m);
    rp.bsj_stream = bsj;
    rp.bsj_block_bytes = rlnc::bsj_block_bytes_public();
    rp.bsj_tile_rows = bsj_rows;
    if (tail != nullptr) {
        rp.tail_status = tail->status;
        rp.tail_len = tail->len;
        rp.tail_need = tail->need;
        rp.tail_L = int64_t(L);
    }
    HIP_TRY(rlnc::launch_rref_batch(rp, ctx->stream, bsj_written));
    return RLNC_OK;
}

// RLNC_FUSED_SCAN=0 (A/B knob, read once): the separate marker-scan launch for every decode
static bool fused_scan_enabled() {
    static const bool on = [] {
        const char *e = getenv("RLNC_FUSED_SCAN");
        return !e || atoi(e) != 0;
    }();
    return on;
}

// The data side's product: decoded = T × the received pieces' data
static rlnc::MatmulParams decode_apply_params(const uint8_t *pieces, size_t obj_stride, size_t k, size_t L, size_t m,
                                              size_t nobj, const uint8_t *T, uint8_t *decoded) {
    rlnc::MatmulParams p{};
    p.in = pieces + k;
    p.in_obj = int64_t(obj_stride);
    p.in_row = int64_t(k + L);
    p.coef = T;
    p.coef_obj = int64_t(k * m);
    p.coef_row = int64_t(m);
    p.out = decoded;
    p.out_obj = int64_t(k * L);
    p.out_row = int64_t(L);
    p.n_out = int(k);
    p.n_in = int(m);
    p.width = int64_t(L);
    p.n_obj = int(nobj);
    return p;
}

// The data side: decoded = T × received data (one matmul), then the marker scan (decoder.rs:136-177).
static int decode_apply_impl(rlnc_context *ctx, const uint8_t *pieces, size_t obj_stride, size_t k, size_t L,
                             size_t m, size_t nobj, const uint8_t *T, const int32_t *rank_dev, uint8_t *decoded,
                             int32_t *ostat_dev, int64_t *len_dev, const void *bsj = nullptr, int bsj_rows = 0,
                             const int32_t *need_dev = nullptr, bool bsj_abs = false) {
    int st;
    rlnc::MatmulParams p = decode_apply_params(pieces, obj_stride, k, L, m, nobj, T, decoded);
    p.bsj_stream = bsj;
    p.bsj_stream_rows = bsj_rows;
    p.bsj_stream_abs = bsj_abs;
    // need_dev: the elimination already wrote every object's status and length from its payload tail; the objects
    // whose tail was all zero are scanned by their product workgroup when each object is one tile (configs[0]'s shape),
    // else the scan kernel runs over all of them
    bool scanned = false;
    if (need_dev != nullptr) {
        p.scan_status = ostat_dev;
        p.scan_need = need_dev;
        p.scan_len = len_dev;
        p.scan_k = int(k);
        p.scan_done = &scanned;
    }
    if ((st = ctx->matmul(p))) return st;
    if (!scanned)
        HIP_TRY(rlnc::launch_final_data_len_ranked(decoded, int64_t(k * L), int64_t(k * L), int(nobj), int(k), rank_dev,
                                                   ostat_dev, len_dev, ctx->stream));
    return RLNC_OK;
}

static int decode_batch_device_impl(rlnc_context *ctx, const uint8_t *pieces, size_t obj_stride, size_t k, size_t L,
                                    size_t m, size_t nobj, uint8_t *decoded, int32_t *pstat_dev, int32_t *ostat_dev,
                                    int64_t *len_dev, int32_t *rank_dev) {
    int st;
    if ((st = ctx->grow(ctx->ws_coef, nobj * k * m))) return st;
    uint8_t *T = ctx->ws_coef.as<uint8_t>();
    // (Eliminating the later objects on a second stream beside the first objects' T x data product measured slower:
    // 8.3-8.6 ms against 7.99 for configs[4]'s 512 objects -- the concurrent elimination slows the product more
    // than it hides; profiles/r02_decode_pipeline_ab.txt.)
    // small objects (the one-wave elimination kernel, products in the 1- or 2-wave bit-sliced program): the elimination
    // also writes the product's block-offset stream, so the product needs no offset launch (configs[0] shape: -6 us)
    const int bsj_rows = rlnc::bsj_unshared_tile_rows(int(k));
    uint32_t *bsj = nullptr;
    if (bsj_rows > 0) {
        if ((st = ctx->grow(ctx->ws_bsj, nobj * m * size_t(bsj_rows) * 4 + 512))) return st;
        bsj = ctx->ws_bsj.as<uint32_t>();
    }
    // one-tile objects (k <= 16 x one 4 KiB column block): the elimination answers the marker scan from the payload
    // tail and the product's workgroups scan the rare all-zero tails (no scan launch: configs[0] shape)
    TailOut tail;
    const bool want_tail = bsj != nullptr && L == 4096 && k % 4 == 0 && obj_stride % 4 == 0 &&
                           reinterpret_cast<uintptr_t>(pieces) % 4 == 0 && fused_scan_enabled();
    if (want_tail) {
        if ((st = ctx->grow(ctx->ws_need, nobj * 4))) return st;
        tail.status = ostat_dev;
        tail.len = len_dev;
        tail.need = ctx->ws_need.as<int32_t>();
    }
    bool written = false;
    if ((st = decode_eliminate_impl(ctx, pieces, obj_stride, k, L, m, nobj, T, pstat_dev, rank_dev, bsj, bsj_rows,
                                    &written, want_tail ? &tail : nullptr)))
        return st;
    return decode_apply_impl(ctx, pieces, obj_stride, k, L, m, nobj, T, rank_dev, decoded, ostat_dev, len_dev,
                             written ? bsj : nullptr, written ? bsj_rows : 0, written && want_tail ? tail.need : nullptr);
}

// Host path (matrices too large for LDS): exact elimination on host threads (elimination.hpp).
static int decode_batch_host_impl(rlnc_context *ctx, const uint8_t *pieces, size_t obj_stride, size_t k, size_t L,
                                  size_t m, size_t nobj, uint8_t *decoded, int32_t *piece_status, int32_t *object_status,
                                  uint64_t *data_len) {
    const size_t full = k + L;
    int st;
    // 1. coefficient headers → host (k bytes of each piece)
    if ((st = ctx->grow(ctx->pin_a, nobj * m * k))) return st;
    uint8_t *hdr = ctx->pin_a.as<uint8_t>();
    if (obj_stride == m * full) {
        HIP_TRY(hipMemcpy2DAsync(hdr, k, pieces, full, k, nobj * m, hipMemcpyDeviceToHost, ctx->stream));
    } else {
        for (size_t o = 0; o < nobj; ++o)
            HIP_TRY(hipMemcpy2DAsync(hdr + o * m * k, k, pieces + o * obj_stride, full, k, m, hipMemcpyDeviceToHost,
                                     ctx->stream));
    }
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    // 2. exact incremental elimination per object (decoder.rs:96-118 for pieces 0..m-1), host threads
    if ((st = ctx->grow(ctx->pin_b, nobj * k * m))) return st;
    uint8_t *T = ctx->pin_b.as<uint8_t>();
    std::vector<int32_t> ranks(nobj, 0);
    std::vector<int32_t> pst(nobj * m, 0);
    auto work = [&](size_t o0, size_t o1) {
        for (size_t o = o0; o < o1; ++o) {
            Elimination e(k, m);
            for (size_t p = 0; p < m; ++p) {
                int slot;
                bool keep;
                pst[o * m + p] = e.push(hdr + (o * m + p) * k, &slot, &keep);
            }
            ranks[o] = int32_t(e.rank());
            std::memset(T + o * k * m, 0, k * m);
            e.transform(T + o * k * m, m);
        }
    };
    const size_t hw = std::max<unsigned>(1, std::thread::hardware_concurrency());
    const size_t nth = std::min<size_t>({nobj, hw, 16});
    if (nth <= 1) {
        work(0, nobj);
    } else {
        std::vector<std::thread> th;
        const size_t per = (nobj + nth - 1) / nth;
        for (size_t t = 0; t < nth; ++t) {
            const size_t a = t * per, b = std::min(nobj, a + per);
            if (a < b) th.emplace_back(work, a, b);
        }
        for (auto &t : th) t.join();
    }
    // 3. T → device, decoded = T × received data rows (one launch for all objects)
    if ((st = ctx->grow(ctx->ws_coef, nobj * k * m)) || (st = ctx->grow(ctx->ws_rank, nobj * 4)) ||
        (st = ctx->grow(ctx->ws_status, nobj * 4)) ||
        (st = ctx->grow(ctx->ws_len, nobj * 8)) || (st = ctx->grow(ctx->pin_c, nobj * 16)))
        return st;
    HIP_TRY(hipMemcpyAsync(ctx->ws_coef.p, T, nobj * k * m, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(ctx->ws_rank.p, ranks.data(), nobj * 4, hipMemcpyHostToDevice, ctx->stream));
    rlnc::MatmulParams p{};
    p.in = pieces + k;
    p.in_obj = int64_t(obj_stride);
    p.in_row = int64_t(full);
    p.coef = T;
    p.coef_obj = int64_t(k * m);
    p.coef_row = int64_t(m);
    p.out = decoded;
    p.out_obj = int64_t(k * L);
    p.out_row = int64_t(L);
    p.n_out = int(k);
    p.n_in = int(m);
    p.width = int64_t(L);
    p.n_obj = int(nobj);
    if ((st = ctx->matmul(p))) return st;
    // 4. get_final_data_len on device (decoder.rs:162-177)
    HIP_TRY(rlnc::launch_final_data_len_ranked(decoded, int64_t(k * L), int64_t(k * L), int(nobj), int(k),
                                               ctx->ws_rank.as<int32_t>(), ctx->ws_status.as<int32_t>(),
                                               ctx->ws_len.as<int64_t>(), ctx->stream));
    int32_t *hst = ctx->pin_c.as<int32_t>();
    int64_t *hlen = reinterpret_cast<int64_t *>(ctx->pin_c.as<uint8_t>() + nobj * 8);
    HIP_TRY(hipMemcpyAsync(hst, ctx->ws_status.p, nobj * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(hlen, ctx->ws_len.p, nobj * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    for (size_t o = 0; o < nobj; ++o) {
        if (object_status) object_status[o] = hst[o];
        if (data_len) data_len[o] = uint64_t(hlen[o]);
    }
    if (piece_status) std::memcpy(piece_status, pst.data(), nobj * m * sizeof(int32_t));
    return RLNC_OK;
}

static int decode_batch_check(rlnc_context *ctx, const uint8_t *pieces, size_t &obj_stride, size_t k, size_t L,
                              size_t m, size_t nobj, uint8_t *decoded) {
    CHECK_ARG(ctx != nullptr);
    if (L == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
    CHECK_ARG(pieces && decoded && m > 0 && m <= 0x7FFFFFFF && k <= 0x7FFFFFFF && nobj <= 0x7FFFFFFF);
    if (obj_stride == 0) obj_stride = m * (k + L);
    CHECK_ARG(obj_stride >= m * (k + L));
    int st = ctx->activate();
    if (st) return st;
    return ctx->note_capture();
}

int rlnc_decode_batch(rlnc_context *ctx, const uint8_t *pieces, size_t obj_stride, size_t k, size_t L, size_t m,
                      size_t nobj, uint8_t *decoded, int32_t *piece_status, int32_t *object_status,
                      uint64_t *data_len) {
    if (nobj == 0 && ctx) return RLNC_OK;
    int st = decode_batch_check(ctx, pieces, obj_stride, k, L, m, nobj, decoded);
    if (st) return st;
    const bool fits = rlnc::rref_lds_bytes(int(k), int(m)) <= rlnc::kRrefMaxLds;
    if (ctx->decode_path >= 2 && !fits)
        return set_error(RLNC_ERR_INVALID_ARGUMENT, "device elimination forced but k=%zu, m=%zu exceed LDS", k, m);
    if (!fits || ctx->decode_path == 1)
        return decode_batch_host_impl(ctx, pieces, obj_stride, k, L, m, nobj, decoded, piece_status, object_status,
                                      data_len);
    if ((st = ctx->grow(ctx->ws_pstat, nobj * m * 4)) || (st = ctx->grow(ctx->ws_status, nobj * 4)) ||
        (st = ctx->grow(ctx->ws_len, nobj * 8)) || (st = ctx->grow(ctx->ws_rank, nobj * 4)) ||
        (st = ctx->grow(ctx->pin_c, nobj * (m * 4 + 16))))
        return st;
    if ((st = decode_batch_device_impl(ctx, pieces, obj_stride, k, L, m, nobj, decoded, ctx->ws_pstat.as<int32_t>(),
                                       ctx->ws_status.as<int32_t>(), ctx->ws_len.as<int64_t>(),
                                       ctx->ws_rank.as<int32_t>())))
        return st;
    uint8_t *h = ctx->pin_c.as<uint8_t>();
    HIP_TRY(hipMemcpyAsync(h, ctx->ws_status.p, nobj * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(h + nobj * 8, ctx->ws_len.p, nobj * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipMemcpyAsync(h + nobj * 16, ctx->ws_pstat.p, nobj * m * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    for (size_t o = 0; o < nobj; ++o) {
        if (object_status) object_status[o] = reinterpret_cast<int32_t *>(h)[o];
        if (data_len) data_len[o] = uint64_t(reinterpret_cast<int64_t *>(h + nobj * 8)[o]);
    }
    if (piece_status) std::memcpy(piece_status, h + nobj * 16, nobj * m * 4);
    return RLNC_OK;
}

int rlnc_decode_batch_device(rlnc_context *ctx, const uint8_t *pieces, size_t obj_stride, size_t k, size_t L, size_t m,
                             size_t nobj, uint8_t *decoded, int32_t *piece_status_dev, int32_t *object_status_dev,
                             int64_t *data_len_dev) {
    if (nobj == 0 && ctx) return RLNC_OK;
    int st = decode_batch_check(ctx, pieces, obj_stride, k, L, m, nobj, decoded);
    if (st) return st;
    CHECK_ARG(piece_status_dev && object_status_dev && data_len_dev);
    if (rlnc::rref_lds_bytes(int(k), int(m)) > rlnc::kRrefMaxLds)
        return set_error(RLNC_ERR_INVALID_ARGUMENT, "k=%zu, m=%zu exceed the device elimination's LDS budget; use "
                         "rlnc_decode_batch", k, m);
    if ((st = ctx->grow(ctx->ws_rank, nobj * 4))) return st;
    return decode_batch_device_impl(ctx, pieces, obj_stride, k, L, m, nobj, decoded, piece_status_dev,
                                    object_status_dev, data_len_dev, ctx->ws_rank.as<int32_t>());
}

int rlnc_decode_batch_eliminate(rlnc_context *ctx, const uint8_t *pieces, size_t obj_stride, size_t k, size_t L,
                                size_t m, size_t nobj, uint8_t *T_dev, int32_t *piece_status_dev, int32_t *rank_dev) {
    if (nobj == 0 && ctx) return RLNC_OK;
    CHECK_ARG(T_dev != nullptr);
    int st = decode_batch_check(ctx, pieces, obj_stride, k, L, m, nobj, T_dev);
    if (st) return st;
    CHECK_ARG(piece_status_dev && rank_dev);
    if (rlnc::rref_lds_bytes(int(k), int(m)) > rlnc::kRrefMaxLds)
        return set_error(RLNC_ERR_INVALID_ARGUMENT, "k=%zu, m=%zu exceed the device elimination's LDS budget; use "
                         "rlnc_decode_batch", k, m);
    return decode_eliminate_impl(ctx, pieces, obj_stride, k, L, m, nobj, T_dev, piece_status_dev, rank_dev);
}

int rlnc_decode_batch_apply(rlnc_context *ctx, const uint8_t *pieces, size_t obj_stride, size_t k, size_t L, size_t m,
                            size_t nobj, const uint8_t *T_dev, const int32_t *rank_dev, uint8_t *decoded,
                            int32_t *object_status_dev, int64_t *data_len_dev) {
    if (nobj == 0 && ctx) return RLNC_OK;
    int st = decode_batch_check(ctx, pieces, obj_stride, k, L, m, nobj, decoded);
    if (st) return st;
    CHECK_ARG(T_dev && rank_dev && object_status_dev && data_len_dev);
    return decode_apply_impl(ctx, pieces, obj_stride, k, L, m, nobj, T_dev, rank_dev, decoded, object_status_dev,
                             data_len_dev);
}

size_t rlnc_decode_batch_apply_plan_bytes(size_t k, size_t m, size_t nobj) {
    if (k == 0 || m == 0 || nobj == 0 || k > 0x7FFFFFFF || m > 0x7FFFFFFF || nobj > 0x7FFFFFFF) return 0;
    return rlnc::bsj_stream_bytes_bound(int(nobj), int(k), int(m));
}

int rlnc_decode_batch_apply_prepare(rlnc_context *ctx, const uint8_t *pieces, size_t obj_stride, size_t k, size_t L,
                                    size_t m, size_t nobj, const uint8_t *T_dev, uint8_t *decoded, void *plan_buf,
                                    size_t plan_bytes) {
    if (nobj == 0 && ctx) return RLNC_OK;
    int st = decode_batch_check(ctx, pieces, obj_stride, k, L, m, nobj, decoded);
    if (st) return st;
    CHECK_ARG(T_dev && plan_buf && plan_bytes >= rlnc_decode_batch_apply_plan_bytes(k, m, nobj));
    const rlnc::MatmulParams p = decode_apply_params(pieces, obj_stride, k, L, m, nobj, T_dev, decoded);
    rlnc::BsjStreamPlan plan;
    if (!(ctx->max_tile_rows > 0 && p.n_out > ctx->max_tile_rows))
        HIP_TRY(rlnc::launch_bsj_stream(p, ctx->variant, ctx->stream, plan_buf, plan_bytes, plan));
    EncodePlanRec rec{ctx->device, pieces, T_dev, decoded, k, L, nobj, m, int(ctx->variant), plan};
    rec.kind = 1;
    rec.obj_stride = obj_stride;
    remember_plan(plan_buf, rec);
    return RLNC_OK;
}

int rlnc_decode_batch_apply_planned(rlnc_context *ctx, const uint8_t *pieces, size_t obj_stride, size_t k, size_t L,
                                    size_t m, size_t nobj, const uint8_t *T_dev, const int32_t *rank_dev,
                                    uint8_t *decoded, int32_t *object_status_dev, int64_t *data_len_dev,
                                    const void *plan_buf) {
    if (nobj == 0 && ctx) return RLNC_OK;
    int st = decode_batch_check(ctx, pieces, obj_stride, k, L, m, nobj, decoded);
    if (st) return st;
    CHECK_ARG(T_dev && rank_dev && object_status_dev && data_len_dev && plan_buf);
    EncodePlanRec rec{};
    if (!find_plan(plan_buf, &rec) || rec.kind != 1 || rec.device != ctx->device || rec.src != pieces ||
        rec.coeffs != T_dev || rec.pieces != decoded || rec.obj_stride != obj_stride || rec.k != k || rec.L != L ||
        rec.nobj != nobj || rec.n != m || rec.variant != int(ctx->variant))
        return set_error(RLNC_ERR_INVALID_ARGUMENT,
                         "decode plan %p was not prepared for this product (same buffers, shape, device and kernel "
                         "variant): call rlnc_decode_batch_apply_prepare with the arguments of this call",
                         plan_buf);
    return decode_apply_impl(ctx, pieces, obj_stride, k, L, m, nobj, T_dev, rank_dev, decoded, object_status_dev,
                             data_len_dev, rec.plan.tile_rows > 0 ? plan_buf : nullptr, rec.plan.tile_rows, nullptr,
                             rec.plan.abs);
}

// ------------------------------------------------------------------------------------------------------
// host-only access to the decoder's elimination engine (no device needed; CPU-testable host logic)
// ------------------------------------------------------------------------------------------------------
struct rlnc_elimination {
    Elimination e;
    explicit rlnc_elimination(size_t k, size_t fixed) : e(k, fixed) {}
};

int rlnc_elimination_new(size_t k, size_t fixed_slots, rlnc_elimination **out) {
    CHECK_ARG(out != nullptr);
    *out = nullptr;
    if (k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
    *out = new (std::nothrow) rlnc_elimination(k, fixed_slots);
    return *out ? RLNC_OK : set_error(RLNC_ERR_OUT_OF_MEMORY, "elimination allocation");
}
void rlnc_elimination_free(rlnc_elimination *e) { delete e; }
int rlnc_elimination_push(rlnc_elimination *e, const uint8_t *coeffs, int32_t *slot, int32_t *keep) {
    CHECK_ARG(e != nullptr && coeffs != nullptr);
    int s = -1;
    bool k = false;
    const int st = e->e.push(coeffs, &s, &k);
    if (slot) *slot = s;
    if (keep) *keep = k ? 1 : 0;
    return st;
}
size_t rlnc_elimination_rank(const rlnc_elimination *e) { return e ? e->e.rank() : 0; }
size_t rlnc_elimination_slots(const rlnc_elimination *e) { return e ? e->e.slots() : 0; }
int rlnc_elimination_transform(const rlnc_elimination *e, uint8_t *T, size_t ld) {
    CHECK_ARG(e != nullptr && T != nullptr && ld >= e->e.slots());
    std::memset(T, 0, e->e.k() * ld);
    e->e.transform(T, ld);
    return RLNC_OK;
}
int rlnc_elimination_coefficients(const rlnc_elimination *e, uint8_t *C) {
    CHECK_ARG(e != nullptr && C != nullptr);
    for (size_t r = 0; r < e->e.rank(); ++r) std::memcpy(C + r * e->e.k(), e->e.row(r), e->e.k());
    return RLNC_OK;
}

}  // extern "C"
