// wire.hip — the data formats either side of the hot path, on the device:
//   * Encoder::new's padded image (encoder.rs:85-106, marker consts.rs:5) written by a kernel from a byte string
//     already in HBM: rlnc_pad_device / rlnc_pad_batch_device / rlnc_encoder_new_device;
//   * ragged batches: objects with their own shapes and buffers in one call -- the sender's encode
//     (rlnc_encode_ragged) and the receiver's recode and decode (rlnc_recode_ragged, rlnc_decode_ragged), as
//     socket or file ingestion produces them.  Each kernel stage is ONE launch over a device-side descriptor table
//     (per wave class of the bit-sliced program), not one launch per object or per shape.
// The coeffs ‖ data framing of a coded piece is written by the matmul kernels themselves (header copy), and the
// decoder's marker scan by a kernel here / in kernels.hip.
#include <algorithm>

#include "context.hpp"
#include "elimination.hpp"
#include "gf256.hpp"

using namespace rlnc::eng;

namespace {

// ---------------------------------------------------------------------------------------------------------------
// Descriptor tables on the device.
//   eager: pinned staging (guarded by an event: the previous upload's copy must have run before the staging buffer
//          is rewritten) → the context's table workspace, one copy on the context stream;
//   inside a HIP stream capture: a region of a capture arena that is never handed out again, filled by kernels
//          that carry the bytes as kernel arguments, so every replay of the graph rewrites exactly the captured
//          table -- a later eager call (which uses the staging path) cannot change what a replay reads, and no host
//          synchronisation on an event recorded inside the capture is needed.  The arena is reserved by eager calls
//          (allocation inside a capture is not allowed): run a call once eagerly before capturing it, as for the
//          workspaces (include/rlnc_hip.h, "HIP graphs").
// ---------------------------------------------------------------------------------------------------------------
constexpr size_t kChunk = 3072;  // table bytes per fill kernel (kernel arguments stay well below 4 KiB)
struct TableChunk {
    uint32_t bytes;
    uint32_t pad;
    uint8_t data[kChunk];
};

__global__ __launch_bounds__(256) void table_fill_kernel(uint8_t *dst, TableChunk c) {
    for (uint32_t i = threadIdx.x; i < c.bytes; i += 256) dst[i] = c.data[i];
}

// eager upload: the device reads the pinned staging buffer itself (one load per thread in flight across PCIe),
// instead of a hipMemcpyAsync host-to-device copy, whose DMA set-up put ~60 us ahead of the first kernel of a
// 256-object ragged recode (scripts/ragged_rate.py)
__global__ __launch_bounds__(256) void table_copy_kernel(uint4 *dst, const uint4 *src, uint32_t n16) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < n16) dst[i] = src[i];
}

int upload_table(rlnc_context *ctx, const void *host, size_t bytes, void **dev) {
    const size_t need = round16(std::max<size_t>(bytes, 16));
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(ctx->stream, &cs));
    if (cs != hipStreamCaptureStatusNone) {
        auto &arenas = ctx->cap_arenas;
        if (arenas.empty() || ctx->cap_used + need > arenas.back()->cap)
            return set_error(RLNC_ERR_INVALID_ARGUMENT,
                             "descriptor table of %zu bytes inside a HIP graph capture: run the same call once "
                             "eagerly before capturing it (that reserves the capture arena)",
                             bytes);
        uint8_t *d = arenas.back()->as<uint8_t>() + ctx->cap_used;
        ctx->cap_used += need;
        for (size_t off = 0; off < bytes; off += kChunk) {
            TableChunk c{};
            c.bytes = uint32_t(std::min(kChunk, bytes - off));
            std::memcpy(c.data, static_cast<const uint8_t *>(host) + off, c.bytes);
            hipLaunchKernelGGL(table_fill_kernel, dim3(1), dim3(256), 0, ctx->stream, d + off, c);
            HIP_TRY(hipGetLastError());
        }
        *dev = d;
        return RLNC_OK;
    }
    // eager: keep room in the capture arena for a captured call of this size (never moved once handed out)
    {
        auto &arenas = ctx->cap_arenas;
        const size_t reserve = 2 * need + (size_t(64) << 10);
        if (!ctx->graph_bound && (arenas.empty() || ctx->cap_used + reserve > arenas.back()->cap)) {
            std::unique_ptr<DevBuf> a(new (std::nothrow) DevBuf);
            if (!a) return set_error(RLNC_ERR_OUT_OF_MEMORY, "capture arena");
            if (int st = a->ensure(std::max<size_t>(size_t(1) << 20, 4 * reserve))) return st;
            arenas.push_back(std::move(a));
            ctx->cap_used = 0;
        }
    }
    int st;
    const int r = ctx->tab_next;
    ctx->tab_next = (r + 1) % rlnc_context::kTabRing;
    PinBuf &pin = ctx->pin_tab[r];
    hipEvent_t &ev = ctx->tab_ev[r];
    if (ev) HIP_TRY(hipEventSynchronize(ev));
    // the eager staging buffer and device table are never referenced by a captured graph (captured calls use the
    // capture arena above), so they grow even on a graph-bound context; each ring slot grows on its own first use
    // of a larger table.  The device table may still be read by earlier eager launches: drain the stream first.
    if (need > ctx->ws_tab.cap) HIP_TRY(hipStreamSynchronize(ctx->stream));
    if ((st = pin.ensure(need)) || (st = ctx->ws_tab.ensure(need))) return st;
    std::memcpy(pin.p, host, bytes);
    if (need / 16 > 0xFFFFFF00u) return set_error(RLNC_ERR_INVALID_ARGUMENT, "descriptor table too large");
    const uint32_t n16 = uint32_t(need / 16);
    hipLaunchKernelGGL(table_copy_kernel, dim3((n16 + 255) / 256), dim3(256), 0, ctx->stream,
                       static_cast<uint4 *>(ctx->ws_tab.p), static_cast<const uint4 *>(pin.p), n16);
    HIP_TRY(hipGetLastError());
    if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(ev, ctx->stream));
    *dev = ctx->ws_tab.p;
    return RLNC_OK;
}

// ---------------------------------------------------------------------------------------------------------------
// Encoder::new's padded image
// ---------------------------------------------------------------------------------------------------------------
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

int launch_pad(rlnc_context *ctx, const std::vector<PadDesc> &d) {
    int64_t max_blocks = 0;
    for (const auto &x : d) max_blocks = std::max<int64_t>(max_blocks, ((x.L + 15) / 16 * x.k + 255) / 256);
    if (max_blocks == 0) return RLNC_OK;
    if (max_blocks > 0x7FFFFFFF || d.size() > 65535) return set_error(RLNC_ERR_INVALID_ARGUMENT, "pad batch too large");
    void *dd = nullptr;
    int st = upload_table(ctx, d.data(), d.size() * sizeof(PadDesc), &dd);
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

// ---------------------------------------------------------------------------------------------------------------
// Ragged matmul: Out_o = Coef_o ⊗ In_o for objects of any shapes, one launch per kernel stage.  Each object's whole
// 4 KiB column blocks go to the bit-sliced program (the hot path of the uniform batches, §4.1 of DESIGN.md) -- one
// launch per tile class: 1, 2 and 4 waves (8-, 16- and 32-row tiles, as the uniform product sizes its tiles) for
// objects of <= 8, <= 16 and <= 32 output rows, 8 waves (64-row tiles) above -- after ONE launch that writes every
// object's block-address stream, and whatever it does not take (the ragged < 4 KiB tail, unaligned operands, < 4
// output rows) to one launch of the perm kernel.  So at most 6 launches, whatever the number of objects and shapes.
// ---------------------------------------------------------------------------------------------------------------
struct MatmulJob {
    const uint8_t *in, *coef;
    uint8_t *out, *hdr;
    int64_t in_row, coef_row, out_row, hdr_row, width;
    int n_out, n_in;
};

bool al16p(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int ragged_matmul(rlnc_context *ctx, const std::vector<MatmulJob> &jobs) {
    using rlnc::RaggedObj;
    std::vector<RaggedObj> cls[4], perm;  // bit-sliced classes of 1, 2, 4, 8 waves
    // the shared-set bit-sliced programs need their block table's address (one probe per device, synchronous the first
    // time; inside a capture that first probe cannot run: their objects then take the perm kernel, bit-identical)
    uint64_t base = 0;
    bool any_bsj = false;
    const bool uv = rlnc::unaligned_vector_ok();  // once per call: hipGetDevice per object was ~0.1 us each
    for (const auto &j : jobs)
        any_bsj |= j.n_out > 0 && j.n_in > 0 && j.width > 0 &&
                   rlnc::ragged_bsj_eligible(j.in, j.out, j.in_row, j.out_row, j.width, j.n_out, uv);
    int st;
    if (any_bsj) {
        if ((st = ctx->grow(ctx->ws_idx, 512))) return st;
        HIP_TRY(rlnc::ragged_bsj_base(ctx->stream, ctx->ws_idx.p, base));
    }
    for (const auto &j : jobs) {
        if (j.n_out <= 0 || j.n_in <= 0 || j.width <= 0) continue;
        int64_t full = 0;
        // (the 1- and 2-wave programs take block offsets, not addresses: no base needed)
        if ((base != 0 || rlnc::ragged_bsj_waves(j.n_out) <= 2) &&
            rlnc::ragged_bsj_eligible(j.in, j.out, j.in_row, j.out_row, j.width, j.n_out, uv)) {
            full = (j.width / rlnc::kRaggedColBlock) * rlnc::kRaggedColBlock;
            const int W = rlnc::ragged_bsj_waves(j.n_out);
            RaggedObj d{};
            d.in = j.in;
            d.coef = j.coef;
            d.out = j.out;
            d.hdr = j.hdr;
            d.in_row = j.in_row;
            d.coef_row = j.coef_row;
            d.out_row = j.out_row;
            d.hdr_row = j.hdr_row;
            d.col0 = 0;
            d.width = full;
            d.n_out = j.n_out;
            d.n_in = j.n_in;
            d.tile_rows = 8 * W;
            d.row_tiles = (j.n_out + d.tile_rows - 1) / d.tile_rows;
            d.col_blocks = int(full / rlnc::kRaggedColBlock);
            cls[W == 8 ? 3 : W == 4 ? 2 : W - 1].push_back(d);
        }
        if (full < j.width) {
            RaggedObj d{};
            d.in = j.in;
            d.coef = j.coef;
            d.out = j.out;
            d.hdr = full ? nullptr : j.hdr;  // the bit-sliced part (column block 0) already wrote the header
            d.in_row = j.in_row;
            d.coef_row = j.coef_row;
            d.out_row = j.out_row;
            d.hdr_row = j.hdr_row;
            d.col0 = full;
            d.width = j.width - full;
            d.n_out = j.n_out;
            d.n_in = j.n_in;
            d.row_tiles = (j.n_out + rlnc::kRaggedPermRows - 1) / rlnc::kRaggedPermRows;
            d.col_blocks = int((d.width + rlnc::kRaggedColBlock - 1) / rlnc::kRaggedColBlock);
            d.aligned = uv ||
                        (al16p(j.in + full) && al16p(j.out + full) && (j.in_row & 15) == 0 && (j.out_row & 15) == 0);
            perm.push_back(d);
        }
    }
    size_t nb = 0;
    for (auto &v : cls) nb += v.size();
    // the 1- and 2-wave classes by source count, most first (a workgroup's time is about its source count; their
    // kernel launches the tiles in table order: gf_matmul_bsj_ragged_kernel)
    for (int c = 0; c < 2; ++c)
        std::stable_sort(cls[c].begin(), cls[c].end(),
                         [](const RaggedObj &a, const RaggedObj &b) { return a.n_in > b.n_in; });
    const size_t np = perm.size();
    if (nb + np == 0) return RLNC_OK;
    if (nb + np > 0x7FFFFFFF) return set_error(RLNC_ERR_INVALID_ARGUMENT, "ragged batch too large");
    // table: [1-wave][2-wave][4-wave][8-wave bit-sliced][perm]; wg0 numbered per launch, idx0 (8-byte units) across
    // all the bit-sliced classes
    std::vector<RaggedObj> tab;
    tab.reserve(nb + np);
    int64_t idx = 0, wgc[4] = {0, 0, 0, 0}, wgp = 0;
    for (int c = 0; c < 4; ++c)
        for (auto &d : cls[c]) {
            d.wg0 = wgc[c];
            d.idx0 = idx;
            wgc[c] += int64_t(d.row_tiles) * d.col_blocks;
            idx += int64_t(d.row_tiles) * d.n_in * d.tile_rows;
            tab.push_back(d);
        }
    for (auto &d : perm) {
        d.wg0 = wgp;
        wgp += int64_t(d.row_tiles) * d.col_blocks;
        tab.push_back(d);
    }
    if (std::max({wgc[0], wgc[1], wgc[2], wgc[3], wgp}) > 0x7FFFFFFF)
        return set_error(RLNC_ERR_INVALID_ARGUMENT, "ragged batch too large for one launch");
    if (idx > 0 && (st = ctx->grow(ctx->ws_idx, size_t(idx) * 8 + 512))) return st;
    void *dtab = nullptr;
    if ((st = upload_table(ctx, tab.data(), tab.size() * sizeof(RaggedObj), &dtab))) return st;
    const RaggedObj *t = static_cast<const RaggedObj *>(dtab);
    HIP_TRY(rlnc::launch_ragged_offsets(t, int(nb), idx, ctx->ws_idx.p, base, ctx->stream));
    size_t at = 0;
    for (int c = 0; c < 4; ++c) {
        HIP_TRY(rlnc::launch_ragged_bsj(1 << c, t + at, int(cls[c].size()), wgc[c], ctx->ws_idx.p, ctx->stream));
        at += cls[c].size();
    }
    HIP_TRY(rlnc::launch_ragged_perm(t + nb, int(np), wgp, ctx->stream));
    return RLNC_OK;
}

// ---------------------------------------------------------------------------------------------------------------
// Ragged get_decoded_data (decoder.rs:136-177): one wave per object scans its padded payload from the end (the last
// nonzero byte must be the 0x81 marker, not at index 0), objects of rank < k report NotAllPiecesReceivedYet.
// ---------------------------------------------------------------------------------------------------------------
struct ScanObj {
    const uint8_t *data;
    const int32_t *rank;
    int32_t *status;
    int64_t *len_out;
    int64_t len;
    int32_t k, pad;
};

__global__ __launch_bounds__(64) void ragged_final_len_kernel(const ScanObj *objs) {
    const ScanObj d = objs[blockIdx.x];
    const int lane = threadIdx.x;
    if (*d.rank < d.k) {  // decoder.rs:137-139
        if (lane == 0) {
            *d.status = RLNC_ERR_NOT_ALL_PIECES_RECEIVED_YET;
            *d.len_out = 0;
        }
        return;
    }
    int64_t last = -1;  // index of the last nonzero byte (wave-uniform after the reduction)
    for (int64_t c = (d.len + 1023) / 1024 - 1; c >= 0 && last < 0; --c) {
        int64_t mine = -1;
        for (int q = 0; q < 16; ++q) {
            const int64_t i = c * 1024 + int64_t(lane) * 16 + q;
            if (i < d.len && d.data[i] != 0) mine = i;
        }
        for (int o = 32; o > 0; o >>= 1) {
            const int64_t v = __shfl_xor(mine, o);
            mine = v > mine ? v : mine;
        }
        last = mine;
    }
    if (lane == 0) {
        const bool ok = last > 0 && d.data[last] == rlnc::kBoundaryMarker;
        *d.status = ok ? RLNC_OK : RLNC_ERR_INVALID_DECODED_DATA_FORMAT;
        *d.len_out = ok ? last : 0;
    }
}

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

// encoder.rs:241-250 for every object: n coded pieces coeffs ‖ Σ coeffs·src each
int rlnc_encode_ragged(rlnc_context *ctx, const rlnc_object_desc *objs, size_t count) {
    CHECK_ARG(ctx != nullptr);
    if (count == 0) return RLNC_OK;
    CHECK_ARG(objs != nullptr);
    std::vector<MatmulJob> jobs;
    jobs.reserve(count);
    for (size_t i = 0; i < count; ++i) {  // every descriptor is checked before anything is launched
        const rlnc_object_desc &o = objs[i];
        if (o.k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;
        if (o.L == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;
        if (o.n == 0) continue;
        CHECK_ARG(o.src && o.coeffs && o.pieces && o.n <= 0x7FFFFFFF && o.k <= 0x7FFFFFFF);
        CHECK_ARG(o.src_row_stride == 0 || o.src_row_stride >= o.L);
        CHECK_ARG(o.piece_row_stride == 0 || o.piece_row_stride >= o.k + o.L);
        const int64_t ss = int64_t(o.src_row_stride ? o.src_row_stride : o.L);
        const int64_t ps = int64_t(o.piece_row_stride ? o.piece_row_stride : o.k + o.L);
        jobs.push_back(MatmulJob{o.src, o.coeffs, o.pieces + o.k, o.pieces, ss, int64_t(o.k), ps, ps, int64_t(o.L),
                                 int(o.n), int(o.k)});
    }
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    return ragged_matmul(ctx, jobs);
}

// recoder.rs:122-153 for every object: out[i] = Σ_j r[i][j] · piece_j over the full pieces (coefficient header and
// data are one linear map)
int rlnc_recode_ragged(rlnc_context *ctx, const rlnc_recode_object_desc *objs, size_t count) {
    CHECK_ARG(ctx != nullptr);
    if (count == 0) return RLNC_OK;
    CHECK_ARG(objs != nullptr);
    std::vector<MatmulJob> jobs;
    jobs.reserve(count);
    for (size_t i = 0; i < count; ++i) {
        const rlnc_recode_object_desc &o = objs[i];
        if (o.n == 0) return RLNC_ERR_NOT_ENOUGH_PIECES_TO_RECODE;  // recoder.rs:69-71
        if (o.k + o.L == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;       // :72-74
        if (o.k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;              // :75-77
        if (o.L == 0) return RLNC_ERR_PIECE_LENGTH_TOO_SHORT;        // :78-80 (full <= k)
        if (o.n_recoded == 0) continue;
        CHECK_ARG(o.pieces && o.r && o.out && o.n <= 0x7FFFFFFF && o.n_recoded <= 0x7FFFFFFF);
        CHECK_ARG(o.piece_row_stride == 0 || o.piece_row_stride >= o.k + o.L);
        CHECK_ARG(o.out_row_stride == 0 || o.out_row_stride >= o.k + o.L);
        const int64_t ps = int64_t(o.piece_row_stride ? o.piece_row_stride : o.k + o.L);
        const int64_t os = int64_t(o.out_row_stride ? o.out_row_stride : o.k + o.L);
        jobs.push_back(MatmulJob{o.pieces, o.r, o.out, nullptr, ps, int64_t(o.n), os, 0, int64_t(o.k + o.L),
                                 int(o.n_recoded), int(o.n)});
    }
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    return ragged_matmul(ctx, jobs);
}

// Decoder::decode over pieces 0..m-1 + get_decoded_data (decoder.rs:96-177) for every object: the exact elimination
// (one launch for the objects whose [coeffs | E] fits a wave's row, k + m <= 256, one for larger ones that fit LDS;
// host threads for any beyond LDS), T × received data (the ragged matmul, <= 4 launches), the marker scan (1 launch)
int rlnc_decode_ragged(rlnc_context *ctx, const rlnc_decode_object_desc *objs, size_t count, int32_t *piece_status_dev,
                       int32_t *object_status_dev, int64_t *data_len_dev) {
    CHECK_ARG(ctx != nullptr);
    if (count == 0) return RLNC_OK;
    CHECK_ARG(objs != nullptr && piece_status_dev && object_status_dev && data_len_dev && count <= 0x7FFFFFFF);
    size_t tot_T = 0;
    for (size_t i = 0; i < count; ++i) {
        const rlnc_decode_object_desc &o = objs[i];
        if (o.L == 0) return RLNC_ERR_PIECE_LENGTH_ZERO;  // decoder.rs:66-68
        if (o.k == 0) return RLNC_ERR_PIECE_COUNT_ZERO;   // :69-71
        CHECK_ARG(o.pieces && o.decoded && o.m > 0 && o.m <= 0x7FFFFFFF && o.k <= 0x7FFFFFFF);
        CHECK_ARG(o.piece_row_stride == 0 || o.piece_row_stride >= o.k + o.L);
        tot_T += o.k * o.m;
    }
    int st = ctx->activate();
    if (st || (st = ctx->note_capture())) return st;
    if ((st = ctx->grow(ctx->ws_coef, tot_T)) || (st = ctx->grow(ctx->ws_rank, count * 4))) return st;
    uint8_t *T = ctx->ws_coef.as<uint8_t>();
    int32_t *rank = ctx->ws_rank.as<int32_t>();
    // 1. the exact elimination
    std::vector<rlnc::RrefObj> blk, wide;
    std::vector<size_t> host, toff(count), soff(count);
    size_t lds_blk = 0;
    int hdr_lds = 1;
    {
        size_t to = 0, so = 0;
        for (size_t i = 0; i < count; ++i) {
            const rlnc_decode_object_desc &o = objs[i];
            const int k = int(o.k), m = int(o.m);
            const size_t ps = o.piece_row_stride ? o.piece_row_stride : o.k + o.L;
            toff[i] = to;
            soff[i] = so;
            rlnc::RrefObj r{o.pieces, int64_t(ps), T + to, piece_status_dev + so, rank + i, k, m, 0, 0};
            if (rlnc::rref_block_eligible(k, m)) {
                blk.push_back(r);
                lds_blk = std::max(lds_blk, rlnc::rref_block_lds_bytes_public(k, m));
            } else if (rlnc::rref_lds_bytes(k, m) <= rlnc::kRrefMaxLds) {
                // k <= 128: the blocked run over the first 256 - k pieces, the general kernel only for an object
                // that did not reach rank k within them (rref.hip launch_rref_batch, two passes)
                if (k <= 128 && rlnc::rref_block_eligible(k, 256 - k)) {
                    r.m_first = 256 - k;
                    r.two_pass = 1;
                    blk.push_back(r);
                    lds_blk = std::max(lds_blk, rlnc::rref_block_lds_bytes_public(k, 256 - k));
                }
                wide.push_back(r);
                if (rlnc::rref_lds_bytes_staged_public(k, m) > rlnc::kRrefMaxLds) hdr_lds = 0;
            } else {
                host.push_back(i);
            }
            to += o.k * o.m;
            so += o.m;
        }
    }
    size_t lds_wide = 0;  // one wide object's headers not fitting beside its matrix: none are staged
    for (const auto &r : wide)
        lds_wide = std::max(lds_wide, hdr_lds ? rlnc::rref_lds_bytes_staged_public(r.k, r.m) : rlnc::rref_lds_bytes(r.k, r.m));
    if (!blk.empty() || !wide.empty()) {
        std::vector<rlnc::RrefObj> tab(blk);
        tab.insert(tab.end(), wide.begin(), wide.end());
        void *dt = nullptr;
        if ((st = upload_table(ctx, tab.data(), tab.size() * sizeof(rlnc::RrefObj), &dt))) return st;
        const auto *t = static_cast<const rlnc::RrefObj *>(dt);
        HIP_TRY(rlnc::launch_rref_ragged(t, int(blk.size()), true, lds_blk, 1, ctx->stream));
        HIP_TRY(rlnc::launch_rref_ragged(t + blk.size(), int(wide.size()), false, lds_wide, hdr_lds, ctx->stream));
    }
    if (!host.empty()) {  // beyond LDS (k of several hundred): host threads' exact elimination, T and statuses uploaded
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        HIP_TRY(hipStreamIsCapturing(ctx->stream, &cs));
        if (cs != hipStreamCaptureStatusNone)
            return set_error(RLNC_ERR_INVALID_ARGUMENT, "a ragged decode with objects beyond LDS cannot be captured");
        for (size_t i : host) {
            const rlnc_decode_object_desc &o = objs[i];
            const size_t ps = o.piece_row_stride ? o.piece_row_stride : o.k + o.L;
            std::vector<uint8_t> hdr(o.m * o.k), Th(o.k * o.m, 0);
            std::vector<int32_t> pst(o.m);
            HIP_TRY(hipMemcpy2DAsync(hdr.data(), o.k, o.pieces, ps, o.k, o.m, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            rlnc::Elimination e(o.k, o.m);
            for (size_t p = 0; p < o.m; ++p) {
                int slot;
                bool keep;
                pst[p] = e.push(hdr.data() + p * o.k, &slot, &keep);
            }
            e.transform(Th.data(), o.m);
            const int32_t r = int32_t(e.rank());
            HIP_TRY(hipMemcpyAsync(T + toff[i], Th.data(), Th.size(), hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(hipMemcpyAsync(piece_status_dev + soff[i], pst.data(), o.m * 4, hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(hipMemcpyAsync(rank + i, &r, 4, hipMemcpyHostToDevice, ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));  // the host vectors go out of scope
        }
    }
    // 2. decoded rows = T × received data rows
    std::vector<MatmulJob> jobs;
    jobs.reserve(count);
    for (size_t i = 0; i < count; ++i) {
        const rlnc_decode_object_desc &o = objs[i];
        const int64_t ps = int64_t(o.piece_row_stride ? o.piece_row_stride : o.k + o.L);
        jobs.push_back(MatmulJob{o.pieces + o.k, T + toff[i], o.decoded, nullptr, ps, int64_t(o.m), int64_t(o.L), 0,
                                 int64_t(o.L), int(o.k), int(o.m)});
    }
    if ((st = ragged_matmul(ctx, jobs))) return st;
    // 3. the marker scan
    std::vector<ScanObj> scan(count);
    for (size_t i = 0; i < count; ++i)
        scan[i] = ScanObj{objs[i].decoded, rank + i, object_status_dev + i, data_len_dev + i,
                          int64_t(objs[i].k * objs[i].L), int32_t(objs[i].k), 0};
    void *ds = nullptr;
    if ((st = upload_table(ctx, scan.data(), scan.size() * sizeof(ScanObj), &ds))) return st;
    hipLaunchKernelGGL(ragged_final_len_kernel, dim3(unsigned(count)), dim3(64), 0, ctx->stream,
                       static_cast<const ScanObj *>(ds));
    HIP_TRY(hipGetLastError());
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
    // pad, then wait for the image, then adopt it: a failed pad or sync leaves nothing behind (*out stays null)
    if ((st = rlnc_pad_batch_device(ctx, &d, 1)) == RLNC_OK) {
        const hipError_t e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess)
            st = set_error(RLNC_ERR_DEVICE, "hipStreamSynchronize after the pad kernel: %s", hipGetErrorString(e));
    }
    if (st == RLNC_OK) st = encoder_adopt_device(ctx, img, k, L, stride, out);
    if (st != RLNC_OK) {
        (void)hipFree(img);
        *out = nullptr;
    }
    return st;
}

}  // extern "C"
