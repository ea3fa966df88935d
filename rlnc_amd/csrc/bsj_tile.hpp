// bsj_tile.hpp — the tile body of the bit-sliced jump programs (the generated inline-asm programs of
// bitslice_jump.inc, gen_bsjump.py): one workgroup's output rows x one 4 KiB column block.  Shared by the uniform and
// ragged kernels of kernels.hip and the column-run A/B variant of kernels_ab.hip (internal to librlnc_hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/rlnc_hip.h"
#include "bitslice_jump.inc"
#include "gf256.hpp"
#include "kernels.hpp"

#ifndef RLNC_BSJ_SOFFSETS
#error "bitslice_jump.inc must be generated with packed blocks (gen_bsjump.py default)"
#endif

namespace rlnc {
namespace {

constexpr int kBsjWaveRows = RLNC_BSJ_NT;  // output rows per wave; a workgroup of W waves = 8 W rows
constexpr int kBsjColBlock = 4096;          // 64 lanes × 64 B, shared by the W waves

// SHARE (W = 4 only): wave w builds one of the four combination sets of each source row and the sets are
// exchanged through LDS (RLNC_BSJ_ASM_W4S) instead of every wave building all four
// probe != nullptr (SHARE only): store the block table's address there and return (launch_bsj, once per device)
// RUN (W = 8 only, variant 9): the workgroup walks `run` consecutive column blocks of one (object, row tile) --
// the column-run program (RLNC_BSJ_ASM_W8R) carries the source-row stream across the tile boundaries, so only the
// first tile pays the prologue (first DMAs, first sets); the grid is objects x row tiles x runs
// The tile of one workgroup: output rows [rt * 8W, +8W) x column block cb of object obj (the uniform batch
// kernel below and the ragged kernel both end here).
// The marker scan of an object whose tile this workgroup holds whole (MatmulParams::scan_need; decoder.rs:162-177: the
// last nonzero byte of the padded payload must be the 0x81 marker, not at index 0), for objects whose payload tail the
// elimination found all zero: every wave's tile stores done and visible to the workgroup, then wave 0 walks the rows
// from the last one, 64 B a lane, the last nonzero byte found by a wave max (DPP row rotations + permlane swaps) of
// (offset + 1) << 8 | byte.  (rank < k never gets here: the elimination answered NotAllPiecesReceivedYet.)
__device__ __forceinline__ uint32_t tile_wave_max(uint32_t a) {
    a = max(a, uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x121, 0xf, 0xf, false)));  // row_ror:1
    a = max(a, uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x122, 0xf, 0xf, false)));  // row_ror:2
    a = max(a, uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x124, 0xf, 0xf, false)));  // row_ror:4
    a = max(a, uint32_t(__builtin_amdgcn_update_dpp(0, int(a), 0x128, 0xf, 0xf, false)));  // row_ror:8
    const auto s16 = __builtin_amdgcn_permlane16_swap(a, a, false, false);
    a = max(s16[0], s16[1]);
    const auto s32 = __builtin_amdgcn_permlane32_swap(a, a, false, false);
    return max(s32[0], s32[1]);
}

__device__ __forceinline__ void bsj_tile_scan(const MatmulParams &p, int obj) {
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's tile stores (issued inside the program)
    __syncthreads();                                       // ... and every other wave's
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    const uint8_t *base = p.out + int64_t(obj) * p.out_obj;
    int64_t hit = -1;
    uint32_t byte = 0;
    for (int r = p.scan_k - 1; r >= 0; --r) {
        const uint4 *q = reinterpret_cast<const uint4 *>(base + int64_t(r) * p.out_row + 64 * lane);
        uint32_t mine = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint4 x = q[u];
            const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (w[t]) {
                    const int b = (31 - __builtin_clz(w[t])) / 8;
                    mine = (uint32_t(64 * lane + 16 * u + 4 * t + b + 1) << 8) | ((w[t] >> (8 * b)) & 0xFFu);
                }
        }
        const uint32_t best = __builtin_amdgcn_readfirstlane(tile_wave_max(mine));
        if (best) {
            hit = int64_t(r) * p.width + int64_t(best >> 8) - 1;
            byte = best & 0xFFu;
            break;
        }
    }
    if (lane == 0) {
        const bool ok = hit > 0 && byte == kBoundaryMarker;
        p.scan_status[obj] = ok ? RLNC_OK : RLNC_ERR_INVALID_DECODED_DATA_FORMAT;
        p.scan_len[obj] = ok ? hit : 0;
    }
}

template <int W, bool SHARE, bool RUN>
__device__ __forceinline__ void bsj_tile(const MatmulParams &p, const void *stream, int row_tiles, int rt, int cb,
                                         int obj, uint32_t tiles, uint64_t *probe) {
    constexpr int kTileRows = kBsjWaveRows * W;
    // W = 8: one workgroup per CU, so a deeper ring and 2 BAR8 set slots (the builders run BAR8 rows ahead); the
    // 4-wave shared program may take the same form (gen_bsjump.py --w4bar: RLNC_BSJ_SLOTS4S ring slots); W = 1: a
    // deeper ring too (its one wave alone keeps the source rows in flight)
    __shared__ __attribute__((aligned(16))) uint8_t
        ring[(W == 8 ? RLNC_BSJ_SLOTS8 : W == 1 ? RLNC_BSJ_SLOTS1 : W == 2 ? RLNC_BSJ_SLOTS2
                                                    : SHARE ? RLNC_BSJ_SLOTS4S : RLNC_BSJ_SLOTS) *
             kBsjColBlock];
    __shared__ __attribute__((aligned(16))) uint8_t cset[SHARE ? (W == 8 ? RLNC_BSJ_CSET_BYTES8 : RLNC_BSJ_CSET_BYTES) : 16];
    const int row0 = rt * kTileRows;
    const int rows = min(kTileRows, p.n_out - row0);
    if (p.hdr != nullptr && cb == 0) {  // coded-piece header (encoder.rs:246-248), 64·W threads
        const uint8_t *coef_base = p.coef + int64_t(obj) * p.coef_obj + int64_t(row0) * p.coef_row;
        uint8_t *h = p.hdr + int64_t(obj) * p.hdr_obj + int64_t(row0) * p.hdr_row;
        for (int e = threadIdx.x; e < rows * p.n_in; e += 64 * W) {
            const int i = e / p.n_in, j = e % p.n_in;
            h[int64_t(i) * p.hdr_row + j] = coef_base[int64_t(i) * p.coef_row + j];
        }
    }
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    // the split 2-wave program (gen_bsjump.py --w2split): wave w owns the 2 KiB half w of the column block in all
    // the tile's rows, instead of rows [8 w, 8 w + 8) in the whole block
#ifdef RLNC_BSJ_W2SPLIT
    constexpr bool kSplit = W == 2;
#else
    constexpr bool kSplit = false;
#endif
    const int wr = kSplit ? 0 : w;  // the wave's first row in the tile (in wave rows)
    const int rows_w =
        __builtin_amdgcn_readfirstlane(kSplit ? rows : max(0, min(kBsjWaveRows, rows - kBsjWaveRows * w)));
    const uint8_t *src = p.in + int64_t(obj) * p.in_obj + int64_t(cb) * kBsjColBlock;
    uint8_t *dst = p.out + int64_t(obj) * p.out_obj + int64_t(row0 + kBsjWaveRows * wr) * p.out_row +
                   int64_t(cb) * kBsjColBlock + (kSplit ? 2048 * w : 0);
    constexpr int kEntry = SHARE ? 8 : 4;  // bytes per stream entry: absolute address / block offset
    const uint8_t *idx = static_cast<const uint8_t *>(stream) +
                         ((int64_t(obj) * row_tiles + rt) * p.n_in * kTileRows + kBsjWaveRows * wr) * kEntry;
    typedef __attribute__((address_space(3))) uint8_t lds_u8;
    const uint32_t ring_lds = uint32_t(reinterpret_cast<uintptr_t>((lds_u8 *)ring));  // addrspacecast
    // W = 8 (shared): waves 0-3 stage the ring and build the sets exactly as in the 4-wave program, waves 4-7
    // (cons = 1) only read the sets and call
    constexpr int kStageWaves = (SHARE && W == 8) ? 4 : W;
    const int ws = w % kStageWaves;
    constexpr uint32_t kShare = kBsjColBlock / kStageWaves;  // bytes of each row a wave moves into the ring
    const uint32_t ldsw = __builtin_amdgcn_readfirstlane(ring_lds + kShare * uint32_t(ws));
    const uint32_t ldsr = ring_lds + 16u * lane;
    const uint32_t dmaoff = kShare * uint32_t(ws) + 16u * lane;
    const uint32_t off = 16u * lane;
    const uint32_t ldsc = uint32_t(reinterpret_cast<uintptr_t>((lds_u8 *)cset)) + 16u * lane;
    // this wave's set (group ws >> 1, half ws & 1) and the second set-slot base: per program (gen_bsjump.py --setregs4 /
    // --setregs8, --banks)
    constexpr uint32_t kCsSet = W == 8 ? uint32_t(RLNC_BSJ_CS_SET8) : uint32_t(RLNC_BSJ_CS_SET);
    constexpr uint32_t kCsBase2 = W == 8 ? uint32_t(RLNC_BSJ_CS_BASE2_8) : uint32_t(RLNC_BSJ_CS_BASE2);
    const uint32_t ldscw = ldsc + kCsSet * uint32_t(ws);
    const uint32_t ldsrg = ldsr + 2048u * uint32_t(kSplit ? ws : ws >> 1);  // this wave's group of the ring chunk
    const uint32_t half = uint32_t(ws & 1);
    const uint32_t cons = uint32_t(w / kStageWaves);
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#define RLNC_BSJ_OPERANDS                                                                                            \
    : [src] "s"(src), [idx] "s"(idx), [dst] "s"(dst), [in_row] "s"(uint32_t(p.in_row)),                           \
      [out_row] "s"(uint32_t(p.out_row)), [n_in] "s"(p.n_in), [rows] "s"(rows_w), [ldsw] "s"(ldsw), [off] "v"(off), \
      [dmaoff] "v"(dmaoff), [ldsr] "v"(ldsr), [ldsc] "v"(ldsc), [ldscw] "v"(ldscw), [ldsrg] "v"(ldsrg),           \
      [half] "s"(half), [probe] "s"(probe), [cons] "s"(cons), [ldsc2] "v"(ldsc + kCsBase2),                      \
      [ldscw2] "v"(ldscw + kCsBase2), [tiles] "s"(tiles)                                                          \
    : RLNC_BSJ_CLOBBER_V, RLNC_BSJ_CLOBBER_S
    if constexpr (W == 1) asm volatile(RLNC_BSJ_ASM_W1 : RLNC_BSJ_OPERANDS);
    if constexpr (W == 2) asm volatile(RLNC_BSJ_ASM_W2 : RLNC_BSJ_OPERANDS);
    if constexpr (W == 4 && !SHARE) asm volatile(RLNC_BSJ_ASM_W4 : RLNC_BSJ_OPERANDS);
    if constexpr (W == 4 && SHARE) asm volatile(RLNC_BSJ_ASM_W4S : RLNC_BSJ_OPERANDS);
    if constexpr (W == 8 && !RUN) asm volatile(RLNC_BSJ_ASM_W8S : RLNC_BSJ_OPERANDS);
    if constexpr (W == 8 && RUN) asm volatile(RLNC_BSJ_ASM_W8R : RLNC_BSJ_OPERANDS);
#undef RLNC_BSJ_OPERANDS
#pragma clang diagnostic pop
    if constexpr (W <= 2 && !SHARE && !RUN)
        if (p.scan_status != nullptr && p.scan_need[obj] != 0) bsj_tile_scan(p, obj);
}

}  // namespace
}  // namespace rlnc
