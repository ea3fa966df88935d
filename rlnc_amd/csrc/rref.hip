// rref.hip — the decoder's coefficient-side elimination on the device, one wave per object.
//
// Replays Decoder::decode (src/full/decoder.rs:96-118) for pieces 0..m-1 of every object, exactly like
// the host engine (elimination.hpp): the diagonal-pivot RREF of DecoderMatrix
// (src/full/decoder_matrix.rs:99-244) is run on [coeffs | E] where E (m columns) tracks every row as a
// combination of the received pieces.  Outputs per object: the status of every decode() call, the rank,
// and T = E (k × m, rows >= rank zero) so that decoded rows = T × received data rows (one matmul).
//
// Two paths, both exact:
//   * generic — the reference algorithm verbatim (pivot test, swap with the first nonzero row below,
//     eliminate every row below/above with q = M[j][i] / M[i][i] from column i on, normalise from column
//     i+1, drop rows whose k coefficient bytes are zero), with the independent row operations of one step
//     done in parallel across the wave;
//   * clean  — used while rows 0..r-1 are a clean RREF (M[i][i] = 1 and every pivot column zero in the
//     other rows).  Then the reference's forward pass only touches the new row r and all its quotients are
//     the ORIGINAL coefficients M[r][i] (row i is zero in every other pivot column), so the whole forward
//     pass is one vector-matrix product; its backward pass only eliminates column r from the rows above
//     and normalises row r.  Same products, same XORs, same bytes — computed with all lanes at once.
//     Leaving the clean state (a zero diagonal after the forward pass: SURVEY.md §0.5) switches to the
//     generic path, which re-checks cleanliness after every piece.
// GF products use v_perm_b32 with the 3-bit split tables of all 256 multipliers staged in LDS (copied from a
// compile-time table), and all m piece headers are staged in LDS up front when they fit: the per-piece loop
// then never waits on HBM.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>

#include "../../include/rlnc_hip.h"
#include "gf256.hpp"
#include "kernels.hpp"
#include "rref_kernels.hpp"

namespace rlnc {

bool rref_block_eligible(int k, int m) {
    return rref_row_dwords(k, m) <= 64 && rref_block_lds_bytes(k, m) <= kRrefMaxLds;
}

size_t rref_lds_bytes(int k, int m) {
    return kTabEntries * kTabDw * 4 + size_t(k + 1) * 4 * size_t(rref_row_dwords(k, m)) + 4 * ((size_t(m) + 3) & ~size_t(3));
}

size_t rref_block_lds_bytes_public(int k, int m) { return rref_block_lds_bytes(k, m); }

// The A/B build (make ab) links rref_ab.hip, whose definition replaces this one
__attribute__((weak)) bool launch_rref_ab(const RrefParams &, hipStream_t, hipError_t *) { return false; }
size_t rref_lds_bytes_staged_public(int k, int m) { return rref_lds_bytes_staged(k, m); }

hipError_t launch_rref_ragged(const RrefObj *objs, int n, bool block, size_t lds, int hdr_lds, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (lds > kRrefMaxLds) return hipErrorInvalidValue;
    RrefParams p{};
    p.objs = objs;
    p.n_obj = n;
    p.skip_full = block ? 0 : 1;  // the general launch skips two-pass objects the blocked launch full-ranked
    // the dynamic-LDS attribute of both kernels (a first launch through launch_rref_batch may not have run yet)
    static std::mutex mu;
    static bool attr_set[64] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    {
        std::lock_guard<std::mutex> lock(mu);
        if (!attr_set[dev]) {
            e = hipFuncSetAttribute(reinterpret_cast<const void *>(&gf_rref_block_kernel<kBlkNW, 8>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, int(kRrefMaxLds));
            if (e == hipSuccess)
                e = hipFuncSetAttribute(reinterpret_cast<const void *>(&gf_rref_batch_kernel<0, 1, 1>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, int(kRrefMaxLds));
            if (e != hipSuccess) return e;
            attr_set[dev] = true;
        }
    }
    if (block)
        hipLaunchKernelGGL((gf_rref_block_kernel<kBlkNW, 8>), dim3(n), dim3(64 * kBlkNW), lds, s, p);
    else
        hipLaunchKernelGGL((gf_rref_batch_kernel<0, 1, 1>), dim3(n), dim3(64), lds, s, p, hdr_lds);
    return hipGetLastError();
}

static hipError_t launch_rref_one(const RrefParams &p, hipStream_t s, bool *bsj_written);

// k + m > 256 with k <= 128: the blocked run over the first 256 - k pieces (>= k), then the general kernel over all m
// pieces for the objects that did not reach rank k within them (with dense coefficients: none).  Same outputs as the
// general kernel alone (RrefParams::m_stride); 32 objects of k = 128, m = 130: 4.0 ms in the one-wave LDS kernel.
hipError_t launch_rref_batch(const RrefParams &p, hipStream_t s, bool *bsj_written) {
    if (bsj_written) *bsj_written = false;
    if (p.n_obj <= 0) return hipSuccess;
    if (p.lds_only == 0 && p.objs == nullptr && p.m_stride == 0 && !p.skip_full && p.k <= 128 &&
        rref_row_dwords(p.k, p.m) > 64 && rref_lds_bytes(p.k, p.m) <= kRrefMaxLds &&
        rref_block_lds_bytes(p.k, 256 - p.k) <= kRrefMaxLds) {
        RrefParams a = p;
        a.m = 256 - p.k;
        a.m_stride = p.m;
        a.bsj_stream = nullptr;
        a.tail_status = nullptr;
        hipError_t e = launch_rref_one(a, s, nullptr);
        if (e != hipSuccess) return e;
        RrefParams b = p;
        b.skip_full = 1;
        b.bsj_stream = nullptr;
        b.tail_status = nullptr;
        return launch_rref_one(b, s, nullptr);
    }
    return launch_rref_one(p, s, bsj_written);
}

static hipError_t launch_rref_one(const RrefParams &p, hipStream_t s, bool *bsj_written) {
    hipError_t ab = hipSuccess;
    if (launch_rref_ab(p, s, &ab)) return ab;  // the A/B build's paths (rref_ab.hip); false in the shipped library
    // many small objects (k <= 16, >= 2048 of them: 8 per CU and more): the one-wave register kernel (path 4's)
    // beats the 4-wave blocked run, whose per-object parallelism the full grid no longer needs -- 4,096 x k = 16:
    // 0.093 vs 0.125 ms, k = 8: 0.051 vs 0.067, k = 16 sparse + dependent: 0.195 vs 0.295; at 512 objects the
    // blocked run stays faster (0.035 vs 0.049) (profiles/r02_elim_small_k.jsonl)
    constexpr int small_min = kSmallMinObjects;
    const bool small_many = p.lds_only == 0 && p.k <= 16 && p.n_obj >= small_min && rref_row_dwords(p.k, p.m) <= 16 &&
                            rref_lds_bytes_staged(p.k, p.m) <= kRrefMaxLds;
    // the blocked clean run (4 waves per object, the default) when the row fits one wave (k + m <= 256)
    if (!small_many && (p.lds_only == 0 || p.lds_only == 3) && rref_row_dwords(p.k, p.m) <= 64 &&
        rref_block_lds_bytes(p.k, p.m) <= kRrefMaxLds) {
        static_assert(kBlkDefault == 8, "the shipped block size");
        auto kern = &gf_rref_block_kernel<kBlkNW, 8>;
        static std::mutex mu;
        static bool attr_set[64] = {};
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
        {
            std::lock_guard<std::mutex> lock(mu);
            if (!attr_set[dev]) {
                for (auto f : {&gf_rref_block_kernel<kBlkNW, 8>}) {
                    e = hipFuncSetAttribute(reinterpret_cast<const void *>(f), hipFuncAttributeMaxDynamicSharedMemorySize,
                                            int(kRrefMaxLds));
                    if (e != hipSuccess) return e;
                }
                attr_set[dev] = true;
            }
        }
        hipLaunchKernelGGL(kern, dim3(p.n_obj), dim3(64 * kBlkNW), rref_block_lds_bytes(p.k, p.m), s, p);
        return hipGetLastError();
    }
    if (small_many && p.k <= 16 && rref_row_dwords(p.k, p.m) <= 16) {
        // kSmallNW objects per workgroup over one table copy (<= 16 KiB + 4 x 2 KiB: under the default LDS limit)
        // rows of 8 dwords or fewer (k + m <= 32): 8 lane groups of 4 registers (123 VGPRs: 4 waves per SIMD) and
        // kSmallNW objects per workgroup; wider rows: 4 groups of 8 (199 VGPRs, 2 waves per SIMD, where the 8 objects
        // per CU the one-object workgroups already hold are all the VGPRs allow) -- profiles/r03_small_elim_ab.txt
        // rows <= k <= 16 = G x RT: 2 registers of 8 lane groups (4 of 4 groups) hold every row; the round-4 forms
        // carried 4 (8) registers per lane, half of them always zero rows (products with q = 0, still issued)
        const bool g8 = rref_row_dwords(p.k, p.m) <= 8;
        auto kern = g8 ? &gf_rref_small_kernel<kSmallNW, 8, 2> : &gf_rref_small_kernel<1, 4, 4>;
        int nw = g8 ? kSmallNW : 1;
        const size_t lds_small = size_t(kTabEntries) * kTabDw * 4 + nw * rref_small_wave_bytes(p.k, p.m) +
                                 (p.tail_status != nullptr ? nw * rref_small_tail_bytes(p.m) : 0);
        hipLaunchKernelGGL(kern, dim3((p.n_obj + nw - 1) / nw), dim3(64 * nw), lds_small, s, p);
        const hipError_t e = hipGetLastError();
        if (e == hipSuccess && bsj_written) *bsj_written = p.bsj_stream != nullptr && p.bsj_tile_rows > 0;
        return e;
    }
    size_t lds = rref_lds_bytes(p.k, p.m);
    if (lds > kRrefMaxLds) return hipErrorInvalidValue;
    const int hdr_lds = rref_lds_bytes_staged(p.k, p.m) <= kRrefMaxLds ? 1 : 0;
    if (hdr_lds) lds = rref_lds_bytes_staged(p.k, p.m);
    // register-resident clean path when the matrix fits: rows <= G·RT, row dwords <= 64 / G; the initial clean
    // run spread over 4 waves (reg_run_mw) up to k = 64
    const int D = rref_row_dwords(p.k, p.m);
    auto kern = &gf_rref_batch_kernel<0, 1, 1>;
    int threads = 64;
    // shipped paths: the blocked run above (k + m <= 256), the one-wave register kernel for many small objects,
    // else the one-wave LDS kernel (the multi-wave register forms of decode paths 3/4/6 are diagnostic builds only)
    if (p.lds_only != 0 || (small_many && !hdr_lds)) return hipErrorInvalidValue;
    if (small_many && D <= 16 && p.k <= 32) kern = &gf_rref_batch_kernel<4, 8, 1>;
    // the 160 KiB dynamic-LDS attribute, once per device (function attributes are per device), under a lock
    {
        static std::mutex mu;
        static bool attr_set[64] = {};
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
        std::lock_guard<std::mutex> lock(mu);
        if (!attr_set[dev]) {
            for (auto f : {&gf_rref_batch_kernel<0, 1, 1>, &gf_rref_batch_kernel<4, 8, 1>}) {
                e = hipFuncSetAttribute(reinterpret_cast<const void *>(f),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, int(kRrefMaxLds));
                if (e != hipSuccess) return e;
            }
            attr_set[dev] = true;
        }
    }
    hipLaunchKernelGGL(kern, dim3(p.n_obj), dim3(threads), lds, s, p, hdr_lds);
    return hipGetLastError();
}

}  // namespace rlnc
