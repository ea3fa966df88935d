// rref_ab.hip — the A/B history of the device elimination (diagnostic build only: make -C rlnc_amd/csrc ab ->
// librlnc_hip_ab.so).  Its dispatch replaces the shipped one (rref.hip) through launch_rref_ab; the kernels are the
// shipped templates of rref_kernels.hpp at the parameters the rounds compared (profiles/r01_*,
// r02_elim_ab.txt, r02_elim_small_k.jsonl, r03_small_elim_ab.txt).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>

#include "kernels.hpp"
#include "rref_kernels.hpp"

namespace rlnc {

static hipError_t launch_rref_one_ab(const RrefParams &p, hipStream_t s);

// The A/B build's dispatch: every elimination launch comes here first and is taken whole (true).  Beyond the shipped
// paths it has decode paths 3, 4 and 6 (lds_only 1, 2, 4: the round-1 LDS-resident and register forms, multi-wave
// for up to k = 64), the 16-piece blocks of the blocked run (RLNC_BLK = 16) and the small-object knobs
// (RLNC_SMALL_MIN, RLNC_SMALL_NW).
bool launch_rref_ab(const RrefParams &p, hipStream_t s, hipError_t *result) {
    // never the payload-tail answer (RrefParams::tail_status): launch_rref_batch reports no block-offset stream written
    // from here, so the product never relies on it and the scan kernel answers every object
    RrefParams q = p;
    q.tail_status = nullptr;
    *result = launch_rref_one_ab(q, s);
    return true;
}

static hipError_t launch_rref_one_ab(const RrefParams &p, hipStream_t s) {
    // many small objects (k <= 16, >= 2048 of them: 8 per CU and more): the one-wave register kernel (path 4's)
    // beats the 4-wave blocked run, whose per-object parallelism the full grid no longer needs -- 4,096 x k = 16:
    // 0.093 vs 0.125 ms, k = 8: 0.051 vs 0.067, k = 16 sparse + dependent: 0.195 vs 0.295; at 512 objects the
    // blocked run stays faster (0.035 vs 0.049) (profiles/r02_elim_small_k.jsonl)
    static const int small_min = [] {
        const char *e = getenv("RLNC_SMALL_MIN");
        return e ? atoi(e) : kSmallMinObjects;
    }();
    const bool small_many = p.lds_only == 0 && p.k <= 16 && p.n_obj >= small_min && rref_row_dwords(p.k, p.m) <= 16 &&
                            rref_lds_bytes_staged(p.k, p.m) <= kRrefMaxLds;
    // the blocked clean run (4 waves per object, the default) when the row fits one wave (k + m <= 256)
    if (!small_many && (p.lds_only == 0 || p.lds_only == 3) && rref_row_dwords(p.k, p.m) <= 64 &&
        rref_block_lds_bytes(p.k, p.m) <= kRrefMaxLds) {
        // A/B knob (read once): RLNC_BLK = 8 or 16 pieces per block (profiles/r02_elim_ab.txt)
        static const int blk = [] {
            const char *e = getenv("RLNC_BLK");
            const int v = e ? atoi(e) : kBlkDefault;
            return v == 8 || v == 16 ? v : kBlkDefault;
        }();
        auto kern = blk == 16 ? &gf_rref_block_kernel<kBlkNW, 16> : &gf_rref_block_kernel<kBlkNW, 8>;
        static std::mutex mu;
        static bool attr_set[64] = {};
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
        {
            std::lock_guard<std::mutex> lock(mu);
            if (!attr_set[dev]) {
                for (auto f : {&gf_rref_block_kernel<kBlkNW, 8>, &gf_rref_block_kernel<kBlkNW, 16>}) {
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
        const bool g8 = rref_row_dwords(p.k, p.m) <= 8;
        auto kern = g8 ? &gf_rref_small_kernel<kSmallNW, 8, 2> : &gf_rref_small_kernel<1, 4, 4>;
        int nw = g8 ? kSmallNW : 1;
        static const int nw_ab = [] {
            const char *e = getenv("RLNC_SMALL_NW");
            return e ? atoi(e) : kSmallNW;
        }();
        if (nw_ab == 1 || nw_ab == 2 || nw_ab == 8) {
            nw = nw_ab;
            if (g8)
                kern = nw == 1 ? &gf_rref_small_kernel<1, 8, 2> : nw == 2 ? &gf_rref_small_kernel<2, 8, 2> : &gf_rref_small_kernel<8, 8, 2>;
            else
                kern = nw == 1 ? &gf_rref_small_kernel<1, 4, 4> : nw == 2 ? &gf_rref_small_kernel<2, 4, 4> : &gf_rref_small_kernel<8, 4, 4>;
        }
        const size_t lds_small = size_t(kTabEntries) * kTabDw * 4 + nw * rref_small_wave_bytes(p.k, p.m);
        if (const char *pe = getenv("RLNC_SMALL_PROF"); pe && g8 && nw == kSmallNW) {
            // per-wave phase timestamps (8 x u64 per object) into the device buffer at this hex address
            RrefParams q = p;
            q.prof = reinterpret_cast<uint64_t *>(strtoull(pe, nullptr, 16));
            hipLaunchKernelGGL((gf_rref_small_kernel<kSmallNW, 8, 2, true>), dim3((p.n_obj + nw - 1) / nw), dim3(64 * nw),
                               lds_small, s, q);
            return hipGetLastError();
        }
        hipLaunchKernelGGL(kern, dim3((p.n_obj + nw - 1) / nw), dim3(64 * nw), lds_small, s, p);
        return hipGetLastError();
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
    if (p.lds_only != 1 && hdr_lds) {  // the register paths read the staged headers
        const bool mw = (p.lds_only == 0 && !small_many) || p.lds_only == 4;
        if (D <= 16 && p.k <= 32) {
            kern = mw ? &gf_rref_batch_kernel<4, 8, 4, 4, 2> : &gf_rref_batch_kernel<4, 8, 1>;
        } else if (D <= 32 && p.k <= 64) {
            kern = mw ? &gf_rref_batch_kernel<2, 32, 4, 2, 8> : &gf_rref_batch_kernel<2, 32, 1>;
        }  // k = 128 (<0, 1, 4, 1, 32>: 3.8 ms for 512 objects) stays on the one-wave LDS path (2.5 ms)
        if (mw && kern != &gf_rref_batch_kernel<0, 1, 1>) threads = 256;
    }
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
            for (auto f : {&gf_rref_batch_kernel<0, 1, 1>, &gf_rref_batch_kernel<4, 8, 1>,
                           &gf_rref_batch_kernel<4, 8, 4, 4, 2>, &gf_rref_batch_kernel<2, 32, 1>,
                           &gf_rref_batch_kernel<2, 32, 4, 2, 8>}) {
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
