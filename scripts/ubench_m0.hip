// ubench_m0.hip — GPR-index mode driven by plain SALU writes of M0 (s_mov/s_lshr_b32 m0, ...) instead of
// s_set_gpr_idx_idx, with indices packed three per SGPR as bytes (0x10 | idx): after the shift,
// M0[7:0] = 0x10 + idx (the base register is named 16 below the table) and M0[15:12] = 1, the upper
// nibble of the next byte, re-enables SRC0-relative addressing (S_SET_GPR_IDX_ON stores its enables there).
// Checks the semantics with back-to-back SALU→VALU use and times the pair.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_m0.hip -o build/ubench_m0 && build/ubench_m0
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int REPS = 129;

#define R2(x) x x
#define R4(x) R2(x) R2(x)
#define R8(x) R4(x) R4(x)

#define CLOB                                                                                                      \
    "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", \
        "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "s20", "s21", "s22", "s23", "s24", "s25", "s26",   \
        "s27", "s28", "m0", "scc"

// s20 = bytes (0x13, 0x1f, 0x10, 0x10): indices 3, 15, 0;  s21 = (0x17, 0x19, 0x11, 0x10): 7, 9, 1
#define INIT_G(lane)                                                                                                 \
    "v_mov_b32 v40, 0\n v_add_u32 v41, 0x100, " lane "\n v_add_u32 v42, 0x200, " lane "\n v_add_u32 v43, 0x300, " lane \
    "\n v_add_u32 v44, 0x400, " lane "\n v_add_u32 v45, 0x500, " lane "\n v_add_u32 v46, 0x600, " lane              \
    "\n v_add_u32 v47, 0x700, " lane "\n v_add_u32 v48, 0x800, " lane "\n v_add_u32 v49, 0x900, " lane               \
    "\n v_add_u32 v50, 0xa00, " lane "\n v_add_u32 v51, 0xb00, " lane "\n v_add_u32 v52, 0xc00, " lane               \
    "\n v_add_u32 v53, 0xd00, " lane "\n v_add_u32 v54, 0xe00, " lane "\n v_add_u32 v55, 0xf00, " lane               \
    "\n s_mov_b32 s20, 0x10101f13\n s_mov_b32 s21, 0x10111917\n"

#define PAIRS8                                                                                                   \
    "s_mov_b32 m0, s20\n v_xor_b32 v56, v24, v56\n s_lshr_b32 m0, s20, 8\n v_xor_b32 v57, v24, v57\n"           \
    "s_lshr_b32 m0, s20, 16\n v_xor_b32 v58, v24, v58\n s_mov_b32 m0, s21\n v_xor_b32 v59, v24, v59\n"           \
    "s_lshr_b32 m0, s21, 8\n v_xor_b32 v60, v24, v60\n s_lshr_b32 m0, s21, 16\n v_xor_b32 v61, v24, v61\n"       \
    "s_lshr_b32 m0, s20, 8\n v_xor_b32 v62, v24, v62\n s_mov_b32 m0, s21\n v_xor_b32 v63, v24, v63\n"

__global__ void sem(uint32_t *out) {
    const uint32_t lane = threadIdx.x;
    uint32_t r[8];
    asm volatile(INIT_G("%8")
                 "v_mov_b32 v56, 0x10000\n v_mov_b32 v57, 0x20000\n v_mov_b32 v58, 0x30000\n v_mov_b32 v59, 0x40000\n"
                 "v_mov_b32 v60, 0x50000\n v_mov_b32 v61, 0x60000\n v_mov_b32 v62, 0x70000\n v_mov_b32 v63, 0x80000\n"
                 "s_mov_b32 s22, 0\n s_set_gpr_idx_on s22, gpr_idx(SRC0)\n" PAIRS8
                 "s_set_gpr_idx_off\n"
                 "v_mov_b32 %0, v56\n v_mov_b32 %1, v57\n v_mov_b32 %2, v58\n v_mov_b32 %3, v59\n"
                 "v_mov_b32 %4, v60\n v_mov_b32 %5, v61\n v_mov_b32 %6, v62\n v_mov_b32 %7, v63"
                 : "=v"(r[0]), "=v"(r[1]), "=v"(r[2]), "=v"(r[3]), "=v"(r[4]), "=v"(r[5]), "=v"(r[6]), "=v"(r[7])
                 : "v"(lane)
                 : CLOB);
    for (int q = 0; q < 8; ++q) out[lane * 8 + q] = r[q];
}

template <int MODE>
__global__ void k(unsigned long long *cyc) {
    const uint32_t lane = threadIdx.x;
    asm volatile(INIT_G("%0") "s_mov_b32 s22, 0" ::"v"(lane) : CLOB);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_set_gpr_idx_on s22, gpr_idx(SRC0)" ::: CLOB);
    for (int r = 0; r < REPS; ++r) {
        if (MODE == 0) asm volatile(R8(PAIRS8) ::: CLOB);
    }
    asm volatile("s_set_gpr_idx_off" ::: CLOB);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

int main() {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    uint32_t *out, ho[64 * 8];
    (void)hipMalloc(&out, sizeof ho);
    hipLaunchKernelGGL(sem, dim3(1), dim3(64), 0, 0, out);
    (void)hipMemcpy(ho, out, sizeof ho, hipMemcpyDeviceToHost);
    const uint32_t idx[8] = {3, 15, 0, 7, 9, 1, 15, 7};
    bool ok = true;
    for (uint32_t l = 0; l < 64; ++l)
        for (int q = 0; q < 8; ++q) {
            const uint32_t g = idx[q] ? 0x100u * idx[q] + l : 0u;
            ok &= ho[l * 8 + q] == ((0x10000u * (q + 1)) ^ g);
        }
    printf("{\"case\": \"semantics: SALU-written M0 (0x10|idx bytes, base-16) indexes SRC0\", \"ok\": %s, "
           "\"lane1\": [%u, %u, %u, %u, %u, %u, %u, %u]}\n",
           ok ? "true" : "false", ho[8], ho[9], ho[10], ho[11], ho[12], ho[13], ho[14], ho[15]);
    if (!ok) return 1;
    for (int wps : {1, 2, 4}) {
        const int threads = 256 * wps, blocks = 256, nw = blocks * threads / 64;
        unsigned long long *cyc;
        (void)hipMalloc(&cyc, nw * 8);
        hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, cyc);
        hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(threads), 0, 0, cyc);
        (void)hipDeviceSynchronize();
        unsigned long long *h = new unsigned long long[nw], mx = 0;
        (void)hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
        for (int i = 0; i < nw; ++i) mx = h[i] > mx ? h[i] : mx;
        printf("{\"case\": \"s_lshr_b32 m0 + v_xor (relative SRC0)\", \"waves_per_simd\": %d, "
               "\"cycles_per_pair_per_simd\": %.3f}\n",
               wps, double(mx) / (double(REPS) * 64 * wps));
        delete[] h;
        (void)hipFree(cyc);
    }
    return 0;
}
