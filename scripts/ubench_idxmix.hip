// ubench_idxmix.hip — issue cost on gfx950 of the instruction MIXES a bit-sliced GF(2^8) multiply-add can use:
// VGPR-relative XORs (GPR-index mode, SRC0 relative) with and without an M0 write in front of each, the
// 1 M0 write : 2 XOR ratio of gf_matmul_bs_kernel, plain SALU beside plain VALU (do SALU and VALU of two
// waves co-issue?), and VOP3 encodings.  Cycles per (SIMD, mix unit) at 1/2/4 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_idxmix.hip -o build/ubench_idxmix && build/ubench_idxmix
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int REPS = 64;

#define CLOB                                                                                                      \
    "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", \
        "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "s20", "s21", "s22", "s23", "s24", "s25", "s26",   \
        "s27", "s28", "m0", "scc"

// 8 units of each mix
#define PLAIN8                                                                                                   \
    "v_xor_b32 v56, v41, v56\n v_xor_b32 v57, v42, v57\n v_xor_b32 v58, v43, v58\n v_xor_b32 v59, v44, v59\n"   \
    "v_xor_b32 v60, v45, v60\n v_xor_b32 v61, v46, v61\n v_xor_b32 v62, v47, v62\n v_xor_b32 v63, v48, v63\n"
// relative XORs, M0 fixed (written once before the loop)
#define REL8                                                                                                     \
    "v_xor_b32 v56, v24, v56\n v_xor_b32 v57, v24, v57\n v_xor_b32 v58, v24, v58\n v_xor_b32 v59, v24, v59\n"   \
    "v_xor_b32 v60, v24, v60\n v_xor_b32 v61, v24, v61\n v_xor_b32 v62, v24, v62\n v_xor_b32 v63, v24, v63\n"
// one M0 write per relative XOR
#define M0X1_8                                                                                                   \
    "s_mov_b32 m0, s20\n v_xor_b32 v56, v24, v56\n s_lshr_b32 m0, s20, 8\n v_xor_b32 v57, v24, v57\n"           \
    "s_mov_b32 m0, s21\n v_xor_b32 v58, v24, v58\n s_lshr_b32 m0, s21, 8\n v_xor_b32 v59, v24, v59\n"           \
    "s_mov_b32 m0, s20\n v_xor_b32 v60, v24, v60\n s_lshr_b32 m0, s20, 8\n v_xor_b32 v61, v24, v61\n"           \
    "s_mov_b32 m0, s21\n v_xor_b32 v62, v24, v62\n s_lshr_b32 m0, s21, 8\n v_xor_b32 v63, v24, v63\n"
// one M0 write per two relative XORs (unit = one XOR)
#define M0X2_8                                                                                                   \
    "s_mov_b32 m0, s20\n v_xor_b32 v56, v24, v56\n v_xor_b32 v57, v25, v57\n"                                   \
    "s_lshr_b32 m0, s20, 8\n v_xor_b32 v58, v24, v58\n v_xor_b32 v59, v25, v59\n"                               \
    "s_mov_b32 m0, s21\n v_xor_b32 v60, v24, v60\n v_xor_b32 v61, v25, v61\n"                                   \
    "s_lshr_b32 m0, s21, 8\n v_xor_b32 v62, v24, v62\n v_xor_b32 v63, v25, v63\n"
// one M0 write per four relative XORs (unit = one XOR)
#define M0X4_8                                                                                                   \
    "s_mov_b32 m0, s20\n v_xor_b32 v56, v24, v56\n v_xor_b32 v57, v25, v57\n v_xor_b32 v58, v26, v58\n v_xor_b32 v59, v27, v59\n" \
    "s_lshr_b32 m0, s21, 8\n v_xor_b32 v60, v24, v60\n v_xor_b32 v61, v25, v61\n v_xor_b32 v62, v26, v62\n v_xor_b32 v63, v27, v63\n"
// plain SALU (not M0) + plain VALU, 1:1 (unit = one pair)
#define SV8                                                                                                      \
    "s_lshr_b32 s22, s20, 1\n v_xor_b32 v56, v41, v56\n s_lshr_b32 s23, s21, 1\n v_xor_b32 v57, v42, v57\n"     \
    "s_lshr_b32 s24, s20, 2\n v_xor_b32 v58, v43, v58\n s_lshr_b32 s25, s21, 2\n v_xor_b32 v59, v44, v59\n"     \
    "s_lshr_b32 s22, s20, 3\n v_xor_b32 v60, v45, v60\n s_lshr_b32 s23, s21, 3\n v_xor_b32 v61, v46, v61\n"     \
    "s_lshr_b32 s24, s20, 4\n v_xor_b32 v62, v47, v62\n s_lshr_b32 s25, s21, 4\n v_xor_b32 v63, v48, v63\n"
// plain VOP3-encoded XOR (unit = one instruction)
#define VOP3X8                                                                                                   \
    "v_xor_b32_e64 v56, v41, v56\n v_xor_b32_e64 v57, v42, v57\n v_xor_b32_e64 v58, v43, v58\n v_xor_b32_e64 v59, v44, v59\n" \
    "v_xor_b32_e64 v60, v45, v60\n v_xor_b32_e64 v61, v46, v61\n v_xor_b32_e64 v62, v47, v62\n v_xor_b32_e64 v63, v48, v63\n"
// relative VOP3 bitop3 XOR3 (SRC0 relative), M0 fixed (unit = one instruction)
#define REL3_8                                                                                                   \
    "v_bitop3_b32 v56, v24, v57, v56 bitop3:0x96\n v_bitop3_b32 v58, v24, v59, v58 bitop3:0x96\n"               \
    "v_bitop3_b32 v60, v24, v61, v60 bitop3:0x96\n v_bitop3_b32 v62, v24, v63, v62 bitop3:0x96\n"               \
    "v_bitop3_b32 v57, v24, v56, v57 bitop3:0x96\n v_bitop3_b32 v59, v24, v58, v59 bitop3:0x96\n"               \
    "v_bitop3_b32 v61, v24, v60, v61 bitop3:0x96\n v_bitop3_b32 v63, v24, v62, v63 bitop3:0x96\n"

#define INIT                                                                                                     \
    "v_mov_b32 v40, 0\n v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n v_mov_b32 v44, 4\n"             \
    "v_mov_b32 v45, 5\n v_mov_b32 v46, 6\n v_mov_b32 v47, 7\n v_mov_b32 v48, 8\n v_mov_b32 v49, 9\n"             \
    "v_mov_b32 v50, 10\n v_mov_b32 v51, 11\n v_mov_b32 v52, 12\n v_mov_b32 v53, 13\n v_mov_b32 v54, 14\n"        \
    "v_mov_b32 v55, 15\n s_mov_b32 s20, 0x10101f13\n s_mov_b32 s21, 0x10111917\n s_mov_b32 s22, 0\n"

template <int MODE>
__global__ void k(unsigned long long *cyc, uint32_t *sink) {
    asm volatile(INIT ::: CLOB);
    if (MODE == 1 || MODE == 7) asm volatile("s_mov_b32 m0, 0x1013" ::: CLOB);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE >= 1 && MODE <= 4 || MODE == 7) asm volatile("s_set_gpr_idx_on s22, gpr_idx(SRC0)" ::: CLOB);
    for (int r = 0; r < REPS; ++r) {
        if (MODE == 0) asm volatile(PLAIN8 PLAIN8 PLAIN8 PLAIN8 ::: CLOB);
        if (MODE == 1) asm volatile(REL8 REL8 REL8 REL8 ::: CLOB);
        if (MODE == 2) asm volatile(M0X1_8 M0X1_8 M0X1_8 M0X1_8 ::: CLOB);
        if (MODE == 3) asm volatile(M0X2_8 M0X2_8 M0X2_8 M0X2_8 ::: CLOB);
        if (MODE == 4) asm volatile(M0X4_8 M0X4_8 M0X4_8 M0X4_8 ::: CLOB);
        if (MODE == 5) asm volatile(SV8 SV8 SV8 SV8 ::: CLOB);
        if (MODE == 6) asm volatile(VOP3X8 VOP3X8 VOP3X8 VOP3X8 ::: CLOB);
        if (MODE == 7) asm volatile(REL3_8 REL3_8 REL3_8 REL3_8 ::: CLOB);
    }
    if (MODE >= 1 && MODE <= 4 || MODE == 7) asm volatile("s_set_gpr_idx_off" ::: CLOB);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t v;
    asm volatile("v_xor_b32 %0, v56, v63" : "=v"(v)::CLOB);
    if (v == 0x12345678u) sink[threadIdx.x] = v;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

static const char *names[] = {"plain v_xor (VOP2)",
                              "relative v_xor, M0 fixed",
                              "1 M0 write : 1 relative v_xor",
                              "1 M0 write : 2 relative v_xor",
                              "1 M0 write : 4 relative v_xor",
                              "plain SALU : plain VALU 1:1 (unit = pair)",
                              "plain v_xor_b32_e64 (VOP3)",
                              "relative v_bitop3 xor3, M0 fixed"};

template <int MODE>
void run(int waves_per_simd, unsigned long long *d, uint32_t *sink) {
    // one workgroup per CU (256 CUs), 4 * waves_per_simd waves per workgroup: waves_per_simd waves per SIMD
    const int blocks = 256, wpb = 4 * waves_per_simd;
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64 * wpb), 0, 0, d, sink);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(64 * wpb), 0, 0, d, sink);
    hipDeviceSynchronize();
    const int n = blocks * wpb;
    unsigned long long *h = new unsigned long long[n];
    hipMemcpy(h, d, n * sizeof(*h), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < n; ++i) s += double(h[i]);
    delete[] h;
    const double units = double(REPS) * 32;  // units per wave
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_unit_per_simd\": %.3f}\n", names[MODE],
           waves_per_simd, s / n / units / waves_per_simd);
}

int main() {
    unsigned long long *d;
    uint32_t *sink;
    hipMalloc(&d, 256 * 32 * sizeof(*d));
    hipMalloc(&sink, 4096 * sizeof(uint32_t));
    for (int w : {1, 2, 4}) {
        run<0>(w, d, sink);
        run<1>(w, d, sink);
        run<2>(w, d, sink);
        run<3>(w, d, sink);
        run<4>(w, d, sink);
        run<5>(w, d, sink);
        run<6>(w, d, sink);
        run<7>(w, d, sink);
    }
    return 0;
}
