// ubench_occ.hip — VALU/SALU issue throughput per SIMD versus waves per SIMD (1..8) on gfx950.
// Occupancy is forced with dynamic LDS: W workgroups of 4 waves (one per SIMD) fit on a CU.  Each wave runs
// the same instruction block; the chip-wide span (s_memrealtime, 100 MHz) and the shader clock
// (s_memtime / s_memrealtime of each wave) give cycles per instruction per SIMD.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_occ.hip -o build/ubench_occ && build/ubench_occ
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int REPS = 256;

#define CLOB                                                                                                      \
    "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", \
        "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "s20", "s21", "s22", "s23", "s24", "s25", "s26",   \
        "s27", "s28", "m0", "scc"

#define PLAIN8                                                                                                   \
    "v_xor_b32 v56, v41, v56\n v_xor_b32 v57, v42, v57\n v_xor_b32 v58, v43, v58\n v_xor_b32 v59, v44, v59\n"   \
    "v_xor_b32 v60, v45, v60\n v_xor_b32 v61, v46, v61\n v_xor_b32 v62, v47, v62\n v_xor_b32 v63, v48, v63\n"
#define REL8                                                                                                     \
    "v_xor_b32 v56, v24, v56\n v_xor_b32 v57, v24, v57\n v_xor_b32 v58, v24, v58\n v_xor_b32 v59, v24, v59\n"   \
    "v_xor_b32 v60, v24, v60\n v_xor_b32 v61, v24, v61\n v_xor_b32 v62, v24, v62\n v_xor_b32 v63, v24, v63\n"
// 1 M0 write : 2 relative XORs; unit = instruction (12 per block)
#define M0X2_8                                                                                                   \
    "s_mov_b32 m0, s20\n v_xor_b32 v56, v24, v56\n v_xor_b32 v57, v25, v57\n"                                   \
    "s_lshr_b32 m0, s20, 8\n v_xor_b32 v58, v24, v58\n v_xor_b32 v59, v25, v59\n"                               \
    "s_mov_b32 m0, s21\n v_xor_b32 v60, v24, v60\n v_xor_b32 v61, v25, v61\n"                                   \
    "s_lshr_b32 m0, s21, 8\n v_xor_b32 v62, v24, v62\n v_xor_b32 v63, v25, v63\n"
#define PERM8                                                                                                    \
    "v_perm_b32 v56, v41, v42, v56\n v_perm_b32 v57, v43, v44, v57\n v_perm_b32 v58, v45, v46, v58\n"           \
    "v_perm_b32 v59, v47, v48, v59\n v_perm_b32 v60, v49, v50, v60\n v_perm_b32 v61, v51, v52, v61\n"           \
    "v_perm_b32 v62, v53, v54, v62\n v_perm_b32 v63, v55, v40, v63\n"
#define BITOP8                                                                                                   \
    "v_bitop3_b32 v56, v41, v42, v56 bitop3:0x96\n v_bitop3_b32 v57, v43, v44, v57 bitop3:0x96\n"               \
    "v_bitop3_b32 v58, v45, v46, v58 bitop3:0x96\n v_bitop3_b32 v59, v47, v48, v59 bitop3:0x96\n"               \
    "v_bitop3_b32 v60, v49, v50, v60 bitop3:0x96\n v_bitop3_b32 v61, v51, v52, v61 bitop3:0x96\n"               \
    "v_bitop3_b32 v62, v53, v54, v62 bitop3:0x96\n v_bitop3_b32 v63, v55, v40, v63 bitop3:0x96\n"
#define SV8                                                                                                      \
    "s_lshr_b32 s22, s20, 1\n v_xor_b32 v56, v41, v56\n s_lshr_b32 s23, s21, 1\n v_xor_b32 v57, v42, v57\n"     \
    "s_lshr_b32 s24, s20, 2\n v_xor_b32 v58, v43, v58\n s_lshr_b32 s25, s21, 2\n v_xor_b32 v59, v44, v59\n"

#define INIT                                                                                                     \
    "v_mov_b32 v40, 0\n v_mov_b32 v41, 1\n v_mov_b32 v42, 2\n v_mov_b32 v43, 3\n v_mov_b32 v44, 4\n"             \
    "v_mov_b32 v45, 5\n v_mov_b32 v46, 6\n v_mov_b32 v47, 7\n v_mov_b32 v48, 8\n v_mov_b32 v49, 9\n"             \
    "v_mov_b32 v50, 10\n v_mov_b32 v51, 11\n v_mov_b32 v52, 12\n v_mov_b32 v53, 13\n v_mov_b32 v54, 14\n"        \
    "v_mov_b32 v55, 15\n v_mov_b32 v56, 0\n v_mov_b32 v57, 0\n v_mov_b32 v58, 0\n v_mov_b32 v59, 0\n"            \
    "v_mov_b32 v60, 0\n v_mov_b32 v61, 0\n v_mov_b32 v62, 0\n v_mov_b32 v63, 0\n"                               \
    "s_mov_b32 s20, 0x10101f13\n s_mov_b32 s21, 0x10111917\n s_mov_b32 s22, 0\n"

constexpr int kInstPerRep[] = {32, 32, 48, 32, 32, 32};  // instructions per loop body, by mode
static const char *names[] = {"plain v_xor (VOP2)", "relative v_xor, M0 fixed", "1 M0 write : 2 relative v_xor",
                              "v_perm_b32", "v_bitop3_b32 (distinct banks)", "plain SALU : plain VALU 1:1"};

template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned long long *out, uint32_t *sink) {
    extern __shared__ uint32_t lds[];
    asm volatile(INIT ::: CLOB);
    if (MODE == 1) asm volatile("s_mov_b32 m0, 0x1013" ::: CLOB);
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 1 || MODE == 2) asm volatile("s_set_gpr_idx_on s22, gpr_idx(SRC0)" ::: CLOB);
    for (int r = 0; r < REPS; ++r) {
        if (MODE == 0) asm volatile(PLAIN8 PLAIN8 PLAIN8 PLAIN8 ::: CLOB);
        if (MODE == 1) asm volatile(REL8 REL8 REL8 REL8 ::: CLOB);
        if (MODE == 2) asm volatile(M0X2_8 M0X2_8 M0X2_8 M0X2_8 ::: CLOB);
        if (MODE == 3) asm volatile(PERM8 PERM8 PERM8 PERM8 ::: CLOB);
        if (MODE == 4) asm volatile(BITOP8 BITOP8 BITOP8 BITOP8 ::: CLOB);
        if (MODE == 5) asm volatile(SV8 SV8 SV8 SV8 ::: CLOB);
    }
    if (MODE == 1 || MODE == 2) asm volatile("s_set_gpr_idx_off" ::: CLOB);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t v;
    asm volatile("v_xor_b32 %0, v56, v63" : "=v"(v)::CLOB);
    if (v == 0x12345678u) sink[threadIdx.x] = v + lds[threadIdx.x];
    if (threadIdx.x % 64 == 0) {
        const int w = blockIdx.x * 4 + threadIdx.x / 64;
        out[4 * w + 0] = t1 - t0;
        out[4 * w + 1] = r0;
        out[4 * w + 2] = r1;
    }
}

template <int MODE>
void run(int W, unsigned long long *d, uint32_t *sink) {
    const int cus = 256, blocks = cus * W;
    const size_t lds = (160 * 1024) / W - 1024;
    hipFuncSetAttribute(reinterpret_cast<const void *>(k<MODE>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int it = 0; it < 2; ++it) hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), lds, 0, d, sink);
    hipDeviceSynchronize();
    const int waves = blocks * 4;
    std::vector<unsigned long long> h(4 * waves);
    hipMemcpy(h.data(), d, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    unsigned long long rmin = ~0ull, rmax = 0;
    double cyc = 0, real = 0;
    for (int w = 0; w < waves; ++w) {
        cyc += double(h[4 * w]);
        real += double(h[4 * w + 2] - h[4 * w + 1]);
        rmin = h[4 * w + 1] < rmin ? h[4 * w + 1] : rmin;
        rmax = h[4 * w + 2] > rmax ? h[4 * w + 2] : rmax;
    }
    const double ghz = cyc / real / 10.0;  // memrealtime: 100 MHz
    const double insts = double(REPS) * kInstPerRep[MODE] * W;  // per SIMD
    const double span_cyc = double(rmax - rmin) * 10.0 * ghz;
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"clock_GHz\": %.3f, \"cyc_per_inst_span\": %.3f, "
           "\"cyc_per_inst_wave\": %.3f}\n",
           names[MODE], W, ghz, span_cyc / insts, cyc / waves / (insts / W) / W);
}

int main() {
    unsigned long long *d;
    uint32_t *sink;
    hipMalloc(&d, 256 * 8 * 4 * 4 * sizeof(unsigned long long));
    hipMalloc(&sink, 4096 * sizeof(uint32_t));
    for (int W : {1, 2, 3, 4, 6, 8}) {
        run<0>(W, d, sink);
        run<1>(W, d, sink);
        run<2>(W, d, sink);
        run<3>(W, d, sink);
        run<4>(W, d, sink);
        run<5>(W, d, sink);
    }
    return 0;
}
