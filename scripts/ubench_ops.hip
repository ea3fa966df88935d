// ubench_ops.hip — issue cost per SIMD (chip-wide span method, 2 and 4 waves per SIMD forced with dynamic LDS)
// of the single VALU operations a bit-sliced GF(2^8) multiply-add can be built from, with controlled VGPR
// banks (bank = register number mod 4) and GPR-index (relative SRC0) forms.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_ops.hip -o build/ubench_ops && build/ubench_ops
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CLOB                                                                                                      \
    "v24", "v25", "v26", "v27", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", \
        "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "s20", "m0", "scc"
// dst/src2 accumulators v56..v63 (banks 0..3 twice); sources chosen per case
#define ACC8(op, a, b)                                                                                          \
    op " v56, " a "0, " b "0\n" op " v57, " a "1, " b "1\n" op " v58, " a "2, " b "2\n" op " v59, " a "3, " b "3\n" \
    op " v60, " a "4, " b "4\n" op " v61, " a "5, " b "5\n" op " v62, " a "6, " b "6\n" op " v63, " a "7, " b "7\n"

// each case: 8 instructions
#define XOR_DB "v_xor_b32 v56, v41, v56\n v_xor_b32 v57, v42, v57\n v_xor_b32 v58, v43, v58\n v_xor_b32 v59, v44, v59\n v_xor_b32 v60, v45, v60\n v_xor_b32 v61, v46, v61\n v_xor_b32 v62, v47, v62\n v_xor_b32 v63, v48, v63\n"
#define XOR_SB "v_xor_b32 v56, v40, v56\n v_xor_b32 v57, v41, v57\n v_xor_b32 v58, v42, v58\n v_xor_b32 v59, v43, v59\n v_xor_b32 v60, v44, v60\n v_xor_b32 v61, v45, v61\n v_xor_b32 v62, v46, v62\n v_xor_b32 v63, v47, v63\n"
#define B3X_DB "v_bitop3_b32 v56, v41, v42, v56 bitop3:0x96\n v_bitop3_b32 v57, v42, v43, v57 bitop3:0x96\n v_bitop3_b32 v58, v43, v40, v58 bitop3:0x96\n v_bitop3_b32 v59, v40, v41, v59 bitop3:0x96\n v_bitop3_b32 v60, v45, v46, v60 bitop3:0x96\n v_bitop3_b32 v61, v46, v47, v61 bitop3:0x96\n v_bitop3_b32 v62, v47, v44, v62 bitop3:0x96\n v_bitop3_b32 v63, v44, v45, v63 bitop3:0x96\n"
#define B3F_DB "v_bitop3_b32 v56, v41, v42, v56 bitop3:0xd8\n v_bitop3_b32 v57, v42, v43, v57 bitop3:0xd8\n v_bitop3_b32 v58, v43, v40, v58 bitop3:0xd8\n v_bitop3_b32 v59, v40, v41, v59 bitop3:0xd8\n v_bitop3_b32 v60, v45, v46, v60 bitop3:0xd8\n v_bitop3_b32 v61, v46, v47, v61 bitop3:0xd8\n v_bitop3_b32 v62, v47, v44, v62 bitop3:0xd8\n v_bitop3_b32 v63, v44, v45, v63 bitop3:0xd8\n"
#define BFI_DB "v_bfi_b32 v56, v41, v42, v56\n v_bfi_b32 v57, v42, v43, v57\n v_bfi_b32 v58, v43, v40, v58\n v_bfi_b32 v59, v40, v41, v59\n v_bfi_b32 v60, v45, v46, v60\n v_bfi_b32 v61, v46, v47, v61\n v_bfi_b32 v62, v47, v44, v62\n v_bfi_b32 v63, v44, v45, v63\n"
#define PERM_DB "v_perm_b32 v56, v41, v42, v56\n v_perm_b32 v57, v42, v43, v57\n v_perm_b32 v58, v43, v40, v58\n v_perm_b32 v59, v40, v41, v59\n v_perm_b32 v60, v45, v46, v60\n v_perm_b32 v61, v46, v47, v61\n v_perm_b32 v62, v47, v44, v62\n v_perm_b32 v63, v44, v45, v63\n"
#define SHL "v_lshlrev_b32 v56, 1, v41\n v_lshlrev_b32 v57, 1, v42\n v_lshlrev_b32 v58, 1, v43\n v_lshlrev_b32 v59, 1, v44\n v_lshlrev_b32 v60, 1, v45\n v_lshlrev_b32 v61, 1, v46\n v_lshlrev_b32 v62, 1, v47\n v_lshlrev_b32 v63, 1, v48\n"
// relative (M0 = 0x1000 | 1: SRC0 = v25 -> bank 1), accumulators banks 0..3
#define RMOV "v_mov_b32 v56, v24\n v_mov_b32 v57, v24\n v_mov_b32 v58, v24\n v_mov_b32 v59, v24\n v_mov_b32 v60, v24\n v_mov_b32 v61, v24\n v_mov_b32 v62, v24\n v_mov_b32 v63, v24\n"
#define RXOR "v_xor_b32 v56, v24, v56\n v_xor_b32 v57, v24, v57\n v_xor_b32 v58, v24, v58\n v_xor_b32 v59, v24, v59\n v_xor_b32 v60, v24, v60\n v_xor_b32 v61, v24, v61\n v_xor_b32 v62, v24, v62\n v_xor_b32 v63, v24, v63\n"
// relative XOR whose other operand is bank 1 too vs never bank 1 (accumulators chosen)
#define RXOR_NB "v_xor_b32 v56, v24, v56\n v_xor_b32 v58, v24, v58\n v_xor_b32 v59, v24, v59\n v_xor_b32 v60, v24, v60\n v_xor_b32 v62, v24, v62\n v_xor_b32 v63, v24, v63\n v_xor_b32 v56, v24, v56\n v_xor_b32 v58, v24, v58\n"
#define RB3 "v_bitop3_b32 v56, v24, v42, v56 bitop3:0x96\n v_bitop3_b32 v57, v24, v43, v57 bitop3:0x96\n v_bitop3_b32 v58, v24, v40, v58 bitop3:0x96\n v_bitop3_b32 v59, v24, v42, v59 bitop3:0x96\n v_bitop3_b32 v60, v24, v42, v60 bitop3:0x96\n v_bitop3_b32 v61, v24, v43, v61 bitop3:0x96\n v_bitop3_b32 v62, v24, v44, v62 bitop3:0x96\n v_bitop3_b32 v63, v24, v42, v63 bitop3:0x96\n"

constexpr int kCases = 11;
static const char *names[kCases] = {"v_xor_b32 VOP2, sources in different banks", "v_xor_b32 VOP2, sources in one bank",
                                    "v_bitop3 xor3, 3 banks", "v_bitop3 as bfi (0xd8), 3 banks", "v_bfi_b32, 3 banks",
                                    "v_perm_b32, 3 banks", "v_lshlrev_b32 const", "relative v_mov_b32 (VOP1)",
                                    "relative v_xor_b32", "relative v_xor_b32, other operand never in the relative bank",
                                    "relative v_bitop3 xor3"};

template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned long long *out, int reps) {
    extern __shared__ uint32_t lds[];
    asm volatile("v_mov_b32 v40, 1\n v_mov_b32 v41, 2\n v_mov_b32 v42, 3\n v_mov_b32 v43, 4\n v_mov_b32 v44, 5\n"
                 "v_mov_b32 v45, 6\n v_mov_b32 v46, 7\n v_mov_b32 v47, 8\n v_mov_b32 v48, 9\n v_mov_b32 v25, 10\n"
                 "s_mov_b32 s20, 1" ::: CLOB);
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE >= 7) asm volatile("s_set_gpr_idx_on s20, gpr_idx(SRC0)" ::: CLOB);
    for (int r = 0; r < reps; ++r) {
#define BODY(X) asm volatile(X X X X X X X X ::: CLOB)
        if (MODE == 0) BODY(XOR_DB);
        if (MODE == 1) BODY(XOR_SB);
        if (MODE == 2) BODY(B3X_DB);
        if (MODE == 3) BODY(B3F_DB);
        if (MODE == 4) BODY(BFI_DB);
        if (MODE == 5) BODY(PERM_DB);
        if (MODE == 6) BODY(SHL);
        if (MODE == 7) BODY(RMOV);
        if (MODE == 8) BODY(RXOR);
        if (MODE == 9) BODY(RXOR_NB);
        if (MODE == 10) BODY(RB3);
    }
    if (MODE >= 7) asm volatile("s_set_gpr_idx_off" ::: CLOB);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x % 64 == 0) {
        const int w = blockIdx.x * 4 + threadIdx.x / 64;
        out[4 * w + 0] = t1 - t0;
        out[4 * w + 1] = r0;
        out[4 * w + 2] = r1;
    }
    if (lds[threadIdx.x] == 0x12345678u) out[0] = 0;
}

template <int MODE>
void run(int W, unsigned long long *d) {
    const int blocks = 256 * W, reps = 256;  // 64 instructions per rep
    const size_t lds = (160 * 1024) / W - 1024;
    hipFuncSetAttribute(reinterpret_cast<const void *>(k<MODE>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int it = 0; it < 2; ++it) hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), lds, 0, d, reps);
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
    const double ghz = cyc / real / 10.0;
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"clock_GHz\": %.3f, \"cyc_per_inst_span\": %.3f}\n", names[MODE],
           W, ghz, double(rmax - rmin) * 10.0 * ghz / (64.0 * reps * W));
}

template <int M>
void all(int W, unsigned long long *d) {
    run<M>(W, d);
    if constexpr (M + 1 < kCases) all<M + 1>(W, d);
}

int main() {
    unsigned long long *d;
    hipMalloc(&d, 256 * 8 * 4 * 4 * sizeof(unsigned long long));
    for (int W : {2, 4}) all<0>(W, d);
    return 0;
}
