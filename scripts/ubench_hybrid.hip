// ubench_hybrid.hip -- can the matrix cores add GF(2^8) multiply-adds beside the bit-sliced XOR3 engine?
// MEASUREMENT ONLY (not part of librlnc_hip).
//
// GF(2^8) c·x is an 8x8 bit matrix over GF(2), so a coded-piece product is a GF(2) GEMM: bit-rows (8 per output
// row) x bit-columns (8 per source row) x byte columns, 64 bit-MACs per GF multiply-add.  With 0/1 operands in
// FP4 (e2m1: 0x0 = 0, 0x2 = 1.0) v_mfma_scale_f32_32x32x64_f8f6f4 does 65,536 bit-MACs = 1,024 GF multiply-adds
// per instruction and the parity of each f32 sum is the GF(2) result (exact: sums <= 256).  This program measures
// the issue rates that decide whether such a path can beat or join the XOR3 engine (256 multiply-adds per
// v_bitop3_b32), on every CU, HIP events around each launch:
//   xor       W waves per SIMD of independent XOR3s (the gf_ceiling pattern)
//   mfma      W waves per SIMD of fp4 MFMAs, 4 independent accumulators per wave (AGPRs)
//   mix<X>    every wave: one MFMA then X XOR3s, repeated (one instruction stream on the SIMD)
//   split     2 waves per SIMD: one runs only MFMAs, the other only XOR3s (two streams on the SIMD)
//
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_hybrid.hip -o build/ubench_hybrid && build/ubench_hybrid
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CLOBX "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"
#define CLOBM                                                                                                       \
    "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7",  \
        "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", \
        "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38",       \
        "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47", "a48", "a49", "a50", "a51", "a52", "a53",       \
        "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63"
#define X1(i, a, b) "v_bitop3_b32 v" #i ", v" #a ", v" #b ", v" #i " bitop3:0x96\n"
#define X8 X1(56, 41, 42) X1(57, 42, 43) X1(58, 43, 40) X1(59, 40, 41) X1(60, 45, 46) X1(61, 46, 47) X1(62, 47, 44) X1(63, 44, 45)
#define X4A X1(56, 41, 42) X1(57, 42, 43) X1(58, 43, 40) X1(59, 40, 41)
#define X4B X1(60, 45, 46) X1(61, 46, 47) X1(62, 47, 44) X1(63, 44, 45)
#define M1(a) "v_mfma_scale_f32_32x32x64_f8f6f4 a[" #a "], v[64:67], v[68:71], a[" #a "], v72, v72 op_sel_hi:[0,0,0] cbsz:4 blgp:4\n"
#define MA M1(0:15)
#define MB M1(16:31)
#define MC M1(32:47)
#define MD M1(48:63)

// MODE 0 xor, 1 mfma, 2 mix (X XOR3s after each MFMA), 3 split (waves >= 4 run XOR3s, the others MFMAs)
template <int MODE, int X>
__global__ __launch_bounds__(512) void hyb_kernel(const uint32_t *seed, uint32_t *out, int reps) {
    extern __shared__ uint32_t lds[];
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t *s = seed + (g % 4096) * 16;
    asm volatile(
        "global_load_dwordx4 v[40:43], %0, off\n global_load_dwordx4 v[44:47], %0, off offset:16\n"
        "global_load_dwordx4 v[56:59], %0, off offset:32\n global_load_dwordx4 v[60:63], %0, off offset:48\n"
        "s_waitcnt vmcnt(0)\n"
        // fp4 operands: every nibble 0x0 or 0x2 (= 1.0), from the random words
        "v_and_b32 v64, 0x22222222, v40\n v_and_b32 v65, 0x22222222, v41\n v_and_b32 v66, 0x22222222, v42\n"
        "v_and_b32 v67, 0x22222222, v43\n v_and_b32 v68, 0x22222222, v44\n v_and_b32 v69, 0x22222222, v45\n"
        "v_and_b32 v70, 0x22222222, v46\n v_and_b32 v71, 0x22222222, v47\n v_mov_b32 v72, 127\n"
        "v_accvgpr_write_b32 a0, 0\n v_accvgpr_write_b32 a16, 0\n v_accvgpr_write_b32 a32, 0\n v_accvgpr_write_b32 a48, 0\n"
        "s_nop 7\n s_nop 7" ::"v"(s)
        : CLOBX, CLOBM);
    const int w = threadIdx.x >> 6;
    for (int r = 0; r < reps; ++r) {
        if constexpr (MODE == 0) asm volatile(X8 X8 X8 X8 X8 X8 X8 X8 ::: CLOBX);  // 64 XOR3s
        if constexpr (MODE == 1) asm volatile(MA MB MC MD MA MB MC MD ::: CLOBM);   // 8 MFMAs
        if constexpr (MODE == 2 && X == 4) asm volatile(MA X4A MB X4B MC X4A MD X4B MA X4A MB X4B MC X4A MD X4B ::: CLOBX, CLOBM);
        if constexpr (MODE == 2 && X == 8) asm volatile(MA X8 MB X8 MC X8 MD X8 MA X8 MB X8 MC X8 MD X8 ::: CLOBX, CLOBM);
        if constexpr (MODE == 2 && X == 12)
            asm volatile(MA X8 X4A MB X4B X8 MC X8 X4A MD X4B X8 MA X8 X4A MB X4B X8 MC X8 X4A MD X4B X8 ::: CLOBX, CLOBM);
        if constexpr (MODE == 2 && X == 16)
            asm volatile(MA X8 X8 MB X8 X8 MC X8 X8 MD X8 X8 MA X8 X8 MB X8 X8 MC X8 X8 MD X8 X8 ::: CLOBX, CLOBM);
        if constexpr (MODE == 3) {
            if (w >= 4)
                asm volatile(X8 X8 X8 X8 X8 X8 X8 X8 ::: CLOBX);
            else
                asm volatile(MA MB MC MD MA MB MC MD ::: CLOBM);
        }
    }
    uint32_t acc;
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n v_accvgpr_read_b32 %0, a0\n v_xor_b32 %0, %0, v56\n v_xor_b32 %0, %0, v63"
                 : "=v"(acc)::CLOBX, CLOBM);
    if (acc == 0x9E3779B9u && lds[threadIdx.x] == 0x12345678u) out[g] = acc;
}

template <int MODE, int X>
static void run(const char *name, int threads, int per_cu, const uint32_t *seed, uint32_t *out, int reps, int cus) {
    auto kern = hyb_kernel<MODE, X>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const size_t lds = (160 * 1024) / per_cu - 1024;
    const int blocks = cus * per_cu;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int it = 0; it < 4; ++it) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds, 0, seed, out, reps);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (it >= 1 && ms < best) best = ms;
    }
    const double waves = double(blocks) * threads / 64;
    double xor3 = 0, mfma = 0;
    if (MODE == 0) xor3 = waves * reps * 64;
    if (MODE == 1) mfma = waves * reps * 8;
    if (MODE == 2) xor3 = waves * reps * 8 * X, mfma = waves * reps * 8;
    if (MODE == 3) xor3 = waves / 2 * reps * 64, mfma = waves / 2 * reps * 8;
    const double t = best * 1e-3;
    const double ma = (xor3 * 256 + mfma * 1024) / t;
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"xor3_T_per_s\": %.4f, \"mfma_T_per_s\": %.5f, "
           "\"T_muladd_per_s\": %.2f, \"of_which_mfma\": %.3f}\n",
           name, threads / 256 * per_cu, best, xor3 / t * 1e-12, mfma / t * 1e-12, ma * 1e-12,
           ma > 0 ? mfma * 1024 / t / ma : 0.0);
}

int main() {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    uint32_t *seed = nullptr, *out = nullptr;
    (void)hipMalloc(&seed, 4096 * 16 * 4);
    (void)hipMalloc(&out, size_t(cus) * 2048 * 4);
    uint32_t *h = new uint32_t[4096 * 16];
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < 4096 * 16; ++i) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        h[i] = uint32_t(z ^ (z >> 31));
    }
    (void)hipMemcpy(seed, h, 4096 * 16 * 4, hipMemcpyHostToDevice);
    const int R = 4096;
    run<0, 0>("xor", 256, 1, seed, out, R * 4, cus);
    run<0, 0>("xor", 512, 1, seed, out, R * 4, cus);
    run<1, 0>("mfma", 256, 1, seed, out, R, cus);
    run<1, 0>("mfma", 512, 1, seed, out, R, cus);
    run<2, 4>("mix4", 256, 1, seed, out, R, cus);
    run<2, 8>("mix8", 256, 1, seed, out, R, cus);
    run<2, 12>("mix12", 256, 1, seed, out, R, cus);
    run<2, 16>("mix16", 256, 1, seed, out, R, cus);
    run<2, 8>("mix8", 512, 1, seed, out, R, cus);
    run<2, 12>("mix12", 512, 1, seed, out, R, cus);
    run<3, 0>("split", 512, 1, seed, out, R, cus);
    (void)hipFree(seed);
    (void)hipFree(out);
    return 0;
}
