// ubench_valu.hip — cycles per wave64 instruction on one gfx950 SIMD for the instructions the GF(2^8)
// kernels are built from, measured with s_memtime inside the kernel (so the result does not depend on the
// clock the chip holds).  Each wave runs REPS blocks of 16 independent instructions written in inline asm
// (nothing for the compiler to fold); one workgroup per CU, W waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_valu.hip -o build/ubench_valu && build/ubench_valu
// Output: cycles per instruction per SIMD (all W waves' instructions / elapsed cycles of the slowest wave).
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int REPS = 256;

#define I(OP, SUF, D) OP " %" #D ", %16, %17, %" #D SUF "\n\t"
#define I2(OP, D) OP " %" #D ", %16, %" #D "\n\t"
#define P16_2(OP)                                                                                                   \
    asm volatile(I2(OP, 0) I2(OP, 1) I2(OP, 2) I2(OP, 3) I2(OP, 4) I2(OP, 5) I2(OP, 6) I2(OP, 7) I2(OP, 8) I2(OP, 9)   \
                     I2(OP, 10) I2(OP, 11) I2(OP, 12) I2(OP, 13) I2(OP, 14) I2(OP, 15)                                \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), \
                   "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]),    \
                   "+v"(a[15])                                                                                 \
                 : "v"(t0))
#define P16S(OP, SUF)                                                                                              \
    asm volatile(I(OP, SUF, 0) I(OP, SUF, 1) I(OP, SUF, 2) I(OP, SUF, 3) I(OP, SUF, 4) I(OP, SUF, 5) I(OP, SUF, 6)   \
                     I(OP, SUF, 7) I(OP, SUF, 8) I(OP, SUF, 9) I(OP, SUF, 10) I(OP, SUF, 11) I(OP, SUF, 12)           \
                         I(OP, SUF, 13) I(OP, SUF, 14) I(OP, SUF, 15)                                                \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), \
                   "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]),    \
                   "+v"(a[15])                                                                                 \
                 : "s"(su), "v"(t1))
#define P16(OP, SUF)                                                                                               \
    asm volatile(I(OP, SUF, 0) I(OP, SUF, 1) I(OP, SUF, 2) I(OP, SUF, 3) I(OP, SUF, 4) I(OP, SUF, 5) I(OP, SUF, 6)   \
                     I(OP, SUF, 7) I(OP, SUF, 8) I(OP, SUF, 9) I(OP, SUF, 10) I(OP, SUF, 11) I(OP, SUF, 12)           \
                         I(OP, SUF, 13) I(OP, SUF, 14) I(OP, SUF, 15)                                                \
                 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), \
                   "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]),    \
                   "+v"(a[15])                                                                                 \
                 : "v"(t0), "v"(t1))

template <int MODE>
__global__ void k(unsigned long long *cyc, uint32_t *out, uint32_t seed) {
    uint32_t a[16];
    uint32_t t0 = seed ^ threadIdx.x, t1 = t0 * 7u + 3u;
    const uint32_t su = __builtin_amdgcn_readfirstlane(t0 * 5u);
    for (int c = 0; c < 16; ++c) a[c] = t0 + c * 0x01010101u;
    __syncthreads();
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < REPS; ++r) {
        if (MODE == 0) P16("v_perm_b32", "");
        if (MODE == 1) P16("v_bitop3_b32", " bitop3:0x96");
        if (MODE == 2) P16("v_xad_u32", "");
        if (MODE == 3) P16("v_and_or_b32", "");
        if (MODE == 4) P16_2("v_xor_b32");
        if (MODE == 5) P16S("v_perm_b32", "");
        if (MODE == 6) P16S("v_bitop3_b32", " bitop3:0x96");
    }
    const unsigned long long t_end = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
    for (int c = 0; c < 16; ++c) x ^= a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t_end - t_start;
}

template <int MODE>
void run(const char *name, int waves_per_simd) {
    const int threads = 256 * waves_per_simd;  // 4 SIMDs per CU
    const int blocks = 256;                    // one workgroup per CU
    unsigned long long *cyc;
    uint32_t *out;
    (void)hipMalloc(&cyc, blocks * threads / 64 * 8);
    (void)hipMalloc(&out, blocks * threads * 4);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, cyc, out, 1u);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, cyc, out, 2u);
    (void)hipDeviceSynchronize();
    const int nw = blocks * threads / 64;
    unsigned long long *h = new unsigned long long[nw];
    (void)hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
    unsigned long long mx = 0;
    double mean = 0;
    for (int i = 0; i < nw; ++i) {
        mx = h[i] > mx ? h[i] : mx;
        mean += h[i];
    }
    mean /= nw;
    // s_memtime ticks at the shader clock (MI355X_MICROARCH.md: tick = shader cycle)
    const double insts_per_simd = double(REPS) * 16 * waves_per_simd;
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_inst_per_simd\": %.3f, \"mean_wave_cycles\": %.0f}\n",
           name, waves_per_simd, mx / insts_per_simd, mean);
    delete[] h;
    (void)hipFree(cyc);
    (void)hipFree(out);
}

int main() {
    for (int w : {2, 4}) {
        run<0>("v_perm_b32 v,v,v", w);
        run<1>("v_bitop3_b32 v,v,v", w);
        run<4>("v_xor_b32 v,v (VOP2)", w);
        run<5>("v_perm_b32 s,v,v", w);
        run<6>("v_bitop3_b32 s,v,v", w);
    }
    return 0;
}
