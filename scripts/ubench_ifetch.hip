// ubench_ifetch.hip — is a long straight-line instruction stream fetch-bound on gfx950?  The same plain
// v_xor_b32 (4-byte VOP2) / v_bfi_b32 (8-byte VOP3) mix, as loop bodies of 32 .. 4096 instructions, at
// 1/2/4 waves per SIMD (forced with dynamic LDS); cycles per instruction per SIMD from the chip-wide span.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_ifetch.hip -o build/ubench_ifetch && build/ubench_ifetch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"
#define X8                                                                                                     \
    "v_xor_b32 v56, v41, v56\n v_xor_b32 v57, v42, v57\n v_xor_b32 v58, v43, v58\n v_xor_b32 v59, v44, v59\n" \
    "v_xor_b32 v60, v45, v60\n v_xor_b32 v61, v46, v61\n v_xor_b32 v62, v47, v62\n v_xor_b32 v63, v40, v63\n"
#define B8                                                                                                             \
    "v_bfi_b32 v56, v41, v42, v56\n v_bfi_b32 v57, v42, v43, v57\n v_bfi_b32 v58, v43, v44, v58\n v_bfi_b32 v59, v44, v45, v59\n" \
    "v_bfi_b32 v60, v45, v46, v60\n v_bfi_b32 v61, v46, v47, v61\n v_bfi_b32 v62, v47, v40, v62\n v_bfi_b32 v63, v40, v41, v63\n"
#define R2(x) x x
#define R4(x) R2(x) R2(x)
#define R8(x) R4(x) R4(x)
#define R16(x) R8(x) R8(x)
#define R32(x) R16(x) R16(x)
#define R64(x) R32(x) R32(x)
#define R128(x) R64(x) R64(x)

template <int MODE>  // 0: 32-instr xor body, 1: 4096-instr xor body, 2: 32-instr bfi body, 3: 4096-instr bfi body
__global__ __launch_bounds__(256) void k(unsigned long long *out, int reps) {
    extern __shared__ uint32_t lds[];
    asm volatile("v_mov_b32 v40, 1\n v_mov_b32 v41, 2\n v_mov_b32 v42, 3\n v_mov_b32 v43, 4\n v_mov_b32 v44, 5\n"
                 "v_mov_b32 v45, 6\n v_mov_b32 v46, 7\n v_mov_b32 v47, 8\n" ::: CLOB);
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (MODE == 0) asm volatile(R4(X8) ::: CLOB);
        if (MODE == 1) asm volatile(R128(R4(X8)) ::: CLOB);
        if (MODE == 2) asm volatile(R4(B8) ::: CLOB);
        if (MODE == 3) asm volatile(R128(R4(B8)) ::: CLOB);
    }
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

static const char *names[] = {"xor VOP2, 32-instr loop", "xor VOP2, 4096-instr loop", "bfi VOP3, 32-instr loop",
                              "bfi VOP3, 4096-instr loop"};

template <int MODE>
void run(int W, unsigned long long *d) {
    const int blocks = 256 * W;
    const int reps = (MODE & 1) ? 4 : 512;  // 16384 instructions per wave either way
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
    const double insts = 16384.0 * W;
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"clock_GHz\": %.3f, \"cyc_per_inst_span\": %.3f}\n", names[MODE],
           W, ghz, double(rmax - rmin) * 10.0 * ghz / insts);
}

int main() {
    unsigned long long *d;
    hipMalloc(&d, 256 * 8 * 4 * 4 * sizeof(unsigned long long));
    for (int W : {1, 2, 4}) {
        run<0>(W, d);
        run<1>(W, d);
        run<2>(W, d);
        run<3>(W, d);
    }
    return 0;
}
