// gf_ceiling.hip — the GF(2^8) multiply-add ceiling of the bit-sliced design, measured live on the device
// (bench.py's roofline "peak").  MEASUREMENT INFRASTRUCTURE, not part of librlnc_hip.
//
// The bit-sliced kernel (rlnc_amd/csrc/gen_bsjump.py) adds c·x for 64 lanes × 32 bytes into 8 accumulator
// bit-planes with 8 v_bitop3_b32 XOR3s (acc[o] ^= G_lo[c,o] ^ G_hi[c,o]): 2,048 multiply-adds per 8
// instructions, 256 GF(2^8) multiply-adds per XOR3.  That is the fewest VALU instructions per multiply-add of
// the design, so the chip's XOR3 issue rate × 256 bounds every kernel built on it.  This kernel issues
// nothing but independent XOR3s (accumulators in four VGPR banks, operands in the other three, random data so
// the toggling — and hence the power-limited clock — matches real pieces) at 2 or 4 waves per SIMD (forced
// with dynamic LDS), timed with HIP events over a ~0.1 s launch.
#include <hip/hip_runtime.h>

#include <cstdint>

#define CLOB                                                                                                       \
    "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"
#define B3X                                                                                                       \
    "v_bitop3_b32 v56, v41, v42, v56 bitop3:0x96\n v_bitop3_b32 v57, v42, v43, v57 bitop3:0x96\n"                \
    "v_bitop3_b32 v58, v43, v40, v58 bitop3:0x96\n v_bitop3_b32 v59, v40, v41, v59 bitop3:0x96\n"                \
    "v_bitop3_b32 v60, v45, v46, v60 bitop3:0x96\n v_bitop3_b32 v61, v46, v47, v61 bitop3:0x96\n"                \
    "v_bitop3_b32 v62, v47, v44, v62 bitop3:0x96\n v_bitop3_b32 v63, v44, v45, v63 bitop3:0x96\n"

__global__ __launch_bounds__(256) void xor3_issue_kernel(const uint32_t *seed, uint32_t *out, int reps) {
    extern __shared__ uint32_t lds[];
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    const uint32_t *s = seed + (g % 4096) * 16;
    // random operands and accumulators (the loads complete before the timed loop's first use)
    asm volatile(
        "global_load_dwordx4 v[40:43], %0, off\n global_load_dwordx4 v[44:47], %0, off offset:16\n"
        "global_load_dwordx4 v[56:59], %0, off offset:32\n global_load_dwordx4 v[60:63], %0, off offset:48\n"
        "s_waitcnt vmcnt(0)" ::"v"(s)
        : CLOB);
    for (int r = 0; r < reps; ++r) asm volatile(B3X B3X B3X B3X B3X B3X B3X B3X ::: CLOB);  // 64 XOR3s
    uint32_t acc;
    asm volatile("v_xor_b32 %0, v56, v57\n v_xor_b32 %0, %0, v58\n v_xor_b32 %0, %0, v59\n v_xor_b32 %0, %0, v60\n"
                 "v_xor_b32 %0, %0, v61\n v_xor_b32 %0, %0, v62\n v_xor_b32 %0, %0, v63"
                 : "=v"(acc)::CLOB);
    if (acc == 0x9E3779B9u && lds[threadIdx.x] == 0x12345678u) out[g] = acc;  // keeps the work observable
}

extern "C" {
// XOR3 instructions per second (wave64 instructions, whole device) at `waves_per_simd` (2 or 4) waves per SIMD;
// < 0 on a HIP error.  Runs on the current device, on the null stream, synchronously.
double gf_xor3_issue_rate(int waves_per_simd, int reps) {
    hipDeviceProp_t prop;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return -1;
    const int W = waves_per_simd;
    const int blocks = prop.multiProcessorCount * W;  // 4 waves per block, one per SIMD
    const size_t lds = (160 * 1024) / W - 1024;       // at most W blocks per CU
    if (hipFuncSetAttribute(reinterpret_cast<const void *>(xor3_issue_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
        return -2;
    uint32_t *seed = nullptr, *out = nullptr;
    if (hipMalloc(&seed, 4096 * 16 * 4) != hipSuccess || hipMalloc(&out, size_t(blocks) * 256 * 4) != hipSuccess)
        return -3;
    uint32_t *h = new uint32_t[4096 * 16];
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < 4096 * 16; ++i) {  // splitmix64
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        h[i] = uint32_t(z ^ (z >> 31));
    }
    (void)hipMemcpy(seed, h, 4096 * 16 * 4, hipMemcpyHostToDevice);
    delete[] h;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    double best = 0;
    for (int it = 0; it < 4; ++it) {  // the first launches ramp the clock
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(xor3_issue_kernel, dim3(blocks), dim3(256), lds, 0, seed, out, reps);
        (void)hipEventRecord(b, 0);
        if (hipEventSynchronize(b) != hipSuccess) return -4;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        const double rate = double(blocks) * 4 * double(reps) * 64 / (ms * 1e-3);
        if (it >= 1 && rate > best) best = rate;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(seed);
    (void)hipFree(out);
    return best;
}
}
