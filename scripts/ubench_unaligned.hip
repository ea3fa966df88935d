// ubench_unaligned.hip -- do 16-byte vector memory instructions at byte-misaligned global addresses return the
// right bytes on this box (SH_MEM_CONFIG alignment mode), and at what rate?  MEASUREMENT ONLY.
//   check   global_load_dwordx4 / global_store_dwordx4 / global_load_lds_dwordx4 at offsets 0..15 against a byte loop
//   rate    a 1 GiB row copy with source and destination offset by 0 / 3 / 8 bytes (dwordx4 per lane)
//
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_unaligned.hip -o build/ubench_unaligned && build/ubench_unaligned
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void vec_kernel(const uint8_t *src, uint8_t *dst, uint8_t *dst_lds, int off_in, int off_out) {
    __shared__ __attribute__((aligned(16))) uint32_t ring[64 * 4];
    const int l = threadIdx.x;
    const uint8_t *s = src + off_in + 16 * l;
    uint8_t *d = dst + off_out + 16 * l;
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    u4 x;
    asm volatile("global_load_dwordx4 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(x) : "v"(s) : "memory");
    asm volatile("global_store_dwordx4 %0, %1, off\n s_waitcnt vmcnt(0)" ::"v"(d), "v"(x) : "memory");
    // LDS-DMA: lane l's 16 bytes land at ring + 16 l
    __builtin_amdgcn_global_load_lds(s, (__attribute__((address_space(3))) void *)ring, 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const u4 y = reinterpret_cast<const u4 *>(ring)[l];
    reinterpret_cast<u4 *>(dst_lds)[l] = y;
}

__global__ __launch_bounds__(256) void copy_kernel(const uint8_t *src, uint8_t *dst, int64_t n16) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n16; i += int64_t(gridDim.x) * 256) {
        u4 x;
        asm volatile("global_load_dwordx4 %0, %1, off\n s_waitcnt vmcnt(0)" : "=v"(x) : "v"(src + 16 * i) : "memory");
        asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(dst + 16 * i), "v"(x) : "memory");
    }
}

int main() {
    uint8_t *src, *dst, *dl;
    (void)hipMalloc(&src, 4096);
    (void)hipMalloc(&dst, 4096);
    (void)hipMalloc(&dl, 4096);
    std::vector<uint8_t> h(4096);
    for (int i = 0; i < 4096; ++i) h[i] = uint8_t(i * 7 + 1);
    (void)hipMemcpy(src, h.data(), 4096, hipMemcpyHostToDevice);
    for (int oi : {0, 1, 3, 4, 8, 13}) {
        for (int oo : {0, 3, 8}) {
            (void)hipMemset(dst, 0, 4096);
            (void)hipMemset(dl, 0, 4096);
            hipLaunchKernelGGL(vec_kernel, dim3(1), dim3(64), 0, 0, src, dst, dl, oi, oo);
            hipError_t e = hipDeviceSynchronize();
            std::vector<uint8_t> g(4096), gl(4096);
            (void)hipMemcpy(g.data(), dst, 4096, hipMemcpyDeviceToHost);
            (void)hipMemcpy(gl.data(), dl, 4096, hipMemcpyDeviceToHost);
            int bad = 0, badl = 0;
            for (int i = 0; i < 1024; ++i) {
                bad += g[oo + i] != h[oi + i];
                badl += gl[i] != h[oi + i];
            }
            int stray = 0;
            for (int i = 0; i < oo; ++i) stray += g[i] != 0;
            for (int i = oo + 1024; i < 4096; ++i) stray += g[i] != 0;
            printf("{\"check\": \"in+%d out+%d\", \"err\": \"%s\", \"vec_bad\": %d, \"stray\": %d, \"lds_dma_bad\": %d}\n", oi, oo,
                   hipGetErrorString(e), bad, stray, badl);
        }
    }
    (void)hipFree(src);
    (void)hipFree(dst);
    (void)hipFree(dl);
    const int64_t n = int64_t(1) << 30;
    (void)hipMalloc(&src, n + 64);
    (void)hipMalloc(&dst, n + 64);
    (void)hipMemset(src, 0x5A, n + 64);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int oi : {0, 3, 8})
        for (int oo : {0, 3}) {
            float best = 1e9f;
            for (int it = 0; it < 5; ++it) {
                (void)hipEventRecord(a, 0);
                hipLaunchKernelGGL(copy_kernel, dim3(256 * 8), dim3(256), 0, 0, src + oi, dst + oo, n / 16);
                (void)hipEventRecord(b, 0);
                (void)hipEventSynchronize(b);
                float ms;
                (void)hipEventElapsedTime(&ms, a, b);
                if (it && ms < best) best = ms;
            }
            printf("{\"rate\": \"in+%d out+%d\", \"ms\": %.4f, \"copy_TBps\": %.3f, \"err\": \"%s\"}\n", oi, oo, best,
                   2.0 * n / (best * 1e-3) * 1e-12, hipGetErrorString(hipGetLastError()));
        }
    return 0;
}
