// ubench_stream.hip -- HBM read patterns for the single-pass encode (one coded piece per pass over the k source
// rows: configs[1]'s 32 objects x k = 32 x 1 MiB read once, 32 MiB written).  MEASUREMENT ONLY.
// XOR in place of the GF product (the arithmetic is ~15 % of the VALU at these rates); random source bytes.
//   colblock<PF>  the shipped kernel's pattern: one 256-thread workgroup per 4 KiB column block (VW 2: 8 KiB),
//                 the k rows walked with PF row pairs in flight per lane
//   span<S>       one workgroup per S KiB column span: each row's span read contiguously (S / 4 16-byte loads
//                 per lane, all in flight), rows walked one after another, accumulators for the whole span
//   ldsdma<D>     one workgroup per 4 KiB column block, the rows streamed through a D-slot LDS ring by
//                 global_load_lds_dwordx4 (D - 1 rows in flight), each lane reading its 16 bytes back
//
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_stream.hip -o build/ubench_stream && build/ubench_stream
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4_t ld_nt(const uint8_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(p));
}

constexpr int K = 32;
constexpr int64_t L = 1 << 20;
constexpr int OBJ = 32;

__device__ __forceinline__ int xcd_map(int b, int total) { return (total & 7) == 0 ? (b & 7) * (total >> 3) + (b >> 3) : b; }

template <int PF>
__global__ __launch_bounds__(256) void colblock_kernel(const uint8_t *src, uint8_t *out) {
    constexpr int CB = int(L / 8192);
    const int w = xcd_map(blockIdx.x, OBJ * CB);
    const int cb = w % CB, obj = w / CB;
    const uint8_t *p = src + int64_t(obj) * K * L + int64_t(cb) * 8192 + threadIdx.x * 16;
    u32x4_t acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    u32x4_t b0[PF], b1[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        b0[u] = ld_nt(p + int64_t(u) * L);
        b1[u] = ld_nt(p + int64_t(u) * L + 4096);
    }
    for (int j = 0; j < K; j += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            acc0 ^= b0[u];
            acc1 ^= b1[u];
            const int n = min(j + u + PF, K - 1);
            b0[u] = ld_nt(p + int64_t(n) * L);
            b1[u] = ld_nt(p + int64_t(n) * L + 4096);
        }
    }
    uint8_t *o = out + int64_t(obj) * L + int64_t(cb) * 8192 + threadIdx.x * 16;
    *reinterpret_cast<u32x4_t *>(o) = acc0;
    *reinterpret_cast<u32x4_t *>(o + 4096) = acc1;
}

template <int S>  // span of S KiB per workgroup: S/4 loads of 16 B per lane per row
__global__ __launch_bounds__(256) void span_kernel(const uint8_t *src, uint8_t *out) {
    constexpr int NS = int(L / (S * 1024));
    constexpr int V = S / 4;
    const int w = xcd_map(blockIdx.x, OBJ * NS);
    const int sp = w % NS, obj = w / NS;
    const uint8_t *p = src + int64_t(obj) * K * L + int64_t(sp) * S * 1024 + threadIdx.x * 16;
    u32x4_t acc[V], buf[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
        acc[v] = u32x4_t{0, 0, 0, 0};
        buf[v] = ld_nt(p + v * 4096);
    }
    for (int j = 1; j <= K; ++j) {
        const uint8_t *q = p + int64_t(min(j, K - 1)) * L;
#pragma unroll
        for (int v = 0; v < V; ++v) {
            acc[v] ^= buf[v];
            buf[v] = ld_nt(q + v * 4096);
        }
    }
    uint8_t *o = out + int64_t(obj) * L + int64_t(sp) * S * 1024 + threadIdx.x * 16;
#pragma unroll
    for (int v = 0; v < V; ++v) *reinterpret_cast<u32x4_t *>(o + v * 4096) = acc[v];
}

template <int D>  // LDS ring of D 4 KiB slots, D - 1 rows in flight
__global__ __launch_bounds__(256) void ldsdma_kernel(const uint8_t *src, uint8_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[D * 4096];
    constexpr int CB = int(L / 4096);
    const int w = xcd_map(blockIdx.x, OBJ * CB);
    const int cb = w % CB, obj = w / CB;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint8_t *p = src + int64_t(obj) * K * L + int64_t(cb) * 4096 + wave * 1024 + lane * 16;
    u32x4_t acc = {0, 0, 0, 0};
    // row j -> slot j % D: every wave moves its 1 KiB quarter of the row
#pragma unroll
    for (int j = 0; j < D - 1; ++j)
        __builtin_amdgcn_global_load_lds(p + int64_t(j) * L, (__attribute__((address_space(3))) void *)(ring + j * 4096 + wave * 1024), 16, 0, 0);
    for (int j = 0; j < K; ++j) {
        // row j landed for this wave's own DMA (D - 2 younger ones may fly), then every wave's
        __builtin_amdgcn_s_waitcnt(0x0F70 | ((D - 2) & 0xf) | ((((D - 2) >> 4) & 3) << 14));
        __builtin_amdgcn_s_barrier();
        const int nj = j + D - 1;
        __builtin_amdgcn_global_load_lds(p + int64_t(min(nj, K - 1)) * L,
                                         (__attribute__((address_space(3))) void *)(ring + (nj % D) * 4096 + wave * 1024), 16, 0, 0);
        acc ^= *reinterpret_cast<const u32x4_t *>(ring + (j % D) * 4096 + threadIdx.x * 16);
    }
    *reinterpret_cast<u32x4_t *>(out + int64_t(obj) * L + int64_t(cb) * 4096 + threadIdx.x * 16) = acc;
}

template <class F>
static void timeit(const char *name, F launch) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float t[9];
    for (int it = 0; it < 9; ++it) {
        (void)hipEventRecord(a, 0);
        launch();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&t[it], a, b);
    }
    float s[7];
    for (int i = 0; i < 7; ++i) s[i] = t[i + 2];
    for (int i = 0; i < 7; ++i)
        for (int j = i + 1; j < 7; ++j)
            if (s[j] < s[i]) {
                const float x = s[i];
                s[i] = s[j];
                s[j] = x;
            }
    const double sec = s[3] * 1e-3;
    const double rd = double(OBJ) * K * L;
    printf("{\"case\": \"%s\", \"ms\": %.4f, \"read_TBps\": %.3f, \"read_frac_8TBps\": %.4f, \"err\": \"%s\"}\n", name,
           s[3], rd / sec * 1e-12, rd / sec / 8e12, hipGetErrorString(hipGetLastError()));
}

__global__ void fill_kernel(uint32_t *p, size_t n) {
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = uint32_t(z ^ (z >> 31));
    }
}

int main() {
    const size_t src_b = size_t(OBJ) * K * L;
    uint8_t *src = nullptr, *out = nullptr;
    if (hipMalloc(&src, src_b) != hipSuccess || hipMalloc(&out, size_t(OBJ) * L) != hipSuccess) return 1;
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t *>(src), src_b / 4);
    (void)hipDeviceSynchronize();
    const int cb8 = OBJ * int(L / 8192), cb4 = OBJ * int(L / 4096);
    for (int rep = 0; rep < 2; ++rep) {
        timeit("colblock_pf1", [&] { hipLaunchKernelGGL(colblock_kernel<1>, dim3(cb8), dim3(256), 0, 0, src, out); });
        timeit("colblock_pf2", [&] { hipLaunchKernelGGL(colblock_kernel<2>, dim3(cb8), dim3(256), 0, 0, src, out); });
        timeit("colblock_pf4", [&] { hipLaunchKernelGGL(colblock_kernel<4>, dim3(cb8), dim3(256), 0, 0, src, out); });
        timeit("span16", [&] { hipLaunchKernelGGL(span_kernel<16>, dim3(OBJ * int(L / 16384)), dim3(256), 0, 0, src, out); });
        timeit("span32", [&] { hipLaunchKernelGGL(span_kernel<32>, dim3(OBJ * int(L / 32768)), dim3(256), 0, 0, src, out); });
        timeit("span64", [&] { hipLaunchKernelGGL(span_kernel<64>, dim3(OBJ * int(L / 65536)), dim3(256), 0, 0, src, out); });
        timeit("ldsdma4", [&] { hipLaunchKernelGGL(ldsdma_kernel<4>, dim3(cb4), dim3(256), 0, 0, src, out); });
        timeit("ldsdma8", [&] { hipLaunchKernelGGL(ldsdma_kernel<8>, dim3(cb4), dim3(256), 0, 0, src, out); });
        timeit("ldsdma16", [&] { hipLaunchKernelGGL(ldsdma_kernel<16>, dim3(cb4), dim3(256), 0, 0, src, out); });
    }
    (void)hipFree(src);
    (void)hipFree(out);
    return 0;
}
