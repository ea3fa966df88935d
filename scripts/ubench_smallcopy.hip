// ubench_smallcopy.hip -- HBM rate of the configs[0]-shape product's memory pattern alone (4,096 objects x 16 rows x
// 4 KiB read, 16 rows written; coded pieces at a 4,112-byte row pitch with the data 16 bytes in).  MEASUREMENT ONLY:
// how far the 2-wave bit-sliced product (108-115 us) is from what a copy of the same shape reaches, and whether the
// occupancy its 243 VGPRs allow (4 workgroups of 2 waves per CU) is what limits it.
//   flat              grid-stride 16-byte copy of the 268 MB, the chip's copy rate
//   tile<DIR,WGS>     one 128-thread workgroup per object, wave w copies rows [8w, 8w+8), 4 x 16 B a lane a row at
//                     16 lane + 1 KiB u (the product's DMA / store footprint), WGS workgroups per CU forced through LDS; DIR 0: aligned rows -> pieces
//                     (encode), 1: pieces -> aligned rows (decode), 2: aligned -> aligned
//
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_smallcopy.hip -o build/ubench_smallcopy && build/ubench_smallcopy
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

constexpr int OBJ = 4096, K = 16, L = 4096, PITCH = K + L;

__global__ __launch_bounds__(256) void flat_kernel(const u32x4_t *src, u32x4_t *dst, int64_t n) {
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256)
        __builtin_nontemporal_store(src[i], dst + i);
}

template <int DIR>
__global__ __launch_bounds__(128) void tile_kernel(const uint8_t *src, uint8_t *dst) {
    extern __shared__ uint8_t pad[];
    const int obj = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t in_row = DIR == 1 ? PITCH : L, out_row = DIR == 0 ? PITCH : L;
    const int in_off = DIR == 1 ? K : 0, out_off = DIR == 0 ? K : 0;
    const uint8_t *s = src + int64_t(obj) * K * in_row + in_off + 16 * lane;
    uint8_t *d = dst + int64_t(obj) * K * out_row + out_off + 16 * lane;
    u32x4_t v[8][4];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int u = 0; u < 4; ++u)
            v[r][u] = *reinterpret_cast<const u32x4_t *>(s + (8 * w + r) * in_row + 1024 * u);
    if (lane == 64) pad[0] = 0;  // keeps the LDS allocation
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int u = 0; u < 4; ++u)
            __builtin_nontemporal_store(v[r][u], reinterpret_cast<u32x4_t *>(d + (8 * w + r) * out_row + 1024 * u));
}

static float time_it(void (*launch)(void *), void *arg) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) launch(arg);
    hipEventRecord(a);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) launch(arg);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

struct Bufs {
    uint8_t *a, *p, *o;
    int dir, lds;
};

template <int DIR>
static void launch_tile(void *arg) {
    Bufs *b = static_cast<Bufs *>(arg);
    const uint8_t *src = DIR == 1 ? b->p : b->a;
    uint8_t *dst = DIR == 0 ? b->p : b->o;
    hipLaunchKernelGGL(tile_kernel<DIR>, dim3(OBJ), dim3(128), b->lds, 0, src, dst);
}

static void launch_flat(void *arg) {
    Bufs *b = static_cast<Bufs *>(arg);
    const int64_t n = int64_t(OBJ) * K * L / 16;
    hipLaunchKernelGGL(flat_kernel, dim3(256 * 32), dim3(256), 0, 0, reinterpret_cast<const u32x4_t *>(b->a),
                       reinterpret_cast<u32x4_t *>(b->o), n);
}

int main() {
    Bufs b{};
    const size_t na = size_t(OBJ) * K * L, np = size_t(OBJ) * K * PITCH;
    hipMalloc(&b.a, na);
    hipMalloc(&b.p, np);
    hipMalloc(&b.o, na);
    hipMemset(b.a, 1, na);
    hipMemset(b.p, 2, np);
    hipMemset(b.o, 3, na);
    hipDeviceSynchronize();
    const double bytes = 2.0 * na;
    const float fms = time_it(launch_flat, &b);
    printf("{\"pattern\": \"flat\", \"ms\": %.4f, \"TBps\": %.3f}\n", fms, bytes / (fms * 1e-3) / 1e12);
    hipFuncSetAttribute(reinterpret_cast<const void *>(tile_kernel<0>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute(reinterpret_cast<const void *>(tile_kernel<1>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute(reinterpret_cast<const void *>(tile_kernel<2>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const int wgs_list[] = {2, 4, 6, 8, 16};
    for (int dir = 0; dir < 3; ++dir)
        for (int wgs : wgs_list) {
            b.lds = 160 * 1024 / wgs - 1024;
            void (*f)(void *) = dir == 0 ? launch_tile<0> : dir == 1 ? launch_tile<1> : launch_tile<2>;
            const float ms = time_it(f, &b);
            printf("{\"pattern\": \"tile\", \"dir\": \"%s\", \"wg_per_cu\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n",
                   dir == 0 ? "rows->pieces" : dir == 1 ? "pieces->rows" : "rows->rows", wgs, ms,
                   bytes / (ms * 1e-3) / 1e12);
        }
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        printf("error %s\n", hipGetErrorString(e));
        return 1;
    }
    return 0;
}
