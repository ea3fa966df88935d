// hbm_ceiling.hip — the HBM rates this box reaches with no GF arithmetic at all, measured live (bench.py's
// `hbm_single_pass_encode.ceiling`).  MEASUREMENT INFRASTRUCTURE, not part of librlnc_hip.
//
// Three access patterns over a buffer far larger than the 256 MiB Infinity Cache, timed with HIP events:
//   copy     — 16 B per lane float4-style copy, grid-stride (the guide's "6.29 TB/s measured" calibration);
//   read     — 16 B per lane contiguous read-only sweep, 4 loads in flight per lane, one 16-B store per lane;
//   pattern  — exactly the single-pass encoder's access pattern (gf_matmul_stream_kernel<1, 2>): one
//              workgroup per 4 KiB column block of one object, the k source rows of that block (row stride L)
//              read with 2 rows in flight per lane, one 4 KiB output row written — XOR in place of the GF product.
// The pattern rate is the ceiling the single-pass encode can reach on this box; the kernel's fraction of it
// separates arithmetic overhead from what the access pattern and HBM allow.
#include <hip/hip_runtime.h>

#include <cstdint>

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4_t ld_nt(const u32x4_t *p) { return __builtin_nontemporal_load(p); }

__global__ __launch_bounds__(256) void copy_kernel(const u32x4_t *src, u32x4_t *dst, size_t n) {
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void read_kernel(const u32x4_t *src, u32x4_t *out, size_t n) {
    u32x4_t acc = {0, 0, 0, 0};
    const size_t stride = size_t(gridDim.x) * 256;
    size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const u32x4_t a = ld_nt(src + i), b = ld_nt(src + i + stride), c = ld_nt(src + i + 2 * stride),
                      d = ld_nt(src + i + 3 * stride);
        acc ^= a ^ b ^ c ^ d;
    }
    for (; i < n; i += stride) acc ^= ld_nt(src + i);
    out[size_t(blockIdx.x) * 256 + threadIdx.x] = acc;
}

// grid = objects × column blocks (XCD-aware as decode_block in kernels.hip), k rows of stride L per block
__global__ __launch_bounds__(256) void pattern_kernel(const uint8_t *src, uint8_t *out, int k, int64_t L, int col_blocks,
                                                      int total) {
    int b = blockIdx.x, w = b;
    if ((total & 7) == 0) w = (b & 7) * (total >> 3) + (b >> 3);
    const int cb = w % col_blocks, obj = w / col_blocks;
    const uint8_t *p = src + int64_t(obj) * k * L + int64_t(cb) * 4096 + threadIdx.x * 16;
    u32x4_t acc = {0, 0, 0, 0};
    u32x4_t x0 = ld_nt(reinterpret_cast<const u32x4_t *>(p));
    u32x4_t x1 = ld_nt(reinterpret_cast<const u32x4_t *>(p + (k > 1 ? L : 0)));
    for (int j = 0; j < k; j += 2) {
        const u32x4_t a = x0, c = x1;
        x0 = ld_nt(reinterpret_cast<const u32x4_t *>(p + int64_t(min(j + 2, k - 1)) * L));
        x1 = ld_nt(reinterpret_cast<const u32x4_t *>(p + int64_t(min(j + 3, k - 1)) * L));
        acc ^= a;
        if (j + 1 < k) acc ^= c;
    }
    *reinterpret_cast<u32x4_t *>(out + int64_t(obj) * L + int64_t(cb) * 4096 + threadIdx.x * 16) = acc;
}

extern "C" {
// Rates in GB/s (bytes moved by the kernel ÷ median time of 7 launches after 2 warm-ups) of the three patterns:
// rates[0] copy (read + write bytes), rates[1] read (read bytes), rates[2] pattern (read bytes; `objects` × k × L
// of source), rates[3] pattern counting read + write bytes.  Returns 0, or < 0 on a HIP error.  Current device,
// null stream, synchronous.  Needs 2 × objects × k × L bytes of device memory.
int hbm_rates(int objects, int k, long long L, double *rates) {
    if (objects <= 0 || k <= 0 || L < 4096 || L % 4096) return -1;
    const size_t src_b = size_t(objects) * k * size_t(L);
    uint8_t *src = nullptr, *dst = nullptr;
    if (hipMalloc(&src, src_b) != hipSuccess) return -2;
    if (hipMalloc(&dst, src_b) != hipSuccess) {
        (void)hipFree(src);
        return -2;
    }
    (void)hipMemset(src, 0x5A, src_b);
    hipDeviceProp_t prop;
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipGetDeviceProperties(&prop, dev);
    const int cu = prop.multiProcessorCount;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    int rc = 0;
    for (int which = 0; which < 3 && rc == 0; ++which) {
        float t[9];
        for (int it = 0; it < 9; ++it) {
            (void)hipEventRecord(a, 0);
            const size_t n = src_b / 16;
            if (which == 0) {
                hipLaunchKernelGGL(copy_kernel, dim3(cu * 8), dim3(256), 0, 0, reinterpret_cast<const u32x4_t *>(src),
                                   reinterpret_cast<u32x4_t *>(dst), n);
            } else if (which == 1) {
                hipLaunchKernelGGL(read_kernel, dim3(cu * 8), dim3(256), 0, 0, reinterpret_cast<const u32x4_t *>(src),
                                   reinterpret_cast<u32x4_t *>(dst), n);
            } else {
                const int cbs = int(L / 4096), total = objects * cbs;
                hipLaunchKernelGGL(pattern_kernel, dim3(total), dim3(256), 0, 0, src, dst, k, int64_t(L), cbs, total);
            }
            (void)hipEventRecord(b, 0);
            if (hipEventSynchronize(b) != hipSuccess) {
                rc = -3;
                break;
            }
            (void)hipEventElapsedTime(&t[it], a, b);
        }
        if (rc) break;
        float s[7];
        for (int i = 0; i < 7; ++i) s[i] = t[i + 2];
        for (int i = 0; i < 7; ++i)
            for (int j = i + 1; j < 7; ++j)
                if (s[j] < s[i]) {
                    const float x = s[i];
                    s[i] = s[j];
                    s[j] = x;
                }
        const double sec = double(s[3]) * 1e-3;
        if (which == 0) rates[0] = 2.0 * double(src_b) / sec / 1e9;
        if (which == 1) rates[1] = double(src_b) / sec / 1e9;
        if (which == 2) {
            rates[2] = double(src_b) / sec / 1e9;
            rates[3] = (double(src_b) + double(objects) * double(L)) / sec / 1e9;
        }
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(src);
    (void)hipFree(dst);
    return rc;
}
}
