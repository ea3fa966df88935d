// the trivial kernel of scripts/ubench_hsa_dispatch.cpp: writes n bytes (write-through) and raises one flag per block
#include <hip/hip_runtime.h>
struct Args {
    unsigned char *dst;
    unsigned *flag;
    unsigned n, epoch;
};
extern "C" __global__ void flag_kernel(Args a) {
    const unsigned i = (blockIdx.x * 256 + threadIdx.x) * 16;
    if (i + 16 <= a.n) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.dst, 0, 0x7FFFFFFF, 0x00020000);
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        const u4 v = {a.epoch, a.epoch, a.epoch, a.epoch};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, int(i), 0, 17);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(a.flag + blockIdx.x, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
