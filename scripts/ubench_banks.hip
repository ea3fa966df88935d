// ubench_banks.hip — does the VGPR bank of the source operands change the issue rate of VOP3 instructions
// on gfx950?  Explicit physical registers (bank = vN mod 4), 64 instructions per block, s_memtime cycles.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_banks.hip -o build/ubench_banks && build/ubench_banks
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int REPS = 128;

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", \
             "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63"

template <int MODE>
__global__ void k(unsigned long long *cyc) {
    asm volatile("v_mov_b32 v41, 0x01020304\n v_mov_b32 v42, 0x05060708\n v_mov_b32 v43, 0x00010203\n"
                 "v_mov_b32 v44, 1\n v_mov_b32 v48, 2\n v_mov_b32 v52, 3\n v_mov_b32 v45, 5\n v_mov_b32 v46, 6" ::: CLOB);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < REPS; ++r) {
        // four different destinations (no dependency chain longer than the 4-instruction rotation)
        if (MODE == 0)  // sources in banks 1,2,3
            asm volatile(R16("v_perm_b32 v56, v41, v42, v43\n v_perm_b32 v57, v41, v42, v43\n"
                             "v_perm_b32 v58, v41, v42, v43\n v_perm_b32 v59, v41, v42, v43\n") ::: CLOB);
        if (MODE == 1)  // sources all in bank 0
            asm volatile(R16("v_perm_b32 v56, v44, v48, v52\n v_perm_b32 v57, v44, v48, v52\n"
                             "v_perm_b32 v58, v44, v48, v52\n v_perm_b32 v59, v44, v48, v52\n") ::: CLOB);
        if (MODE == 2)  // bitop3, banks 1,2,3
            asm volatile(R16("v_bitop3_b32 v56, v41, v42, v43 bitop3:0x96\n v_bitop3_b32 v57, v41, v42, v43 bitop3:0x96\n"
                             "v_bitop3_b32 v58, v41, v42, v43 bitop3:0x96\n v_bitop3_b32 v59, v41, v42, v43 bitop3:0x96\n") ::: CLOB);
        if (MODE == 3)  // bitop3, bank 0
            asm volatile(R16("v_bitop3_b32 v56, v44, v48, v52 bitop3:0x96\n v_bitop3_b32 v57, v44, v48, v52 bitop3:0x96\n"
                             "v_bitop3_b32 v58, v44, v48, v52 bitop3:0x96\n v_bitop3_b32 v59, v44, v48, v52 bitop3:0x96\n") ::: CLOB);
        if (MODE == 4)  // VOP2 xor, banks 1,2
            asm volatile(R16("v_xor_b32 v56, v41, v42\n v_xor_b32 v57, v41, v42\n v_xor_b32 v58, v41, v42\n"
                             "v_xor_b32 v59, v41, v42\n") ::: CLOB);
        if (MODE == 5)  // VOP2 xor, bank 0
            asm volatile(R16("v_xor_b32 v56, v44, v48\n v_xor_b32 v57, v44, v48\n v_xor_b32 v58, v44, v48\n"
                             "v_xor_b32 v59, v44, v48\n") ::: CLOB);
        if (MODE == 6)  // VOP3 encoding of a 2-source op (v_xor_b32_e64), banks 1,2
            asm volatile(R16("v_xor_b32_e64 v56, v41, v42\n v_xor_b32_e64 v57, v41, v42\n v_xor_b32_e64 v58, v41, v42\n"
                             "v_xor_b32_e64 v59, v41, v42\n") ::: CLOB);
        if (MODE == 7)  // perm with two distinct + repeated operand (t2 form: perm(t2, t2, sel)), banks 1,1,3
            asm volatile(R16("v_perm_b32 v56, v41, v41, v43\n v_perm_b32 v57, v41, v41, v43\n"
                             "v_perm_b32 v58, v41, v41, v43\n v_perm_b32 v59, v41, v41, v43\n") ::: CLOB);
        if (MODE == 8)  // v_perm with an SGPR hi table and VGPR lo/sel in banks 2,3
            asm volatile(R16("v_perm_b32 v56, s4, v42, v43\n v_perm_b32 v57, s4, v42, v43\n"
                             "v_perm_b32 v58, s4, v42, v43\n v_perm_b32 v59, s4, v42, v43\n") ::: CLOB, "s4");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
void run(const char *name, int wps) {
    const int threads = 256 * wps, blocks = 256, nw = blocks * threads / 64;
    unsigned long long *cyc;
    (void)hipMalloc(&cyc, nw * 8);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, cyc);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, cyc);
    (void)hipDeviceSynchronize();
    unsigned long long *h = new unsigned long long[nw], mx = 0;
    (void)hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
    for (int i = 0; i < nw; ++i) mx = h[i] > mx ? h[i] : mx;
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_inst_per_simd\": %.3f}\n", name, wps,
           double(mx) / (double(REPS) * 64 * wps));
    delete[] h;
    (void)hipFree(cyc);
}

int main() {
    for (int w : {1, 2, 4}) {
        run<0>("perm v,v,v banks 1,2,3", w);
        run<1>("perm v,v,v banks 0,0,0", w);
        run<7>("perm v,v,v banks 1,1,3 (t2 form)", w);
        run<8>("perm s,v,v banks -,2,3", w);
        run<2>("bitop3 banks 1,2,3", w);
        run<3>("bitop3 banks 0,0,0", w);
        run<4>("xor VOP2 banks 1,2", w);
        run<5>("xor VOP2 banks 0,0", w);
        run<6>("xor VOP3(e64) banks 1,2", w);
    }
    return 0;
}
