// ubench_gpridx.hip — issue cost on gfx950 of VGPR-indexed XORs (s_set_gpr_idx_idx + v_xor_b32 with a relative
// SRC0), the inner operation of a bit-sliced GF(2^8) multiply-add whose 4-bit combination index is wave-uniform.
// Also checks the semantics (first launch of each mode verifies the XOR result against the host).
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_gpridx.hip -o build/ubench_gpridx && build/ubench_gpridx
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int REPS = 129;  // odd: the accumulators end as one pass's XOR

#define R2(x) x x
#define R4(x) R2(x) R2(x)
#define R8(x) R4(x) R4(x)

// G = v40..v55 (16 combination registers), acc = v56..v63, indices in s[20:27]
#define CLOB                                                                                                      \
    "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", \
        "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "s20", "s21", "s22", "s23", "s24", "s25", "s26",   \
        "s27", "s28", "m0", "scc"

#define IDX8(op)                                                                                           \
    "s_set_gpr_idx_idx s20\n " op " v56, v40, v56\n s_set_gpr_idx_idx s21\n " op " v57, v40, v57\n"         \
    "s_set_gpr_idx_idx s22\n " op " v58, v40, v58\n s_set_gpr_idx_idx s23\n " op " v59, v40, v59\n"         \
    "s_set_gpr_idx_idx s24\n " op " v60, v40, v60\n s_set_gpr_idx_idx s25\n " op " v61, v40, v61\n"         \
    "s_set_gpr_idx_idx s26\n " op " v62, v40, v62\n s_set_gpr_idx_idx s27\n " op " v63, v40, v63\n"

#define IDX8_SHR                                                                                          \
    "s_set_gpr_idx_idx s20\n s_lshr_b32 s28, s28, 1\n v_xor_b32 v56, v40, v56\n"                         \
    "s_set_gpr_idx_idx s21\n s_lshr_b32 s28, s28, 1\n v_xor_b32 v57, v40, v57\n"                         \
    "s_set_gpr_idx_idx s22\n s_lshr_b32 s28, s28, 1\n v_xor_b32 v58, v40, v58\n"                         \
    "s_set_gpr_idx_idx s23\n s_lshr_b32 s28, s28, 1\n v_xor_b32 v59, v40, v59\n"                         \
    "s_set_gpr_idx_idx s24\n s_lshr_b32 s28, s28, 1\n v_xor_b32 v60, v40, v60\n"                         \
    "s_set_gpr_idx_idx s25\n s_lshr_b32 s28, s28, 1\n v_xor_b32 v61, v40, v61\n"                         \
    "s_set_gpr_idx_idx s26\n s_lshr_b32 s28, s28, 1\n v_xor_b32 v62, v40, v62\n"                         \
    "s_set_gpr_idx_idx s27\n s_lshr_b32 s28, s28, 1\n v_xor_b32 v63, v40, v63\n"

#define PLAIN8                                                                                            \
    "v_xor_b32 v56, v41, v56\n v_xor_b32 v57, v42, v57\n v_xor_b32 v58, v43, v58\n v_xor_b32 v59, v44, v59\n" \
    "v_xor_b32 v60, v45, v60\n v_xor_b32 v61, v46, v61\n v_xor_b32 v62, v47, v62\n v_xor_b32 v63, v48, v63\n"

template <int MODE>
__global__ void k(unsigned long long *cyc, uint32_t *out) {
    const uint32_t lane = threadIdx.x;
    asm volatile(
        "v_mov_b32 v40, 0\n v_add_u32 v41, 0x100, %0\n v_add_u32 v42, 0x200, %0\n v_add_u32 v43, 0x300, %0\n"
        "v_add_u32 v44, 0x400, %0\n v_add_u32 v45, 0x500, %0\n v_add_u32 v46, 0x600, %0\n v_add_u32 v47, 0x700, %0\n"
        "v_add_u32 v48, 0x800, %0\n v_add_u32 v49, 0x900, %0\n v_add_u32 v50, 0xa00, %0\n v_add_u32 v51, 0xb00, %0\n"
        "v_add_u32 v52, 0xc00, %0\n v_add_u32 v53, 0xd00, %0\n v_add_u32 v54, 0xe00, %0\n v_add_u32 v55, 0xf00, %0\n"
        "v_mov_b32 v56, 0\n v_mov_b32 v57, 0\n v_mov_b32 v58, 0\n v_mov_b32 v59, 0\n"
        "v_mov_b32 v60, 0\n v_mov_b32 v61, 0\n v_mov_b32 v62, 0\n v_mov_b32 v63, 0\n"
        "s_mov_b32 s20, 3\n s_mov_b32 s21, 15\n s_mov_b32 s22, 0\n s_mov_b32 s23, 7\n"
        "s_mov_b32 s24, 9\n s_mov_b32 s25, 1\n s_mov_b32 s26, 12\n s_mov_b32 s27, 5\n s_mov_b32 s28, -1" ::"v"(lane)
        : CLOB);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (MODE == 0 || MODE == 1 || MODE == 3) asm volatile("s_set_gpr_idx_on s20, gpr_idx(SRC0)" ::: CLOB);
    for (int r = 0; r < REPS; ++r) {
        if (MODE == 0) asm volatile(R8(IDX8("v_xor_b32")) ::: CLOB);
        if (MODE == 1) asm volatile(R8(IDX8_SHR) ::: CLOB);
        if (MODE == 2) asm volatile(R8(PLAIN8) ::: CLOB);
        if (MODE == 3) asm volatile(R8(IDX8("v_xor_b32_e64")) ::: CLOB);
    }
    if (MODE == 0 || MODE == 1 || MODE == 3) asm volatile("s_set_gpr_idx_off" ::: CLOB);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t a0, a1, a7;
    asm volatile("v_mov_b32 %0, v56\n v_mov_b32 %1, v57\n v_mov_b32 %2, v63" : "=v"(a0), "=v"(a1), "=v"(a7)::CLOB);
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        out[threadIdx.x * 3 + 0] = a0;
        out[threadIdx.x * 3 + 1] = a1;
        out[threadIdx.x * 3 + 2] = a7;
    }
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE>
void run(const char *name, int wps, bool idx) {
    const int threads = 256 * wps, blocks = 256, nw = blocks * threads / 64;
    unsigned long long *cyc;
    uint32_t *out;
    (void)hipMalloc(&cyc, nw * 8);
    (void)hipMalloc(&out, 64 * 3 * 4);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, cyc, out);
    hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(threads), 0, 0, cyc, out);
    (void)hipDeviceSynchronize();
    unsigned long long *h = new unsigned long long[nw], mx = 0;
    uint32_t ho[192];
    (void)hipMemcpy(h, cyc, nw * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ho, out, sizeof ho, hipMemcpyDeviceToHost);
    for (int i = 0; i < nw; ++i) mx = h[i] > mx ? h[i] : mx;
    // expected (8 XORs per pass into each acc, odd pass count): acc0 = G[3] x8 -> 0 (even count per pass)...
    // each acc receives 8 XORs of the same register per pass: result 0 for idx modes; plain: 0 as well.
    // So check with a single distinguishing pass instead: G values are (lane + 0x100*m); 8 XORs of one value = 0.
    bool ok = true;
    for (int l = 0; l < 64; ++l) ok &= ho[l * 3] == 0 && ho[l * 3 + 1] == 0 && ho[l * 3 + 2] == 0;
    printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_valu_per_simd\": %.3f, \"zero_check\": %s}\n",
           name, wps, double(mx) / (double(REPS) * 64 * wps), ok ? "true" : "false");
    (void)idx;
    delete[] h;
    (void)hipFree(cyc);
    (void)hipFree(out);
}

// semantics check: one indexed XOR per accumulator
__global__ void sem(uint32_t *out) {
    const uint32_t lane = threadIdx.x;
    uint32_t a0, a1, a7;
    asm volatile(
        "v_mov_b32 v40, 0\n v_add_u32 v41, 0x100, %3\n v_add_u32 v42, 0x200, %3\n v_add_u32 v43, 0x300, %3\n"
        "v_add_u32 v44, 0x400, %3\n v_add_u32 v45, 0x500, %3\n v_add_u32 v46, 0x600, %3\n v_add_u32 v47, 0x700, %3\n"
        "v_add_u32 v48, 0x800, %3\n v_add_u32 v49, 0x900, %3\n v_add_u32 v50, 0xa00, %3\n v_add_u32 v51, 0xb00, %3\n"
        "v_add_u32 v52, 0xc00, %3\n v_add_u32 v53, 0xd00, %3\n v_add_u32 v54, 0xe00, %3\n v_add_u32 v55, 0xf00, %3\n"
        "v_mov_b32 v56, 0x10000\n v_mov_b32 v57, 0x20000\n v_mov_b32 v63, 0x30000\n"
        "s_mov_b32 s20, 3\n s_mov_b32 s21, 15\n s_mov_b32 s27, 5\n"
        "s_set_gpr_idx_on s20, gpr_idx(SRC0)\n v_xor_b32 v56, v40, v56\n"
        "s_set_gpr_idx_idx s21\n v_xor_b32 v57, v40, v57\n"
        "s_set_gpr_idx_idx s27\n v_xor_b32 v63, v40, v63\n"
        "s_set_gpr_idx_off\n"
        "v_mov_b32 %0, v56\n v_mov_b32 %1, v57\n v_mov_b32 %2, v63"
        : "=v"(a0), "=v"(a1), "=v"(a7)
        : "v"(lane)
        : CLOB);
    out[lane * 3 + 0] = a0;
    out[lane * 3 + 1] = a1;
    out[lane * 3 + 2] = a7;
}

int main() {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    uint32_t *out, ho[192];
    (void)hipMalloc(&out, sizeof ho);
    hipLaunchKernelGGL(sem, dim3(1), dim3(64), 0, 0, out);
    (void)hipMemcpy(ho, out, sizeof ho, hipMemcpyDeviceToHost);
    bool ok = true;
    for (uint32_t l = 0; l < 64; ++l)
        ok &= ho[l * 3] == (0x10000u ^ (0x300u + l)) && ho[l * 3 + 1] == (0x20000u ^ (0xf00u + l)) &&
              ho[l * 3 + 2] == (0x30000u ^ (0x500u + l));
    printf("{\"case\": \"semantics s_set_gpr_idx SRC0-relative xor\", \"ok\": %s, \"lane1\": [%u, %u, %u]}\n",
           ok ? "true" : "false", ho[3], ho[4], ho[5]);
    for (int w : {1, 2, 4}) {
        run<0>("idx_idx + v_xor (VOP2)", w, true);
        run<3>("idx_idx + v_xor_e64 (VOP3)", w, true);
        run<1>("idx_idx + s_lshr + v_xor", w, true);
        run<2>("plain v_xor (VOP2)", w, false);
    }
    return 0;
}
