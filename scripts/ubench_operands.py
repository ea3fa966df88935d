#!/usr/bin/env python3
"""Microbenchmark generator: is the issue rate of independent v_bitop3_b32 XOR3s on gfx950 limited by how many
DISTINCT VGPRs the instruction stream reads (register-file read bandwidth / operand reuse), rather than by VGPR
banks?  The product kernel's inline products (16 XOR3s per (row, source), accumulators over 128 registers,
combinations over 64) issue at ~3.4 cycles each with random data (profiles/r02_ubench_tables.jsonl, inline_abs),
the live ceiling kernel (8 accumulators, 8 operands) at ~2.33.  Each case is 256 straight-line XOR3s per loop trip
with random register contents, at 2 waves per SIMD, cycles from s_memtime.

    python3 scripts/ubench_operands.py --gen   # writes build/ubench_operands.hip
    hipcc --offload-arch=gfx950 -O3 build/ubench_operands.hip -o build/ubench_operands && build/ubench_operands
"""
import argparse
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 256


def seq(case, rnd):
    """(dst/src0, src1, src2) register triples; accumulators live in v0-v127, operands in v128-v191."""
    out = []
    for k in range(N):
        if case == "ceil":  # the ceiling kernel's pattern: 8 accumulators, 8 operands
            a = k % 8
            x, y = 128 + (k % 4), 132 + ((k + 1) % 4)
        elif case == "acc128_op8":
            a = k % 128
            x, y = 128 + (k % 4), 132 + ((k + 1) % 4)
        elif case == "acc8_op64":
            a = k % 8
            x, y = 128 + rnd.randrange(32), 160 + rnd.randrange(32)
        elif case == "acc128_op64":  # the product's pattern
            a = k % 128
            x, y = 128 + rnd.randrange(32), 160 + rnd.randrange(32)
        elif case == "acc128_op64_bank":  # same, three banks per instruction
            a = 4 * rnd.randrange(32) + 2 + rnd.randrange(2)
            x, y = 128 + 4 * rnd.randrange(8), 129 + 4 * rnd.randrange(8)
        elif case == "acc128_op64_pairx":  # consecutive pairs of instructions share src1
            a = k % 128
            x, y = 128 + rnd.randrange(32) if k % 2 == 0 else out[-1][1], 160 + rnd.randrange(32)
        elif case == "acc128_op64_pairxy":  # consecutive pairs share both sources
            a = k % 128
            if k % 2:
                x, y = out[-1][1], out[-1][2]
            else:
                x, y = 128 + rnd.randrange(32), 160 + rnd.randrange(32)
        elif case == "acc16_op64":
            a = k % 16
            x, y = 128 + rnd.randrange(32), 160 + rnd.randrange(32)
        elif case == "acc128_op16":
            a = k % 128
            x, y = 128 + rnd.randrange(8), 160 + rnd.randrange(8)
        elif case == "xor2_acc128_op64":  # VOP2 XORs (two sources)
            a = k % 128
            x, y = 128 + rnd.randrange(64), None
        else:
            raise ValueError(case)
        # every register the case names must be one the kernel clobbers (v0-v191): a write outside them
        # corrupts the compiler's own registers
        assert 0 <= a < 128 and 128 <= x < 192 and (y is None or 128 <= y < 192), (case, a, x, y)
        out.append((a, x, y))
    return out


CASES = ["ceil", "acc128_op8", "acc8_op64", "acc16_op64", "acc128_op16", "acc128_op64", "acc128_op64_bank",
         "acc128_op64_pairx", "acc128_op64_pairxy", "xor2_acc128_op64"]


def gen(path):
    rnd = random.Random(7)
    clob = ", ".join(f'"v{r}"' for r in range(192))
    # every register a distinct pseudo-random word (odd multiplier per register, then a second word mixed in)
    movs = "\n".join(f'        "v_mov_b32 v{r}, {hex((0x9E3779B1 * (r + 1)) & 0xFFFFFFFF | 1)}\\n v_mul_lo_u32 v{r}, v{r}, v{r % 4}\\n'
                      f' v_xor_b32 v{r}, v{r}, v{(r + 1) % 4}\\n"' for r in range(4, 192))
    src = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdint>', '#include <vector>']
    for ci, case in enumerate(CASES):
        ins = []
        for a, x, y in seq(case, rnd):
            ins.append(f"v_xor_b32 v{a}, v{a}, v{x}" if y is None else f"v_bitop3_b32 v{a}, v{a}, v{x}, v{y} bitop3:0x96")
        body = "\\n".join(ins)
        src.append(f'''
__global__ __launch_bounds__(256) void k{ci}(unsigned long long *out, const uint32_t *seed, int reps) {{
    extern __shared__ uint32_t lds[];
    const uint32_t *sd = seed + ((blockIdx.x * 256 + threadIdx.x) % 4096) * 4;
    asm volatile("global_load_dwordx4 v[0:3], %0, off\\n s_waitcnt vmcnt(0)" ::"v"(sd) : {clob});
    asm volatile(""
{movs}
        ::: {clob});
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) asm volatile("{body}" ::: {clob});
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc;
    asm volatile("v_xor_b32 %0, v0, v77\\n v_xor_b32 %0, %0, v127" : "=v"(acc) :: {clob});
    if (threadIdx.x % 64 == 0) out[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
    if (acc == 0x12345678u && lds[threadIdx.x] == 1u) out[0] = acc;
}}''')
    runs = "\n".join(f'    run("{c}", k{i}, d, seed, cus);' for i, c in enumerate(CASES))
    src.append(f'''
template <typename K>
void run(const char *name, K kern, unsigned long long *d, const uint32_t *seed, int cus) {{
    const int W = 2, blocks = cus * W, reps = 512;
    hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 79 * 1024, 0, d, seed, reps);
    if (hipDeviceSynchronize() != hipSuccess) {{ printf("launch failed\\n"); return; }}
    std::vector<unsigned long long> h(blocks * 4);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double mx = 0;
    for (auto v : h) mx = double(v) > mx ? double(v) : mx;
    printf("{{\\"case\\": \\"%s\\", \\"waves_per_simd\\": %d, \\"cycles_per_inst_per_simd\\": %.3f}}\\n", name, W,
           mx / (double(reps) * {N} * W));
}}

int main() {{
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    unsigned long long *d;
    uint32_t *seed;
    (void)hipMalloc(&d, size_t(cus) * 64 * 8);
    (void)hipMalloc(&seed, 4096 * 16);
    std::vector<uint32_t> hs(4096 * 4);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto &v : hs) {{
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        v = uint32_t(z ^ (z >> 31));
    }}
    (void)hipMemcpy(seed, hs.data(), hs.size() * 4, hipMemcpyHostToDevice);
{runs}
    return 0;
}}
''')
    with open(path, "w") as f:
        f.write("\n".join(src))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--gen", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "build", "ubench_operands.hip"))
    a = ap.parse_args()
    gen(a.out)
    print(a.out)
