#!/usr/bin/env python3
"""Microbenchmark generator: the cost of one call into a coefficient-specialised code block of 16 v_bitop3 XOR3s
(the bit-sliced jump kernel's unit, gen_bsjump.py), for three block organisations, at 2 and 4 waves per SIMD:

  rel1  one table of 256 blocks whose accumulator operands (DST, SRC2) are GPR-index relative (M0 = 0xC000 | 16 i
        selects row slot i) -- the product kernel's form;
  abs8  eight tables of 256 blocks, one per row slot, every operand absolute (no GPR-index mode; 270 KB of code:
        instruction-cache pressure);
  abs1  one table of absolute blocks, every call into slot 0 (the absolute form without the code-size cost).

Each iteration loads 8 random block offsets (s_load_dwordx8) and makes 8 calls (row slots 0..7), like one source
row of the product kernel; 128 iterations per wave.  Accumulators v0-v127, combinations v128-v191 (random).

    python3 scripts/ubench_tables.py --gen          # writes build/ubench_tables.hip (CPU)
    hipcc --offload-arch=gfx950 -O3 build/ubench_tables.hip -o build/ubench_tables && build/ubench_tables
"""
import argparse
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BLOCK = 16 * 8 + 4


def xtime(a):
    a <<= 1
    return (a ^ 0x11B) & 0xFF if a & 0x100 else a


def block_indices(c):
    m = [c]
    for _ in range(7):
        m.append(xtime(m[-1]))
    lo = [sum(((m[b] >> o) & 1) << b for b in range(4)) for o in range(8)]
    hi = [sum(((m[4 + b] >> o) & 1) << b for b in range(4)) for o in range(8)]
    return lo, hi


# Register maps.  "std": the product kernel's (accumulators v0-v127 with row slot i at 16 i, combinations
# v128-v191); "bank": every XOR3's three sources in three different VGPR banks (bank = vN mod 4) -- accumulators
# in banks 2 and 3 (row slot i at 32 i, M0 steps by 32), the low-half combinations in bank 0, the high-half ones
# in bank 1 (v0-v125).
MAP = "std"


def G(g, h, v):
    if MAP == "bank":
        return 4 * (16 * g + v) + h
    return 128 + g * 32 + h * 16 + v


def ACC(i, g, p):
    if MAP == "bank":
        return 32 * i + 4 * (4 * g + p // 2) + 2 + p % 2
    return 16 * i + 8 * g + p


def SLOT_STEP():
    return 32 if MAP == "bank" else 16


def REGS():
    return sorted({ACC(i, g, p) for i in range(8) for g in range(2) for p in range(8)} |
                  {G(g, h, v) for g in range(2) for h in range(2) for v in range(16)})


def block_body(c, slot, relative, reps=1, pack=False):
    lo, hi = block_indices(c)
    L = []
    for _ in range(reps):
        v3, v2 = [], []
        for g in range(2):
            for o in range(8):
                a = ACC(0 if relative else slot, g, o)
                if pack:  # the product kernel's packed form: accumulator as SRC0, VOP2 XOR for a one-half product
                    if lo[o] and hi[o]:
                        v3.append(f"v_bitop3_b32 v{a}, v{a}, v{G(g, 0, lo[o])}, v{G(g, 1, hi[o])} bitop3:0x96")
                    elif lo[o] or hi[o]:
                        v2.append(f"v_xor_b32 v{a}, v{a}, v{G(g, 0, lo[o]) if lo[o] else G(g, 1, hi[o])}")
                    continue
                x = f"v{G(g, 0, lo[o])}" if lo[o] else "0"
                y = f"v{G(g, 1, hi[o])}" if hi[o] else "0"
                L.append(f"v_bitop3_b32 v{a}, {x}, {y}, v{a} bitop3:0x96")
        L += v3 + v2
    return L


def body_bytes(c, reps, pack):
    if not pack:
        return 16 * reps * 8
    return sum(8 if x.startswith("v_bitop3") else 4 for x in block_body(c, 0, True, reps, True))


def blocks(slot, relative, reps=1, stride=None, empty=False, pack=False):
    """256 blocks; each 16 * reps XOR3s (none if empty) + s_setpc, padded with s_nop to `stride` bytes."""
    L = []
    stride = stride or (0 if empty else 16 * reps * 8) + 4
    for c in range(256):
        size = (0 if empty else body_bytes(c, reps, pack)) + 4
        if not empty:
            L += block_body(c, slot, relative, reps, pack)
        L.append("s_setpc_b64 s[40:41]")
        L += ["s_nop 0"] * ((stride - size) // 4)
    return L


MODES = {  # name: (tables, relative, xor3 reps per block, stride, empty, inline, map, pack)
    "rel1": (1, True, 1, None, False, False, "std", False),
    "abs1": (1, False, 1, None, False, False, "std", False),
    "rel1_a256": (1, True, 1, 256, False, False, "std", False),
    "empty": (1, False, 1, None, True, False, "std", False),
    "rel1_x2": (1, True, 2, None, False, False, "std", False),
    "inline_rel": (0, True, 1, None, False, True, "std", False),
    "inline_abs": (0, False, 1, None, False, True, "std", False),
    # round 2: the packed blocks of the product kernel (stride 136), standard and bank-separated register maps
    "relp": (1, True, 1, 136, False, False, "std", True),
    "relp_bank": (1, True, 1, 136, False, False, "bank", True),
    "inline_relp": (0, True, 1, None, False, True, "std", True),
    "inline_relp_bank": (0, True, 1, None, False, True, "bank", True),
    "inline_abs_bank": (0, False, 1, None, False, True, "bank", False),
}


def block_stride(mode):
    tables, rel, reps, stride, empty, inl, mp, pack = MODES[mode]
    size = (0 if empty else 16 * reps * 8) + 4
    return stride or size


def program(mode):
    global MAP
    tables, rel, reps, stride, empty, inl, MAP, pack = MODES[mode]
    bs = block_stride(mode)
    # the tables sit first and the entry jumps over them with s_setpc (big tables are beyond s_branch's range)
    L = ["s_getpc_b64 s[36:37]", "2:", "s_add_u32 s36, s36, (9f - 2b)", "s_addc_u32 s37, s37, 0",
         "s_mov_b64 s[52:53], %[offs]", "s_mov_b32 s43, %[reps]",
         "s_getpc_b64 s[54:55]", "3:", "s_add_u32 s54, s54, (7f - 3b)", "s_addc_u32 s55, s55, 0",
         "s_setpc_b64 s[54:55]", ".p2align 8", "9:"]
    for t in range(tables):
        L += blocks(t, rel, reps, stride, empty, pack)
    L.append("7:")
    if rel:
        L.append(f"s_set_gpr_idx_on 0, {'gpr_idx(SRC0,DST)' if pack else 'gpr_idx(SRC2,DST)'}")
    L.append("1:")
    L += ["s_load_dwordx8 s[44:51], s[52:53], 0", "s_add_u32 s52, s52, 32", "s_addc_u32 s53, s53, 0",
          "s_waitcnt lgkmcnt(0)"]
    for i in range(8):
        if rel:
            L.append(f"s_mov_b32 m0, {hex((0x9000 if pack else 0xC000) | (SLOT_STEP() * i))}")
        if inl:  # the products of a fixed coefficient per row, no call
            L += block_body(0x53 + i, i, rel, 1, pack)
            continue
        L += [f"s_add_u32 s38, s36, s{44 + i}", "s_addc_u32 s39, s37, 0"]  # offsets hold c * this stride
        L.append("s_swappc_b64 s[40:41], s[38:39]")
    L += ["s_sub_u32 s43, s43, 1", "s_cmp_eq_u32 s43, 0", "s_cbranch_scc0 1b"]
    if rel:
        L.append("s_set_gpr_idx_off")
    return "\\n\\t".join(L)


def gen(path):
    global MAP
    modes = list(MODES)
    src = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <vector>', '#include <cstdint>']
    for mi, mode in enumerate(modes):
        prog = program(mode)
        regs = REGS()
        MAP = "std"
        regs = sorted(set(regs) | set(range(4)))
        clob = ", ".join(f'"v{r}"' for r in regs) + ", " + ", ".join(f'"s{r}"' for r in range(36, 56))
        movs = "\n".join(f'                 "v_mov_b32 v{r}, v{r % 4}\\n"' for r in regs if r >= 4)
        src.append(f'''
__global__ __launch_bounds__(256) void k_{mode}(unsigned long long *out, int reps, const uint32_t *offs,
                                                 const uint32_t *seed) {{
    extern __shared__ uint32_t lds[];
    const uint32_t *sd = seed + ((blockIdx.x * 256 + threadIdx.x) % 4096) * 4;
    // random accumulators and combinations (every register gets one of 4 random words)
    asm volatile("global_load_dwordx4 v[0:3], %0, off\\n s_waitcnt vmcnt(0)" ::"v"(sd) : {clob});
    asm volatile(""
{movs}
                 ::: {clob});
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    offs += {mi} * 64 * 8 * 128;  // this mode's offsets (c * its block stride)
    asm volatile("{prog}" : : [offs] "s"(offs + (blockIdx.x % 64) * 8 * 128), [reps] "s"(reps) : {clob}, "m0", "scc", "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc;
    asm volatile("v_xor_b32 %0, v0, v{regs[17]}\\n v_xor_b32 %0, %0, v{regs[-1]}" : "=v"(acc) :: {clob});
    if (threadIdx.x % 64 == 0) {{
        const int w = blockIdx.x * 4 + threadIdx.x / 64;
        out[4 * w + 0] = t1 - t0;
        out[4 * w + 1] = r0;
        out[4 * w + 2] = r1;
    }}
    if (acc == 0x12345678u && lds[threadIdx.x] == 1u) out[0] = acc;
}}''')
    src.append('''
template <typename K>
void run(const char *name, K kern, int W, unsigned long long *d, const uint32_t *offs, const uint32_t *seed, int cus) {
    const int blocks = cus * W, reps = 128;
    const size_t lds = (160 * 1024) / W - 1024;
    hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, d, reps, offs, seed);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\\n"); return; }
    const int waves = blocks * 4;
    std::vector<unsigned long long> h(4 * waves);
    (void)hipMemcpy(h.data(), d, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    unsigned long long rmin = ~0ull, rmax = 0;
    double cyc = 0, real = 0;
    for (int w = 0; w < waves; ++w) {
        cyc += double(h[4 * w]);
        real += double(h[4 * w + 2] - h[4 * w + 1]);
        rmin = h[4 * w + 1] < rmin ? h[4 * w + 1] : rmin;
        rmax = h[4 * w + 2] > rmax ? h[4 * w + 2] : rmax;
    }
    const double ghz = cyc / real / 10.0;  // s_memtime ticks per 10 ns s_memrealtime tick
    const double calls = 8.0 * reps;       // per wave
    printf("{\\"case\\": \\"%s\\", \\"waves_per_simd\\": %d, \\"clock_GHz\\": %.3f, \\"simd_cycles_per_call\\": %.2f}\\n",
           name, W, ghz, double(rmax - rmin) * 10.0 * ghz / (calls * W));
}

int main() {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    unsigned long long *d;
    uint32_t *offs;
    (void)hipMalloc(&d, size_t(cus) * 4 * 4 * 4 * sizeof(unsigned long long));
    uint32_t *seed;
    const int nmodes = NMODES;
    const int strides[NMODES] = {STRIDES};
    const char *names[NMODES] = {NAMES};
    (void)hipMalloc(&offs, size_t(nmodes) * 64 * 8 * 128 * sizeof(uint32_t));
    (void)hipMalloc(&seed, 4096 * 4 * sizeof(uint32_t));
    std::vector<uint32_t> h(size_t(nmodes) * 64 * 8 * 128), hs(4096 * 4);
    uint32_t x = 12345;
    for (size_t i = 0; i < 64 * 8 * 128; ++i) {
        x = x * 1103515245u + 12345u;
        const uint32_t c = (x >> 16) & 255u;
        for (int mm = 0; mm < nmodes; ++mm) h[size_t(mm) * 64 * 8 * 128 + i] = c * uint32_t(strides[mm]);
    }
    for (auto &v : hs) {
        x = x * 1103515245u + 12345u;
        v = x ^ (x >> 13) * 2654435761u;
    }
    (void)hipMemcpy(offs, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(seed, hs.data(), hs.size() * 4, hipMemcpyHostToDevice);
    for (int W : {2, 4}) {
RUNS
    }
    return 0;
}
''')
    text = "\n".join(src)
    text = text.replace("NMODES", str(len(modes)))
    text = text.replace("{STRIDES}", "{" + ", ".join(str(block_stride(m)) for m in modes) + "}")
    text = text.replace("{NAMES}", "{" + ", ".join(f'"{m}"' for m in modes) + "}")
    text = text.replace("RUNS", "\n".join(f"        run(names[{i}], k_{m}, W, d, offs, seed, cus);" for i, m in enumerate(modes)))
    src = [text]
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write("\n".join(src))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--gen", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "build", "ubench_tables.hip"))
    a = ap.parse_args()
    gen(a.out)
    print(a.out)
