#!/usr/bin/env python3
"""Generate bitslice_asm.inc: the gfx950 inner program of the bit-sliced GF(2^8) matmul (kernels.hip).

Why generated: the kernel keeps 128 accumulators, 64 combination registers and 16 staging registers in
FIXED physical VGPRs so that (a) the per-(row, source) work is 16 wave-uniform register-indexed XORs
(s_set_gpr_idx_idx + v_xor_b32 with a relative SRC0), which no compiler emits in this form, and (b) the
operand banks are chosen by hand.  Run `python3 gen_bitslice.py` after editing; the output is committed.

Algorithm (one workgroup = 8 output rows x 16 KiB of columns; one lane = 64 bytes as two 32-byte groups):
  * bit-slicing: a group's 8 dwords (32 bytes) are transposed into 8 bit-planes, plane b holding bit b of
    each of the 32 bytes, by three delta-swap stages (register-index bit k <-> bit-position bit k);
  * for source row j, G[h][v] = XOR of planes {4h + b : bit b of v} for v = 0..15 (h = low/high half);
  * GF(2^8) multiply-add by c is linear over GF(2): output plane o = XOR_b bit_o(c * 2^b) . plane b,
    i.e. acc[o] ^= G[0][idx_lo(c, o)] ^ G[1][idx_hi(c, o)] -- 16 indexed XORs per group per (row, source);
    the 16 indices are wave-uniform and come from the prep kernel's stream (s_load_dwordx16, one ahead);
  * after all sources, the accumulators are transposed back (the swaps are involutions) and stored.

Index delivery: GPR-index mode takes its enables from M0[15:12] (S_SET_GPR_IDX_ON stores them there), so a
plain SALU write of M0 both selects and enables.  Indices are packed three per SGPR as bytes 0x10 | idx
(byte 3 = 0x10): `s_lshr_b32 m0, s, 8*b` leaves M0[7:0] = 16 + idx and M0[15:12] = 1 (the next byte's
upper nibble), and the XOR names its base register 16 below the table.  One row's 16 indices take 6
SGPRs, so a 4-row step (24 SGPRs) is loaded a whole step ahead (scripts/ubench_m0.hip checks the
semantics and measures 4.1 cycles per SALU+VALU pair at 2 waves/SIMD, the same as s_set_gpr_idx_idx).
"""
import os

NT = 8  # output rows per workgroup
STEP = 4  # rows per index step (one SMEM batch)
ROW_DW = 6  # index dwords per (row, source)

# ---- register map (see kernels.hip gf_matmul_bs_kernel) -------------------------------------------
def ACC(i, g, p):  # output row i, group g, plane/dword p
    return i * 16 + g * 8 + p

def G(g, h, v):  # combination v of half h of group g
    return 128 + g * 32 + h * 16 + v

def RAW(g, d, buf=0):  # staging registers: two buffers, source rows j+1 and j+2 in flight
    return (192 if buf == 0 else 220) + g * 8 + d

TMP0 = 208  # 8 temporaries v208..v215
V_MASK = (216, 217, 218)  # 0xAAAAAAAA, 0xCCCCCCCC, 0xF0F0F0F0

# SGPRs: s32-s34 are the ABI stack/frame/base pointers (reserved even in a stackless kernel), so the block
# starts at s36; the compiler keeps its own values (kernel arguments, the asm operands) in s0-s31.
S_BUF = (36, 60)  # two 24-dword index buffers (4 rows x 6 dwords), 4-aligned for s_load_dwordx16/x8
S_SRC, S_IDX, S_DST = 84, 86, 88
S_INROW, S_OUTROW, S_CNT, S_ROWS, S_T0 = 90, 91, 92, 93, 94
FIRST_SGPR = S_BUF[0]
LAST_VGPR = RAW(1, 7, 1)
LAST_SGPR = S_T0
STREAM_ROW_BYTES = ROW_DW * 4
STREAM_J_BYTES = NT * STREAM_ROW_BYTES


def v(n):
    return f"v{n}"


def bank(r):
    return r % 4


def transpose(regs_in, regs_out, lines):
    """Three delta-swap stages on 8 registers (in place except the last stage, which writes regs_out)."""
    cur = list(regs_in)
    for k in range(3):
        s = 1 << k
        pairs = [(r, r + s) for r in range(8) if not (r >> k) & 1]
        # shifts for all 4 pairs first (8 temporaries), then the bit-field inserts
        for n, (a, b) in enumerate(pairs):
            lines.append(f"v_lshlrev_b32 v{TMP0 + 2 * n}, {s}, {v(cur[b])}")
            lines.append(f"v_lshrrev_b32 v{TMP0 + 2 * n + 1}, {s}, {v(cur[a])}")
        dst = cur if k < 2 else regs_out
        for n, (a, b) in enumerate(pairs):
            # a' = (a & ~m) | ((b << s) & m);  b' = (b & m) | ((a >> s) & ~m)
            lines.append(f"v_bfi_b32 {v(dst[a])}, v{V_MASK[k]}, v{TMP0 + 2 * n}, {v(cur[a])}")
            lines.append(f"v_bfi_b32 {v(dst[b])}, v{V_MASK[k]}, {v(cur[b])}, v{TMP0 + 2 * n + 1}")
        if k == 2:
            cur = list(regs_out)


def combos(g, h, lines):
    """G[v] for the 11 composite v from the 4 planes (entries 1, 2, 4, 8): one VOP2 XOR each."""
    b = lambda x: v(G(g, h, x))
    lines += [f"v_xor_b32 {b(x)}, {b(y)}, {b(z)}" for x, y, z in
              [(3, 1, 2), (5, 1, 4), (6, 2, 4), (7, 3, 4), (9, 1, 8), (10, 2, 8), (11, 3, 8), (12, 4, 8), (13, 5, 8),
               (14, 6, 8), (15, 7, 8)]]


DIAG = set()  # diagnostic builds only (scripts/bs_diag.sh): "novm" drops source loads, "nosmem" index reloads


def loads(lines, buf=0):
    if "novm" in DIAG:
        return
    for g in range(2):
        for half in range(2):
            q = 2 * g + half
            r0 = RAW(g, 4 * half, buf)
            off = f" offset:{q * 1024}" if q else ""
            lines.append(f"global_load_dwordx4 v[{r0}:{r0 + 3}], %[off], s[{S_SRC}:{S_SRC + 1}]{off}")


def idx_load(buf, byte_off, lines):
    """24 dwords = one 4-row step of the index stream."""
    if "nosmem" in DIAG and byte_off:
        return
    lines.append(f"s_load_dwordx16 s[{buf}:{buf + 15}], s[{S_IDX}:{S_IDX + 1}], {hex(byte_off)}")
    lines.append(f"s_load_dwordx8 s[{buf + 16}:{buf + 23}], s[{S_IDX}:{S_IDX + 1}], {hex(byte_off + 64)}")


def row_update(i, buf, lines):
    """acc[i] ^= M_c . planes for both groups: 16 M0 writes, 32 relative XORs."""
    # (h, o) order: the two updates of one accumulator are 24 instructions apart, not 3 (dependent VALU
    # issue); "oh" keeps the old (o, h) order for A/B
    order = [(o, h) for o in range(8) for h in range(2)] if "oh" in DIAG else [(o, h) for h in range(2) for o in range(8)]
    for o, h in order:
            n = 2 * o + h
            reg = buf + ROW_DW * (i % STEP) + n // 3
            sh = 8 * (n % 3)
            if "plainxor" not in DIAG and "nom0" not in DIAG:
                lines.append(f"s_mov_b32 m0, s{reg}" if sh == 0 else f"s_lshr_b32 m0, s{reg}, {sh}")
            for g in range(2):
                a = ACC(i, g, o)
                if "plainxor" in DIAG:  # timing only: a fixed combination, no GPR-index mode
                    lines.append(f"v_xor_b32 v{a}, v{G(g, h, 1 + (n % 15))}, v{a}")
                else:
                    lines.append(f"v_xor_b32 v{a}, v{G(g, h, 0) - 16}, v{a}")


def body(L, buf):
    """One source row: its planes come from staging buffer `buf` (loaded two rows earlier), which is then
    refilled with row j+2 (the last row again past the end: no branch, always in bounds)."""
    if "novm" not in DIAG:
        L.append("s_waitcnt vmcnt(4)")  # the other buffer's 4 loads (issued later) may stay in flight
    for g in range(2):
        outs = [G(g, b // 4, 1 << (b % 4)) for b in range(8)]
        if "notrans" in DIAG:  # timing only: planes = raw dwords
            L += [f"v_mov_b32 v{o}, v{RAW(g, d, buf)}" for d, o in enumerate(outs)]
        else:
            transpose([RAW(g, d, buf) for d in range(8)], outs, L)
    L += [
        f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1",
        f"s_cmp_gt_u32 s{S_CNT}, 1",  # row j+2 exists
        f"s_cselect_b32 s{S_T0}, s{S_INROW}, 0",
        f"s_add_u32 s{S_SRC}, s{S_SRC}, s{S_T0}",
        f"s_addc_u32 s{S_SRC + 1}, s{S_SRC + 1}, 0",
    ]
    loads(L, buf)
    for g in range(2):
        for h in range(2):
            if "nocombo" not in DIAG:
                combos(g, h, L)
    if "plainxor" not in DIAG:
        L.append("s_set_gpr_idx_on 0, gpr_idx(SRC0)")
    nsteps = NT // STEP
    for st in range(nsteps):
        cur, nxt = S_BUF[st & 1], S_BUF[(st + 1) & 1]
        if "nosmem" not in DIAG or st == 0:
            L.append("s_waitcnt lgkmcnt(0)")
        # the next step: this source's next rows, or the next source's first rows (stream is [j][row])
        idx_load(nxt, (st + 1) * STEP * STREAM_ROW_BYTES, L)
        for i in range(st * STEP, (st + 1) * STEP):
            row_update(i, cur, L)
    L += [
        "s_set_gpr_idx_off" if "plainxor" not in DIAG else "s_nop 0",
        f"s_add_u32 s{S_IDX}, s{S_IDX}, {STREAM_J_BYTES}",
        f"s_addc_u32 s{S_IDX + 1}, s{S_IDX + 1}, 0",
    ]


def program():
    L = []
    L += [
        f"s_mov_b64 s[{S_SRC}:{S_SRC + 1}], %[src]",
        f"s_mov_b64 s[{S_IDX}:{S_IDX + 1}], %[idx]",
        f"s_mov_b64 s[{S_DST}:{S_DST + 1}], %[dst]",
        f"s_mov_b32 s{S_INROW}, %[in_row]",
        f"s_mov_b32 s{S_OUTROW}, %[out_row]",
        f"s_mov_b32 s{S_CNT}, %[n_in]",
        f"s_mov_b32 s{S_ROWS}, %[rows]",
        f"v_mov_b32 v{V_MASK[0]}, 0xaaaaaaaa",
        f"v_mov_b32 v{V_MASK[1]}, 0xcccccccc",
        f"v_mov_b32 v{V_MASK[2]}, 0xf0f0f0f0",
    ]
    # prologue: source rows 0 and 1 in flight (row 0 again when n_in == 1)
    loads(L, 0)
    L += [
        f"s_cmp_gt_u32 s{S_CNT}, 1",
        f"s_cselect_b32 s{S_T0}, s{S_INROW}, 0",
        f"s_add_u32 s{S_SRC}, s{S_SRC}, s{S_T0}",
        f"s_addc_u32 s{S_SRC + 1}, s{S_SRC + 1}, 0",
    ]
    loads(L, 1)
    idx_load(S_BUF[0], 0, L)
    for r in range(128):
        L.append(f"v_mov_b32 v{r}, 0")
    for g in range(2):
        for h in range(2):
            L.append(f"v_mov_b32 {v(G(g, h, 0))}, 0")
    # loop over source rows j, two per trip (staging buffers alternate); S_CNT = rows not yet consumed
    L.append("1:")
    body(L, 0)
    L += [f"s_cmp_eq_u32 s{S_CNT}, 0", "s_cbranch_scc1 3f"]
    body(L, 1)
    L += [f"s_cmp_eq_u32 s{S_CNT}, 0", "s_cbranch_scc0 1b", "3:", "s_waitcnt vmcnt(0) lgkmcnt(0)"]
    # ---- epilogue: transpose back and store the rows that exist
    for i in range(NT):
        L += [f"s_cmp_gt_u32 s{S_ROWS}, {i}", "s_cbranch_scc0 2f"]
        for g in range(2):
            regs = [ACC(i, g, p) for p in range(8)]
            transpose(regs, regs, L)
        for g in range(2):
            for half in range(2):
                q = 2 * g + half
                r0 = ACC(i, g, 4 * half)
                off = f" offset:{q * 1024}" if q else ""
                L.append(f"global_store_dwordx4 %[off], v[{r0}:{r0 + 3}], s[{S_DST}:{S_DST + 1}]{off}")
        L += [f"s_add_u32 s{S_DST}, s{S_DST}, s{S_OUTROW}", f"s_addc_u32 s{S_DST + 1}, s{S_DST + 1}, 0"]
    L.append("2:")
    return L


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "bitslice_asm.inc"))
    ap.add_argument("--diag", default="", help="comma list: novm, nosmem (timing diagnostics, wrong results), nobanks (A/B)")
    args = ap.parse_args()
    DIAG.update(x for x in args.diag.split(",") if x)
    lines = program()
    clob_v = ", ".join(f'"v{r}"' for r in range(LAST_VGPR + 1))
    clob_s = ", ".join(f'"s{r}"' for r in range(FIRST_SGPR, LAST_SGPR + 1))
    body = "\\n\\t".join(lines)
    with open(args.out, "w") as f:
        f.write("// GENERATED by gen_bitslice.py -- do not edit.  Inner program of gf_matmul_bs_kernel (kernels.hip).\n")
        f.write(f"// {sum(1 for l in lines if l.startswith('v_'))} VALU, "
                f"{sum(1 for l in lines if l.startswith('s_'))} SALU/SMEM, "
                f"{sum(1 for l in lines if l.startswith('global_'))} VMEM instructions in the text.\n")
        f.write(f"#define RLNC_BS_NT {NT}\n")
        f.write(f"#define RLNC_BS_ROW_DWORDS {ROW_DW}\n")
        f.write(f"#define RLNC_BS_STEP_BYTES {STEP * STREAM_ROW_BYTES}\n")
        f.write(f'#define RLNC_BS_ASM "{body}"\n')
        f.write(f"#define RLNC_BS_CLOBBER_V {clob_v}\n")
        f.write(f'#define RLNC_BS_CLOBBER_S {clob_s}, "m0", "scc", "memory"\n')


if __name__ == "__main__":
    main()
