#!/usr/bin/env python3
"""Generate bitslice_jump.inc: the gfx950 inner program of gf_matmul_bsj_kernel (kernels.hip), the bit-sliced
GF(2^8) matmul whose per-(row, source) work is ONE call into a code block specialised for the coefficient.

Why: on gfx950 (scripts/ubench_ops.hip, profiles/r01_ubench_ops.jsonl) every GPR-index-relative VALU
instruction issues at ~4.4 cycles per wave64, whatever its form, while v_xor_b32 / v_bitop3_b32 with absolute
operands issue at ~2.3.  gf_matmul_bs_kernel spends 32 relative XORs + 16 M0 writes per (row, source);
here the coefficient c selects one of 256 straight-line blocks (s_swappc_b64 / s_setpc_b64) holding the 16
products of that c as v_bitop3_b32 XOR3s whose combination operands are absolute registers baked into the
block, only the accumulator (DST and SRC2) relative to the row slot (M0 = 0xC000 | 16 * row).  One call
costs ~105 cycles at 2 waves/SIMD (scripts/ubench_jump.hip) against ~165 for the relative-XOR form.

Algorithm (one workgroup = 4 waves = 32 output rows x 4 KiB of columns; wave w owns rows 8w..8w+7 of the
tile; one lane = 64 bytes as two 32-byte groups):
  * the 4 KiB source chunk of row j reaches LDS once per workgroup, each wave moving a quarter by LDS-DMA
    (global_load_lds_dwordx4) into a 3-slot ring two rows ahead, one s_barrier per row; every wave then reads
    the whole chunk with 4 ds_read_b128 (per-CU load traffic is a quarter of 8-row-per-wave tiling's, whose
    vector-memory path measured ~24 % of the kernel: profiles/r01_bsj_diag.txt);
  * bit-slicing: a group's 8 dwords (32 bytes) are transposed into 8 bit-planes (plane b = bit b of each
    of the 32 bytes) by three delta-swap stages; 64-bit shifts move two registers per instruction and the
    bit-field merges are v_bitop3_b32 (full rate; v_bfi_b32 and 32-bit shifts issue at quarter rate);
  * for source row j, G[h][v] = XOR of planes {4h + b : bit b of v} (v = 0..15, h = low/high half);
  * multiply-add by c: acc[o] ^= G[0][lo(c, o)] ^ G[1][hi(c, o)], bit b of lo(c, o) = bit o of c * 2^b and
    bit b of hi(c, o) = bit o of c * 2^(4 + b) (GF(2)-linearity of x -> c * x) -- block c holds these 16
    XOR3s for both groups;
  * the block offsets c * BLOCK_BYTES of all (row, source) pairs come from the prep kernel's stream
    (s_load_dwordx8 per source, one source ahead); source rows are loaded two ahead into two staging buffers;
  * after all sources, the accumulators are transposed back and stored.
A call is 4 scalar instructions (M0, low address half, s_swappc_b64, the block's s_setpc_b64): the high half
is preset once the prologue has checked that the block table does not straddle a 4 GiB line (else the loop
copy with the carry runs), and rows past n_out have c = 0, whose block returns at once.

Shared-combination program (RLNC_BSJ_ASM_W4S, variant 7) calls absolute block addresses: the offset kernel writes
base + offset of block c (64-bit; the base is read once per device by a probe launch of this program, which stores
it and exits), two s_load_dwordx16 buffers of 8 addresses, so a call is an M0 step (s_add_u32 m0, m0, 16) +
s_swappc_b64 + s_setpc_b64.  Its blocks are packed (--pack): the accumulator is SRC0 (GPR-index mode SRC0 + DST),
so a product whose low or high half selects nothing is a 4-byte v_xor_b32 instead of an XOR3 with a zero operand.
With 4 waves on one column block, wave w transposes
only set w = (group w >> 1, half w & 1) of the planes -- half of one group's transpose instead of two full ones --
and since round 6 only the four planes of each set (1 KiB) go through LDS, every wave building the 11 composite
combinations of the four sets from them (--no-setplanes: whole 4 KiB sets, built by their builder, the round-1..5
form); the sets are exchanged through two 16 KiB
LDS slots.  Per source row j: barrier; 4 ds_read_b128 of row j's set planes; the staging read of row j + 2 (the
wave's group only); the DMA of row j + 4; the own set planes of row j + 1 (hides the set reads' latency); the 44
composite XORs of row j; row j's calls.  Cost attribution of the round-5 form (profiles/r01_bsj_diag.txt): calls
~10 %, the barrier ~7 %, the own set ~9 %; of the 8-wave program at round 6's start
(profiles/r06_unit_breakdown.json): set reads 11.7 %, barrier 10.1 %, calls 10.0 %, set building 5.1 %.
Run `python3 gen_bsjump.py` after editing; the output is committed.
"""
import argparse
import os

NT = 8  # output rows per wave
WAVES = 4  # waves per workgroup (all on the same 4 KiB column chunk)
WG_ROWS = NT * WAVES
SLOTS = 3  # LDS ring slots of 4 KiB (rows j, j+1, j+2)
BLOCK_BYTES = 16 * 8 + 4  # 16 VOP3 (8 bytes) + s_setpc_b64 (4 bytes); --stride pads with s_nop (never run)
# Default layout: blocks on an 8-byte grid (stride 136, table 8-byte aligned) so that no 8-byte VOP3 straddles an
# 8-byte boundary: encode launch -1.6 %, bench +0.9 % against stride 132; 256-byte-aligned blocks (a 64 KB table)
# made the encode launch 12 % slower and 64-byte-aligned ones (stride 192) 5 %: instruction-cache capacity, not alignment, dominates in the
# product kernel (profiles/r02_bsj_layout_ab.txt; the isolated call microbenchmark, scripts/ubench_tables.py, gains
# 10 % from 256-byte alignment).
DEFAULT_STRIDE, DEFAULT_ALIGN = 136, 3
STREAM_J_BYTES = WG_ROWS * 4  # one dword (block offset) per row of the workgroup tile


# ---- register map ---------------------------------------------------------------------------------------
# --banks (A/B, round 6): a register map in which no XOR3 of a block reads two operands from one VGPR bank (bank =
# register mod 4): group 0's accumulators in banks 2-3 and its low / high combinations in banks 0 / 1, group 1's
# accumulators in banks 0-1 and its combinations in banks 2 / 3.  Entry k of the four sets of a source row is then the
# register quad 128 + 4k (set st = 2g + h in bank st), so the set exchange through LDS is laid out by entry: one
# ds_read_b128 per entry for every wave, one ds_write_b32 per entry for its builder.
BANKS = False


def ACC(i, g, p):  # output row i, group g, plane p (the blocks name row 0; M0 adds 16 * i)
    if BANKS:  # consecutive even-aligned plane pairs (the epilogue transpose's 64-bit shifts), banks 2-3 / 0-1
        return i * 16 + 4 * (p // 2) + (p % 2) + (2 if g == 0 else 0)
    return i * 16 + g * 8 + p


# Set planes (round 6, default; --no-setplanes = the round-1..5 form): the shared programs exchange only the 4
# transposed planes of a set through LDS (one ds_write_b128 per builder, one ds_read_b128 per set and wave instead of
# four) and every wave builds the 11 composite entries of each set itself (44 VOP2 XORs per source row per wave): a
# quarter of the LDS read traffic for more VALU.  The set reads were the largest term of the 8-wave unit (11.7 %,
# profiles/r06_unit_breakdown.json); interleaved A/B (profiles/r06_setplanes_ab.txt): encode launch -2.3 %, the 4-wave
# 32-row product -7.5 %, bench +3.3 %.  The planes sit first in each set's 16 registers (a contiguous quad), entry 0 last.
SETPLANES = True
SP_POS = {1: 0, 2: 1, 4: 2, 8: 3, 3: 4, 5: 5, 6: 6, 7: 7, 9: 8, 10: 9, 11: 10, 12: 11, 13: 12, 14: 13, 15: 14, 0: 15}
# --setregs R (8 or 12, A/B): R entries of each set go through LDS (the planes and the first R - 4 composites of
# SR_ORDER, built by the set's builder), the other 15 - R composites are built by every wave; R = 4 is the planes-only
# form above.  Each composite is one XOR of two entries earlier in SR_ORDER (SR_RECIPE).
SETREGS = 4
SR_ORDER = [1, 2, 4, 8, 3, 12, 5, 10, 6, 9, 7, 11, 13, 14, 15, 0]
SR_RECIPE = {3: (1, 2), 12: (4, 8), 5: (1, 4), 10: (2, 8), 6: (2, 4), 9: (1, 8), 7: (3, 4), 11: (3, 8), 13: (5, 8),
             14: (6, 8), 15: (7, 8)}


def set_pos(v):  # the entry index of combination v in a set (set planes: the exchanged entries first)
    if not SETPLANES:
        return v
    return SR_ORDER.index(v) if SR_MAP else SP_POS[v]


SR_MAP = False  # the SR_ORDER register map (any program exchanging more than the planes; the blocks follow it)


def G(g, h, v):  # combination v of half h of group g (G[g][h][0] = 0)
    if BANKS:
        return 128 + 4 * set_pos(v) + 2 * g + h
    return 128 + g * 32 + h * 16 + set_pos(v)


def RAW(g, d):  # the current source row's 64 bytes, read from the LDS ring
    return 192 + g * 8 + d


TMP0 = 208  # 8 temporaries v208..v215 (4 pairs for 64-bit shifts)
V_X = 216  # 8 registers v216..v223: the transposes' middle stage / the epilogue's store buffer
V_MASK = (224, 225, 226)  # 0xAAAAAAAA, 0xCCCCCCCC, 0xF0F0F0F0
LAST_VGPR = 226
S_OFF = (36, 44, 52)  # block offsets of rows j % 3 (8 dwords each, 4-aligned for s_load_dwordx8)
S_SRC, S_IDX, S_DST, S_BASE, S_TGT, S_RET = 60, 62, 64, 66, 68, 70
S_INROW, S_OUTROW, S_CNT, S_ROWS, S_T0, S_LDSW = 72, 73, 74, 75, 76, 77
FIRST_SGPR, LAST_SGPR = S_OFF[0], S_LDSW
BFI = "0xca"  # v_bitop3_b32 truth table of S0 ? S1 : S2 (index = S0 S1 S2)

# shared-combination program (W = 4, gen --share): wave w builds only set w = (group w >> 1, half w & 1) of
# the next source row and exchanges the four sets through LDS (two 16 KiB set slots)
def RB(x, d):  # source-row staging buffer x (rows alternate), the wave's group only: 8 dwords
    return 192 + 8 * x + d


def OWN(x):  # the wave's own set of the next row, built here and written to LDS (OWN(0) = 0)
    return 228 + x


S_NDMA, S_H = 78, 79  # source rows still to advance over; the wave's half h
CS_SLOT, CS_SET = 16384, 4096
# the shared program reads absolute 64-bit block addresses (the offset kernel adds the table base found by a probe
# launch): two buffers of 8 address pairs (s_load_dwordx16), the other scalars moved up
S_ADDR = (36, 52)
SHARED_SGPRS = dict(S_SRC=68, S_IDX=70, S_DST=72, S_BASE=74, S_TGT=76, S_RET=78, S_INROW=80, S_OUTROW=81, S_CNT=82,
                    S_ROWS=83, S_T0=84, S_LDSW=85, S_NDMA=86, S_H=87)
S_CONS = 88  # 8-wave program: 1 for the consumer waves 4-7
# column-run programs (--run, variant 9): one workgroup walks `tiles` consecutive 4 KiB column blocks of one
# (object, row tile); the source-row stream runs on across the tile boundaries (DMA, staging, set building and the
# block addresses continue into the next tile's rows), so a tile's prologue costs nothing but its epilogue
S_IDXM = 74  # 64-bit: the wave's block-address stream start minus one row (S_BASE is unused by the 8-wave program)
S_DTL, S_SRCT, S_DST0, S_TL, S_POS, S_NIN = 89, 90, 92, 94, 95, 96
# Measured and not kept (profiles/r02_run_ab.txt): builders waiting on vmcnt at the barrier rows only, with
# vmcnt(1 + 32) for the two rows after a tile switch (so the next rows' DMA waits do not include the epilogue's
# stores, which retire in issue order ahead of them): 1.4 % slower than a vmcnt(1) wait in every row.
LAST_VGPR_ALL, LAST_SGPR_ALL = 243, 96

DIAG = set()
# The shared program raises the wave priority (s_setprio) for the calls from PRIO_AT[0] on and drops it after
# the next barrier: the wave finishing a row (which the other 3 waves of its workgroup wait for at the barrier) wins
# issue over the co-resident wave of the other workgroup.  Calls 2.. at level 2: -2..4 % encode time (A/B in
# profiles/r01_bsj_diag.txt, levels 1-3 and first calls 0/2/4/6 within noise of each other).  --prio K,L / --prio off.
PRIO_AT = (2, 2)
ALIGN = 0  # log2 alignment of the first block (--align)


def v(n):
    return f"v{n}"


# ---- bit transpose --------------------------------------------------------------------------------------
# The delta-swap stage k exchanges bit k of the register index with bit k of the bit position (s = 2^k):
#   a' = (a & ~m) | ((b << s) & m),  b' = (b & m) | ((a >> s) & ~m)   for pairs (a, b = a + s), m = MASK[k].
# The three stages act on disjoint index bits, so they commute; all three are involutions, hence so is the
# transpose.  A 64-bit shift of a register pair is exact here: the bits that cross the dword boundary land in
# the low s bits (left shift) or the high s bits (right shift) of the other dword, which m (resp. ~m)
# clears -- provided both registers of the pair need the same shift, i.e. have the same bit k.  Stages 1 and
# 2 find such pairs adjacent in the natural order (stage 1: (2,3), (6,7) left, (0,1), (4,5) right; stage 2:
# (4,5), (6,7) left, (0,1), (2,3) right); stage 0 runs last, on the order PHYS0 written by stage 2
# (pairs (1,3), (5,7) left, (0,2), (4,6) right).  Every stage writes a register set disjoint from the one
# it reads: natural src -> X -> src registers in PHYS0 order -> dst.
PHYS0 = [0, 2, 1, 3, 4, 6, 5, 7]  # physical slot d holds logical register PHYS0[d]
SHIFT_PAIRS = {0: ([(1, 3), (5, 7)], [(0, 2), (4, 6)]), 1: ([(2, 3), (6, 7)], [(0, 1), (4, 5)]),
               2: ([(4, 5), (6, 7)], [(0, 1), (2, 3)])}


def stage(k, cur, out, lines, need=range(8)):
    """Outputs `need` (logical indices) of stage k; only the shifts those outputs read are issued."""
    s = 1 << k
    need = set(need)
    left, right = SHIFT_PAIRS[k]
    used_shl = {a + s for a in need if not (a >> k) & 1}  # output a (bit k clear) reads b << s, b = a + s
    used_shr = {b - s for b in need if (b >> k) & 1}  # output b (bit k set) reads a >> s, a = b - s
    shl, shr = {}, {}
    t = TMP0
    for pairs, op, dst, used in ((left, "v_lshlrev_b64", shl, used_shl), (right, "v_lshrrev_b64", shr, used_shr)):
        for x, y in pairs:
            if not {x, y} & used:
                continue
            assert cur[y] == cur[x] + 1 and cur[x] % 2 == 0, (k, x, y, cur)
            lines.append(f"{op} v[{t}:{t + 1}], {s}, v[{cur[x]}:{cur[y]}]")
            dst[x], dst[y] = t, t + 1
            t += 2
    assert not {cur[a] for a in cur} & {out[a] for a in need}
    for a in range(8):
        if (a >> k) & 1:
            continue
        b = a + s
        if a in need:
            lines.append(f"v_bitop3_b32 {v(out[a])}, v{V_MASK[k]}, v{shl[b]}, {v(cur[a])} bitop3:{BFI}")  # m ? b<<s : a
        if b in need:
            lines.append(f"v_bitop3_b32 {v(out[b])}, v{V_MASK[k]}, {v(cur[b])}, v{shr[a]} bitop3:{BFI}")  # m ? b : a>>s


def transpose(src, dst, lines, half=None):
    """src: natural order (logical r in src[r], aligned consecutive registers); dst: any layout, disjoint
    from src and X.  half = h: only planes 4h..4h+3 (stage 1 in full, stages 2 and 0 on half the outputs)."""
    X = {r: V_X + r for r in range(8)}
    regs = [src[r] for r in range(8)]
    mid = {PHYS0[d]: regs[d] for d in range(8)}
    need = range(8) if half is None else range(4 * half, 4 * half + 4)
    stage(1, src, X, lines)
    stage(2, X, mid, lines, need)
    stage(0, mid, dst, lines, need)


# --combo3 (A/B, round 6): the composite combinations as VOP3 v_bitop3_b32 (S0 ^ S1, S2 = 0) instead of VOP2 v_xor_b32:
# at 2 waves per SIMD the VOP2 XOR measured 2.97 cycles per wave64 instruction against 2.38 for v_bitop3
# (profiles/r01_ubench_ops.jsonl; equal at 4 waves per SIMD)
COMBO3 = False


def xor2(d, a, b):
    """d = a ^ b for the composite combinations (register names as strings)."""
    if COMBO3:
        return f"v_bitop3_b32 {d}, {a}, {b}, 0 bitop3:0x3c"
    return f"v_xor_b32 {d}, {a}, {b}"


def combos(g, h, lines):
    """G[v] for the 11 composite v from the 4 planes (entries 1, 2, 4, 8): one VOP2 XOR each."""
    b = lambda x: v(G(g, h, x))
    lines += [xor2(b(x), b(y), b(z)) for x, y, z in
              [(3, 1, 2), (5, 1, 4), (6, 2, 4), (7, 3, 4), (9, 1, 8), (10, 2, 8), (11, 3, 8), (12, 4, 8), (13, 5, 8),
               (14, 6, 8), (15, 7, 8)]]


# ---- GF(2^8) (0x11B) for the block tables ---------------------------------------------------------------
def xtime(a):
    a <<= 1
    return (a ^ 0x11B) & 0xFF if a & 0x100 else a


def block_indices(c):
    """lo[o], hi[o]: bit b of lo[o] = bit o of c * 2^b, of hi[o] = bit o of c * 2^(4 + b)."""
    m = [c]
    for _ in range(7):
        m.append(xtime(m[-1]))
    lo = [sum(((m[b] >> o) & 1) << b for b in range(4)) for o in range(8)]
    hi = [sum(((m[4 + b] >> o) & 1) << b for b in range(4)) for o in range(8)]
    return lo, hi


def blocks(lines):
    for c in range(256):
        lo, hi = block_indices(c)
        if c == 0:  # no products (and the rows past n_out): return at once
            lines.append(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
            lines += ["s_nop 0"] * ((BLOCK_BYTES - 4) // 4)
            continue
        for g in range(2):
            for o in range(8):
                a = ACC(0, g, o)
                if lo[o] == 0 and hi[o] == 0:  # nothing to add: keep the block size (8 bytes), issue no VALU
                    lines += ["s_nop 0", "s_nop 0"]
                    continue
                x = f"v{G(g, 0, lo[o])}" if lo[o] else "0"  # G[.][0] = 0: an inline constant reads no VGPR bank
                y = f"v{G(g, 1, hi[o])}" if hi[o] else "0"
                lines.append(f"v_bitop3_b32 v{a}, {x}, {y}, v{a} bitop3:0x96")
        lines.append(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
        lines += ["s_nop 0"] * ((BLOCK_BYTES - (16 * 8 + 4)) // 4)


# ---- main program ---------------------------------------------------------------------------------------
FAST = True  # the loop being generated: True = high half of every block address preset (no carry, checked)


# The shared programs step M0 by 16 between calls (a 4-byte SALU) instead of moving an 8-byte literal (--no-m0step);
# with --pack (default) the two are worth -0.3 % encode and -1.1 % decode time, 5 interleaved passes
# (profiles/r02_bsj_thread_ab.txt)
M0STEP = True


# --pack: the shared programs' blocks with the accumulator as SRC0 (GPR-index mode SRC0 + DST), so that a product
# whose low or high half selects nothing is a 4-byte VOP2 v_xor_b32 instead of an 8-byte XOR3 with a zero operand;
# blocks packed at their own size (XOR3s first, 8-byte grid), the offset kernel reads the block offsets from a table
PACK = True


def idx_mode():
    return "gpr_idx(SRC0,DST)" if PACK else "gpr_idx(SRC2,DST)"


def m0_slot(i):
    """M0 = row slot i's GPR-index base (after slot i - 1's call when stepping)."""
    if M0STEP and i:
        return "s_add_u32 m0, m0, 16"
    return f"s_mov_b32 m0, {hex((0x9000 if PACK else 0xC000) | (16 * i))}"


def blocks_packed(lines):
    """The 256 blocks at their own sizes; returns their byte offsets from the table start."""
    offs, pos = [], 0
    for c in range(256):
        lo, hi = block_indices(c)
        v3, v2 = [], []
        for g in range(2):
            for o in range(8):
                a = ACC(0, g, o)
                if c == 0 or (lo[o] == 0 and hi[o] == 0):
                    continue
                if lo[o] and hi[o]:
                    v3.append(f"v_bitop3_b32 v{a}, v{a}, v{G(g, 0, lo[o])}, v{G(g, 1, hi[o])} bitop3:0x96")
                else:
                    v2.append(f"v_xor_b32 v{a}, v{a}, v{G(g, 0, lo[o]) if lo[o] else G(g, 1, hi[o])}")
        size = 8 * len(v3) + 4 * len(v2) + 4
        pad = (-size) % 8
        offs.append(pos)
        lines += v3 + v2 + [f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]"] + ["s_nop 0"] * (pad // 4)
        pos += size + pad
    return offs


def call(L, cur, i):
    """Row i's product of the current source: M0 = its accumulator slot, then the call into block c (whose
    offset c * BLOCK_BYTES is s[cur + i]).  Rows past n_out have c = 0, whose block returns at once.  The fast
    loop adds the low half only: the prologue has checked that the block table does not cross a 4 GiB line."""
    L += [f"s_mov_b32 m0, {hex(0xC000 | (16 * i))}", f"s_add_u32 s{S_TGT}, s{S_BASE}, s{cur + i}"]
    if not FAST:
        L.append(f"s_addc_u32 s{S_TGT + 1}, s{S_BASE + 1}, 0")
    L.append(f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]")


def loops(L, body_fn, unroll):
    """The main loop twice: fast (high address half preset) and, for a block table straddling a 4 GiB line,
    with the carry; both leave through 3:."""
    global FAST
    L += [f"s_add_u32 s{S_T0}, s{S_BASE}, {256 * BLOCK_BYTES}",
          "s_cbranch_scc1 12f" if "safe" not in DIAG else "s_branch 12f",  # --diag=safe: test the carry loop
          f"s_mov_b32 s{S_TGT + 1}, s{S_BASE + 1}"]
    for fast, top in ((True, 1), (False, 11)):
        FAST = fast
        L.append(f"{top}:" if fast else "12:")
        if not fast:
            L.append(f"{top}:")
        for j in range(unroll):
            body_fn(L, j)
            L += [f"s_cmp_eq_u32 s{S_CNT}, 0", "s_cbranch_scc1 3f" if j < unroll - 1 else f"s_cbranch_scc0 {top}b"]
        if fast:
            L.append("s_branch 3f")
    FAST = True
    L += ["3:", "s_waitcnt vmcnt(0) lgkmcnt(0)"]

def dma(lines, slot):
    """This wave's share (4 / WAVES KiB) of the row at S_SRC into ring slot `slot`, 1 KiB per LDS-DMA
    instruction (M0 = wave-uniform LDS base, lane l writes base + 16 l; one wait state after the M0 write)."""
    if "novm" in DIAG:
        return
    # the instruction offset applies to the global AND the LDS address (LDS = M0 + offset + 16 lane)
    lines += [f"s_add_u32 m0, s{S_LDSW}, {slot * 4096}", "s_nop 0"]
    for d in range(4 // WAVES):
        off = f" offset:{d * 1024}" if d else ""
        lines.append(f"global_load_lds_dwordx4 %[dmaoff], s[{S_SRC}:{S_SRC + 1}]{off}")


def advance(lines):
    """S_SRC -> the next source row if it exists (else stays: the re-read is harmless, always in bounds)."""
    lines += [
        f"s_cmp_gt_u32 s{S_CNT}, 1",
        f"s_cselect_b32 s{S_T0}, s{S_INROW}, 0",
        f"s_add_u32 s{S_SRC}, s{S_SRC}, s{S_T0}",
        f"s_addc_u32 s{S_SRC + 1}, s{S_SRC + 1}, 0",
    ]


def body(L, slot):
    """Source row j (slot = j % 3): its chunk is in ring slot `slot`, its block offsets in S_OFF[slot]."""
    if "novm" not in DIAG and "novmw" not in DIAG:
        L.append(f"s_waitcnt vmcnt({4 // WAVES})")  # this wave's DMAs of row j done (row j+1's may stay in flight)
    if "nobar" not in DIAG:
        L.append("s_barrier")  # every wave's quarter of row j landed; every wave is done reading row j-1's slot
    L.append(f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1")
    advance(L)
    dma(L, (slot + 2) % SLOTS)  # row j+2 into the slot row j-1 used
    for g in range(2):
        for h in range(2):
            q = 2 * g + h
            if "nods" not in DIAG:
                L.append(f"ds_read_b128 v[{RAW(g, 4 * h)}:{RAW(g, 4 * h) + 3}], %[ldsr] offset:{slot * 4096 + q * 1024}")
    if "nosmem" not in DIAG or "nods" not in DIAG:
        L.append("s_waitcnt lgkmcnt(0)")  # the chunk, and row j's block offsets (SMEM, issued a row earlier)
    for g in range(2):
        planes = {b: G(g, b // 4, 1 << (b % 4)) for b in range(8)}
        if "notrans" in DIAG:  # timing only
            L += [f"v_mov_b32 v{planes[b]}, v{RAW(g, b)}" for b in range(8)]
        else:
            transpose({d: RAW(g, d) for d in range(8)}, planes, L)
    for g in range(2):
        for h in range(2):
            if "nocombo" not in DIAG:
                combos(g, h, L)
    cur, nxt = S_OFF[slot], S_OFF[(slot + 1) % SLOTS]
    L += [
        f"s_load_dwordx8 s[{nxt}:{nxt + 7}], s[{S_IDX}:{S_IDX + 1}], {STREAM_J_BYTES}" if "nosmem" not in DIAG
        else "s_nop 0",  # timing only: every row reuses the prologue's offsets of rows 0-2
        f"s_add_u32 s{S_IDX}, s{S_IDX}, {STREAM_J_BYTES}",
        f"s_addc_u32 s{S_IDX + 1}, s{S_IDX + 1}, 0",
        "s_set_gpr_idx_on 0, gpr_idx(SRC2,DST)" if "absinline" not in DIAG else "s_nop 0",
    ]
    for i in range(NT):
        if "inline" in DIAG:  # timing only: the products of a fixed coefficient inline, no call
            L.append(f"s_mov_b32 m0, {hex(0xC000 | (16 * i))}")
            lo, hi = block_indices(0x53 + i)
            L += [f"v_bitop3_b32 v{ACC(0, g, o)}, v{G(g, 0, lo[o])}, v{G(g, 1, hi[o])}, v{ACC(0, g, o)} bitop3:0x96"
                  for g in range(2) for o in range(8)]
            continue
        if "absinline" in DIAG:  # timing only: as "inline" with absolute accumulators (no GPR-index mode)
            lo, hi = block_indices(0x53 + i)
            if "nobank" in DIAG:  # ... with the three sources of every XOR3 in three different banks
                lo = [4 * ((x // 4) % 4) + (o + 1) % 4 for o, x in enumerate(lo)]
                hi = [4 * ((x // 4) % 4) + (o + 2) % 4 for o, x in enumerate(hi)]
            L += [f"v_bitop3_b32 v{ACC(i, g, o)}, v{G(g, 0, lo[o])}, v{G(g, 1, hi[o])}, v{ACC(i, g, o)} bitop3:0x96"
                  for g in range(2) for o in range(8)]
            continue
        call(L, cur, i)
    L.append("s_set_gpr_idx_off" if "absinline" not in DIAG else "s_nop 0")


def advance_s(L):
    """S_SRC -> the next source row while one is left (S_NDMA counts them down; SCC is read twice)."""
    L += [
        f"s_cmp_gt_u32 s{S_NDMA}, 0",
        f"s_cselect_b32 s{S_T0}, s{S_INROW}, 0",
        f"s_cselect_b32 s{S_TGT}, 1, 0",
        f"s_sub_u32 s{S_NDMA}, s{S_NDMA}, s{S_TGT}",
        f"s_add_u32 s{S_SRC}, s{S_SRC}, s{S_T0}",
        f"s_addc_u32 s{S_SRC + 1}, s{S_SRC + 1}, 0",
    ]


def advance_run(L):
    """advance_s for the column-run program: past the tile's last source row the DMA stream moves on to row 0 of
    the next column block (S_SRCT + 4 KiB) while the workgroup has one (S_DTL counts the tiles the DMA stream
    has still to enter), else stays (the re-read is harmless, always in bounds)."""
    L += [
        f"s_cmp_gt_u32 s{S_NDMA}, 0",
        "s_cbranch_scc0 30f",
        f"s_sub_u32 s{S_NDMA}, s{S_NDMA}, 1",
        f"s_add_u32 s{S_SRC}, s{S_SRC}, s{S_INROW}",
        f"s_addc_u32 s{S_SRC + 1}, s{S_SRC + 1}, 0",
        "s_branch 31f",
        "30:",
        f"s_cmp_gt_u32 s{S_DTL}, 1",
        "s_cbranch_scc0 31f",
        f"s_sub_u32 s{S_DTL}, s{S_DTL}, 1",
        f"s_add_u32 s{S_SRCT}, s{S_SRCT}, 4096",
        f"s_addc_u32 s{S_SRCT + 1}, s{S_SRCT + 1}, 0",
        f"s_mov_b64 s[{S_SRC}:{S_SRC + 1}], s[{S_SRCT}:{S_SRCT + 1}]",
        f"s_sub_u32 s{S_NDMA}, s{S_NIN}, 1",
        "31:",
    ]


RUN = False  # the 8-wave program being generated is the column-run form


def own_set(L, rb, cslot):
    """Set (g, h) of the row staged in RB[rb]: planes 4h..4h+3 by the half transpose, the 11 composite
    entries by VOP2 XORs, then 4 ds_write_b128 to set slot `cslot` (entry 0 is the zero register)."""
    L += [f"s_cmp_eq_u32 s{S_H}, 0", "s_cbranch_scc0 4f"]
    for h in range(2):
        if SETPLANES:  # the 4 planes as one contiguous quad OWN(0..3), then the exchanged composites OWN(4..R-1)
            planes = {4 * h + b: OWN(b) for b in range(4)}
            transpose({d: RB(rb, d) for d in range(8)}, planes, L, half=h)
            for pos in range(4, SETREGS):
                x, y = SR_RECIPE[SR_ORDER[pos]]
                L.append(xor2(f"v{OWN(pos)}", f"v{OWN(SR_ORDER.index(x))}", f"v{OWN(SR_ORDER.index(y))}"))
        else:
            planes = {4 * h + b: OWN(1 << b) for b in range(4)}
            transpose({d: RB(rb, d) for d in range(8)}, planes, L, half=h)
            L += [f"v_xor_b32 v{OWN(x)}, v{OWN(y)}, v{OWN(z)}" for x, y, z in
                  [(3, 1, 2), (5, 1, 4), (6, 2, 4), (7, 3, 4), (9, 1, 8), (10, 2, 8), (11, 3, 8), (12, 4, 8),
                   (13, 5, 8), (14, 6, 8), (15, 7, 8)]]
        L.append("s_branch 6f" if h == 0 else "6:")
        if h == 0:
            L.append("4:")
    sfx, base = cslot_addr(cslot)
    if BANKS:  # entry k of this wave's set into its dword of the entry's 16 bytes (ldscw = ldsc + 4 * set)
        for k in range(SETREGS):
            L.append(f"ds_write_b32 %[ldscw{sfx}], v{OWN(k)} offset:{base + k * 1024}")
        return
    for q in range(SETREGS // 4 if SETPLANES else 4):
        L.append(f"ds_write_b128 %[ldscw{sfx}], v[{OWN(4 * q)}:{OWN(4 * q) + 3}] offset:{base + q * 1024}")


def set_reads(L, sfx, base):
    """The four sets of a source row from LDS: 16 ds_read_b128 (whole sets), or with --setplanes one per set (the
    planes) into the set's first quad."""
    if BANKS:  # entry k of all four sets: one quad
        for k in range(SETREGS):
            L.append(f"ds_read_b128 v[{128 + 4 * k}:{128 + 4 * k + 3}], %[ldsc{sfx}] offset:{base + k * 1024}")
        return
    for st in range(4):
        for q in range(SETREGS // 4 if SETPLANES else 4):
            r = G(st >> 1, st & 1, 1) + 4 * q if SETPLANES else G(st >> 1, st & 1, 4 * q)
            L.append(f"ds_read_b128 v[{r}:{r + 3}], %[ldsc{sfx}] offset:{base + st * CS_SET + q * 1024}")


def set_combos(L):
    """Set planes: the 11 composite entries of the four sets from their planes, in every wave (--diag=s8nocombo:
    skipped, timing only)."""
    if SETPLANES and "s8nocombo" not in DIAG:
        for st in range(4):
            if not SR_MAP:
                combos(st >> 1, st & 1, L)
                continue
            g, h = st >> 1, st & 1
            for v in SR_ORDER[SETREGS:15]:
                x, y = SR_RECIPE[v]
                L.append(xor2(f"v{G(g, h, v)}", f"v{G(g, h, x)}", f"v{G(g, h, y)}"))


SET_WAIT = 3  # LDS ops a builder leaves in flight at the set-read wait: 2 staging reads + the set write(s) (1, or 4)


def apply_setregs(r):
    """The set exchange of the program about to be generated: r entries per set through LDS (set planes)."""
    global SETREGS, CS_SET, CS_SLOT, SET_WAIT
    SETREGS = r
    if BANKS:  # laid out by entry: 1 KiB per entry of the four sets, a wave's set at +4 B
        CS_SET, CS_SLOT, SET_WAIT = 4, r * 1024, 2 + r
    else:
        CS_SET, CS_SLOT, SET_WAIT = r * 256, r * 1024, 2 + r // 4


def body_s(L, j, cons=False):
    """Source row j (j = the row index mod 6): sets of row j from LDS, row j + 2's staging read, row j + 4's
    DMA, the own set of row j + 1, then row j's products.  cons (8-wave program): waves 4-7 (S_CONS != 0) only
    read the sets and call; waves 0-3 stage, build and write the sets for all eight."""
    L += ["s_waitcnt vmcnt(1) lgkmcnt(0)",  # row j+2's DMA landed (row j+3's may fly); own set j + RB[j+1] done
          "s_barrier" if "snobar" not in DIAG else "s_nop 0",  # every wave's set of row j written, row j+2
          f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1"]                   # landed, row j+1's ring slot read by all
    if PRIO_AT is not None:
        L.append("s_setprio 0")
    if "sprio2" in DIAG:
        L.append("s_setprio 2")  # experiment: set building (what the other waves wait for next row) first
    set_reads(L, "", (j % 2) * CS_SLOT)
    if cons:
        L += [f"s_cmp_lg_u32 s{S_CONS}, 0", "s_cbranch_scc1 20f"]
    for hh in range(2):
        r = RB(j % 2, 4 * hh)
        L.append(f"ds_read_b128 v[{r}:{r + 3}], %[ldsrg] offset:{((j + 2) % SLOTS) * 4096 + hh * 1024}")
    advance_s(L)
    L += [f"s_add_u32 m0, s{S_LDSW}, {((j + 1) % SLOTS) * 4096}", "s_nop 0",
          "global_load_lds_dwordx4 %[dmaoff], s[{0}:{1}]".format(S_SRC, S_SRC + 1)]  # row j+4
    if "snoown" in DIAG:  # timing only: the set writes without building the set
        L += [f"ds_write_b128 %[ldscw], v[{OWN(4 * q)}:{OWN(4 * q) + 3}] offset:{((j + 1) % 2) * CS_SLOT + q * 1024}"
              for q in range(4)]
    else:
        own_set(L, (j + 1) % 2, (j + 1) % 2)
    cur, nxt = S_ADDR[j % 2], S_ADDR[(j + 1) % 2]
    if "sprio2" in DIAG:
        L.append("s_setprio 0")
    L += [
        # the 16 set reads (LDS returns in order; 2 staging reads + 4 writes may fly)
        f"s_waitcnt lgkmcnt({SET_WAIT})" if "snowait" not in DIAG else "s_nop 0",
    ]
    if cons:  # consumer waves: no staging reads or set writes in flight, the 16 set reads are the last
        L += ["s_branch 21f", "20:", "s_waitcnt lgkmcnt(0)", "21:"]
    set_combos(L)
    L += [
        f"s_load_dwordx16 s[{nxt}:{nxt + 15}], s[{S_IDX}:{S_IDX + 1}], {STREAM_J_BYTES}",
        f"s_add_u32 s{S_IDX}, s{S_IDX}, {STREAM_J_BYTES}",
        f"s_addc_u32 s{S_IDX + 1}, s{S_IDX + 1}, 0",
        f"s_set_gpr_idx_on 0, {idx_mode()}",
    ]
    for i in range(NT):
        if "sinline" in DIAG:  # timing only: a fixed coefficient's products inline (relative), no call
            L.append(f"s_mov_b32 m0, {hex(0xC000 | (16 * i))}")
            lo, hi = block_indices(0x53 + i)
            L += [f"v_bitop3_b32 v{ACC(0, g, o)}, v{G(g, 0, lo[o])}, v{G(g, 1, hi[o])}, v{ACC(0, g, o)} bitop3:0x96"
                  for g in range(2) for o in range(8)]
            continue
        if PRIO_AT is not None and i == PRIO_AT[0]:  # the calls closest to the next barrier at raised priority
            L.append(f"s_setprio {PRIO_AT[1]}")
        # row i: M0 = its accumulator slot, then the call to the absolute address of block c (rows past
        # n_out have c = 0, whose block returns at once)
        L += [m0_slot(i), f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{cur + 2 * i}:{cur + 2 * i + 1}]"]
    L.append("s_set_gpr_idx_off")


def program_shared(cons=False):
    assert WAVES == (8 if cons else 4)
    saved = {n: globals()[n] for n in SHARED_SGPRS}
    globals().update(SHARED_SGPRS)
    try:
        if not cons and W4BAR:
            return program_shared4b()
        return program_shared_body(cons)
    finally:
        globals().update(saved)


def program_shared_body(cons=False):
    """cons: the 8-wave program (64-row tile): waves 0-3 are the 4-wave program's builders, waves 4-7 (rows
    32-63) only read the sets and call.  It has no block table of its own: the offset kernel's absolute
    addresses point into the 4-wave program's blocks (same register map, same return register)."""
    if cons:
        return program_shared8()
    L = [
        f"s_mov_b64 s[{S_SRC}:{S_SRC + 1}], %[src]",
        f"s_mov_b64 s[{S_IDX}:{S_IDX + 1}], %[idx]",
        f"s_mov_b64 s[{S_DST}:{S_DST + 1}], %[dst]",
        f"s_mov_b32 s{S_INROW}, %[in_row]",
        f"s_mov_b32 s{S_OUTROW}, %[out_row]",
        f"s_mov_b32 s{S_CNT}, %[n_in]",
        f"s_sub_u32 s{S_NDMA}, %[n_in], 1",
        f"s_mov_b32 s{S_H}, %[half]",
        f"s_mov_b32 s{S_ROWS}, %[rows]",
        f"v_mov_b32 v{V_MASK[0]}, 0xaaaaaaaa",
        f"v_mov_b32 v{V_MASK[1]}, 0xcccccccc",
        f"v_mov_b32 v{V_MASK[2]}, 0xf0f0f0f0",
        f"s_getpc_b64 s[{S_BASE}:{S_BASE + 1}]",
        "5:",
        f"s_add_u32 s{S_BASE}, s{S_BASE}, (9f - 5b)",
        f"s_addc_u32 s{S_BASE + 1}, s{S_BASE + 1}, 0",
        f"s_mov_b32 s{S_LDSW}, %[ldsw]",
        # probe launch (probe != 0): store the block table's address for the offset kernel and leave
        "s_cmp_lg_u64 %[probe], 0",
        "s_cbranch_scc0 10f",
        f"v_mov_b32 v{V_X}, s{S_BASE}",
        f"v_mov_b32 v{V_X + 1}, s{S_BASE + 1}",
        f"v_mov_b32 v{V_X + 2}, 0",
        f"global_store_dwordx2 v{V_X + 2}, v[{V_X}:{V_X + 1}], %[probe]",
        "s_waitcnt vmcnt(0)",
        "s_branch 8f",
        "10:",
    ]
    dmai = "global_load_lds_dwordx4 %[dmaoff], s[{0}:{1}]".format(S_SRC, S_SRC + 1)
    for slot in range(3):  # rows 0, 1, 2 (clamped to the last row) into ring slots 0, 1, 2
        if slot:
            advance_s(L)
        L += [f"s_add_u32 m0, s{S_LDSW}, {slot * 4096}", "s_nop 0", dmai]
    L.append(f"s_load_dwordx16 s[{S_ADDR[0]}:{S_ADDR[0] + 15}], s[{S_IDX}:{S_IDX + 1}], 0")
    L += [f"v_mov_b32 v{r}, 0" for r in range(128)]
    L.append(f"v_mov_b32 v{OWN(0)}, 0")
    L += ["s_waitcnt vmcnt(1)", "s_barrier"]  # rows 0 and 1 landed (all waves)
    for x in range(2):
        for hh in range(2):
            r = RB(x, 4 * hh)
            L.append(f"ds_read_b128 v[{r}:{r + 3}], %[ldsrg] offset:{x * 4096 + hh * 1024}")
    L += ["s_waitcnt lgkmcnt(0)", "s_barrier"]  # every wave has read slot 0: row 3 may overwrite it
    advance_s(L)
    L += [f"s_add_u32 m0, s{S_LDSW}, 0", "s_nop 0", dmai]
    own_set(L, 0, 0)  # row 0's own set into set slot 0
    L.append("1:")  # absolute addresses: one loop (no carry case)
    for j in range(6):
        body_s(L, j)
        L += [f"s_cmp_eq_u32 s{S_CNT}, 0", "s_cbranch_scc1 3f" if j < 5 else "s_cbranch_scc0 1b"]
    L += ["3:", "s_waitcnt vmcnt(0) lgkmcnt(0)"]
    epilogue(L)
    L.append("s_branch 8f")
    if ALIGN:
        L.append(f".p2align {ALIGN}")
    L.append("9:")
    global SOFFS
    if PACK:
        SOFFS = blocks_packed(L)
    else:
        blocks(L)
        SOFFS = None
    L.append("8:")
    return L


SOFFS = None  # byte offsets of the shared programs' packed blocks (--pack)


def run_tail(L, unroll, body_fn):
    """The column-run main loop: `unroll` bodies, a tile ending after any of them (labels: 40 + j = body j,
    60 + j = tile end after body j); the tile end records the position (S_POS), runs the epilogue into the
    tile's rows, clears the accumulators and continues with the next body while the run has tiles."""
    L.append("1:")
    for j in range(unroll):
        if j:
            L.append(f"{40 + j}:")
        body_fn(L, j)
        L += [f"s_cmp_eq_u32 s{S_CNT}, 0", f"s_cbranch_scc1 {60 + j}f" if j < unroll - 1 else "s_cbranch_scc0 1b"]
    for j in [unroll - 1] + list(range(unroll - 1)):
        L += [f"{60 + j}:", f"s_mov_b32 s{S_POS}, {j}", "s_branch 7f"]
    L.append("7:")
    # the run's last tile: the DMA stream's last (re-)reads must land before the workgroup ends (LDS); no other
    # vmcnt wait follows its stores
    L += [f"s_cmp_eq_u32 s{S_TL}, 1", "s_cbranch_scc0 26f", "s_waitcnt vmcnt(0)", "26:"]
    L.append(f"s_mov_b64 s[{S_DST}:{S_DST + 1}], s[{S_DST0}:{S_DST0 + 1}]")
    epilogue(L)  # the tile's rows (its own rows: S_ROWS), then fresh accumulators
    L += [f"v_mov_b32 v{r}, 0" for r in range(128)]
    L += [f"s_sub_u32 s{S_TL}, s{S_TL}, 1",
          f"s_cmp_eq_u32 s{S_TL}, 0",
          "s_cbranch_scc1 3f",
          f"s_add_u32 s{S_DST0}, s{S_DST0}, 4096",
          f"s_addc_u32 s{S_DST0 + 1}, s{S_DST0 + 1}, 0",
          f"s_mov_b32 s{S_CNT}, s{S_NIN}"]
    for j in range(unroll):  # continue with body j + 1
        nb = "1b" if j == unroll - 1 else f"{40 + j + 1}b"
        L += [f"s_cmp_eq_u32 s{S_POS}, {j}", f"s_cbranch_scc1 {nb}"]
    L += ["3:", "s_waitcnt lgkmcnt(0)"]


def run_init(L):
    L += [f"s_mov_b64 s[{S_SRCT}:{S_SRCT + 1}], %[src]",
          f"s_mov_b64 s[{S_DST0}:{S_DST0 + 1}], %[dst]",
          f"s_mov_b32 s{S_TL}, %[tiles]",
          f"s_mov_b32 s{S_DTL}, %[tiles]",
          f"s_mov_b32 s{S_NIN}, %[n_in]"]


# 8-wave program: one workgroup per CU leaves LDS for SLOTS8 ring slots and CSLOTS8 = 2 BAR8 set slots, so the
# builders run BAR8 rows ahead (staging read of row j + BAR8 + 1, set of row j + BAR8, DMA of row j + DMA8 during
# row j) and the workgroup meets at a barrier every BAR8-th row instead of every row.  Conditions (vmcnt(1) at
# every row top): DMA8 >= 2 BAR8 + 2 (rows <= x + 2 BAR8 landed at barrier x), SLOTS8 >= DMA8 - 1 (a ring slot is
# refilled only after a barrier that follows its staging reads); set slot r % CSLOTS8 is rewritten BAR8 rows after
# its last read, with one barrier in between.  BAR8 = 2: DMA8 = SLOTS8 = 6 (88 KiB); BAR8 = 3: DMA8 = 8,
# SLOTS8 = 12 (144 KiB; set slots 4-5 through the second base, ds offsets are 16-bit).
BAR8 = 3
DMA8 = SLOTS8 = CSLOTS8 = 0
# 8-wave program: calls 4.. of each row at s_setprio 1, back to 0 at the next row's top (round 6 with set planes:
# encode launch -0.9 %, bench +0.7 % interleaved, profiles/r06_prio_ab.txt; round 1's program measured no priority
# best, -0.8 % against calls 2.. at level 2, profiles/r01_launch_size.txt)
PRIO8 = (4, 1)


def set_bar8(b):
    global BAR8, DMA8, SLOTS8, CSLOTS8
    BAR8, DMA8, SLOTS8, CSLOTS8 = b, 2 * b + 2, {2: 6, 3: 12, 4: 16}[b], 2 * b


set_bar8(3)


def cs_base2():
    """Byte offset of the second set-slot base (%[ldsc2] / %[ldscw2]: ds offsets are 16-bit): the first slot that
    does not end within 64 KiB of the first base (RLNC_BSJ_CS_BASE2 for the host)."""
    first = 0
    while (first + 1) * CS_SLOT <= 65536:
        first += 1
    return first * CS_SLOT


def cslot_addr(slot):  # (base operand, offset) of set slot `slot` for reads / the wave's own write
    o, b2 = slot * CS_SLOT, cs_base2()
    return ("", o) if o < b2 else ("2", o - b2)


def lcm(*xs):
    import math
    out = 1
    for x in xs:
        out = out * x // math.gcd(out, x)
    return out


def body_s8(L, j):
    """Source row j (j = the row index mod the unroll): sets of row j, then -- builders only -- the staging read of
    row j + BAR8 + 1, the DMA of row j + DMA8 and the own set of row j + BAR8; then row j's products.  Barrier
    when j % BAR8 == 0: it orders the set writes of rows j .. j + BAR8 - 1 before their reads, the ring landing of
    rows <= j + 2 BAR8 before their staging reads and every read of a slot before its reuse."""
    if RUN:  # consumers have no loads in flight, only the last tile's stores: never wait on those
        L += [f"s_cmp_lg_u32 s{S_CONS}, 0", "s_cbranch_scc1 24f", "s_waitcnt vmcnt(1)", "24:", "s_waitcnt lgkmcnt(0)"]
    else:
        L.append("s_waitcnt vmcnt(1) lgkmcnt(0)")  # rows <= j+DMA8-2 landed; own LDS ops + addresses done
    if j % BAR8 == 0:  # --diag=s8nobar: no barrier in the loop at all (timing only, wrong results): the most any
        L.append("s_barrier" if "s8nobar" not in DIAG else "s_nop 0")  # barrier replacement could gain
    L.append(f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1")
    if PRIO8 is not None:
        L.append("s_setprio 0")
    sfx, base = cslot_addr(j % CSLOTS8)
    # per-term diagnostics of the 8-wave unit (timing only, wrong results; scripts/archive/r06_unit_breakdown.sh):
    # s8noread no set reads, s8nodma no LDS-DMA of source rows, s8nostage no staging reads, s8noown the set writes
    # without building the set, s8nosmem no address-stream loads (the prologue's two rows reused), s8inline a fixed
    # coefficient's products inline per row (relative, no call)
    if "s8noread" not in DIAG:
        set_reads(L, sfx, base)
    L += [f"s_cmp_lg_u32 s{S_CONS}, 0", "s_cbranch_scc1 20f"]
    if "bprio" in DIAG:  # experiment: builders at raised priority while staging and building the sets
        L.append("s_setprio 1")
    nx = j + BAR8 + 1  # staged now into RB[nx % 2] (it held row nx - 2, whose set was built during row j - 1)
    if "s8nostage" not in DIAG:
        for hh in range(2):
            r = RB(nx % 2, 4 * hh)
            L.append(f"ds_read_b128 v[{r}:{r + 3}], %[ldsrg] offset:{(nx % SLOTS8) * 4096 + hh * 1024}")
    advance_run(L) if RUN else advance_s(L)
    if "s8nodma" not in DIAG:
        L += [f"s_add_u32 m0, s{S_LDSW}, {((j + DMA8) % SLOTS8) * 4096}", "s_nop 0",
              "global_load_lds_dwordx4 %[dmaoff], s[{0}:{1}]".format(S_SRC, S_SRC + 1)]  # row j + DMA8
    if "s8noown" in DIAG:
        sfx2, base2 = cslot_addr((j + BAR8) % CSLOTS8)
        L += [f"ds_write_b128 %[ldscw{sfx2}], v[{OWN(4 * q)}:{OWN(4 * q) + 3}] offset:{base2 + q * 1024}"
              for q in range(4)]
    else:
        own_set(L, (j + BAR8) % 2, (j + BAR8) % CSLOTS8)  # row j + BAR8's set
    if "bprio" in DIAG:
        L.append("s_setprio 0")
    L += [f"s_waitcnt lgkmcnt({SET_WAIT})",  # the 16 set reads (2 staging reads + 4 set writes may fly)
          "s_branch 21f", "20:", "s_waitcnt lgkmcnt(0)", "21:"]
    set_combos(L)
    cur, nxt = S_ADDR[j % 2], S_ADDR[(j + 1) % 2]
    if RUN:  # row j is the tile's last: the next row's addresses are row 0's (the next column block, same rows)
        L += [f"s_cmp_eq_u32 s{S_CNT}, 0",
              f"s_cselect_b64 s[{S_IDX}:{S_IDX + 1}], s[{S_IDXM}:{S_IDXM + 1}], s[{S_IDX}:{S_IDX + 1}]"]
    L += [
        f"s_load_dwordx16 s[{nxt}:{nxt + 15}], s[{S_IDX}:{S_IDX + 1}], {STREAM_J_BYTES}" if "s8nosmem" not in DIAG
        else "s_nop 0",
        f"s_add_u32 s{S_IDX}, s{S_IDX}, {STREAM_J_BYTES}",
        f"s_addc_u32 s{S_IDX + 1}, s{S_IDX + 1}, 0",
        f"s_set_gpr_idx_on 0, {idx_mode()}",
    ]
    for i in range(NT):
        if PRIO8 is not None and i == PRIO8[0]:
            L.append(f"s_setprio {PRIO8[1]}")
        if "s8inline" in DIAG:  # the block of a fixed coefficient inline, in the packed blocks' form
            L.append(m0_slot(i))
            L += inline_block(0x53 + 11 * i)
            continue
        L += [m0_slot(i), f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{cur + 2 * i}:{cur + 2 * i + 1}]"]
    L.append("s_set_gpr_idx_off")


def inline_block(c):
    """Block c's XOR3s / XORs without its return (packed form: the accumulator is SRC0, GPR-index relative)."""
    lo, hi = block_indices(c)
    v3, v2 = [], []
    for g in range(2):
        for o in range(8):
            a = ACC(0, g, o)
            if lo[o] and hi[o]:
                v3.append(f"v_bitop3_b32 v{a}, v{a}, v{G(g, 0, lo[o])}, v{G(g, 1, hi[o])} bitop3:0x96")
            elif lo[o] or hi[o]:
                v2.append(f"v_xor_b32 v{a}, v{a}, v{G(g, 0, lo[o]) if lo[o] else G(g, 1, hi[o])}")
    return v3 + v2


W4BAR = 0  # --w4bar B: the 4-wave shared program in the 8-wave program's form (all four waves builders)


def program_shared4b():
    """The 4-wave shared program (32-row tiles: the decode's products) in the 8-wave program's form: the four waves
    build the sets BAR8 rows ahead of their reads and meet at a barrier every BAR8-th row instead of every row (LDS:
    SLOTS8 ring slots + CSLOTS8 set slots; with set planes 72 KiB at BAR8 = 3, two workgroups per CU).  Carries the
    probe entry and the block table the 8-wave program calls into, like program_shared_body."""
    assert WAVES == 4
    L = [
        f"s_getpc_b64 s[{S_BASE}:{S_BASE + 1}]",
        "5:",
        f"s_add_u32 s{S_BASE}, s{S_BASE}, (9f - 5b)",
        f"s_addc_u32 s{S_BASE + 1}, s{S_BASE + 1}, 0",
        # probe launch (probe != 0): store the block table's address for the offset kernel and leave
        "s_cmp_lg_u64 %[probe], 0",
        "s_cbranch_scc0 10f",
        f"v_mov_b32 v{V_X}, s{S_BASE}",
        f"v_mov_b32 v{V_X + 1}, s{S_BASE + 1}",
        f"v_mov_b32 v{V_X + 2}, 0",
        f"global_store_dwordx2 v{V_X + 2}, v[{V_X}:{V_X + 1}], %[probe]",
        "s_waitcnt vmcnt(0)",
        "s_branch 8f",
        "10:",
    ]
    L += program_shared8()
    L.append("s_branch 8f")
    if ALIGN:
        L.append(f".p2align {ALIGN}")
    L.append("9:")
    global SOFFS
    SOFFS = blocks_packed(L)
    L.append("8:")
    return L


def program_shared8():
    L = []
    if RUN:
        run_init(L)
    L += [
        f"s_mov_b64 s[{S_SRC}:{S_SRC + 1}], %[src]",
        f"s_mov_b64 s[{S_IDX}:{S_IDX + 1}], %[idx]",
        f"s_mov_b64 s[{S_DST}:{S_DST + 1}], %[dst]",
        f"s_mov_b32 s{S_INROW}, %[in_row]",
        f"s_mov_b32 s{S_OUTROW}, %[out_row]",
        f"s_mov_b32 s{S_CNT}, %[n_in]",
        f"s_sub_u32 s{S_NDMA}, %[n_in], 1",
        f"s_mov_b32 s{S_H}, %[half]",
        f"s_mov_b32 s{S_ROWS}, %[rows]",
        f"s_mov_b32 s{S_CONS}, %[cons]",
    ]
    if RUN:  # the wave's block-address stream start minus one row
        L += [f"s_sub_u32 s{S_IDXM}, s{S_IDX}, {STREAM_J_BYTES}", f"s_subb_u32 s{S_IDXM + 1}, s{S_IDX + 1}, 0"]
    L += [
        f"v_mov_b32 v{V_MASK[0]}, 0xaaaaaaaa",
        f"v_mov_b32 v{V_MASK[1]}, 0xcccccccc",
        f"v_mov_b32 v{V_MASK[2]}, 0xf0f0f0f0",
        f"s_mov_b32 s{S_LDSW}, %[ldsw]",
        f"s_cmp_lg_u32 s{S_CONS}, 0",
        "s_cbranch_scc1 22f",
    ]
    dmai = "global_load_lds_dwordx4 %[dmaoff], s[{0}:{1}]".format(S_SRC, S_SRC + 1)
    for slot in range(DMA8):  # builders: rows 0 .. DMA8 - 1 (clamped to the last row) into ring slots
        if slot:
            advance_run(L) if RUN else advance_s(L)
        L += [f"s_add_u32 m0, s{S_LDSW}, {slot * 4096}", "s_nop 0", dmai]
    L.append("22:")
    L.append(f"s_load_dwordx16 s[{S_ADDR[0]}:{S_ADDR[0] + 15}], s[{S_IDX}:{S_IDX + 1}], 0")
    if "s8nosmem" in DIAG:  # both address buffers once, reused for every row
        L.append(f"s_load_dwordx16 s[{S_ADDR[1]}:{S_ADDR[1] + 15}], s[{S_IDX}:{S_IDX + 1}], {STREAM_J_BYTES}")
    L += [f"v_mov_b32 v{r}, 0" for r in range(128)]
    L.append(f"v_mov_b32 v{OWN(0)}, 0")
    L += [f"s_waitcnt vmcnt({DMA8 - 1 - BAR8})", "s_barrier"]  # rows 0..BAR8 landed (consumers have no loads)
    L += [f"s_cmp_lg_u32 s{S_CONS}, 0", "s_cbranch_scc1 23f"]
    for x in range(2):  # rows 0, 1 into RB[0], RB[1]
        for hh in range(2):
            r = RB(x, 4 * hh)
            L.append(f"ds_read_b128 v[{r}:{r + 3}], %[ldsrg] offset:{x * 4096 + hh * 1024}")
    L.append("s_waitcnt lgkmcnt(0)")
    for r in range(BAR8):  # the sets of rows 0 .. BAR8 - 1; RB[BAR8 % 2] ends with row BAR8
        own_set(L, r % 2, r)
        if r + 2 <= BAR8:
            for hh in range(2):
                x = RB(r % 2, 4 * hh)
                L.append(f"ds_read_b128 v[{x}:{x + 3}], %[ldsrg] offset:{(r + 2) * 4096 + hh * 1024}")
        L.append("s_waitcnt lgkmcnt(0)")  # the set writes have read OWN; the staged row is in
    L += ["23:", "s_waitcnt lgkmcnt(0)"]
    unroll = lcm(BAR8, CSLOTS8, SLOTS8, 2)  # set slots, ring slots and the two RB / address buffers (12 at BAR8 = 3)
    if not RUN:
        L.append("1:")
        for j in range(unroll):
            body_s8(L, j)
            L += [f"s_cmp_eq_u32 s{S_CNT}, 0", "s_cbranch_scc1 3f" if j < unroll - 1 else "s_cbranch_scc0 1b"]
        L += ["3:", "s_waitcnt vmcnt(0) lgkmcnt(0)"]
        epilogue(L)
        return L
    # column runs (run_tail): ring slots, set slots and address buffers are positions of the unbroken
    # source-row stream, so the next tile continues with the body after the one its predecessor ended in
    run_tail(L, unroll, body_s8)
    return L


def epilogue(L):
    """Accumulator planes -> bytes (the same involution), into X, stored from there (memory dword d in X + d)."""
    for i in range(NT):
        L += [f"s_cmp_gt_u32 s{S_ROWS}, {i}", "s_cbranch_scc0 2f"]
        for g in range(2):
            transpose({p: ACC(i, g, p) for p in range(8)}, {d: V_X + d for d in range(8)}, L)
            for half in range(2):
                q = 2 * g + half
                off = f" offset:{q * 1024}" if q else ""
                if RUN and "rnostore" in DIAG:  # timing only: the column-run program without its tile stores
                    continue
                L.append(f"global_store_dwordx4 %[off], v[{V_X + 4 * half}:{V_X + 4 * half + 3}], "
                         f"s[{S_DST}:{S_DST + 1}]{off}")
        L += [f"s_add_u32 s{S_DST}, s{S_DST}, s{S_OUTROW}", f"s_addc_u32 s{S_DST + 1}, s{S_DST + 1}, 0"]
    L.append("2:")


def body_deep(L, j, slots):
    """body() with a deeper ring (the 1-wave program): `slots` ring slots, source rows j + 1 .. j + slots - 2 in
    flight while row j is used and row j + slots - 1 issued here; block-offset buffers alternate (j % 2)."""
    D = slots - 1
    slot = j % slots
    L.append(f"s_waitcnt vmcnt({(D - 1) * (4 // WAVES)})")  # this wave's DMAs of row j done
    if WAVES > 1:
        L.append("s_barrier")
    L.append(f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1")
    advance_s(L)
    dma(L, (j + D) % slots)  # row j + D into the slot row j - 1 used (read, and waited for, in body j - 1)
    for g in range(2):
        for h in range(2):
            q = 2 * g + h
            L.append(f"ds_read_b128 v[{RAW(g, 4 * h)}:{RAW(g, 4 * h) + 3}], %[ldsr] offset:{slot * 4096 + q * 1024}")
    L.append("s_waitcnt lgkmcnt(0)")
    for g in range(2):
        planes = {b: G(g, b // 4, 1 << (b % 4)) for b in range(8)}
        transpose({d: RAW(g, d) for d in range(8)}, planes, L)
    for g in range(2):
        for h in range(2):
            combos(g, h, L)
    cur, nxt = S_OFF[j % 2], S_OFF[(j + 1) % 2]
    L += [
        f"s_load_dwordx8 s[{nxt}:{nxt + 7}], s[{S_IDX}:{S_IDX + 1}], {STREAM_J_BYTES}",
        f"s_add_u32 s{S_IDX}, s{S_IDX}, {STREAM_J_BYTES}",
        f"s_addc_u32 s{S_IDX + 1}, s{S_IDX + 1}, 0",
        "s_set_gpr_idx_on 0, gpr_idx(SRC2,DST)",
    ]
    for i in range(NT):
        call(L, cur, i)
    L.append("s_set_gpr_idx_off")


def program(slots=SLOTS):
    """slots > 3: the deeper-ring form (body_deep); slots = 3: rows j + 1, j + 2 in flight (body)."""
    L = [
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
        f"s_getpc_b64 s[{S_BASE}:{S_BASE + 1}]",
        "5:",
        f"s_add_u32 s{S_BASE}, s{S_BASE}, (9f - 5b)",
        f"s_addc_u32 s{S_BASE + 1}, s{S_BASE + 1}, 0",
        f"s_mov_b32 s{S_LDSW}, %[ldsw]",
    ]
    if slots > 3:  # rows 0 .. slots - 2 on their way (the last row again past n_in), row 0's offsets
        L.append(f"s_sub_u32 s{S_NDMA}, %[n_in], 1")
        for r in range(slots - 1):
            if r:
                advance_s(L)
            dma(L, r)
        L.append(f"s_load_dwordx8 s[{S_OFF[0]}:{S_OFF[0] + 7}], s[{S_IDX}:{S_IDX + 1}], 0")
        L += [f"v_mov_b32 v{r}, 0" for r in range(128)]
        L += [f"v_mov_b32 {v(G(g, h, 0))}, 0" for g in range(2) for h in range(2)]
        unroll = slots if slots % 2 == 0 else 2 * slots
        loops(L, lambda LL, j: body_deep(LL, j, slots), unroll)
        epilogue(L)
        L.append("s_branch 8f")
        if ALIGN:
            L.append(f".p2align {ALIGN}")
        L.append("9:")
        blocks(L)
        L.append("8:")
        return L
    # prologue: rows 0 and 1 on their way into slots 0 and 1 (row 0 again when n_in == 1), row 0's offsets
    dma(L, 0)
    advance(L)
    dma(L, 1)
    L.append(f"s_load_dwordx8 s[{S_OFF[0]}:{S_OFF[0] + 7}], s[{S_IDX}:{S_IDX + 1}], 0")
    if "nosmem" in DIAG:
        L += [f"s_load_dwordx8 s[{S_OFF[b]}:{S_OFF[b] + 7}], s[{S_IDX}:{S_IDX + 1}], {b * STREAM_J_BYTES}"
              for b in (1, 2)]
        L.append("s_waitcnt lgkmcnt(0)")
    L += [f"v_mov_b32 v{r}, 0" for r in range(128)]
    L += [f"v_mov_b32 {v(G(g, h, 0))}, 0" for g in range(2) for h in range(2)]
    # loop over source rows j, three per trip (ring slot and offset buffer j % 3 are immediates)
    loops(L, body, 3)
    epilogue(L)
    L.append("s_branch 8f")
    if ALIGN:
        L.append(f".p2align {ALIGN}")
    L.append("9:")
    blocks(L)
    L.append("8:")
    return L


# ---- split 2-wave program (--w2split) ----------------------------------------------------------------------
# Tiles of <= 16 rows (many small objects: configs[0]'s 16 x 4 KiB): wave w owns byte group w of every lane (the 2 KiB
# half [2048 w, 2048 w + 2 KiB) of the column block) for ALL 16 rows, instead of both groups of 8 rows.  A wave then
# transposes and combines one group per source row instead of two (half the set building, which is ~20 % of the
# 2-wave program on configs[0]: profiles/r05_sets_ab.jsonl), and it reads only the half of the ring chunk it moved in by
# DMA itself, so the two waves never wait for each other (no barrier).  The price: 16 calls of 8 XOR3s per source row
# instead of 8 calls of 16.  Same block-offset stream as the 2-wave program (16 entries per source row, both waves read
# all 16), same 136-byte block stride (blocks half used).
SPLIT_NT = 16


def ACCS(i, p):  # row i (0..15), plane p of the wave's group
    return 8 * i + p


def GS(h, v):  # combination v of half h of the wave's group
    return 128 + 16 * h + v


def RAWS(d):
    return 160 + d


SPLIT_MAP = dict(TMP0=168, V_X=176, V_MASK=(184, 185, 186))
SPLIT_SGPRS = dict(S_OFF=(36, 52), S_SRC=68, S_IDX=70, S_DST=72, S_BASE=74, S_TGT=76, S_RET=78, S_INROW=80,
                   S_OUTROW=81, S_CNT=82, S_ROWS=83, S_T0=84, S_LDSW=85)


def call_split(L, cur, i):
    L += [f"s_mov_b32 m0, {hex(0xC000 | (8 * i))}", f"s_add_u32 s{S_TGT}, s{S_BASE}, s{cur + i}"]
    if not FAST:
        L.append(f"s_addc_u32 s{S_TGT + 1}, s{S_BASE + 1}, 0")
    L.append(f"s_swappc_b64 s[{S_RET}:{S_RET + 1}], s[{S_TGT}:{S_TGT + 1}]")


def body_split(L, j):
    """Source row j (ring slot j % 3, offset buffer j % 2): this wave's own DMA of it done, then its group's set."""
    slot = j % SLOTS
    L += [f"s_waitcnt vmcnt({4 // WAVES})",  # this wave's DMAs of row j done (row j + 1's may fly)
          f"s_sub_u32 s{S_CNT}, s{S_CNT}, 1"]
    advance(L)
    dma(L, (slot + 2) % SLOTS)  # row j + 2 into the slot row j - 1 used (read and waited for in row j - 1)
    for h in range(2):
        L.append(f"ds_read_b128 v[{RAWS(4 * h)}:{RAWS(4 * h) + 3}], %[ldsrg] offset:{slot * 4096 + h * 1024}")
    L.append("s_waitcnt lgkmcnt(0)")  # the chunk, and row j's block offsets (SMEM, issued a row earlier)
    transpose({d: RAWS(d) for d in range(8)}, {b: GS(b // 4, 1 << (b % 4)) for b in range(8)}, L)
    for h in range(2):
        b = lambda x: v(GS(h, x))
        L += [f"v_xor_b32 {b(x)}, {b(y)}, {b(z)}" for x, y, z in
              [(3, 1, 2), (5, 1, 4), (6, 2, 4), (7, 3, 4), (9, 1, 8), (10, 2, 8), (11, 3, 8), (12, 4, 8), (13, 5, 8),
               (14, 6, 8), (15, 7, 8)]]
    cur, nxt = S_OFF[j % 2], S_OFF[(j + 1) % 2]
    L += [f"s_load_dwordx16 s[{nxt}:{nxt + 15}], s[{S_IDX}:{S_IDX + 1}], {STREAM_J_BYTES}",
          f"s_add_u32 s{S_IDX}, s{S_IDX}, {STREAM_J_BYTES}",
          f"s_addc_u32 s{S_IDX + 1}, s{S_IDX + 1}, 0",
          "s_set_gpr_idx_on 0, gpr_idx(SRC2,DST)"]
    for i in range(SPLIT_NT):
        call_split(L, cur, i)
    L.append("s_set_gpr_idx_off")


def blocks_split(L):
    for c in range(256):
        lo, hi = block_indices(c)
        if c == 0:
            L.append(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
            L += ["s_nop 0"] * ((BLOCK_BYTES - 4) // 4)
            continue
        for o in range(8):
            a = ACCS(0, o)
            if lo[o] == 0 and hi[o] == 0:
                L += ["s_nop 0", "s_nop 0"]
                continue
            x = f"v{GS(0, lo[o])}" if lo[o] else "0"
            y = f"v{GS(1, hi[o])}" if hi[o] else "0"
            L.append(f"v_bitop3_b32 v{a}, {x}, {y}, v{a} bitop3:0x96")
        L.append(f"s_setpc_b64 s[{S_RET}:{S_RET + 1}]")
        L += ["s_nop 0"] * ((BLOCK_BYTES - (8 * 8 + 4)) // 4)


def epilogue_split(L):
    for i in range(SPLIT_NT):
        L += [f"s_cmp_gt_u32 s{S_ROWS}, {i}", "s_cbranch_scc0 2f"]
        transpose({p: ACCS(i, p) for p in range(8)}, {d: V_X + d for d in range(8)}, L)
        for half in range(2):
            off = f" offset:{half * 1024}" if half else ""
            L.append(f"global_store_dwordx4 %[off], v[{V_X + 4 * half}:{V_X + 4 * half + 3}], s[{S_DST}:{S_DST + 1}]{off}")
        L += [f"s_add_u32 s{S_DST}, s{S_DST}, s{S_OUTROW}", f"s_addc_u32 s{S_DST + 1}, s{S_DST + 1}, 0"]
    L.append("2:")


def program_split():
    assert WAVES == 2 and STREAM_J_BYTES == 4 * SPLIT_NT
    saved = {n: globals()[n] for n in list(SPLIT_MAP) + list(SPLIT_SGPRS)}
    globals().update(SPLIT_MAP)
    globals().update(SPLIT_SGPRS)
    try:
        L = [
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
            f"s_getpc_b64 s[{S_BASE}:{S_BASE + 1}]",
            "5:",
            f"s_add_u32 s{S_BASE}, s{S_BASE}, (9f - 5b)",
            f"s_addc_u32 s{S_BASE + 1}, s{S_BASE + 1}, 0",
            f"s_mov_b32 s{S_LDSW}, %[ldsw]",
        ]
        dma(L, 0)
        advance(L)
        dma(L, 1)
        L.append(f"s_load_dwordx16 s[{S_OFF[0]}:{S_OFF[0] + 15}], s[{S_IDX}:{S_IDX + 1}], 0")
        L += [f"v_mov_b32 v{r}, 0" for r in range(8 * SPLIT_NT)]
        L += [f"v_mov_b32 v{GS(h, 0)}, 0" for h in range(2)]
        loops(L, body_split, 6)  # lcm of the 3 ring slots and the 2 offset buffers
        epilogue_split(L)
        L.append("s_branch 8f")
        if ALIGN:
            L.append(f".p2align {ALIGN}")
        L.append("9:")
        blocks_split(L)
        L.append("8:")
        return L
    finally:
        globals().update(saved)


# cache-policy modifiers of the source DMA loads and the tile stores (--load-hint / --store-hint, A/B only; the
# default program carries none)
HINTS = {"load": "", "store": ""}


def hinted(lines):
    out = []
    for ln in lines:
        if HINTS["load"] and ln.startswith("global_load_lds_dwordx4"):
            ln += " " + HINTS["load"]
        if HINTS["store"] and ln.startswith("global_store_dwordx4"):
            ln += " " + HINTS["store"]
        out.append(ln)
    return out


def main():
    global BLOCK_BYTES, ALIGN, WAVES, WG_ROWS, STREAM_J_BYTES
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "bitslice_jump.inc"))
    ap.add_argument("--diag", default="", help="comma list: novm, inline, absinline (timing diagnostics, wrong results)")
    ap.add_argument("--stride", type=int, default=DEFAULT_STRIDE, help="bytes per code block (>= 132, multiple of 4)")
    ap.add_argument("--align", type=int, default=DEFAULT_ALIGN, help="log2 alignment of the block table")
    ap.add_argument("--prio8", default="4,1", help="K,L: 8-wave program's calls K.. of each row at s_setprio L (off)")
    ap.add_argument("--no-m0step", action="store_true", help="shared programs: M0 moved as a literal per call")
    ap.add_argument("--no-pack", action="store_true",
                    help="shared programs: fixed-stride XOR3-only blocks (A/B history: bsj_tile.hpp requires packed)")
    ap.add_argument("--prio", default="", help="K,L: shared program's calls K.. of each row at s_setprio L")
    ap.add_argument("--load-hint", default="", help="cache-policy modifiers of the DMA loads, e.g. 'nt' (A/B)")
    # 5 slots (4 rows in flight) measured equal to 3 on the 8-row ragged recode of scripts/ragged_rate.py
    # (0.2228 / 0.2205 ms against 0.2188 / 0.2233, profiles/r04_ragged_ab.txt): the 1-wave program is not waiting on
    # its source rows there
    ap.add_argument("--slots1", type=int, default=3, help="ring slots of the 1-wave program (3 = the 2-row form)")
    ap.add_argument("--slots2", type=int, default=3, help="ring slots of the 2-wave program (3 = the 2-row form)")
    ap.add_argument("--store-hint", default="", help="cache-policy modifiers of the tile stores, e.g. 'nt' (A/B)")
    # the 1- and 2-wave programs (<= 16 output rows: many small objects, HBM-bound) store non-temporally: configs[0]'s
    # 4,096 x 16 x 4 KiB encode 0.149 -> 0.142 ms, decode 0.179 -> 0.169 (profiles/r04_hint_cfg0_ab.txt); the 4- and
    # 8-wave programs keep plain stores (no gain on the VALU-bound bench, profiles/r02_cache_hint_ab.txt)
    ap.add_argument("--store-hint-small", default="nt", help="tile-store modifiers of the 1- and 2-wave programs")
    ap.add_argument("--w2split", action="store_true", help="2-wave program: waves split the byte groups, not the rows")
    ap.add_argument("--w4bar", type=int, default=0, choices=(0, 2, 3),
                    help="4-wave shared program in the 8-wave form with a barrier every N rows (0: every row)")
    ap.add_argument("--bar8", type=int, default=3, choices=(2, 3, 4), help="8-wave program: a barrier every N rows")
    ap.add_argument("--setregs", type=int, default=4, choices=(4, 8, 12),
                    help="set planes: entries of each set exchanged through LDS (4 = the planes only)")
    # the shipped split (profiles/r06_banks_r48_ab.txt): the 4-wave program exchanges the planes only, the 8-wave
    # program (four builders for eight waves) the planes and the first 4 composites
    ap.add_argument("--setregs4", type=int, default=0, choices=(0, 4, 8, 12),
                    help="--setregs of the 4-wave program (0: --setregs)")
    ap.add_argument("--setregs8", type=int, default=8, choices=(0, 4, 8, 12),
                    help="--setregs of the 8-wave program (0: --setregs)")
    ap.add_argument("--combo3", action="store_true", help="composite combinations as v_bitop3_b32 in every program (A/B)")
    ap.add_argument("--combo3-8", action="store_true", help="... in the 8-wave programs only")
    ap.add_argument("--banks", action="store_true",
                    help="set planes: the bank-conflict-free register map, sets exchanged by entry")
    ap.add_argument("--no-setplanes", action="store_true",
                    help="shared programs: exchange whole sets through LDS (the round-1..5 form) instead of planes only")
    args = ap.parse_args()
    HINTS["load"], HINTS["store"] = args.load_hint, args.store_hint
    global PRIO_AT
    if args.prio:
        PRIO_AT = None if args.prio == "off" else tuple(int(x) for x in args.prio.split(","))
    DIAG.update(x for x in args.diag.split(",") if x)
    global M0STEP
    M0STEP = not args.no_m0step
    global PACK
    PACK = not args.no_pack
    global COMBO3
    COMBO3 = args.combo3
    global SETPLANES, SET_WAIT, CS_SLOT, CS_SET, W4BAR, SETREGS
    if args.no_setplanes:
        SETPLANES, SET_WAIT = False, 6  # 2 staging reads + 4 set writes in flight
    else:  # set planes: a set slot holds the four sets' exchanged entries (4 x R x 256 B)
        global BANKS, SR_MAP
        BANKS = args.banks
        R4 = args.setregs4 or args.setregs
        R8 = args.setregs8 or args.setregs
        SR_MAP = max(R4, R8) > 4 or BANKS
        apply_setregs(R4)
    W4BAR = args.w4bar
    set_bar8(args.bar8)
    global PRIO8
    PRIO8 = None if args.prio8 == "off" else tuple(int(x) for x in args.prio8.split(","))
    assert args.stride >= BLOCK_BYTES and args.stride % 4 == 0
    BLOCK_BYTES, ALIGN = args.stride, args.align
    clob_v = ", ".join(f'"v{r}"' for r in range(LAST_VGPR_ALL + 1))
    clob_s = ", ".join(f'"s{r}"' for r in range(FIRST_SGPR, LAST_SGPR_ALL + 1))
    with open(args.out, "w") as f:
        f.write("// GENERATED by gen_bsjump.py -- do not edit.  Inner programs of gf_matmul_bsj_kernel<W> (kernels.hip),\n"
                "// W = 1, 2, 4 waves per workgroup (8 W output rows per tile).\n")
        f.write(f"#define RLNC_BSJ_NT {NT}\n")
        f.write(f"#define RLNC_BSJ_SLOTS {SLOTS}\n")
        f.write(f"#define RLNC_BSJ_BLOCK_BYTES {BLOCK_BYTES}\n")
        f.write(f"#define RLNC_BSJ_SLOTS1 {args.slots1}\n")
        f.write(f"#define RLNC_BSJ_SLOTS2 {args.slots2}\n")
        if args.w2split:
            f.write("#define RLNC_BSJ_W2SPLIT 1\n")
        for w in (1, 2, 4):
            WAVES, WG_ROWS = w, NT * w
            STREAM_J_BYTES = WG_ROWS * 4
            saved = HINTS["store"]
            if w <= 2 and not HINTS["store"]:
                HINTS["store"] = args.store_hint_small
            if w == 2 and args.w2split:
                body_txt = "\\n\\t".join(hinted(program_split()))
            else:
                body_txt = "\\n\\t".join(hinted(program({1: args.slots1, 2: args.slots2}.get(w, SLOTS))))
            HINTS["store"] = saved
            f.write(f'#define RLNC_BSJ_ASM_W{w} "{body_txt}"\n')
        WAVES, WG_ROWS = 4, NT * 4
        STREAM_J_BYTES = WG_ROWS * 8  # 64-bit block addresses
        if W4BAR:
            set_bar8(W4BAR)
        body_txt = "\\n\\t".join(hinted(program_shared()))
        f.write(f'#define RLNC_BSJ_ASM_W4S "{body_txt}"\n')
        f.write(f"#define RLNC_BSJ_SLOTS4S {SLOTS8 if W4BAR else SLOTS}\n")
        f.write(f"#define RLNC_BSJ_CSET_BYTES {(CSLOTS8 if W4BAR else 2) * CS_SLOT}\n")
        f.write(f"#define RLNC_BSJ_CS_SET {CS_SET}\n")
        f.write(f"#define RLNC_BSJ_CS_BASE2 {cs_base2()}\n")
        set_bar8(args.bar8)
        if SETPLANES:
            apply_setregs(R8)
        if args.combo3_8:
            COMBO3 = True
        WAVES, WG_ROWS = 8, NT * 8
        STREAM_J_BYTES = WG_ROWS * 8
        body_txt = "\\n\\t".join(hinted(program_shared(cons=True)))
        f.write(f'#define RLNC_BSJ_ASM_W8S "{body_txt}"\n')
        global RUN
        RUN = True
        body_txt = "\\n\\t".join(hinted(program_shared(cons=True)))
        RUN = False
        f.write(f'#define RLNC_BSJ_ASM_W8R "{body_txt}"\n')
        f.write(f"#define RLNC_BSJ_SLOTS8 {SLOTS8}\n")
        if SOFFS is not None:  # block offsets of the shared programs' packed table (bsj_offset_kernel<true>)
            f.write("#define RLNC_BSJ_SOFFSETS {" + ", ".join(str(x) for x in SOFFS) + "}\n")
        f.write(f"#define RLNC_BSJ_CSET_BYTES8 {CSLOTS8 * CS_SLOT}\n")
        f.write(f"#define RLNC_BSJ_CS_SET8 {CS_SET}\n")
        f.write(f"#define RLNC_BSJ_CS_BASE2_8 {cs_base2()}\n")
        f.write(f"#define RLNC_BSJ_CLOBBER_V {clob_v}\n")
        f.write(f'#define RLNC_BSJ_CLOBBER_S {clob_s}, "m0", "scc", "memory"\n')


if __name__ == "__main__":
    main()
