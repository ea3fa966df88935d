"""GPU parity: librlnc_hip (through the C ABI) against the oracle and the committed golden vectors.

Bit-exact for every byte (GF(2^8) is integer work; no tolerance).
"""
import numpy as np
import pytest

from oracle import np_oracle as npo
from oracle.oracle import OracleDecoder
from tests.conftest import hexarr
from tests.gpu_util import AB_BUILD, MUL, decode_paths, dev, host, np_matmul, variants

pytestmark = pytest.mark.gpu

DEFAULT_VARIANT = 8  # rlnc_context default (bit-sliced jump with shared combinations, 8-wave tiles above 32 rows)

S = ["Ok", "CodingVectorLengthMismatch", "DataLengthMismatch", "PieceCountZero", "DataLengthZero",
     "PieceLengthZero", "NotEnoughPiecesToRecode", "PieceLengthTooShort", "PieceNotUseful", "ReceivedAllPieces",
     "NotAllPiecesReceivedYet", "InvalidDecodedDataFormat", "InvalidPieceLength", "InvalidOutputBuffer"]


@pytest.fixture(scope="module")
def ctx():
    import torch

    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    import rlnc_amd

    c = rlnc_amd.Context(0)
    yield c
    c.set_kernel_variant(DEFAULT_VARIANT, 0)


# ------------------------------------------------------------------------------------------------
# L1 primitives (simd/mod.rs:18-119): all scalars incl. the 0/1 early-outs, aligned and unaligned
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n,off", [(1, 0), (15, 0), (16, 0), (17, 3), (1000, 1), (4096, 0), (65537, 5),
                                   (1 << 20, 0)])
def test_primitives(ctx, n, off):
    import torch
    from rlnc_amd import batch

    rng = np.random.default_rng(n + off)
    a = rng.integers(0, 256, n, dtype=np.uint8)
    b = rng.integers(0, 256, n, dtype=np.uint8)
    for c in [0, 1, 2, 0x53, 0x80, 0xFF]:
        ta = torch.zeros(n + off, dtype=torch.uint8, device="cuda:0")
        tb = torch.zeros(n + off, dtype=torch.uint8, device="cuda:0")
        ta[off:] = dev(a)
        tb[off:] = dev(b)
        va, vb = ta[off:], tb[off:]
        batch.mul_vec_by_scalar(va, c, ctx)
        assert np.array_equal(host(va), MUL[c][a]), c
        ta[off:] = dev(a)
        batch.mul_vec_by_scalar_then_add_into_vec(vb, va, c, ctx)
        assert np.array_equal(host(vb), b ^ MUL[c][a]), c
        tb[off:] = dev(b)
        batch.add_vectors(vb, va, ctx)
        assert np.array_equal(host(vb), a ^ b)


# ------------------------------------------------------------------------------------------------
# the matrix operator: shapes around every tile/row/column boundary, both kernel variants
# ------------------------------------------------------------------------------------------------
SHAPES = [(1, 1, 1, 1), (1, 3, 17, 1), (2, 2, 16, 2), (3, 5, 4095, 1), (4, 32, 4096, 2), (5, 33, 4097, 1),
          (8, 7, 100, 3), (16, 16, 8192, 1), (17, 31, 5000, 2), (32, 32, 12288, 1), (33, 64, 4096, 1),
          (64, 32, 4096 * 3 + 48, 1), (70, 65, 333, 2), (16, 32, 8192 * 2, 2), (24, 9, 8192 + 4096 + 16, 1),
          (9, 40, 32768, 1), (1, 32, 8192 + 16, 2), (2, 7, 4096, 1), (3, 33, 12288 + 48, 2), (1, 70, 4096 * 5, 1)]


@pytest.mark.parametrize("variant", variants(0, 1, 2, 3, 4, 5, 6, 7, 8, 9))
@pytest.mark.parametrize("n_out,n_in,W,nobj", SHAPES)
def test_matmul(ctx, variant, n_out, n_in, W, nobj):
    from rlnc_amd import batch

    rng = np.random.default_rng(n_out * 1000 + n_in * 10 + W + nobj)
    coef = rng.integers(0, 256, (nobj, n_out, n_in), dtype=np.uint8)
    coef[:, 0, :] = 1
    if n_out > 1:
        coef[:, 1, ::2] = 0
    inp = rng.integers(0, 256, (nobj, n_in, W), dtype=np.uint8)
    out = dev(np.zeros((nobj, n_out, W), np.uint8))
    ctx.set_kernel_variant(variant, 0)
    try:
        batch.matmul(dev(coef), dev(inp), out, ctx)
        got = host(out)
    finally:
        ctx.set_kernel_variant(DEFAULT_VARIANT, 0)
    for o in range(nobj):
        assert np.array_equal(got[o], np_matmul(coef[o], inp[o])), o


# the bit-sliced kernel takes whole 16 KiB column blocks of >= 4 output rows (8-row tiles, zero-padded
# index stream for a partial last tile); shapes around those boundaries, ragged tails to the perm kernel
BS_SHAPES = [(4, 1, 16384, 1), (5, 2, 16384 + 16, 2), (8, 32, 32768, 1), (9, 31, 16384 * 3 + 4096 + 7, 1),
             (16, 33, 16384 * 2, 3), (64, 32, 16384 * 2 + 48, 1), (32, 100, 16384, 2), (13, 7, 65536 + 5, 1),
             (3, 5, 16384, 1)]


@pytest.mark.parametrize("variant", variants(5, 6, 7, 8, 9))
@pytest.mark.parametrize("n_out,n_in,W,nobj", BS_SHAPES)
def test_matmul_bitsliced(ctx, variant, n_out, n_in, W, nobj):
    from rlnc_amd import batch

    rng = np.random.default_rng(n_out * 7 + n_in * 3 + W + nobj)
    coef = rng.integers(0, 256, (nobj, n_out, n_in), dtype=np.uint8)
    coef[:, 0, :] = 1
    coef[:, -1, :3] = [0, 2, 0x80][: min(3, n_in)]
    inp = rng.integers(0, 256, (nobj, n_in, W), dtype=np.uint8)
    inp[:, 0, :256] = np.arange(256, dtype=np.uint8)  # every byte value against every coefficient row
    out = dev(np.zeros((nobj, n_out, W), np.uint8))
    ctx.set_kernel_variant(variant, 0)
    try:
        batch.matmul(dev(coef), dev(inp), out, ctx)
        got = host(out)
    finally:
        ctx.set_kernel_variant(DEFAULT_VARIANT, 0)
    for o in range(nobj):
        assert np.array_equal(got[o], np_matmul(coef[o], inp[o])), o


# variant 8: 64-row tiles of 8 waves above 32 output rows (waves 4-7 read the sets built by waves 0-3)
W8_SHAPES = [(33, 32, 4096, 1), (64, 32, 8192, 2), (65, 3, 4096 * 3 + 17, 1), (100, 17, 8192, 2), (128, 128, 4096, 1),
             (40, 1, 4096, 3), (64, 64, 4096 * 4, 1)]


@pytest.mark.parametrize("n_out,n_in,W,nobj", W8_SHAPES)
def test_matmul_eight_wave_tiles(ctx, n_out, n_in, W, nobj):
    from rlnc_amd import batch

    rng = np.random.default_rng(n_out * 11 + n_in * 5 + W + nobj)
    coef = rng.integers(0, 256, (nobj, n_out, n_in), dtype=np.uint8)
    coef[:, 0, :] = 1
    coef[:, -1, :] = 0
    coef[:, 33 % n_out, : min(3, n_in)] = [0, 2, 0x80][: min(3, n_in)]
    inp = rng.integers(0, 256, (nobj, n_in, W), dtype=np.uint8)
    inp[:, 0, :256] = np.arange(256, dtype=np.uint8)
    out = dev(np.zeros((nobj, n_out, W), np.uint8))
    ctx.set_kernel_variant(8, 0)
    try:
        batch.matmul(dev(coef), dev(inp), out, ctx)
        got = host(out)
    finally:
        ctx.set_kernel_variant(DEFAULT_VARIANT, 0)
    for o in range(nobj):
        assert np.array_equal(got[o], np_matmul(coef[o], inp[o])), o


# variant 9: column runs (a workgroup walks `run` column blocks with its source-row stream unbroken); forced run
# lengths against ragged runs, fewer sources than the DMA depth (the stream crosses several tiles at once), source
# counts off the 12-row unroll, partial row tiles and the ragged byte tail
# (17-32 output rows: the 4-wave run program)
RUN_SHAPES = [(64, 32, 4096 * 5, 2), (33, 1, 4096 * 7 + 17, 1), (70, 2, 4096 * 4, 2), (40, 3, 4096 * 9, 1),
              (100, 13, 4096 * 6 + 48, 1), (128, 25, 4096 * 3, 2), (64, 12, 4096 * 8, 1), (65, 7, 4096 * 5, 3),
              (32, 32, 4096 * 5, 2), (17, 1, 4096 * 7 + 17, 1), (24, 2, 4096 * 4, 2), (20, 5, 4096 * 9, 1),
              (32, 13, 4096 * 6 + 48, 1), (30, 7, 4096 * 3, 3),
              # guided runs need 8 | run units and run | column blocks (whole runs first, single blocks last)
              (64, 32, 4096 * 8, 8), (70, 5, 4096 * 4, 4), (128, 25, 4096 * 6 + 48, 4), (64, 3, 4096 * 16, 4)]


@pytest.mark.skipif(not AB_BUILD, reason="variant 9 (column runs) is in the diagnostic A/B build only")
@pytest.mark.parametrize("run", [0, 1, 2, 3, 8])
@pytest.mark.parametrize("n_out,n_in,W,nobj", RUN_SHAPES)
def test_matmul_column_runs(ctx, run, n_out, n_in, W, nobj):
    from rlnc_amd import batch

    rng = np.random.default_rng(n_out * 13 + n_in * 7 + W + nobj + run)
    coef = rng.integers(0, 256, (nobj, n_out, n_in), dtype=np.uint8)
    coef[:, 0, :] = 1
    coef[:, -1, :] = 0
    inp = rng.integers(0, 256, (nobj, n_in, W), dtype=np.uint8)
    inp[:, 0, :256] = np.arange(256, dtype=np.uint8)
    out = dev(np.zeros((nobj, n_out, W), np.uint8))
    ctx.set_kernel_variant(9, 0)
    ctx.set_column_run(run)
    try:
        batch.matmul(dev(coef), dev(inp), out, ctx)
        got = host(out)
    finally:
        ctx.set_kernel_variant(DEFAULT_VARIANT, 0)
        ctx.set_column_run(0)
    for o in range(nobj):
        assert np.array_equal(got[o], np_matmul(coef[o], inp[o])), o


def test_matmul_every_coefficient_eight_waves(ctx):
    """All 256 coefficients in a 64-row tile (64 rows x 4 sources), each against every byte value."""
    from rlnc_amd import batch

    rng = np.random.default_rng(257)
    coef = np.arange(256, dtype=np.uint8).reshape(1, 64, 4)
    inp = rng.integers(0, 256, (1, 4, 8192), dtype=np.uint8)
    inp[0, :, :256] = np.arange(256, dtype=np.uint8)
    out = dev(np.zeros((1, 64, 8192), np.uint8))
    ctx.set_kernel_variant(8, 0)
    try:
        batch.matmul(dev(coef), dev(inp), out, ctx)
        got = host(out)
    finally:
        ctx.set_kernel_variant(DEFAULT_VARIANT, 0)
    assert np.array_equal(got[0], np_matmul(coef[0], inp[0]))


@pytest.mark.parametrize("variant", variants(5, 6, 7))
def test_matmul_every_coefficient(ctx, variant):
    """All 256 coefficients (16 rows x 16 sources = 0..255) against every byte value: each of the jump
    variant's 256 code blocks, and every index pattern of the relative-XOR variant."""
    from rlnc_amd import batch

    rng = np.random.default_rng(256)
    coef = np.arange(256, dtype=np.uint8).reshape(1, 16, 16)
    inp = rng.integers(0, 256, (1, 16, 16384), dtype=np.uint8)
    inp[0, :, :256] = np.arange(256, dtype=np.uint8)
    out = dev(np.zeros((1, 16, 16384), np.uint8))
    ctx.set_kernel_variant(variant, 0)
    try:
        batch.matmul(dev(coef), dev(inp), out, ctx)
        got = host(out)
    finally:
        ctx.set_kernel_variant(DEFAULT_VARIANT, 0)
    assert np.array_equal(got[0], np_matmul(coef[0], inp[0]))


@pytest.mark.parametrize("variant", variants(5, 6, 7, 8, 9))
@pytest.mark.parametrize("n_out", [12, 40, 70])
def test_matmul_bitsliced_strided_with_header(ctx, variant, n_out):
    """Padded row strides and the coded-piece header copy, through the raw C ABI descriptor; n_out > 32 reaches
    variant 8's 64-row, 8-wave tile (and its ragged second tile at 70)."""
    import ctypes as C

    import torch

    from rlnc_amd import _lib
    from rlnc_amd.errors import check

    rng = np.random.default_rng(5 + n_out)
    nobj, n_in, W, pad = 2, 20, 16384 * 2 + 32, 48
    hdr_w = n_in
    coef = rng.integers(0, 256, (nobj, n_out, n_in), dtype=np.uint8)
    inp = rng.integers(0, 256, (nobj, n_in, W + pad), dtype=np.uint8)
    pieces = dev(np.zeros((nobj, n_out, 64 + W + pad), np.uint8))  # [header (64 B slot) | data | pad]
    dcoef, dinp = dev(coef), dev(inp)
    base = pieces.data_ptr()
    row = 64 + W + pad
    d = _lib.MatmulDesc(dinp.data_ptr(), n_in * (W + pad), W + pad, dcoef.data_ptr(), n_out * n_in, n_in,
                        base + 64, n_out * row, row, base, n_out * row, row, n_out, n_in, W, nobj)
    ctx.set_kernel_variant(variant, 0)
    try:
        check(ctx.lib.rlnc_gf256_matmul(ctx.h, C.byref(d)), ctx.lib)
        torch.cuda.synchronize()
        got = host(pieces)
    finally:
        ctx.set_kernel_variant(DEFAULT_VARIANT, 0)
    for o in range(nobj):
        assert np.array_equal(got[o, :, :hdr_w], coef[o])
        assert np.array_equal(got[o, :, 64:64 + W], np_matmul(coef[o], inp[o, :, :W]))
        assert not got[o, :, 64 + W:].any() and not got[o, :, hdr_w:64].any()


@pytest.mark.parametrize("tile", [1, 2, 4, 8, 16, 32])
def test_matmul_tile_caps(ctx, tile):
    from rlnc_amd import batch

    rng = np.random.default_rng(tile)
    coef = rng.integers(0, 256, (1, 40, 12), dtype=np.uint8)
    inp = rng.integers(0, 256, (1, 12, 4096 + 16), dtype=np.uint8)
    out = dev(np.zeros((1, 40, 4096 + 16), np.uint8))
    ctx.set_kernel_variant(0, tile)
    try:
        batch.matmul(dev(coef), dev(inp), out, ctx)
        got = host(out)
    finally:
        ctx.set_kernel_variant(DEFAULT_VARIANT, 0)
    assert np.array_equal(got[0], np_matmul(coef[0], inp[0]))


# ------------------------------------------------------------------------------------------------
# golden vectors through the object API (rlnc::full mirror → C ABI)
# ------------------------------------------------------------------------------------------------
def test_golden_encode(ctx, golden):
    from rlnc_amd.full import Encoder

    for v in golden["encode"]:
        k, L, n = v["k"], v["L"], v["n"]
        enc = Encoder.without_padding(hexarr(v["src"]), k, ctx=ctx)
        co = hexarr(v["coeffs"]).reshape(n, k)
        want = hexarr(v["out"]).reshape(n, k + L)
        for i in range(n):
            full = np.zeros(k + L, np.uint8)

            class R:  # the "rng" hands out the committed coefficient row
                def fill_bytes(self, m, row=co[i]):
                    return row[:m].tobytes()

            enc.code_with_buf(R(), full)
            assert np.array_equal(full, want[i]), (k, L, i)


def test_golden_pad(ctx, golden):
    from rlnc_amd.full import Encoder

    for v in golden["pad"]:
        k, L = v["k"], v["L"]
        enc = Encoder.new(hexarr(v["data"]), k, ctx=ctx)
        assert enc.get_piece_byte_len() == L and enc.get_full_coded_piece_byte_len() == k + L
        rows = []
        for i in range(k):  # unit coding vectors read the padded pieces back
            out = np.zeros(L, np.uint8)
            cv = np.zeros(k, np.uint8)
            cv[i] = 1
            enc.code_with_coding_vector(cv, out)
            rows.append(out)
        assert np.concatenate(rows).tobytes().hex() == v["padded"]


def test_golden_recode(ctx, golden):
    from rlnc_amd.full import Recoder

    for v in golden["recode"]:
        k, L, n = v["k"], v["L"], v["n"]
        rec = Recoder.new(hexarr(v["pieces"]), k + L, k, ctx=ctx)
        assert rec.get_num_pieces_recoded_together() == n and rec.get_piece_byte_len() == L
        out = np.zeros(k + L, np.uint8)
        rec.recode_with_coding_vector(hexarr(v["r"]), out)
        assert out.tobytes().hex() == v["out"]


def test_golden_decode_object_api(ctx, golden):
    from rlnc_amd.full import Decoder
    from rlnc_amd.errors import RLNCError

    for v in golden["decode"]:
        d = Decoder.new(v["L"], v["k"], ctx=ctx)
        sts = []
        for p in v["pieces"]:
            try:
                d.decode(hexarr(p))
                sts.append("Ok")
            except RLNCError as e:
                sts.append(e.name)
        assert sts == v["statuses"], v["name"]
        try:
            data = d.get_decoded_data()
            assert v["final_status"] == "Ok" and data.tobytes().hex() == v["data"], v["name"]
        except RLNCError as e:
            assert e.name == v["final_status"], v["name"]


@pytest.mark.parametrize("path", decode_paths(1, 2, 3, 4, 5, 6))
def test_golden_decode_batch(ctx, golden, path):
    from rlnc_amd import batch

    ctx.set_decode_path(path)
    for v in golden["decode"]:
        k, L = v["k"], v["L"]
        ps = [hexarr(p) for p in v["pieces"]]
        if any(p.size != k + L for p in ps):
            continue
        pieces = dev(np.stack(ps)[None])
        decoded = dev(np.zeros((1, k, L), np.uint8))
        pst, ost, dl = batch.decode_batch(pieces, k, decoded, ctx)
        assert [S[s] for s in pst[0]] == v["statuses"], v["name"]
        got = host(decoded)[0]
        assert got[: v["rows"]].tobytes().hex() == v["payload"], v["name"]
        assert S[ost[0]] == v["final_status"], v["name"]
        if v["final_status"] == "Ok":
            assert got.reshape(-1)[: dl[0]].tobytes().hex() == v["data"]
    ctx.set_decode_path(0)


def _sequences(rng, nobj, k, m, L, sparsity, dep_frac):
    """nobj piece sequences: random coefficient vectors (a fraction zeroed), some pieces replaced by
    combinations of earlier ones (dependent), random data bytes."""
    seqs = np.zeros((nobj, m, k + L), np.uint8)
    for o in range(nobj):
        for p in range(m):
            if p >= 2 and rng.random() < dep_frac:
                a, b = rng.integers(0, p, 2)
                c = int(rng.integers(0, 256))
                seqs[o, p] = seqs[o, a] ^ MUL[c][seqs[o, b]]
            else:
                cv = rng.integers(0, 256, k, dtype=np.uint8)
                cv[rng.random(k) < sparsity] = 0
                seqs[o, p, :k] = cv
                seqs[o, p, k:] = rng.integers(0, 256, L, dtype=np.uint8)
    return seqs


@pytest.mark.parametrize("path", decode_paths(1, 2, 3, 4, 5, 6))
@pytest.mark.parametrize("k,m,L,sparsity,dep", [(32, 32, 40, 0.0, 0.0), (64, 64, 24, 0.0, 0.1), (128, 128, 20, 0.0, 0.0),
                                                (100, 120, 9, 0.0, 0.1), (120, 128, 16, 0.9, 0.02),
                                                (48, 56, 10, 0.4, 0.1), (64, 70, 9, 0.85, 0.05), (8, 14, 5, 0.7, 0.1), (8, 12, 33, 0.9, 0.0), (32, 40, 64, 0.0, 0.2),
                                                (32, 36, 16, 0.6, 0.1), (17, 30, 7, 0.5, 0.2), (70, 80, 16, 0.3, 0.05),
                                                (1, 3, 4, 0.5, 0.0), (128, 130, 16, 0.0, 0.02),
                                                (16, 300, 8, 0.2, 0.1), (100, 170, 12, 0.8, 0.1)])
def test_decode_batch_vs_oracle_sequences(ctx, path, k, m, L, sparsity, dep):
    """Device (and host) elimination: every decode() status, the rank and the padded payload rows equal the
    oracle's full-row RREF, for dense, sparse (diagonal-pivot quirk) and dependent pieces."""
    from rlnc_amd import batch

    from rlnc_amd.errors import RLNCError

    rng = np.random.default_rng(k * 1000 + m + int(100 * sparsity))
    nobj = 12
    seqs = _sequences(rng, nobj, k, m, L, sparsity, dep)
    decoded = dev(np.zeros((nobj, k, L), np.uint8))
    ctx.set_decode_path(path)
    try:
        if path == 5 and k + m > 256:  # the blocked run does not apply: an error, not another kernel
            with pytest.raises(RLNCError) as ei:
                batch.decode_batch(dev(seqs), k, decoded, ctx)
            assert ei.value == RLNCError.InvalidArgument
            return
        pst, ost, dl = batch.decode_batch(dev(seqs), k, decoded, ctx)
    finally:
        ctx.set_decode_path(0)
    got = host(decoded)
    for o in range(nobj):
        od = OracleDecoder(L, k)
        want = [S[od.decode(p)] for p in seqs[o]]
        assert [S[x] for x in pst[o]] == want, (o, [S[x] for x in pst[o]], want)
        pay = od.padded_payload()
        assert np.array_equal(got[o, : pay.shape[0]], pay), o
        assert not got[o, pay.shape[0]:].any()
        st, data = od.get_decoded_data()
        assert S[ost[o]] == S[st], o
        if st == 0:
            assert int(dl[o]) == data.size


@pytest.mark.parametrize("k,m,sparsity,dep", [(32, 48, 0.5, 0.05), (64, 64, 0.3, 0.02), (16, 40, 0.6, 0.1),
                                               (128, 128, 0.05, 0.0), (48, 64, 0.8, 0.0), (96, 100, 0.2, 0.05),
                                               (32, 20, 0.0, 0.0), (64, 40, 0.3, 0.1), (128, 100, 0.5, 0.0)])
def test_decode_blocked_path_stress(ctx, k, m, sparsity, dep):
    """The blocked elimination (path 5) against the oracle on 64 objects per shape: sparse coefficients drive the
    matrix in and out of the clean state (zero pivots, kept dirty rows, prefix re-extension, the many-dirty-rows
    fallback), dependent pieces hit PieceNotUseful; statuses, rank and payload rows must all match."""
    from rlnc_amd import batch

    rng = np.random.default_rng(5000 + k * 7 + m)
    nobj, L = 64, 8
    seqs = _sequences(rng, nobj, k, m, L, sparsity, dep)
    decoded = dev(np.zeros((nobj, k, L), np.uint8))
    ctx.set_decode_path(5)
    try:
        pst, ost, dl = batch.decode_batch(dev(seqs), k, decoded, ctx)
    finally:
        ctx.set_decode_path(0)
    got = host(decoded)
    for o in range(nobj):
        od = OracleDecoder(L, k)
        want = [S[od.decode(p)] for p in seqs[o]]
        assert [S[x] for x in pst[o]] == want, (o, [S[x] for x in pst[o]], want)
        pay = od.padded_payload()
        assert np.array_equal(got[o, : pay.shape[0]], pay), o
        assert not got[o, pay.shape[0]:].any()


def test_decode_batch_many_objects(ctx):
    """160 objects in one batch decode (one elimination launch of 160 workgroups, one product); every object's
    statuses, payload rows and final status against the oracle."""
    from rlnc_amd import batch

    rng = np.random.default_rng(160)
    nobj, k, m, L = 160, 16, 20, 64
    seqs = _sequences(rng, nobj, k, m, L, 0.2, 0.1)
    decoded = dev(np.zeros((nobj, k, L), np.uint8))
    pst, ost, dl = batch.decode_batch(dev(seqs), k, decoded, ctx)
    got = host(decoded)
    for o in range(nobj):
        od = OracleDecoder(L, k)
        want = [S[od.decode(p)] for p in seqs[o]]
        assert [S[x] for x in pst[o]] == want, o
        pay = od.padded_payload()
        assert np.array_equal(got[o, : pay.shape[0]], pay), o
        st, data = od.get_decoded_data()
        assert S[ost[o]] == S[st], o


def test_decode_batch_device_async_outputs(ctx, orc):
    import torch

    from rlnc_amd import batch

    k, L, nobj, m = 32, 4096, 6, 34
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, (nobj, k * L - 1), dtype=np.uint8)
    src = np.stack([orc.pad(d, k) for d in data])
    pieces = np.stack([orc.encode(src[o], rng.integers(0, 256, (m, k), dtype=np.uint8)) for o in range(nobj)])
    decoded = torch.zeros((nobj, k, L), dtype=torch.uint8, device="cuda:0")
    ps = torch.zeros((nobj, m), dtype=torch.int32, device="cuda:0")
    os_ = torch.zeros(nobj, dtype=torch.int32, device="cuda:0")
    dl = torch.zeros(nobj, dtype=torch.int64, device="cuda:0")
    batch.decode_batch_device(dev(pieces), k, decoded, ps, os_, dl, ctx)
    torch.cuda.synchronize()
    for o in range(nobj):
        od = OracleDecoder(L, k)
        assert ps[o].cpu().tolist() == [od.decode(p) for p in pieces[o]]
        if int(os_[o]) == 0:
            assert int(dl[o]) == data[o].size
            assert np.array_equal(decoded[o].cpu().numpy().reshape(-1)[: data[o].size], data[o])


@pytest.mark.parametrize("k,L,n,m,dep", [(32, 4096 * 3 + 16, 40, 32, 0.0), (16, 5000, 24, 20, 0.3), (64, 8192, 64, 64, 0.0)])
def test_split_encode_decode_pipeline(ctx, orc, k, L, n, m, dep):
    """encode_batch_headers + encode_batch_data == encode_batch, and decode_batch_eliminate on a second context /
    stream (ordered by HIP events) + decode_batch_apply == decode_batch_device, byte for byte (bench.py's
    pipelined step)."""
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    rng = np.random.default_rng(k * 7 + m)
    nobj = 5
    src = dev(rng.integers(0, 256, (nobj, k, L), dtype=np.uint8))
    co = rng.integers(0, 256, (nobj, n, k), dtype=np.uint8)
    for o in range(nobj):  # some dependent coding vectors: useless pieces and rank < k objects
        for p in range(2, m):
            if rng.random() < dep:
                co[o, p] = co[o, p - 1] ^ co[o, p - 2]
    co = dev(co)
    ref = torch.empty((nobj, n, k + L), dtype=torch.uint8, device="cuda:0")
    batch.encode_batch(src, co, ref, ctx)
    pieces = torch.zeros_like(ref)
    ctx2 = rlnc_amd.Context(0)
    side = torch.cuda.Stream()
    ev_h, ev_e = torch.cuda.Event(), torch.cuda.Event()
    T = torch.empty((nobj, k, m), dtype=torch.uint8, device="cuda:0")
    pst = torch.full((nobj, m), -1, dtype=torch.int32, device="cuda:0")
    rank = torch.empty(nobj, dtype=torch.int32, device="cuda:0")
    dec = torch.zeros((nobj, k, L), dtype=torch.uint8, device="cuda:0")
    ost = torch.empty(nobj, dtype=torch.int32, device="cuda:0")
    dl = torch.empty(nobj, dtype=torch.int64, device="cuda:0")
    batch.encode_batch_headers(co, pieces, ctx)
    ev_h.record()
    batch.encode_batch_data(src, co, pieces, ctx)
    with torch.cuda.stream(side):
        side.wait_event(ev_h)
        batch.decode_batch_eliminate(pieces[:, :m], k, T, pst, rank, ctx2)
        ev_e.record()
    torch.cuda.current_stream().wait_event(ev_e)
    batch.decode_batch_apply(pieces[:, :m], k, T, rank, dec, ost, dl, ctx)
    torch.cuda.synchronize()
    assert torch.equal(pieces, ref)
    want_dec = torch.zeros_like(dec)
    want_ps = torch.empty_like(pst)
    want_os = torch.empty_like(ost)
    want_dl = torch.empty_like(dl)
    batch.decode_batch_device(ref[:, :m], k, want_dec, want_ps, want_os, want_dl, ctx)
    torch.cuda.synchronize()
    assert torch.equal(pst, want_ps) and torch.equal(ost, want_os) and torch.equal(dec, want_dec)
    assert torch.equal(dl[ost == 0], want_dl[want_os == 0])
    assert torch.equal(rank, (pst == 0).sum(1).to(torch.int32))
    hs = host(src)
    for o in range(nobj):
        if int(rank[o]) == k:
            assert np.array_equal(host(dec)[o], hs[o]), o
    ctx2.close()


# ------------------------------------------------------------------------------------------------
# ports of src/full/tests.rs (round trips with random sizes, recoders, useless pieces)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("seed", range(4))
def test_prop_encoder_decoder(ctx, seed):
    # full/tests.rs:7-47
    from rlnc_amd.errors import RLNCError
    from rlnc_amd.full import Decoder, Encoder

    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, int(rng.integers(1 << 10, 1 << 16)), dtype=np.uint8)
    k = int(rng.integers(1 << 5, 1 << 8))
    enc = Encoder.new(data, k, ctx=ctx)
    dec = Decoder.new(enc.get_piece_byte_len(), enc.get_piece_count(), ctx=ctx)
    while True:
        try:
            dec.decode(enc.code(rng))
        except RLNCError as e:
            if e == RLNCError.ReceivedAllPieces:
                break
            assert e == RLNCError.PieceNotUseful
    assert dec.is_already_decoded()
    assert np.array_equal(dec.get_decoded_data(), data)


@pytest.mark.parametrize("seed", range(3))
def test_prop_encoder_recoder_decoder(ctx, seed):
    # full/tests.rs:49-119 (counts reduced)
    from rlnc_amd.errors import RLNCError
    from rlnc_amd.full import Decoder, Encoder, Recoder

    rng = np.random.default_rng(10 + seed)
    data = rng.integers(0, 256, int(rng.integers(1 << 10, 1 << 15)), dtype=np.uint8)
    k = int(rng.integers(1 << 5, 1 << 7))
    enc = Encoder.new(data, k, ctx=ctx)
    dec = Decoder.new(enc.get_piece_byte_len(), enc.get_piece_count(), ctx=ctx)
    done = False
    while not done:
        nrec = int(rng.integers(2, k))
        coded = np.concatenate([enc.code(rng) for _ in range(nrec)])
        rec = Recoder.new(coded, enc.get_full_coded_piece_byte_len(), enc.get_piece_count(), ctx=ctx)
        for _ in range(int(rng.integers(0, 2 * k))):
            try:
                dec.decode(rec.recode(rng))
            except RLNCError as e:
                if e == RLNCError.ReceivedAllPieces:
                    done = True
                    break
                assert e == RLNCError.PieceNotUseful
        if done:
            break
        try:
            dec.decode(enc.code(rng))
        except RLNCError as e:
            if e == RLNCError.ReceivedAllPieces:
                break
            assert e == RLNCError.PieceNotUseful
    assert np.array_equal(dec.get_decoded_data(), data)


@pytest.mark.parametrize("seed", range(3))
def test_prop_decoding_with_useless_pieces(ctx, seed):
    # full/tests.rs:121-203
    from rlnc_amd.errors import RLNCError
    from rlnc_amd.full import Decoder, Encoder, Recoder

    rng = np.random.default_rng(20 + seed)
    data = rng.integers(0, 256, int(rng.integers(1 << 10, 1 << 16)), dtype=np.uint8)
    k = int(rng.integers(1 << 5, 1 << 8))
    enc = Encoder.new(data, k, ctx=ctx)
    dec = Decoder.new(enc.get_piece_byte_len(), enc.get_piece_count(), ctx=ctx)
    seen = []
    for _ in range(k // 2):
        p = enc.code(rng)
        try:
            dec.decode(p)
            seen.append(p)
        except RLNCError as e:
            assert e == RLNCError.PieceNotUseful
    rec = Recoder.new(np.concatenate(seen), enc.get_full_coded_piece_byte_len(), enc.get_piece_count(), ctx=ctx)
    for _ in range(2 * len(seen)):
        with pytest.raises(RLNCError) as ei:
            dec.decode(rec.recode(rng))
        assert ei.value == RLNCError.PieceNotUseful
    while dec.get_remaining_piece_count() > 0:
        try:
            dec.decode(enc.code(rng))
        except RLNCError as e:
            assert e == RLNCError.PieceNotUseful
    assert np.array_equal(dec.get_decoded_data(), data)


# ------------------------------------------------------------------------------------------------
# BASELINE.json configs at full size, bit-exact against the C oracle
# ------------------------------------------------------------------------------------------------
def test_config2_encode_32x1MiB_to_64(ctx, orc):
    from rlnc_amd import batch

    k, L, n = 32, 1 << 20, 64
    rng = np.random.default_rng(0x524C4E43)
    src = rng.integers(0, 256, (1, k, L), dtype=np.uint8)
    co = rng.integers(0, 256, (1, n, k), dtype=np.uint8)
    out = dev(np.zeros((1, n, k + L), np.uint8))
    batch.encode_batch(dev(src), dev(co), out, ctx)
    got = host(out)[0]
    assert np.array_equal(got, orc.encode(src[0], co[0]))


def test_config3_decode_32x1MiB(ctx, orc):
    from rlnc_amd import batch

    k, L = 32, 1 << 20
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, k * L - 1, dtype=np.uint8)  # Encoder::new pads to exactly L = 2^20
    src = orc.pad(data, k)
    assert src.shape == (k, L)
    co = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
    coded = orc.encode(src, co)
    pieces = dev(coded[None])
    decoded = dev(np.zeros((1, k, L), np.uint8))
    pst, ost, dl = batch.decode_batch(pieces, k, decoded, ctx)
    od = OracleDecoder(L, k)
    want = [S[od.decode(p)] for p in coded]
    assert [S[s] for s in pst[0]] == want
    got = host(decoded)[0]
    assert np.array_equal(got, od.padded_payload())
    assert S[ost[0]] == "Ok" and int(dl[0]) == data.size
    assert np.array_equal(got.reshape(-1)[: data.size], data)


def test_config4_recode_64x256KiB(ctx, orc):
    from rlnc_amd import batch

    k, L, n, count = 64, 1 << 18, 64, 64
    rng = np.random.default_rng(4)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    pieces = orc.encode(src, rng.integers(0, 256, (n, k), dtype=np.uint8))
    r = rng.integers(0, 256, (1, count, n), dtype=np.uint8)
    out = dev(np.zeros((1, count, k + L), np.uint8))
    batch.recode_batch(dev(pieces[None]), dev(r), out, k, ctx)
    got = host(out)[0]
    for c in [0, 1, count - 1]:
        assert np.array_equal(got[c], orc.recode(pieces, k + L, k, r[0, c]))
    # all 64 at once against the independent numpy matmul on a column slice
    assert np.array_equal(got[:, :4096 + k], np_matmul(r[0], pieces[:, :4096 + k]))


def test_config5_batch_objects_k128_64KiB(ctx, orc):
    from rlnc_amd import batch

    k, L, nobj = 128, 1 << 16, 8
    rng = np.random.default_rng(5)
    src = rng.integers(0, 256, (nobj, k, L), dtype=np.uint8)
    co = rng.integers(0, 256, (nobj, k, k), dtype=np.uint8)
    pieces = dev(np.zeros((nobj, k, k + L), np.uint8))
    batch.encode_batch(dev(src), dev(co), pieces, ctx)
    hp = host(pieces)
    assert np.array_equal(hp[0], orc.encode(src[0], co[0]))
    decoded = dev(np.zeros((nobj, k, L), np.uint8))
    pst, ost, dl = batch.decode_batch(pieces, k, decoded, ctx)
    got = host(decoded)
    od = OracleDecoder(L, k)
    want = [S[od.decode(p)] for p in hp[1]]
    assert [S[s] for s in pst[1]] == want
    assert np.array_equal(got[1], od.padded_payload())
    for o in range(nobj):
        if (pst[o] == 0).sum() == k:  # full rank: decode must return the source rows
            assert np.array_equal(got[o], src[o])


# ------------------------------------------------------------------------------------------------
# large piece counts: k at and past 255/256 (the reference takes any piece_count, encoder.rs:85-106), full encode
# through the batch API, decode with the default path (k + m > 256: the round-1 device kernel, or the host
# elimination once [coeffs | E] outgrows LDS) and with the host elimination (path 1)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("k,extra,L", [(255, 3, 4096 + 16), (256, 4, 4096), (300, 8, 8192 + 48)])
@pytest.mark.parametrize("path", [0, 1])
def test_large_piece_counts(ctx, orc, k, extra, L, path):
    import torch

    from rlnc_amd import batch

    rng = np.random.default_rng(k * 31 + extra + path)
    nobj, n = 2, k + extra
    src = rng.integers(0, 256, (nobj, k, L), dtype=np.uint8)
    coeffs = rng.integers(0, 256, (nobj, n, k), dtype=np.uint8)
    coeffs[:, k, :] = coeffs[:, 0, :]  # a repeated coefficient vector: PieceNotUseful mid-sequence
    pieces = torch.zeros((nobj, n, k + L), dtype=torch.uint8, device="cuda:0")
    batch.encode_batch(dev(src), dev(coeffs), pieces, ctx)
    hp = host(pieces)
    for o in range(nobj):
        assert np.array_equal(hp[o], orc.encode(src[o], coeffs[o])), o
    decoded = dev(np.zeros((nobj, k, L), np.uint8))
    ctx.set_decode_path(path)
    try:
        pst, ost, dl = batch.decode_batch(pieces, k, decoded, ctx)
    finally:
        ctx.set_decode_path(0)
    got = host(decoded)
    for o in range(nobj):
        od = OracleDecoder(L, k)
        want = [S[od.decode(p)] for p in hp[o]]
        assert [S[x] for x in pst[o]] == want, o
        pay = od.padded_payload()
        assert np.array_equal(got[o, : pay.shape[0]], pay), o
        st, _ = od.get_decoded_data()
        assert S[ost[o]] == S[st], o
        if want.count("Ok") == k:
            assert np.array_equal(got[o], src[o]), o


@pytest.mark.parametrize("k,n,count", [(256, 260, 70), (300, 300, 33)])
def test_large_piece_count_recode(ctx, orc, k, n, count):
    """Recode of n coded pieces with k ≥ 256 (recoder.rs:122-153: the coefficient fold and the data combination
    as one linear map over the full pieces): every recoded piece against the oracle's recode."""
    import torch

    from rlnc_amd import batch

    rng = np.random.default_rng(k + n + count)
    L = 4096 + 32
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    pieces = orc.encode(src, rng.integers(0, 256, (n, k), dtype=np.uint8))
    r = rng.integers(0, 256, (1, count, n), dtype=np.uint8)
    out = torch.zeros((1, count, k + L), dtype=torch.uint8, device="cuda:0")
    batch.recode_batch(dev(pieces[None]), dev(r), out, k, ctx)
    got = host(out)[0]
    for c in range(count):
        assert np.array_equal(got[c], orc.recode(pieces, k + L, k, r[0, c])), c


@pytest.mark.parametrize("k,m,sparsity,dep,nobj", [(16, 16, 0.0, 0.0, 2048), (16, 24, 0.5, 0.1, 2051),
                                                  (8, 12, 0.7, 0.1, 2049), (16, 16, 0.3, 0.1, 6001),
                                                  (12, 20, 0.6, 0.2, 5000)])
def test_decode_many_small_objects(ctx, k, m, sparsity, dep, nobj):
    """>= 2,048 objects with k <= 16: the default path takes the multi-object kernel (rref.hip gf_rref_small_kernel,
    4 objects per workgroup: 2,049 and 2,051 leave the last workgroup part-empty; rows of <= 8 dwords on 8 lane
    groups, else 4; 5,000 and 6,001 objects: more than one round of waves); every object's statuses and payload rows
    against the oracle."""
    from rlnc_amd import batch

    rng = np.random.default_rng(2048 + k * 3 + m)
    L = 8
    seqs = _sequences(rng, nobj, k, m, L, sparsity, dep)
    decoded = dev(np.zeros((nobj, k, L), np.uint8))
    pst, ost, dl = batch.decode_batch(dev(seqs), k, decoded, ctx)
    got = host(decoded)
    for o in range(nobj):
        od = OracleDecoder(L, k)
        want = [S[od.decode(p)] for p in seqs[o]]
        assert [S[x] for x in pst[o]] == want, o
        pay = od.padded_payload()
        assert np.array_equal(got[o, : pay.shape[0]], pay), o
        st, _ = od.get_decoded_data()
        assert S[ost[o]] == S[st], o


@pytest.mark.parametrize("k,m,sparsity,dep,nobj,L", [(16, 16, 0.0, 0.0, 2048, 4096), (16, 24, 0.5, 0.1, 2051, 4096 + 40),
                                                    (8, 12, 0.7, 0.1, 2049, 8192)])
def test_decode_many_small_objects_block_products(ctx, k, m, sparsity, dep, nobj, L):
    """As above with whole 4 KiB column blocks: the T x data product takes the 1- / 2-wave bit-sliced program, whose
    block-offset stream the small-object elimination writes itself (engine.cpp decode_batch_device_impl, RrefParams::
    bsj_stream) -- rank-deficient and dependent objects included, a ragged tail after the blocks in one case."""
    from rlnc_amd import batch

    rng = np.random.default_rng(4096 + k * 5 + m)
    seqs = _sequences(rng, nobj, k, m, L, sparsity, dep)
    decoded = dev(np.zeros((nobj, k, L), np.uint8))
    pst, ost, dl = batch.decode_batch(dev(seqs), k, decoded, ctx)
    got = host(decoded)
    for o in range(nobj):
        od = OracleDecoder(L, k)
        want = [S[od.decode(p)] for p in seqs[o]]
        assert [S[x] for x in pst[o]] == want, o
        pay = od.padded_payload()
        assert np.array_equal(got[o, : pay.shape[0]], pay), o
        st, _ = od.get_decoded_data()
        assert S[ost[o]] == S[st], o


@pytest.mark.parametrize("path", [0, 2])
def test_decode_two_pass_beyond_one_wave_row(ctx, path):
    """k + m > 256 with k <= 128: the blocked run over the first 256 - k pieces, the general kernel only for objects
    not full-ranked within them (rref.hip launch_rref_batch).  Objects 0-3 reach rank k early (the later pieces are
    ReceivedAllPieces, T columns zero); objects 4-5 have their first 256 - k pieces spanning only 40 dimensions, so
    the general pass must redo them over all m pieces; object 6 never reaches rank k."""
    from rlnc_amd import batch

    from oracle.oracle import Oracle

    orc = Oracle()
    rng = np.random.default_rng(4242)
    k, m, L, nobj = 64, 230, 24, 7
    first = 256 - k
    seqs = np.zeros((nobj, m, k + L), np.uint8)
    for o in range(nobj):
        src = rng.integers(0, 256, (k, L), dtype=np.uint8)
        co = rng.integers(0, 256, (m, k), dtype=np.uint8)
        if o >= 4:
            base = rng.integers(0, 256, (40, k), dtype=np.uint8)
            co[:first] = orc.encode(base, rng.integers(0, 256, (first, 40), dtype=np.uint8))[:, 40:]
        if o == 6:
            co[first:] = orc.encode(co[:8], rng.integers(0, 256, (m - first, 8), dtype=np.uint8))[:, 8:]
        seqs[o] = orc.encode(src, co)
    decoded = dev(np.zeros((nobj, k, L), np.uint8))
    ctx.set_decode_path(path)
    try:
        pst, ost, dl = batch.decode_batch(dev(seqs), k, decoded, ctx)
    finally:
        ctx.set_decode_path(0)
    got = host(decoded)
    for o in range(nobj):
        od = OracleDecoder(L, k)
        want = [S[od.decode(p)] for p in seqs[o]]
        assert [S[x] for x in pst[o]] == want, o
        pay = od.padded_payload()
        assert np.array_equal(got[o, : pay.shape[0]], pay), o
        st, _ = od.get_decoded_data()
        assert S[ost[o]] == S[st], o
    assert all(S[x] == "ReceivedAllPieces" for x in pst[0, first:])
    assert (pst[4] == 0).sum() == k and (pst[6] == 0).sum() < k


@pytest.mark.parametrize("variant", [8, 7, 6])
@pytest.mark.parametrize("k,L,n", [(32, 4096 * 2, 64), (32, 4096 * 3 + 17, 40), (16, 8192, 12), (8, 4096, 2),
                                   (20, 3000, 24)])
def test_encode_plan_written_ahead(orc, variant, k, L, n):
    """rlnc_encode_batch_prepare on a second context / stream writes the code-block address stream ahead;
    rlnc_encode_batch_data_planned (ordered after it by an event) writes exactly what encode_batch does, checked
    against the oracle (encoder.rs:128-144) -- for the 8-wave absolute-address program, the 4-wave one, the
    unshared 1- / 2-wave ones, the single-pass kernel (n = 2: no stream) and narrow shapes (perm kernel: no
    stream).  A plan is refused for any other product (another coefficient buffer)."""
    import torch

    import rlnc_amd
    from rlnc_amd import batch
    from rlnc_amd.errors import RLNCError

    rng = np.random.default_rng(k * 131 + n + variant)
    nobj = 3
    src_h = rng.integers(0, 256, (nobj, k, L), dtype=np.uint8)
    co_h = rng.integers(0, 256, (nobj, n, k), dtype=np.uint8)
    src, co = dev(src_h), dev(co_h)
    c1, c2 = rlnc_amd.Context(0), rlnc_amd.Context(0)
    for c in (c1, c2):
        c.set_kernel_variant(variant)
    plan = torch.zeros(batch.encode_plan_bytes(k, nobj, n), dtype=torch.uint8, device="cuda:0")
    pieces = torch.zeros((nobj, n, k + L), dtype=torch.uint8, device="cuda:0")
    side = torch.cuda.Stream()
    ev = torch.cuda.Event()
    with torch.cuda.stream(side):
        batch.encode_batch_prepare(src, co, pieces, plan, c2)
        ev.record()
    batch.encode_batch_headers(co, pieces, c1)
    torch.cuda.current_stream().wait_event(ev)
    batch.encode_batch_data_planned(src, co, pieces, plan, c1)
    torch.cuda.synchronize()
    got = host(pieces)
    for o in range(nobj):
        assert np.array_equal(got[o], orc.encode(src_h[o], co_h[o])), o
    other = co.clone()
    with pytest.raises(RLNCError):
        batch.encode_batch_data_planned(src, other, pieces, plan, c1)
    c1.close()
    c2.close()



@pytest.mark.parametrize("variant", [8, 7])
@pytest.mark.parametrize("k,L,m", [(32, 4096 * 2, 32), (40, 4096 * 3 + 17, 44), (16, 8192, 16), (16, 4096, 20),
                                   (8, 3000, 8)])
def test_decode_apply_plan_written_ahead(orc, variant, k, L, m):
    """rlnc_decode_batch_apply_prepare on the elimination's context / stream writes the T x data product's address
    stream once T is final; rlnc_decode_batch_apply_planned (ordered after it by an event) writes exactly what
    decode_batch_apply writes -- decoded rows, object statuses and lengths -- and full-rank objects decode to the
    oracle's padded source with its data length (decoder.rs:136-177).  Shapes: 32-row products (the 4-wave program),
    40 rows (the 8-wave program, misaligned rows), small objects (1- / 2-wave programs), a narrow shape (no stream);
    one object with a rank-deficient draw.  A plan is refused for any other product (another output buffer) and an
    encode plan is refused by the decode."""
    import torch

    import rlnc_amd
    from rlnc_amd import batch
    from rlnc_amd.errors import RLNCError

    rng = np.random.default_rng(k * 7 + m + variant)
    nobj = 3
    lens = [k * L - 1 - o for o in range(nobj)]
    srcs = [orc.pad(rng.integers(0, 256, n, dtype=np.uint8), k) for n in lens]
    pieces_h = np.zeros((nobj, m, k + L), np.uint8)
    for o in range(nobj):
        co = rng.integers(0, 256, (m, k), dtype=np.uint8)
        if o == 2:
            co[:, 0] = 0  # rank-deficient: column 0 never pivots
        pieces_h[o] = orc.encode(srcs[o], co)
    pieces = dev(pieces_h)
    c1, c2 = rlnc_amd.Context(0), rlnc_amd.Context(0)
    for c in (c1, c2):
        c.set_kernel_variant(variant)

    def z(shape, dtype):
        return torch.zeros(shape, dtype=dtype, device="cuda:0")

    T, pst, rank = z((nobj, k, m), torch.uint8), z((nobj, m), torch.int32), z(nobj, torch.int32)
    outs = [(z((nobj, k, L), torch.uint8), z(nobj, torch.int32), z(nobj, torch.int64)) for _ in range(2)]
    plan = z(batch.decode_apply_plan_bytes(k, m, nobj), torch.uint8)
    side = torch.cuda.Stream()
    ev = torch.cuda.Event()
    with torch.cuda.stream(side):
        batch.decode_batch_eliminate(pieces, k, T, pst, rank, c2)
        batch.decode_batch_apply_prepare(pieces, k, T, outs[0][0], plan, c2)
        ev.record()
    torch.cuda.current_stream().wait_event(ev)
    batch.decode_batch_apply_planned(pieces, k, T, rank, *outs[0], plan, c1)
    batch.decode_batch_apply(pieces, k, T, rank, *outs[1], c1)
    torch.cuda.synchronize()
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    dec, ost, dl = (host(t) for t in outs[0])
    rk = host(rank)
    for o in range(nobj):
        if rk[o] == k:
            assert np.array_equal(dec[o], srcs[o]), o
            assert ost[o] == 0 and dl[o] == lens[o], (o, ost[o], dl[o])
        else:
            assert o == 2 and ost[o] == 10, (o, rk[o], ost[o])  # NotAllPiecesReceivedYet
    with pytest.raises(RLNCError):  # another output buffer: not the product the plan was prepared for
        batch.decode_batch_apply_planned(pieces, k, T, rank, *outs[1], plan, c1)
    eplan = z(batch.encode_plan_bytes(k, nobj, m), torch.uint8)
    src_d = z((nobj, k, L), torch.uint8)
    batch.encode_batch_prepare(src_d, z((nobj, m, k), torch.uint8), z((nobj, m, k + L), torch.uint8), eplan, c1)
    with pytest.raises(RLNCError):  # an encode plan
        batch.decode_batch_apply_planned(pieces, k, T, rank, *outs[0], eplan, c1)
    torch.cuda.synchronize()
    c1.close()
    c2.close()


@pytest.mark.parametrize("k", [16, 8, 5])
def test_decode_small_objects_marker_outcomes(ctx, k):
    """Objects of k <= 16 pieces x one 4 KiB column block (the small-object elimination + 1- / 2-wave product, then
    the marker scan of decoder.rs:162-177, 16 lanes an object).  Payload tails chosen to hit every outcome: the marker as the very last byte, early in row 0, alone at the start of the last row, at index 0 only
    (invalid), an all-zero payload (invalid), a last nonzero byte other than 0x81 (invalid), and rank-deficient
    objects (NotAllPiecesReceivedYet, length 0)."""
    import torch

    from rlnc_amd import batch

    nobj, L = 2056, 4096
    rng = np.random.default_rng(77 + k)
    src = rng.integers(0, 256, (nobj, k * L), dtype=np.uint8)
    want_len = np.zeros(nobj, np.int64)
    for o in range(nobj):
        c = o % 6
        if c == 0:
            src[o, -1] = 0x81
            want_len[o] = k * L - 1
        elif c == 1:
            src[o, 101:] = 0
            src[o, 100] = 0x81
            want_len[o] = 100
        elif c == 2:
            src[o] = 0
        elif c == 3:
            src[o] = 0
            src[o, 0] = 0x81
        elif c == 4:
            src[o, -1] = 0x7E
        else:
            src[o, (k - 1) * L:] = 0
            src[o, (k - 1) * L] = 0x81
            want_len[o] = (k - 1) * L
    co = rng.integers(0, 256, (nobj, k, k), dtype=np.uint8)
    deficient = np.arange(nobj) % 11 == 7
    co[deficient, 1] = co[deficient, 0]  # a repeated coding vector: rank k - 1 at most
    src_d = dev(src.reshape(nobj, k, L))
    pieces = torch.empty((nobj, k, k + L), dtype=torch.uint8, device=src_d.device)
    batch.encode_batch(src_d, dev(co), pieces, ctx)
    decoded = dev(np.zeros((nobj, k, L), np.uint8))
    pst, ost, dl = batch.decode_batch(pieces, k, decoded, ctx)
    got = host(decoded).reshape(nobj, k * L)
    for o in range(nobj):
        od = OracleDecoder(L, k)
        for p in host(pieces[o]):
            od.decode(p)
        st, data = od.get_decoded_data()
        assert S[ost[o]] == S[st], o
        assert int(dl[o]) == (len(data) if S[st] == "Ok" else 0), o
        if deficient[o] or S[st] == "NotAllPiecesReceivedYet":  # (a random 16 x 16 matrix is singular at ~1/256)
            assert S[ost[o]] == "NotAllPiecesReceivedYet", o
            continue
        assert np.array_equal(got[o], src[o]), o
        if o % 6 in (0, 1, 5):
            assert S[ost[o]] == "Ok" and int(dl[o]) == want_len[o], o
        else:
            assert S[ost[o]] == "InvalidDecodedDataFormat", o
