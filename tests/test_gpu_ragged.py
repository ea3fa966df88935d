"""GPU: ragged batches on the receiver side (rlnc_decode_ragged, rlnc_recode_ragged) and the sender side
(rlnc_encode_ragged through batch.encode_ragged): objects of many shapes, one launch per kernel stage, bit-exact
against the oracle -- every decode() status of every object (decoder.rs:96-118), its get_decoded_data outcome
(decoder.rs:136-177) and payload, every recoded piece (recoder.rs:122-153).  Shapes cover the elimination's three
homes (blocked run k + m <= 256, the one-wave LDS kernel, host threads beyond LDS), < 4 KiB and unaligned tails,
padded row strides, rank-deficient objects, dependent / sparse coefficients and payloads without a valid marker."""
import numpy as np
import pytest

from oracle.oracle import OracleDecoder
from tests.gpu_util import dev, host

pytestmark = pytest.mark.gpu

# (k, L, m, objects, dependent-piece fraction, zero-coefficient fraction, padded stride)
DECODE_SHAPES = [
    (16, 4096, 16, 40, 0.0, 0.0, 0),
    (16, 4096 + 7, 20, 40, 0.2, 0.3, 0),
    (32, 8192, 32, 40, 0.0, 0.0, 64),
    (32, 1000, 40, 40, 0.1, 0.0, 0),
    (64, 3 * 4096 + 48, 64, 30, 0.0, 0.0, 0),
    (100, 2 * 4096, 110, 20, 0.05, 0.5, 16),
    (128, 8192, 128, 16, 0.0, 0.0, 0),
    (8, 64, 6, 24, 0.0, 0.0, 0),  # m < k: NotAllPiecesReceivedYet
    (200, 4096, 204, 4, 0.0, 0.0, 0),  # k + m > 256, k > 128: the one-wave LDS kernel
    (100, 4096 + 32, 180, 6, 0.1, 0.6, 0),  # k + m > 256, k <= 128: blocked run over 156 pieces, general pass if needed
    (400, 64, 402, 2, 0.0, 0.0, 0),  # beyond LDS: host threads
]


@pytest.fixture(scope="module")
def ctx():
    import torch

    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    import rlnc_amd

    return rlnc_amd.Context(0)


def _pieces(orc, rng, k, L, m, dep, sparse, valid):
    """m received pieces of one object: random source (Encoder::new-padded when `valid`), coefficients with
    `sparse` zeros and a `dep` fraction of pieces that are combinations of earlier ones."""
    if valid:
        data = rng.integers(0, 256, int(rng.integers(max(1, k * L - k), k * L)), dtype=np.uint8)
        src = orc.pad(data, k)
        assert src.shape == (k, L)
    else:
        data, src = None, rng.integers(0, 256, (k, L), dtype=np.uint8)
    co = rng.integers(0, 256, (m, k), dtype=np.uint8)
    co[rng.random((m, k)) < sparse] = 0
    for i in range(1, m):
        if rng.random() < dep:
            a, b = rng.integers(0, i, 2)
            co[i] = orc.encode(co[[a, b]].astype(np.uint8), rng.integers(0, 256, (1, 2), dtype=np.uint8))[0, 2:]
    return data, orc.encode(src, co)


def test_decode_ragged_many_shapes_vs_oracle(ctx, orc):
    import torch

    from rlnc_amd import batch

    rng = np.random.default_rng(0x52414744)
    objs, meta, keep = [], [], []
    for si, (k, L, m, count, dep, sparse, pad) in enumerate(DECODE_SHAPES):
        for o in range(count):
            valid = (o % 7) != 3  # some payloads carry no valid marker: InvalidDecodedDataFormat
            data, pc = _pieces(orc, rng, k, L, m, dep, sparse, valid)
            buf = torch.zeros((m, k + L + pad), dtype=torch.uint8, device="cuda:0")
            buf[:, : k + L] = dev(pc)
            dec = torch.zeros((k, L), dtype=torch.uint8, device="cuda:0")
            objs.append((buf[:, : k + L], k, dec))
            meta.append((k, L, m, data, pc))
            keep.append(buf)
    order = rng.permutation(len(objs))  # shapes interleaved: nothing relies on grouping
    objs = [objs[i] for i in order]
    meta = [meta[i] for i in order]
    assert len(objs) >= 256 and len({(k, L, m) for k, L, m, _, _ in meta}) >= 8
    ps, ost, dl = batch.decode_ragged(objs, ctx)
    ps, ost, dl = host(ps), host(ost), host(dl)
    off = 0
    for i, ((k, L, m, data, pc), (_, _, dec)) in enumerate(zip(meta, objs)):
        od = OracleDecoder(L, k)
        want = [od.decode(p) for p in pc]
        assert list(ps[off: off + m]) == want, (i, k, L, m)
        off += m
        st, payload = od.get_decoded_data()
        assert int(ost[i]) == st, (i, k, L, m, int(ost[i]), st)
        if od.is_already_decoded():
            assert np.array_equal(host(dec), od.padded_payload()), (i, k, L, m)
        if st == 0:
            assert int(dl[i]) == payload.size and np.array_equal(payload, data), i


def test_decode_ragged_matches_uniform_batch(ctx, orc):
    """Same objects through rlnc_decode_ragged and rlnc_decode_batch_device: identical outputs."""
    import torch

    from rlnc_amd import batch

    rng = np.random.default_rng(3)
    k, L, m, B = 32, 4 * 4096, 34, 12
    src = np.stack([orc.pad(rng.integers(0, 256, k * L - 5, dtype=np.uint8), k) for _ in range(B)])
    co = rng.integers(0, 256, (B, m, k), dtype=np.uint8)
    pieces = dev(np.stack([orc.encode(src[o], co[o]) for o in range(B)]))
    d1 = torch.zeros((B, k, L), dtype=torch.uint8, device="cuda:0")
    d2 = torch.zeros_like(d1)
    ps1, os1, dl1 = batch.decode_ragged([(pieces[o], k, d1[o]) for o in range(B)], ctx)
    ps2 = torch.empty((B, m), dtype=torch.int32, device="cuda:0")
    os2 = torch.empty(B, dtype=torch.int32, device="cuda:0")
    dl2 = torch.empty(B, dtype=torch.int64, device="cuda:0")
    batch.decode_batch_device(pieces, k, d2, ps2, os2, dl2, ctx)
    torch.cuda.synchronize()
    assert torch.equal(d1, d2) and torch.equal(ps1, ps2.reshape(-1)) and torch.equal(os1, os2)
    assert torch.equal(dl1, dl2)
    assert np.array_equal(host(d1), src)


@pytest.mark.parametrize("seed", [0, 1])
def test_recode_ragged_many_shapes_vs_oracle(ctx, orc, seed):
    import torch

    from rlnc_amd import batch

    rng = np.random.default_rng(100 + seed)
    # (k, L, n received, recoded, padded stride)
    shapes = [(16, 4096, 20, 8, 0), (32, 8192 + 3, 40, 16, 0), (64, 262144, 64, 5, 0), (8, 100, 12, 3, 7),
              (128, 4096 * 2, 130, 40, 32), (20, 4076, 24, 2, 0), (3, 9000, 2, 4, 0), (700, 94, 513, 3, 0)]
    objs, want = [], []
    for k, L, n, cnt, pad in shapes:
        for _ in range(3):
            src = rng.integers(0, 256, (k, L), dtype=np.uint8)
            coded = orc.encode(src, rng.integers(0, 256, (n, k), dtype=np.uint8))
            r = rng.integers(0, 256, (cnt, n), dtype=np.uint8)
            r[0] = 0
            buf = torch.zeros((n, k + L + pad), dtype=torch.uint8, device="cuda:0")
            buf[:, : k + L] = dev(coded)
            out = torch.zeros((cnt, k + L + pad), dtype=torch.uint8, device="cuda:0")
            objs.append((buf[:, : k + L], dev(r), out[:, : k + L], k))
            want.append([orc.recode(coded, k + L, k, r[i]) for i in range(cnt)])
    batch.recode_ragged(objs, ctx)
    torch.cuda.synchronize()
    for (_, _, out, k), w in zip(objs, want):
        got = host(out)
        for i, wi in enumerate(w):
            assert np.array_equal(got[i], wi), (k, i)


def test_encode_ragged_many_shapes_vs_oracle(ctx, orc):
    import torch

    from rlnc_amd import batch

    rng = np.random.default_rng(77)
    shapes = [(16, 4096, 16), (32, 1 << 20, 64), (32, 3 * 4096 + 16, 33), (5, 999, 7), (128, 65536, 128),
              (64, 8192, 2), (40, 4096, 100), (1, 4096, 1)]
    objs, want = [], []
    for k, L, n in shapes:
        for _ in range(2):
            src = rng.integers(0, 256, (k, L), dtype=np.uint8)
            co = rng.integers(0, 256, (n, k), dtype=np.uint8)
            co[0] = 0
            co[-1] = 1
            pc = torch.zeros((n, k + L), dtype=torch.uint8, device="cuda:0")
            objs.append((dev(src), dev(co), pc))
            want.append(orc.encode(src, co))
    batch.encode_ragged(objs, ctx)
    torch.cuda.synchronize()
    for (_, _, pc), w in zip(objs, want):
        assert np.array_equal(host(pc), w)


def test_ragged_errors_checked_before_launch(ctx):
    import torch

    from rlnc_amd import _lib
    from rlnc_amd.errors import RLNCError

    p = torch.zeros((4, 40), dtype=torch.uint8, device="cuda:0")
    d = torch.zeros((8, 32), dtype=torch.uint8, device="cuda:0")
    ps = torch.zeros(8, dtype=torch.int32, device="cuda:0")
    arr = (_lib.DecodeObjDesc * 2)(_lib.DecodeObjDesc(p.data_ptr(), 0, d.data_ptr(), 8, 32, 4),
                                   _lib.DecodeObjDesc(p.data_ptr(), 0, d.data_ptr(), 8, 0, 4))
    assert ctx.lib.rlnc_decode_ragged(ctx.h, arr, 2, ps.data_ptr(), ps.data_ptr(), ps.data_ptr()) == \
        RLNCError.PieceLengthZero.code
    arr[1].L, arr[1].k = 32, 0
    assert ctx.lib.rlnc_decode_ragged(ctx.h, arr, 2, ps.data_ptr(), ps.data_ptr(), ps.data_ptr()) == \
        RLNCError.PieceCountZero.code
    r = (_lib.RecodeObjDesc * 1)(_lib.RecodeObjDesc(p.data_ptr(), 0, p.data_ptr(), d.data_ptr(), 0, 8, 32, 0, 1))
    assert ctx.lib.rlnc_recode_ragged(ctx.h, r, 1) == RLNCError.NotEnoughPiecesToRecode.code
    r[0].n, r[0].k, r[0].L = 4, 0, 40
    assert ctx.lib.rlnc_recode_ragged(ctx.h, r, 1) == RLNCError.PieceCountZero.code
    r[0].k, r[0].L = 40, 0
    assert ctx.lib.rlnc_recode_ragged(ctx.h, r, 1) == RLNCError.PieceLengthTooShort.code
