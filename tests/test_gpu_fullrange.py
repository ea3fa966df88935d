"""GPU parity at the reference's own property-test range (src/full/tests.rs:11-15, :53-60, :125-131): data of
1 KiB..64 KiB, 32..2048 source pieces (so piece lengths down to ONE byte, k >> L), recoders over up to
(32 + 2048) / 2 = 1,040 received pieces.

Every coded piece is compared with the C oracle's encode of the same coefficient bytes (its own first k bytes),
every recoded piece with the oracle's recode of the same recoding coefficients (drawn from a twin of the RNG the
recoder used), and every decode() status with the oracle's exact replica of Decoder::decode (decoder.rs:96-118)
fed the same pieces; the decoded bytes must equal the source.  Both the object API (rlnc_amd.full over the C ABI)
and the batch API (encode_batch / decode_batch, decode path 0 = automatic and 1 = host elimination) run.
"""
import copy

import numpy as np
import pytest

from oracle.oracle import OracleDecoder
from tests.gpu_util import dev, host

pytestmark = pytest.mark.gpu

MIN_LEN, MAX_LEN = 1 << 10, 1 << 16  # full/tests.rs:11-12
MIN_K, MAX_K = 1 << 5, 1 << 11  # full/tests.rs:14-15
MAX_RECODE = (MIN_K + MAX_K) // 2  # full/tests.rs:60


@pytest.fixture(scope="module")
def ctx():
    import torch

    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    import rlnc_amd

    c = rlnc_amd.Context(0)
    yield c
    c.set_decode_path(0)


def _shape(seed):
    """(data length, k): the two edges first (k = 2048 with 1 KiB -> L = 1; k = 32 with 64 KiB), then random."""
    if seed == 0:
        return MIN_LEN, MAX_K
    if seed == 1:
        return MAX_LEN, MIN_K
    rng = np.random.default_rng(1000 + seed)
    return int(rng.integers(MIN_LEN, MAX_LEN + 1)), int(rng.integers(MIN_K, MAX_K + 1))


def _decode_and_check(orc, dec, od, piece):
    """decode() on the device path and on the oracle replica; statuses and counters must agree."""
    from rlnc_amd.errors import RLNCError

    want = od.decode(piece)
    try:
        dec.decode(piece)
        got = 0
    except RLNCError as e:
        got = e.code
    assert got == want, (got, want)
    assert dec.get_useful_piece_count() == od.useful and dec.get_received_piece_count() == od.received
    return got


@pytest.mark.parametrize("seed", range(5))
def test_fullrange_encoder_decoder(ctx, orc, seed):
    # full/tests.rs:7-47 at its full range, bit-exact piece by piece
    from rlnc_amd.full import Decoder, Encoder

    n_bytes, k = _shape(seed)
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, n_bytes, dtype=np.uint8)
    enc = Encoder.new(data, k, ctx=ctx)
    src = orc.pad(data, k)
    L = enc.get_piece_byte_len()
    assert src.shape == (k, L) and L == (n_bytes + 1 + k - 1) // k
    dec = Decoder.new(L, k, ctx=ctx)
    od = OracleDecoder(L, k)
    while True:
        piece = enc.code(rng)
        assert np.array_equal(piece, orc.encode(src, piece[None, :k])[0])
        if _decode_and_check(orc, dec, od, piece) == 9:  # ReceivedAllPieces
            break
    assert dec.is_already_decoded()
    assert np.array_equal(dec.get_decoded_data(), data)
    st, want = od.get_decoded_data()
    assert st == 0 and np.array_equal(want, data)


@pytest.mark.parametrize("seed", range(4))
def test_fullrange_encoder_recoder_decoder(ctx, orc, seed):
    # full/tests.rs:49-119: recoders over 2..1,040 coded pieces feed the decoder, fresh pieces in between
    from rlnc_amd.full import Decoder, Encoder, Recoder, fill_bytes

    n_bytes, k = _shape(seed)
    rng = np.random.default_rng(100 + seed)
    data = rng.integers(0, 256, n_bytes, dtype=np.uint8)
    enc = Encoder.new(data, k, ctx=ctx)
    src = orc.pad(data, k)
    full = enc.get_full_coded_piece_byte_len()
    dec = Decoder.new(enc.get_piece_byte_len(), k, ctx=ctx)
    od = OracleDecoder(enc.get_piece_byte_len(), k)
    recoders = 0
    while not dec.is_already_decoded():
        n = int(rng.integers(2, MAX_RECODE + 1)) if recoders else MAX_RECODE  # the largest recoder first
        coded = np.stack([enc.code(rng) for _ in range(n)])
        assert np.array_equal(coded, orc.encode(src, coded[:, :k]))
        rec = Recoder.new(coded.reshape(-1), full, k, ctx=ctx)
        assert rec.get_num_pieces_recoded_together() == n
        recoders += 1
        # full/tests.rs:70-72 recodes up to 2k pieces per recoder; past the recoder's n every piece is redundant,
        # so the loop stops a few pieces after that (each redundant piece costs the oracle a full RREF)
        for _ in range(min(int(rng.integers(1, 2 * k + 1)), n + 4)):
            twin = copy.deepcopy(rng)
            piece = rec.recode(rng)
            assert np.array_equal(piece, orc.recode(coded, full, k, fill_bytes(twin, n)))
            if _decode_and_check(orc, dec, od, piece) == 9:
                break
        if not dec.is_already_decoded():
            _decode_and_check(orc, dec, od, enc.code(rng))
    assert np.array_equal(dec.get_decoded_data(), data)


@pytest.mark.parametrize("seed", range(3))
def test_fullrange_useless_recoded_pieces(ctx, orc, seed):
    # full/tests.rs:121-203: pieces recoded only from pieces the decoder has seen are always PieceNotUseful
    from rlnc_amd.full import Decoder, Encoder, Recoder

    n_bytes, k = _shape(seed)
    rng = np.random.default_rng(200 + seed)
    data = rng.integers(0, 256, n_bytes, dtype=np.uint8)
    enc = Encoder.new(data, k, ctx=ctx)
    full = enc.get_full_coded_piece_byte_len()
    dec = Decoder.new(enc.get_piece_byte_len(), k, ctx=ctx)
    od = OracleDecoder(enc.get_piece_byte_len(), k)
    seen = []
    for _ in range(k // 2):
        p = enc.code(rng)
        if _decode_and_check(orc, dec, od, p) == 0:
            seen.append(p)
    rec = Recoder.new(np.concatenate(seen), full, k, ctx=ctx)
    for _ in range(min(2 * len(seen), 64)):
        assert _decode_and_check(orc, dec, od, rec.recode(rng)) == 8  # PieceNotUseful
    while not dec.is_already_decoded():
        _decode_and_check(orc, dec, od, enc.code(rng))
    assert np.array_equal(dec.get_decoded_data(), data)


@pytest.mark.parametrize("path", [0, 1])
@pytest.mark.parametrize("k,n_bytes,nobj", [(2048, 1024, 2), (2048, 1 << 16, 1), (1024, 4096, 3), (333, 40000, 2),
                                            (32, 1 << 16, 4)])
def test_fullrange_batch_api(ctx, orc, path, k, n_bytes, nobj):
    """encode_batch / decode_batch at the same shapes: k + 3 coded pieces per object, all fed to the decoder."""
    from rlnc_amd import batch

    import torch

    rng = np.random.default_rng(k * 7 + n_bytes + path)
    data = rng.integers(0, 256, (nobj, n_bytes), dtype=np.uint8)
    src = np.stack([orc.pad(d, k) for d in data])
    L = src.shape[2]
    n = k + 3
    co = rng.integers(0, 256, (nobj, n, k), dtype=np.uint8)
    pieces = torch.zeros((nobj, n, k + L), dtype=torch.uint8, device="cuda:0")
    batch.encode_batch(dev(src), dev(co), pieces, ctx)
    hp = host(pieces)
    ctx.set_decode_path(path)
    try:
        decoded = torch.zeros((nobj, k, L), dtype=torch.uint8, device="cuda:0")
        ps, ost, dl = batch.decode_batch(pieces, k, decoded, ctx)
    finally:
        ctx.set_decode_path(0)
    hd = host(decoded)
    for o in range(nobj):
        assert np.array_equal(hp[o], orc.encode(src[o], co[o])), o
        od = OracleDecoder(L, k)
        assert list(ps[o]) == [od.decode(p) for p in hp[o]], o
        assert np.array_equal(hd[o], od.padded_payload()), o
        assert ost[o] == 0 and int(dl[o]) == n_bytes
        assert np.array_equal(hd[o].reshape(-1)[:n_bytes], data[o])


@pytest.mark.parametrize("k,n,L,count", [(2048, 1040, 1, 3), (32, 1040, 2049, 4), (700, 513, 94, 5)])
def test_fullrange_recode_batch(ctx, orc, k, n, L, count):
    """recode_batch over up to 1,040 received pieces (recoder.rs:122-153 × count), k >> L included."""
    from rlnc_amd import batch

    import torch

    rng = np.random.default_rng(k + n + L)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    co = rng.integers(0, 256, (n, k), dtype=np.uint8)
    coded = orc.encode(src, co)
    r = rng.integers(0, 256, (1, count, n), dtype=np.uint8)
    r[0, 0, :] = 0
    r[0, 1 % count, :] = 0
    r[0, 1 % count, n - 1] = 1  # a unit vector: the recoded piece is the last received piece
    out = torch.zeros((1, count, k + L), dtype=torch.uint8, device="cuda:0")
    batch.recode_batch(dev(coded[None]), dev(r), out, k, ctx)
    got = host(out)[0]
    for i in range(count):
        assert np.array_equal(got[i], orc.recode(coded, k + L, k, r[0, i])), i
    assert not got[0].any() and np.array_equal(got[1 % count], coded[n - 1])
