"""GPU: the rlnc::full API mirror — error variants, check order, getters and state rules, ported from the
reference's own unit tests (encoder.rs:277-544, decoder.rs:186-350, recoder.rs:180-331)."""
import numpy as np
import pytest

from tests.conftest import hexarr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import rlnc_amd

    return rlnc_amd.Context(0)


def rnd(n, seed=0):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


def raises(kind, fn, *a):
    from rlnc_amd.errors import RLNCError

    with pytest.raises(RLNCError) as ei:
        fn(*a)
    assert ei.value == getattr(RLNCError, kind), (ei.value, kind)


def test_encoder_without_padding_invalid_data(ctx):
    from rlnc_amd.full import Encoder

    raises("DataLengthZero", Encoder.without_padding, rnd(0), 10, ctx)
    raises("PieceCountZero", Encoder.without_padding, rnd(100), 0, ctx)
    raises("DataLengthMismatch", Encoder.without_padding, rnd(1001), 32, ctx)
    Encoder.without_padding(rnd(100), 10, ctx)


def test_encoder_new_invalid_inputs(ctx):
    from rlnc_amd.full import Encoder

    raises("DataLengthZero", Encoder.new, rnd(0), 5, ctx)
    raises("PieceCountZero", Encoder.new, rnd(100), 0, ctx)
    raises("DataLengthZero", Encoder.new, rnd(0), 0, ctx)
    Encoder.new(rnd(1024), 32, ctx)


def test_encoder_code_with_coding_vector_invalid_inputs(ctx):
    from rlnc_amd.full import Encoder

    enc = Encoder.new(rnd(1024), 32, ctx)
    k, L = enc.get_piece_count(), enc.get_piece_byte_len()
    raises("CodingVectorLengthMismatch", enc.code_with_coding_vector, rnd(k - 1), np.zeros(L, np.uint8))
    raises("InvalidOutputBuffer", enc.code_with_coding_vector, rnd(k), np.zeros(L - 1, np.uint8))
    raises("CodingVectorLengthMismatch", enc.code_with_coding_vector, rnd(k + 1), np.zeros(L, np.uint8))
    raises("InvalidOutputBuffer", enc.code_with_coding_vector, rnd(k), np.zeros(L + 1, np.uint8))
    raises("CodingVectorLengthMismatch", enc.code_with_coding_vector, rnd(0), np.zeros(k + L, np.uint8))
    raises("InvalidOutputBuffer", enc.code_with_coding_vector, rnd(k), np.zeros(0, np.uint8))
    enc.code_with_coding_vector(rnd(k), np.zeros(L, np.uint8))


def test_encoder_code_with_buf_invalid_inputs(ctx):
    from rlnc_amd.full import Encoder

    enc = Encoder.new(rnd(1024), 32, ctx)
    rng = np.random.default_rng(1)
    full = enc.get_full_coded_piece_byte_len()
    raises("InvalidOutputBuffer", enc.code_with_buf, rng, np.zeros(full - 1, np.uint8))
    raises("InvalidOutputBuffer", enc.code_with_buf, rng, np.zeros(full + 1, np.uint8))
    raises("InvalidOutputBuffer", enc.code_with_buf, rng, np.zeros(0, np.uint8))
    enc.code_with_buf(rng, np.zeros(full, np.uint8))


def test_encoder_getters(ctx):
    from rlnc_amd.full import Encoder

    e = Encoder.new(rnd(100), 1, ctx)
    assert (e.get_piece_count(), e.get_piece_byte_len(), e.get_full_coded_piece_byte_len()) == (1, 101, 102)
    e = Encoder.new(bytes([42]), 1, ctx)
    assert (e.get_piece_byte_len(), e.get_full_coded_piece_byte_len()) == (2, 3)
    e = Encoder.new(rnd(10), 10, ctx)
    assert (e.get_piece_byte_len(), e.get_full_coded_piece_byte_len()) == (2, 12)
    e = Encoder.new(rnd(100), 50, ctx)
    assert (e.get_piece_count(), e.get_piece_byte_len()) == (50, 3)


def test_decoder_new_invalid_inputs(ctx):
    from rlnc_amd.full import Decoder

    raises("PieceLengthZero", Decoder.new, 0, 10, ctx)
    raises("PieceCountZero", Decoder.new, 10, 0, ctx)
    raises("PieceLengthZero", Decoder.new, 0, 0, ctx)
    Decoder.new(10, 5, ctx)


def test_decoder_decode_invalid_piece_length(ctx):
    from rlnc_amd.errors import RLNCError
    from rlnc_amd.full import Decoder, Encoder

    rng = np.random.default_rng(2)
    enc = Encoder.new(rnd(1024), 32, ctx)
    dec = Decoder.new(enc.get_piece_byte_len(), enc.get_piece_count(), ctx)
    full = enc.get_full_coded_piece_byte_len()
    raises("InvalidPieceLength", dec.decode, rnd(full - 1))
    raises("InvalidPieceLength", dec.decode, rnd(full + 1))
    raises("InvalidPieceLength", dec.decode, rnd(0))
    assert dec.get_received_piece_count() == 0 and dec.get_useful_piece_count() == 0
    assert not dec.is_already_decoded()
    try:
        dec.decode(enc.code(rng))
        useful = True
    except RLNCError as e:
        assert e == RLNCError.PieceNotUseful
        useful = False
    assert dec.get_received_piece_count() == 1
    assert dec.get_useful_piece_count() == (1 if useful else 0)


def test_decoder_getters(ctx):
    from rlnc_amd.errors import RLNCError
    from rlnc_amd.full import Decoder, Encoder

    rng = np.random.default_rng(3)
    enc = Encoder.new(rnd(1024), 32, ctx)
    k = enc.get_piece_count()
    dec = Decoder.new(enc.get_piece_byte_len(), k, ctx)
    assert dec.get_num_pieces_coded_together() == k
    assert dec.get_piece_byte_len() == enc.get_piece_byte_len()
    assert dec.get_full_coded_piece_byte_len() == enc.get_full_coded_piece_byte_len()
    assert dec.get_remaining_piece_count() == k
    raises("NotAllPiecesReceivedYet", dec.get_decoded_data)
    useful = 0
    for _ in range(k // 2):
        try:
            dec.decode(enc.code(rng))
            useful += 1
        except RLNCError as e:
            assert e == RLNCError.PieceNotUseful
    assert dec.get_received_piece_count() == k // 2 and dec.get_useful_piece_count() == useful
    assert dec.get_remaining_piece_count() == k - useful
    total = k // 2
    while not dec.is_already_decoded():
        try:
            dec.decode(enc.code(rng))
        except RLNCError as e:
            assert e == RLNCError.PieceNotUseful
        total += 1
    assert dec.get_useful_piece_count() == k and dec.get_remaining_piece_count() == 0
    assert dec.get_received_piece_count() == total
    raises("ReceivedAllPieces", dec.decode, enc.code(rng))
    assert dec.get_received_piece_count() == total


def test_recoder_new_invalid_inputs(ctx):
    from rlnc_amd.full import Encoder, Recoder

    rng = np.random.default_rng(4)
    enc = Encoder.new(rnd(1024), 32, ctx)
    full, k = enc.get_full_coded_piece_byte_len(), enc.get_piece_count()
    raises("NotEnoughPiecesToRecode", Recoder.new, rnd(0), full, k, ctx)
    raises("PieceLengthZero", Recoder.new, rnd(3), 0, k, ctx)
    raises("PieceCountZero", Recoder.new, rnd(3), full, 0, ctx)
    raises("PieceLengthTooShort", Recoder.new, rnd(3), k, k, ctx)
    raises("PieceLengthTooShort", Recoder.new, rnd(3), k - 1, k, ctx)
    coded = np.concatenate([enc.code(rng) for _ in range(5)])
    r = Recoder.new(coded, full, k, ctx)
    assert r.get_original_num_pieces_coded_together() == k and r.get_num_pieces_recoded_together() == 5


def test_recoder_recode_with_buf_invalid_inputs(ctx):
    from rlnc_amd.full import Encoder, Recoder

    rng = np.random.default_rng(5)
    enc = Encoder.new(rnd(1024), 32, ctx)
    coded = np.concatenate([enc.code(rng) for _ in range(16)])
    r = Recoder.new(coded, enc.get_full_coded_piece_byte_len(), enc.get_piece_count(), ctx)
    full = r.get_full_coded_piece_byte_len()
    raises("InvalidOutputBuffer", r.recode_with_buf, rng, np.zeros(full - 1, np.uint8))
    raises("InvalidOutputBuffer", r.recode_with_buf, rng, np.zeros(full + 1, np.uint8))
    raises("InvalidOutputBuffer", r.recode_with_buf, rng, np.zeros(0, np.uint8))
    r.recode_with_buf(rng, np.zeros(full, np.uint8))


def test_recoder_getters(ctx):
    from rlnc_amd.full import Encoder, Recoder

    rng = np.random.default_rng(6)
    enc = Encoder.new(rnd(1024), 32, ctx)
    coded = np.concatenate([enc.code(rng) for _ in range(10)])
    r = Recoder.new(coded, enc.get_full_coded_piece_byte_len(), 32, ctx)
    assert r.get_original_num_pieces_coded_together() == 32
    assert r.get_num_pieces_recoded_together() == 10
    assert r.get_piece_byte_len() == enc.get_piece_byte_len()
    assert r.get_full_coded_piece_byte_len() == enc.get_full_coded_piece_byte_len()


def test_final_data_len_edge_cases_all_paths(ctx, golden):
    """decoder.rs:162-177 through the host path, the device path and the batch kernel (k = 1 pieces
    with coefficient 1 decode to exactly their payload)."""
    import torch

    from rlnc_amd import batch
    from rlnc_amd.errors import RLNCError
    from rlnc_amd.full import Decoder

    for v in golden["final_data_len"]:
        payload = hexarr(v["padded"])
        L = payload.size
        piece = np.concatenate([[1], payload]).astype(np.uint8)
        d = Decoder.new(L, 1, ctx)
        d.decode(piece)
        try:
            got = d.get_decoded_data()
            assert v["status"] == "Ok" and got.size == v["len"]
        except RLNCError as e:
            assert e.name == v["status"]
        out = torch.zeros(L, dtype=torch.uint8, device="cuda:0")
        try:
            n = d.get_decoded_data_device(out.data_ptr(), L)
            assert v["status"] == "Ok" and n == v["len"]
        except RLNCError as e:
            assert e.name == v["status"]
        dec = torch.zeros((1, 1, L), dtype=torch.uint8, device="cuda:0")
        _, ost, dl = batch.decode_batch(torch.from_numpy(piece[None, None]).cuda(), 1, dec, ctx)
        assert (ost[0] == 0) == (v["status"] == "Ok")
        if ost[0] == 0:
            assert int(dl[0]) == v["len"]


def test_decode_device_pieces(ctx):
    """Decoder::decode on pieces already in HBM (only the coefficient bytes cross PCIe)."""
    import torch

    from rlnc_amd.errors import RLNCError
    from rlnc_amd.full import Decoder, Encoder

    rng = np.random.default_rng(8)
    data = rnd(50000, 8)
    enc = Encoder.new(data, 24, ctx)
    dec = Decoder.new(enc.get_piece_byte_len(), 24, ctx)
    while not dec.is_already_decoded():
        p = torch.from_numpy(enc.code(rng)).cuda()
        try:
            dec.decode_device(p.data_ptr(), p.numel())
        except RLNCError as e:
            assert e == RLNCError.PieceNotUseful
    assert np.array_equal(dec.get_decoded_data(), data)
