"""BASELINE.json configs end to end on the GPU, bit-exact against the C oracle.

* configs[0]: the reference example workflow (examples/full_rlnc.rs:11-149) — encode, half the pieces decoded
  directly, a recoder over exactly those pieces (all its output useless), a second recoder over fresh pieces,
  then direct pieces until decoded — through the rlnc::full mirror (C ABI), at the BASELINE shape 16 × 4 KiB and
  at the example's own 10 KiB / 32 pieces.  Every coded/recoded piece and every decode() status is compared with
  the oracle fed the same coefficient bytes (a recording RNG hands them out, like rng.fill_bytes).
* configs[3]: all 64 recoded pieces of the 64 × (64 + 256 KiB) recoder against the oracle's recode.
* configs[4]: the real per-GPU share of the 8-GPU batch — 512 objects × k=128 × 64 KiB (4 GiB of source, coded
  pieces past byte offset 2^32) — 8 sampled objects' coded pieces and decoded rows against the oracle, every
  object's decode() statuses against the oracle's decisions, and decoded == source for every full-rank object.
"""
import numpy as np
import pytest

from oracle.oracle import OracleDecoder
from tests.gpu_util import dev, host

pytestmark = pytest.mark.gpu

S = ["Ok", "CodingVectorLengthMismatch", "DataLengthMismatch", "PieceCountZero", "DataLengthZero",
     "PieceLengthZero", "NotEnoughPiecesToRecode", "PieceLengthTooShort", "PieceNotUseful", "ReceivedAllPieces",
     "NotAllPiecesReceivedYet", "InvalidDecodedDataFormat", "InvalidPieceLength", "InvalidOutputBuffer"]


@pytest.fixture(scope="module")
def ctx():
    import torch

    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    import rlnc_amd

    return rlnc_amd.Context(0)


class RecordingRng:
    """rng.fill_bytes stand-in: draws from a seeded numpy generator and keeps every draw."""

    def __init__(self, seed):
        self.g = np.random.default_rng(seed)
        self.draws = []

    def fill_bytes(self, n):
        b = self.g.integers(0, 256, n, dtype=np.uint8)
        self.draws.append(b)
        return b.tobytes()

    def last(self):
        return self.draws[-1]


def _status(fn):
    from rlnc_amd.errors import RLNCError

    try:
        fn()
        return "Ok"
    except RLNCError as e:
        return e.name


@pytest.mark.parametrize("data_len,k", [(16 * 4096 - 1, 16), (10 * 1024, 32)])
def test_config0_example_workflow(ctx, orc, data_len, k):
    """examples/full_rlnc.rs:11-149, step for step, every byte and status against the oracle."""
    from rlnc_amd.full import Decoder, Encoder, Recoder

    rng = RecordingRng(data_len + k)
    data = np.random.default_rng(k).integers(0, 256, data_len, dtype=np.uint8)
    src = orc.pad(data, k)  # Encoder::new's padded image (encoder.rs:85-106)
    L = src.shape[1]
    enc = Encoder.new(data, k, ctx=ctx)  # :17
    assert (enc.get_piece_count(), enc.get_piece_byte_len(), enc.get_full_coded_piece_byte_len()) == (k, L, k + L)
    if data_len == 16 * 4096 - 1:
        assert L == 4096  # BASELINE configs[0]: 16 pieces × 4 KiB
    dec = Decoder.new(enc.get_piece_byte_len(), enc.get_piece_count(), ctx=ctx)  # :36
    od = OracleDecoder(L, k)
    full = k + L

    def code():
        p = enc.code(rng)
        assert np.array_equal(p, orc.encode(src, rng.last())[0])
        return p

    def feed(p):
        got = _status(lambda: dec.decode(p))
        want = S[od.decode(p)]
        assert got == want
        assert dec.get_received_piece_count() == od.received and dec.get_useful_piece_count() == od.useful
        return got

    # 4. half the pieces straight from the sender, each also collected for the recoder (:39-56)
    half = k // 2
    for_recoder = []
    for _ in range(half):
        p = code()
        for_recoder.append(p)
        if feed(p) == "ReceivedAllPieces":
            break
    # 5./6. a recoder over exactly the pieces the decoder has seen: nothing it makes is useful (:58-85)
    seen = np.concatenate(for_recoder)
    rec = Recoder.new(seen, full, k, ctx=ctx)
    assert rec.get_num_pieces_recoded_together() == len(for_recoder)
    for _ in range(2 * k):
        if dec.is_already_decoded():
            break
        rp = rec.recode(rng)
        assert np.array_equal(rp, orc.recode(seen, full, k, rng.last()))
        assert feed(rp) == "PieceNotUseful"  # full/tests.rs:171-184
    # 7./8. a second recoder over fresh pieces: its output is useful (:87-120)
    fresh = np.concatenate([code() for _ in range(half)])
    rec2 = Recoder.new(fresh, full, k, ctx=ctx)
    useful = 0
    for _ in range(half // 2):
        if dec.is_already_decoded():
            break
        rp = rec2.recode(rng)
        assert np.array_equal(rp, orc.recode(fresh, full, k, rng.last()))
        useful += feed(rp) == "Ok"
    assert useful > 0
    # 9. direct pieces until decoded (:122-142)
    while not dec.is_already_decoded():
        feed(code())
    assert od.is_already_decoded()
    assert _status(lambda: dec.decode(code())) == "ReceivedAllPieces"
    # retrieve and verify (:144-149)
    out = dec.get_decoded_data()
    st, want = od.get_decoded_data()
    assert st == 0 and np.array_equal(out, want) and np.array_equal(out, data)


def test_config3_recode_all_64_vs_oracle(ctx, orc):
    from rlnc_amd import batch

    k, L, n, count = 64, 1 << 18, 64, 64
    rng = np.random.default_rng(44)
    src = rng.integers(0, 256, (k, L), dtype=np.uint8)
    pieces = orc.encode(src, rng.integers(0, 256, (n, k), dtype=np.uint8))
    r = rng.integers(0, 256, (1, count, n), dtype=np.uint8)
    r[0, 0] = 0  # an all-zero recoding vector and unit vectors (the c=0 / c=1 early-outs)
    r[0, 1] = 0
    r[0, 1, 5] = 1
    out = dev(np.zeros((1, count, k + L), np.uint8))
    batch.recode_batch(dev(pieces[None]), dev(r), out, k, ctx)
    got = host(out)[0]
    for c in range(count):
        assert np.array_equal(got[c], orc.recode(pieces, k + L, k, r[0, c])), c
    assert not got[0].any() and np.array_equal(got[1], pieces[5])


def test_config4_full_gpu_share_512x_k128_64KiB(ctx, orc):
    """512 objects (4,096 / 8 GPUs) × k=128 × 64 KiB: 4 GiB of source, 4.03 GiB of coded pieces (object 511's
    pieces end past byte offset 2^32), encode 128 + decode 128 per object."""
    import torch

    from rlnc_amd import batch

    k, L, nobj = 128, 1 << 16, 512
    full = k + L
    g = torch.Generator(device="cuda:0")
    g.manual_seed(0x524C4E43)
    src = torch.randint(0, 256, (nobj, k, L), dtype=torch.uint8, device="cuda:0", generator=g)
    # tails that fix get_final_data_len (decoder.rs:162-177): even objects end in the 0x81 marker (Ok, k·L-1),
    # odd ones in a non-marker byte (InvalidDecodedDataFormat), object 2 has 100 zero bytes after its marker
    src[0::2, -1, -1] = 0x81
    src[1::2, -1, -1] = 0x37
    src[2, -1, -100:] = 0
    src[2, -1, -101] = 0x81
    want_len = {o: k * L - 1 for o in range(0, nobj, 2)}
    want_len[2] = k * L - 101
    co_h = np.random.default_rng(45).integers(0, 256, (nobj, k, k), dtype=np.uint8)
    co_h[7, 9] = co_h[7, 3] ^ co_h[7, 4]  # a dependent piece: object 7 ends rank-deficient unless 128 others span
    pieces = torch.empty((nobj, k, full), dtype=torch.uint8, device="cuda:0")
    assert pieces[nobj - 1, k - 1].data_ptr() - pieces.data_ptr() > (1 << 32)  # object 511's last pieces
    batch.encode_batch(src, dev(co_h), pieces, ctx)
    decoded = torch.empty((nobj, k, L), dtype=torch.uint8, device="cuda:0")
    pst, ost, dl = batch.decode_batch(pieces, k, decoded, ctx)
    torch.cuda.synchronize()

    # every object's decode() statuses against the oracle's decisions: they read only the coefficient columns
    # (decoder_matrix.rs:120-244), so the oracle decoder fed [coeffs | first data byte] decides identically
    heads = pieces[:, :, : k + 1].cpu().numpy()
    full_rank = []
    for o in range(nobj):
        od = OracleDecoder(1, k)
        want = [od.decode(p) for p in heads[o]]
        assert list(pst[o]) == want, o
        full_rank.append(od.is_already_decoded())
        if not od.is_already_decoded():
            assert S[ost[o]] == "NotAllPiecesReceivedYet", o
        elif o in want_len:
            assert S[ost[o]] == "Ok" and int(dl[o]) == want_len[o], o
        else:
            assert S[ost[o]] == "InvalidDecodedDataFormat", o
    assert (pst[7] == 8).any()  # the dependent piece 9 of object 7 is rejected
    assert sum(full_rank) >= nobj - 8
    # decoded == source for every full-rank object (on the device)
    mismatch = (decoded != src).view(nobj, -1).any(1).cpu().numpy()
    for o in range(nobj):
        if full_rank[o]:
            assert not mismatch[o], o
    # sampled objects, bytes against the oracle: coded pieces and the padded payload rows of the full decode
    for o in [0, 1, 7, 255, 256, 383, 510, 511]:
        s = src[o].cpu().numpy()
        hp = pieces[o].cpu().numpy()
        assert np.array_equal(hp, orc.encode(s, co_h[o])), o
        od = OracleDecoder(L, k)
        for p in hp:
            od.decode(p)
        pay = od.padded_payload()
        got = decoded[o].cpu().numpy()
        assert np.array_equal(got[: pay.shape[0]], pay), o
        st, _ = od.get_decoded_data()
        assert S[ost[o]] == S[st], o
