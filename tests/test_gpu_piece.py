"""GPU: the object API's call-latency path (piece.hip: sources split across the waves of a workgroup, output rows
written into pinned host memory, per-chunk completion flags) against the oracle -- Encoder::code_with_coding_vector /
code_with_buf, Recoder::recode_with_buf and Decoder::get_decoded_data at the reference's bench shapes and at the
edges: one source, k not a power of two, k = 512 / 2048 with pieces <= 8 KiB (several coefficient batches of 64 per
wave), pieces of 1 byte to 1 MiB + 1 (one flag chunk to many), hundreds of calls on one workspace (epochs and counter
re-arming), concurrent calls on one encoder from several threads."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import rlnc_amd

    return rlnc_amd.Context(0)


def _src(rng, k, L):
    return rng.integers(0, 256, (k, L), dtype=np.uint8)


@pytest.mark.parametrize("k,L", [(1, 1), (1, 4096), (2, 17), (3, 1000), (16, 65537), (17, 1023), (32, 32769),
                                 (64, 16385), (128, 8193), (256, 4097), (512, 2048), (512, 8192), (2048, 8),
                                 (2048, 8192), (33, 1 << 20), (16, (1 << 20) + 1)])
def test_code_with_coding_vector_matches_oracle(ctx, orc, k, L):
    from rlnc_amd.full import Encoder

    rng = np.random.default_rng(k * 7919 + L)
    src = _src(rng, k, L)
    enc = Encoder.without_padding(src.reshape(-1), k, ctx)
    out = np.zeros(L, np.uint8)
    for trial in range(3):
        cv = rng.integers(0, 256, k, dtype=np.uint8)
        if trial == 1:
            cv[rng.random(k) < 0.5] = 0  # zero coefficients (early-outs in the reference, simd/mod.rs:93-95)
        if trial == 2:
            cv[:] = 1
        enc.code_with_coding_vector(cv, out)
        st, want = orc.code_with_coding_vector(src, cv)
        assert st == 0 and np.array_equal(out, want), (k, L, trial)


@pytest.mark.parametrize("size,k", [(1 << 20, 16), (1 << 20, 128), (1 << 20, 256), (1000, 7)])
def test_code_with_buf_padded_encoder(ctx, orc, size, k):
    from rlnc_amd.full import Encoder

    rng = np.random.default_rng(size + k)
    data = rng.integers(0, 256, size, dtype=np.uint8)
    enc = Encoder.new(data, k, ctx)
    src = orc.pad(data, k)
    full = np.zeros(enc.get_full_coded_piece_byte_len(), np.uint8)
    for _ in range(4):
        enc.code_with_buf(rng, full)
        assert np.array_equal(full, orc.encode(src, full[:k])[0])


def test_many_calls_one_workspace(ctx, orc):
    """300 calls in a row (one leased workspace: the epoch advances, each chunk counter re-arms itself), alternating a
    one-chunk and a 17-chunk piece so stale flags of the other shape are never mistaken for this call's."""
    from rlnc_amd.full import Encoder

    rng = np.random.default_rng(5)
    shapes = [(16, 4096), (16, 17 * 65536 - 5)]
    encs = []
    for k, L in shapes:
        src = _src(rng, k, L)
        encs.append((Encoder.without_padding(src.reshape(-1), k, ctx), src, np.zeros(L, np.uint8)))
    for i in range(300):
        enc, src, out = encs[i % 2]
        cv = rng.integers(0, 256, src.shape[0], dtype=np.uint8)
        enc.code_with_coding_vector(cv, out)
        if i % 7 == 0 or i > 290:
            assert np.array_equal(out, orc.code_with_coding_vector(src, cv)[1]), i


def test_many_split_calls_one_workspace(ctx, orc):
    """Products split across workgroups (more than 128 sources over few column blocks, piece.hip piece_split): 200
    calls in a row on one leased workspace alternating 5 blocks x 4 workgroups and 20 blocks x 5, so each block's
    counter must be re-armed by its last workgroup, and the partial slabs of the other shape are never read."""
    from rlnc_amd.full import Encoder

    rng = np.random.default_rng(6)
    shapes = [(256, 4097), (300, 20000)]
    encs = []
    for k, L in shapes:
        src = _src(rng, k, L)
        encs.append((Encoder.without_padding(src.reshape(-1), k, ctx), src, np.zeros(L, np.uint8)))
    for i in range(200):
        enc, src, out = encs[i % 2]
        cv = rng.integers(0, 256, src.shape[0], dtype=np.uint8)
        enc.code_with_coding_vector(cv, out)
        if i % 5 == 0 or i > 190:
            assert np.array_equal(out, orc.code_with_coding_vector(src, cv)[1]), i


@pytest.mark.parametrize("k,L", [(64, 40000), (256, 4097)])
def test_concurrent_calls_one_encoder(ctx, orc, k, L):
    """Encoder::code is &self on a Send + Sync type (encoder.rs:264): four threads on one encoder, each call on its
    own leased workspace (k = 256: the split product, each call with its own slabs and counters)."""
    from rlnc_amd.full import Encoder

    rng = np.random.default_rng(11)
    src = _src(rng, k, L)
    enc = Encoder.without_padding(src.reshape(-1), k, ctx)
    cvs = rng.integers(0, 256, (4, 40, k), dtype=np.uint8)
    outs = np.zeros((4, 40, L), np.uint8)

    def work(t):
        for i in range(40):
            enc.code_with_coding_vector(cvs[t, i], outs[t, i])

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for t in range(4):
        for i in (0, 17, 39):
            assert np.array_equal(outs[t, i], orc.code_with_coding_vector(src, cvs[t, i])[1]), (t, i)


@pytest.mark.parametrize("size,k", [(1 << 20, 16), (1 << 20, 64), (1 << 20, 256), (1 << 24, 128), (5000, 3)])
def test_recode_with_buf_matches_oracle(ctx, orc, size, k):
    from rlnc_amd.full import Encoder, Recoder

    rng = np.random.default_rng(size ^ k)
    data = rng.integers(0, 256, size, dtype=np.uint8)
    enc = Encoder.new(data, k, ctx)
    full = enc.get_full_coded_piece_byte_len()
    nrec = max(1, k // 2)
    coded = np.concatenate([enc.code(rng) for _ in range(nrec)])
    rec = Recoder.new(coded, full, k, ctx)
    out = np.zeros(full, np.uint8)
    for _ in range(3):
        r = rng.integers(0, 256, nrec, dtype=np.uint8)
        rec.recode_with_coding_vector(r, out)
        assert np.array_equal(out, orc.recode(coded, full, k, r))


@pytest.mark.parametrize("size,k", [(1 << 20, 16), (1 << 20, 32), (1 << 20, 128), (1 << 20, 256), (1 << 24, 16),
                                    (1 << 24, 32), ((1 << 25) + 12345, 64), (3000, 5)])
def test_get_decoded_data_recovers_source(ctx, size, k):
    """The decoder's T x data product through the piece kernel (k output rows, one flag chunk per 64 KiB of a row)
    returns the source bytes (decoder.rs:136-177), with dependent pieces mixed in.  Objects above 4 MiB take the batch
    kernels and one device-to-host copy."""
    from rlnc_amd.full import Decoder, Encoder

    rng = np.random.default_rng(size + 3 * k)
    data = rng.integers(0, 256, size, dtype=np.uint8)
    enc = Encoder.new(data, k, ctx)
    dec = Decoder.new(enc.get_piece_byte_len(), k, ctx)
    pieces = [enc.code(rng) for _ in range(k + 3)]
    pieces.insert(k // 2, pieces[0].copy())  # a duplicate: PieceNotUseful
    for p in pieces:
        if dec.is_already_decoded():
            break
        try:
            dec.decode(p)
        except Exception:
            pass
    got = dec.get_decoded_data()
    assert np.array_equal(got, data)


def test_get_decoded_data_large_objects_from_threads(ctx):
    """Large decodes' copy-out (pinned ring + the host copy pool, pre-faulting fresh caller buffers) from four threads
    at once, each on its own decoder of a 9-33 MiB object (fresh numpy buffers above glibc's mmap threshold and heap
    reuse below it): every result equals its source.  The pool serialises concurrent copies; each call's ring and
    events are its own workspace's."""
    import threading

    from rlnc_amd.full import Decoder, Encoder

    sizes = [(33 << 20) + 5, (9 << 20) + 77, (16 << 20) - 3, (24 << 20) + 1]
    decs, datas = [], []
    for i, size in enumerate(sizes):
        rng = np.random.default_rng(500 + i)
        data = rng.integers(0, 256, size, dtype=np.uint8)
        k = 16 if i % 2 else 32
        enc = Encoder.new(data, k, ctx)
        dec = Decoder.new(enc.get_piece_byte_len(), k, ctx)
        while not dec.is_already_decoded():
            try:
                dec.decode(enc.code(rng))
            except Exception:
                pass
        decs.append(dec)
        datas.append(data)
    results = [None] * len(decs)
    errors = []

    def work(i):
        try:
            for _ in range(2):  # the second call reuses the same workspace pool and pinned ring
                results[i] = decs[i].get_decoded_data()
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=work, args=(i,)) for i in range(len(decs))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors
    for got, data in zip(results, datas):
        assert np.array_equal(got, data)
