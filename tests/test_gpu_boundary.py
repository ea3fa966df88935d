"""GPU: the boundary contract of include/rlnc_hip.h beyond single-threaded use.

* Encoder::code(&self) from 8 threads at once on ONE encoder (the reference Encoder is Send + Sync,
  encoder.rs:264): every coded piece equals the oracle's for the same coefficient bytes.
* #[derive(Clone)] of Encoder / Decoder / Recoder (encoder.rs:18, decoder.rs:8, recoder.rs:12).
* Objects outlive the context handle they were created with (the context is reference counted).
* Batch calls without an explicit context on two torch streams: each stream gets its own context (its
  workspaces are stream-ordered), results against the numpy matmul.
* Decoder::decode staged through the pinned upload ring (caller buffer reuse, chunked pieces, clone / drop with
  uploads in flight).
* The 8-wave (variant 8) program with padded row strides, a header slot and several objects.
"""
import ctypes as C
import threading

import numpy as np
import pytest

from oracle.oracle import OracleDecoder
from tests.gpu_util import dev, host, np_matmul

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import torch

    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    import rlnc_amd

    return rlnc_amd.Context(0)


class SeqRng:
    def __init__(self, seed):
        self.g = np.random.default_rng(seed)
        self.draws = []

    def fill_bytes(self, n):
        b = self.g.integers(0, 256, n, dtype=np.uint8)
        self.draws.append(b)
        return b.tobytes()


@pytest.mark.parametrize("data_len,k", [(1 << 20, 32), (200_000, 16)])
def test_encoder_code_from_8_threads(ctx, orc, data_len, k):
    from rlnc_amd.full import Encoder

    data = np.random.default_rng(data_len).integers(0, 256, data_len, dtype=np.uint8)
    enc = Encoder.new(data, k, ctx=ctx)
    src = orc.pad(data, k)
    nth, per = 8, 12
    out = [[] for _ in range(nth)]
    rngs = [SeqRng(100 + t) for t in range(nth)]
    errors = []
    barrier = threading.Barrier(nth)

    def work(t):
        try:
            barrier.wait()
            for _ in range(per):
                out[t].append(enc.code(rngs[t]))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    ths = [threading.Thread(target=work, args=(t,)) for t in range(nth)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors
    for t in range(nth):
        want = orc.encode(src, np.stack(rngs[t].draws))
        assert np.array_equal(np.stack(out[t]), want), t


def test_recoders_and_decoders_on_threads_share_a_context(ctx, orc):
    """Distinct decoders / recoders used concurrently from threads on one context (each call leases its own
    workspace)."""
    from rlnc_amd.full import Decoder, Encoder, Recoder

    k = 16
    datas = [np.random.default_rng(s).integers(0, 256, 30_000 + s, dtype=np.uint8) for s in range(6)]
    results = [None] * len(datas)

    def work(i):
        rng = np.random.default_rng(50 + i)
        enc = Encoder.new(datas[i], k, ctx=ctx)
        coded = np.concatenate([enc.code(rng) for _ in range(k + 4)])
        rec = Recoder.new(coded, enc.get_full_coded_piece_byte_len(), k, ctx=ctx)
        dec = Decoder.new(enc.get_piece_byte_len(), k, ctx=ctx)
        while not dec.is_already_decoded():
            try:
                dec.decode(rec.recode(rng))
            except Exception:
                pass
        results[i] = dec.get_decoded_data()

    ths = [threading.Thread(target=work, args=(i,)) for i in range(len(datas))]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    for i, d in enumerate(datas):
        assert np.array_equal(results[i], d), i


def test_clone_encoder_decoder_recoder(ctx, orc):
    import copy

    from rlnc_amd.errors import RLNCError
    from rlnc_amd.full import Decoder, Encoder, Recoder

    k = 20
    data = np.random.default_rng(3).integers(0, 256, 50_001, dtype=np.uint8)
    enc = Encoder.new(data, k, ctx=ctx)
    enc2 = enc.clone()
    del enc  # the clone owns its own copy of the source
    a, b = SeqRng(1), SeqRng(1)
    enc3 = copy.copy(enc2)
    assert np.array_equal(enc2.code(a), enc3.code(b))
    rng = SeqRng(2)
    dec = Decoder.new(enc2.get_piece_byte_len(), k, ctx=ctx)
    seen = []
    for _ in range(k // 2):
        p = enc2.code(rng)
        dec.decode(p)
        seen.append(p)
    dec2 = dec.clone()
    assert (dec2.get_received_piece_count(), dec2.get_useful_piece_count()) == (k // 2, k // 2)
    # the original continues with pieces the clone never sees, and vice versa
    r1, r2 = np.random.default_rng(7), np.random.default_rng(8)
    for d, r in [(dec, r1), (dec2, r2)]:
        while not d.is_already_decoded():
            try:
                d.decode(enc2.code(r))
            except RLNCError as e:
                assert e == RLNCError.PieceNotUseful
    assert np.array_equal(dec.get_decoded_data(), data) and np.array_equal(dec2.get_decoded_data(), data)
    rec = Recoder.new(np.concatenate(seen), enc2.get_full_coded_piece_byte_len(), k, ctx=ctx)
    rec2 = rec.clone()
    del rec
    x, y = SeqRng(9), SeqRng(9)
    got = rec2.recode(x)
    assert np.array_equal(got, orc.recode(np.concatenate(seen), k + enc2.get_piece_byte_len(), k, x.draws[0]))
    assert np.array_equal(rec2.clone().recode(y), got)


@pytest.mark.parametrize("data_len,k", [(1 << 20, 16), ((9 << 20) + 5, 2), (4_500_000, 64), (300_000, 200)])
def test_decoder_staged_uploads(ctx, data_len, k):
    """Decoder::decode returns once its piece is staged in pinned memory, before the DMA: one caller buffer reused
    for every piece, interleaved decoders packing one staging slot and cycling the ring (the 4.5 MB / k = 64 case
    wraps it several times), pieces over the 4 MiB slot (several slots per piece), a clone and a drop taken with
    pieces still staged -- every decoded object equals its source."""
    from rlnc_amd.errors import RLNCError
    from rlnc_amd.full import Decoder, Encoder

    rng = np.random.default_rng(data_len)
    datas = [rng.integers(0, 256, data_len + i, dtype=np.uint8) for i in range(3)]
    encs = [Encoder.new(d, k, ctx=ctx) for d in datas]
    decs = [Decoder.new(e.get_piece_byte_len(), k, ctx=ctx) for e in encs]
    bufs = [np.empty(e.get_full_coded_piece_byte_len(), np.uint8) for e in encs]
    clone = None
    while not all(d.is_already_decoded() for d in decs):
        for i, (e, d) in enumerate(zip(encs, decs)):
            if d.is_already_decoded():
                continue
            bufs[i][:] = e.code(rng)  # the caller's one buffer, rewritten after every call
            try:
                d.decode(bufs[i])
            except RLNCError as err:
                assert err == RLNCError.PieceNotUseful
            bufs[i][:] = 0
            if i == 0 and clone is None and d.get_useful_piece_count() == k // 2:
                clone = d.clone()
                scratch = Decoder.new(e.get_piece_byte_len(), k, ctx=ctx)
                scratch.decode(e.code(rng))
                del scratch  # dropped with its upload possibly still queued
    for d, data in zip(decs, datas):
        assert np.array_equal(d.get_decoded_data(), data)
    while not clone.is_already_decoded():
        try:
            clone.decode(encs[0].code(rng))
        except RLNCError as err:
            assert err == RLNCError.PieceNotUseful
    assert np.array_equal(clone.get_decoded_data(), datas[0])


def test_objects_outlive_their_context_handle(orc):
    import rlnc_amd
    from rlnc_amd.full import Decoder, Encoder

    c = rlnc_amd.Context(0)
    data = np.random.default_rng(11).integers(0, 256, 9_999, dtype=np.uint8)
    enc = Encoder.new(data, 8, ctx=c)
    dec = Decoder.new(enc.get_piece_byte_len(), 8, ctx=c)
    c.close()  # drops the creator's reference only
    rng = np.random.default_rng(12)
    while not dec.is_already_decoded():
        try:
            dec.decode(enc.code(rng))
        except rlnc_amd.RLNCError:
            pass
    assert np.array_equal(dec.get_decoded_data(), data)


def test_batch_default_contexts_per_stream():
    """No explicit context, two streams in flight at once: each stream gets its own default context."""
    import torch

    from rlnc_amd import batch

    rng = np.random.default_rng(21)
    shapes = [(3, 24, 4096 * 6, 40), (5, 16, 4096 * 4 + 32, 70)]
    jobs = []
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for rep in range(3):
        for (nobj, k, L, n), s in zip(shapes, streams):
            src = rng.integers(0, 256, (nobj, k, L), dtype=np.uint8)
            co = rng.integers(0, 256, (nobj, n, k), dtype=np.uint8)
            with torch.cuda.stream(s):
                dsrc, dco = dev(src), dev(co)
                out = torch.empty((nobj, n, k + L), dtype=torch.uint8, device="cuda:0")
                batch.encode_batch(dsrc, dco, out)
            jobs.append((src, co, out, dsrc, dco))
    torch.cuda.synchronize()
    for src, co, out, _, _ in jobs:
        got = host(out)
        for o in range(src.shape[0]):
            assert np.array_equal(got[o, :, : co.shape[2]], co[o])
            assert np.array_equal(got[o, :, co.shape[2]:], np_matmul(co[o], src[o]))


@pytest.mark.parametrize("n_out", [40, 70])
def test_variant8_strided_with_header(ctx, n_out):
    """The 8-wave program (n_out > 32) with padded strides, a 64-byte header slot and 2 objects."""
    import torch

    from rlnc_amd import _lib
    from rlnc_amd.errors import check

    rng = np.random.default_rng(n_out)
    nobj, n_in, W, pad = 2, 20, 4096 * 5 + 32, 48
    coef = rng.integers(0, 256, (nobj, n_out, n_in), dtype=np.uint8)
    inp = rng.integers(0, 256, (nobj, n_in, W + pad), dtype=np.uint8)
    row = 64 + W + pad
    pieces = dev(np.zeros((nobj, n_out, row), np.uint8))
    dcoef, dinp = dev(coef), dev(inp)
    base = pieces.data_ptr()
    d = _lib.MatmulDesc(dinp.data_ptr(), n_in * (W + pad), W + pad, dcoef.data_ptr(), n_out * n_in, n_in,
                        base + 64, n_out * row, row, base, n_out * row, row, n_out, n_in, W, nobj)
    ctx.set_kernel_variant(8, 0)
    check(ctx.lib.rlnc_gf256_matmul(ctx.h, C.byref(d)), ctx.lib)
    torch.cuda.synchronize()
    got = host(pieces)
    for o in range(nobj):
        assert np.array_equal(got[o, :, :n_in], coef[o])
        assert np.array_equal(got[o, :, 64:64 + W], np_matmul(coef[o], inp[o, :, :W]))
        assert not got[o, :, 64 + W:].any() and not got[o, :, n_in:64].any()


def test_stream_contexts_stay_bounded():
    """batch calls without an explicit context on many torch streams keep at most STREAM_CONTEXTS_PER_THREAD
    default contexts per thread (each holds grow-only workspaces), and every call stays correct."""
    import torch

    from rlnc_amd import batch, context
    from tests.gpu_util import dev, host, np_matmul

    rng = np.random.default_rng(21)
    src = rng.integers(0, 256, (1, 8, 4096), dtype=np.uint8)
    co = rng.integers(0, 256, (1, 12, 8), dtype=np.uint8)
    want = np_matmul(co[0], src[0])
    streams = [torch.cuda.Stream() for _ in range(12)]
    for rep in range(2):
        for s in streams:
            with torch.cuda.stream(s):
                out = torch.zeros((1, 12, 8 + 4096), dtype=torch.uint8, device="cuda:0")
                batch.encode_batch(dev(src), dev(co), out)
            s.synchronize()
            assert np.array_equal(host(out)[0, :, 8:], want)
            assert len(context._tls.sctxs) <= context.STREAM_CONTEXTS_PER_THREAD
    context.release_stream_contexts()
    assert len(context._tls.sctxs) == 0
