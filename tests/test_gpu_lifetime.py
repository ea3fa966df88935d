"""GPU: object lifetimes on a shared context (engine.cpp / context.hpp ObjUse).  Dropping an Encoder / Recoder /
Decoder waits for that object's own stream-ordered uses only -- never for unrelated work queued on the context's
stream -- and a dropped object's device block is reused by the next object only after every launch that read it,
whichever stream the context used then."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _long_batch(torch, ctx, reps):
    """`reps` encode launches of 16 objects x k = 32 x 1 MiB x 32 coded pieces on the context's current stream:
    ~0.6 ms each.  Returns the tensors (kept alive until the stream has run)."""
    from rlnc_amd import batch

    g = torch.Generator(device="cuda").manual_seed(1)
    src = torch.randint(0, 256, (16, 32, 1 << 20), dtype=torch.uint8, device="cuda", generator=g)
    co = torch.randint(0, 256, (16, 32, 32), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty((16, 32, 32 + (1 << 20)), dtype=torch.uint8, device="cuda")
    for _ in range(reps):
        batch.encode_batch(src, co, out, ctx)
    return src, co, out


def test_drop_does_not_wait_for_unrelated_stream_work():
    """Objects built and used first (a decoder that decoded and returned its data, an encoder that also ran a
    code_batch_device launch, a recoder); then ~100 ms of batch encodes queued on the context's stream; then the
    objects are dropped: the drops return at once and the batch is still running after them.  (Round 3 synchronised
    the whole context stream on every drop.)"""
    import torch

    import rlnc_amd
    from rlnc_amd.full import Decoder, Encoder, Recoder

    ctx = rlnc_amd.Context(0)
    ctx.use_torch_stream()
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    enc = Encoder.new(data, 16, ctx)
    pieces = [enc.code(rng) for _ in range(18)]
    dec = Decoder.new(enc.get_piece_byte_len(), 16, ctx)
    for p in pieces:
        if dec.is_already_decoded():
            break
        try:
            dec.decode(p)
        except Exception:
            pass
    assert np.array_equal(dec.get_decoded_data(), data)
    rec = Recoder.new(np.concatenate(pieces[:4]), enc.get_full_coded_piece_byte_len(), 16, ctx)
    rec.recode(rng)
    co = torch.from_numpy(rng.integers(0, 256, (4, 16), dtype=np.uint8)).cuda()
    out = torch.empty((4, enc.get_full_coded_piece_byte_len()), dtype=torch.uint8, device="cuda")
    enc.code_batch_device(co.data_ptr(), 4, out.data_ptr())
    torch.cuda.synchronize()
    keep = _long_batch(torch, ctx, 160)
    t0 = time.perf_counter()
    del dec, enc, rec
    drop_ms = (time.perf_counter() - t0) * 1e3
    still_running = not torch.cuda.current_stream().query()
    torch.cuda.synchronize()
    del keep
    print(f"drops {drop_ms:.3f} ms, batch still running after them: {still_running}")
    assert still_running, "the drops waited for the unrelated batch"
    assert drop_ms < 5.0


def test_dropped_encoder_block_reused_only_after_its_launches():
    """code_batch_device queued on stream A (with unrelated work ahead of it), the context switched to stream B, the
    encoder dropped, a new encoder of the same size built at once (the block cache hands it the old block; its upload
    would overwrite the source): the launch on A still reads the old source (advisor round 3)."""
    import torch

    import rlnc_amd
    from oracle.oracle import Oracle, build
    from rlnc_amd.full import Encoder

    build()
    orc = Oracle()
    ctx = rlnc_amd.Context(0)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    rng = np.random.default_rng(9)
    k, L = 32, 1 << 16
    data = rng.integers(0, 256, k * L, dtype=np.uint8)
    enc = Encoder.without_padding(data, k, ctx)
    n = 64
    coeffs = rng.integers(0, 256, (n, k), dtype=np.uint8)
    with torch.cuda.stream(sa):
        co_dev = torch.from_numpy(coeffs).cuda()
        out_dev = torch.zeros((n, k + L), dtype=torch.uint8, device="cuda")
        ctx.use_torch_stream()
        keep = _long_batch(torch, ctx, 60)  # ~40 ms ahead of the launch below on stream A
        enc.code_batch_device(co_dev.data_ptr(), n, out_dev.data_ptr())
    ctx.set_stream(sb.cuda_stream)
    del enc
    other = rng.integers(0, 256, k * L, dtype=np.uint8)
    enc2 = Encoder.without_padding(other, k, ctx)  # same size: the cached block
    sa.synchronize()
    got = out_dev.cpu().numpy()
    want = orc.encode(data.reshape(k, L), coeffs)
    assert np.array_equal(got, want)
    del enc2, keep


def test_block_reused_only_after_uses_on_two_streams():
    """An encoder used on stream A (behind a GPU spin of tens of ms that touches none of the context's workspaces) and
    then on stream B (nothing ahead): dropping it must wait for A's launch too, not only for the latest use on B,
    before the block cache hands the block to a new encoder whose upload overwrites the source.  (The context's
    workspaces are stream-ordered: the two launches never overlap here, A's runs after B's.)  Where B shares a
    hardware queue with A, B's launch itself runs after A's and the case passes either way.)"""
    import torch

    import rlnc_amd
    from oracle.oracle import Oracle, build
    from rlnc_amd.full import Encoder

    build()
    orc = Oracle()
    ctx = rlnc_amd.Context(0)
    # B at high priority: a hardware queue of its own, so its launch runs while A still spins (two streams of one
    # priority may share a queue and serialise, which would hide the case)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream(priority=-1)
    rng = np.random.default_rng(11)
    k, L = 32, 1 << 16
    data = rng.integers(0, 256, k * L, dtype=np.uint8)
    enc = Encoder.without_padding(data, k, ctx)
    n = 64
    ca, cb = (rng.integers(0, 256, (n, k), dtype=np.uint8) for _ in range(2))
    ca_dev, cb_dev = torch.from_numpy(ca).cuda(), torch.from_numpy(cb).cuda()
    out_a = torch.zeros((n, k + L), dtype=torch.uint8, device="cuda")
    out_b = torch.zeros((n, k + L), dtype=torch.uint8, device="cuda")
    # one launch first: the context's workspaces grow to this shape now (a growth frees the old buffer, and hipFree
    # waits for the whole device, which would run A's spin out before B's launch)
    enc.code_batch_device(cb_dev.data_ptr(), n, out_b.data_ptr())
    torch.cuda.synchronize()
    out_b.zero_()
    with torch.cuda.stream(sa):
        torch.cuda._sleep(200_000_000)
        ctx.use_torch_stream()
        enc.code_batch_device(ca_dev.data_ptr(), n, out_a.data_ptr())
    with torch.cuda.stream(sb):
        ctx.use_torch_stream()
        enc.code_batch_device(cb_dev.data_ptr(), n, out_b.data_ptr())
        still_waiting = not sa.query()  # A's launch has not run yet when the encoder is dropped
        del enc
        other = rng.integers(0, 256, k * L, dtype=np.uint8)
        enc2 = Encoder.without_padding(other, k, ctx)  # same size: the cached block
    torch.cuda.synchronize()
    src = data.reshape(k, L)
    assert still_waiting, "stream A's spin ended before the drop: the case was not exercised"
    assert np.array_equal(out_b.cpu().numpy(), orc.encode(src, cb))
    assert np.array_equal(out_a.cpu().numpy(), orc.encode(src, ca))
    del enc2
