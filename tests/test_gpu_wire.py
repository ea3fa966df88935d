"""GPU: the wire formats either side of the hot path and host-resident streaming (§8(f1)).

* Encoder::new's padding + 0x81 marker built on the device (rlnc_pad_device / rlnc_pad_batch_device /
  rlnc_encoder_new_device) against the committed golden pad vectors (encoder.rs:85-106, consts.rs:5) and the
  oracle's pad, including unaligned sources, padded row strides and Encoder::new's error order.
* rlnc_encode_ragged: objects of different k, L and n (and scattered buffers) in one call, against the oracle.
* rlnc_encode_host_stream / rlnc_decode_host_stream from pageable and from pinned host memory, against the oracle
  and the device-resident batch calls.
"""
import ctypes as C

import numpy as np
import pytest

from oracle.oracle import OracleDecoder
from tests.conftest import hexarr
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


def _pad_dev(ctx, data_t, k, out_t, stride=0):
    return ctx.lib.rlnc_pad_device(ctx.h, C.c_void_p(data_t.data_ptr()), data_t.numel(), k,
                                   C.c_void_p(out_t.data_ptr()), stride)


def test_golden_pad_on_device(ctx, golden):
    import torch

    for v in golden["pad"]:
        data, k, L = hexarr(v["data"]), v["k"], v["L"]
        assert ctx.lib.rlnc_padded_piece_byte_len(data.size, k) == L
        want = np.frombuffer(bytes.fromhex(v["padded"]), np.uint8).reshape(k, L)
        for off, stride in [(0, 0), (3, 0), (1, L + 37)]:  # unaligned source bytes, padded row stride
            buf = torch.zeros(data.size + off, dtype=torch.uint8, device="cuda:0")
            buf[off:] = dev(data)
            rows = stride or L
            out = torch.full((k * rows + 64,), 0xEE, dtype=torch.uint8, device="cuda:0")
            assert _pad_dev(ctx, buf[off:], k, out, stride) == 0
            got = host(out)
            img = got[: k * rows].reshape(k, rows)
            assert np.array_equal(img[:, :L], want), (v["k"], off, stride)
            assert (got[k * rows:] == 0xEE).all()  # nothing written past the image
            if stride:
                assert (img[:, L:] == 0xEE).all()  # row padding untouched


def test_encoder_new_device_matches_host_encoder(ctx, orc):
    import torch

    from rlnc_amd import _lib
    from rlnc_amd.full import Encoder

    rng = np.random.default_rng(8)
    for n_bytes, k in [(1, 1), (100, 3), (4096 * 16 - 1, 16), (1 << 20, 32), (77_777, 20)]:
        data = rng.integers(0, 256, n_bytes, dtype=np.uint8)
        data[-1] = 0x81 if n_bytes % 2 else 0  # data ending in the marker / in zeros
        d = dev(data)
        h = C.c_void_p()
        assert ctx.lib.rlnc_encoder_new_device(ctx.h, C.c_void_p(d.data_ptr()), d.numel(), k, C.byref(h)) == 0
        enc_d = Encoder(h, ctx)
        enc_h = Encoder.new(data, k, ctx=ctx)
        assert enc_d.get_piece_byte_len() == enc_h.get_piece_byte_len() == orc.piece_byte_len(n_bytes, k)
        src = orc.pad(data, k)
        r1, r2 = np.random.default_rng(n_bytes), np.random.default_rng(n_bytes)
        for _ in range(3):
            p = enc_d.code(r1)
            assert np.array_equal(p, enc_h.code(r2))
            assert np.array_equal(p, orc.encode(src, p[:k])[0])
        del d
        torch.cuda.synchronize()
    # Encoder::new's error order on the device path
    z = dev(np.zeros(4, np.uint8))
    h = C.c_void_p()
    assert S[ctx.lib.rlnc_encoder_new_device(ctx.h, C.c_void_p(z.data_ptr()), 0, 0, C.byref(h))] == "DataLengthZero"
    assert S[ctx.lib.rlnc_encoder_new_device(ctx.h, C.c_void_p(z.data_ptr()), 4, 0, C.byref(h))] == "PieceCountZero"
    assert _lib.header_symbols()  # noqa: the header parses


def test_pad_batch_ragged_one_launch(ctx, orc):
    import torch

    from rlnc_amd import _lib

    rng = np.random.default_rng(9)
    shapes = [(5, 1), (4095, 16), (4096, 16), (10_000, 7), (1, 1), (300_001, 64)]
    datas = [rng.integers(0, 256, n, dtype=np.uint8) for n, _ in shapes]
    dd = [dev(x) for x in datas]
    outs, descs = [], []
    for (n, k), d in zip(shapes, dd):
        L = orc.piece_byte_len(n, k)
        o = torch.zeros(k * L, dtype=torch.uint8, device="cuda:0")
        outs.append(o)
        descs.append(_lib.PadDesc(d.data_ptr(), n, k, o.data_ptr(), 0))
    arr = (_lib.PadDesc * len(descs))(*descs)
    assert ctx.lib.rlnc_pad_batch_device(ctx.h, arr, len(descs)) == 0
    torch.cuda.synchronize()
    for (n, k), x, o in zip(shapes, datas, outs):
        assert np.array_equal(host(o), orc.pad(x, k).reshape(-1)), (n, k)


def test_encode_ragged_vs_oracle(ctx, orc):
    """Mixed k, L, n in one call: two runs at a constant object stride (one launch each), scattered objects,
    padded strides, and objects with n = 0."""
    import torch

    from rlnc_amd import _lib

    rng = np.random.default_rng(10)
    objs, keep, want = [], [], []

    def add(k, L, n, src_t, co_t, pc_t, ss=0, ps=0):
        objs.append(_lib.ObjectDesc(src_t.data_ptr(), ss, co_t.data_ptr(), pc_t.data_ptr(), ps, k, L, n))
        keep.extend([src_t, co_t, pc_t])

    # a run of 5 objects k=16 L=8192 n=20 in one contiguous buffer (one launch)
    k, L, n, B = 16, 8192, 20, 5
    src = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    co = rng.integers(0, 256, (B, n, k), dtype=np.uint8)
    ts, tc = dev(src), dev(co)
    tp = torch.zeros((B, n, k + L), dtype=torch.uint8, device="cuda:0")
    for o in range(B):
        add(k, L, n, ts[o], tc[o], tp[o])
        want.append((tp[o], orc.encode(src[o], co[o])))
    # scattered objects of other shapes, one with padded row strides, interleaved with the run's shape
    for k, L, n in [(32, 4096 * 3 + 5, 40), (7, 100, 3), (16, 8192, 20), (64, 4096, 70), (3, 1, 2)]:
        s_ = rng.integers(0, 256, (k, L), dtype=np.uint8)
        c_ = rng.integers(0, 256, (n, k), dtype=np.uint8)
        pad_s, pad_p = (48, 32) if k == 32 else (0, 0)
        ts_ = torch.zeros((k, L + pad_s), dtype=torch.uint8, device="cuda:0")
        ts_[:, :L] = dev(s_)
        tp_ = torch.zeros((n, k + L + pad_p), dtype=torch.uint8, device="cuda:0")
        add(k, L, n, ts_, dev(c_), tp_, L + pad_s if pad_s else 0, k + L + pad_p if pad_p else 0)
        want.append((tp_[:, : k + L], orc.encode(s_, c_)))
    empty = dev(np.zeros(16, np.uint8))
    add(4, 4, 0, empty, empty, empty)  # n = 0: nothing to do
    arr = (_lib.ObjectDesc * len(objs))(*objs)
    assert ctx.lib.rlnc_encode_ragged(ctx.h, arr, len(objs)) == 0
    torch.cuda.synchronize()
    for t, w in want:
        assert np.array_equal(host(t.contiguous()), w)


@pytest.mark.parametrize("window", [1, 2])
@pytest.mark.parametrize("pinned", [False, True])
def test_host_stream_encode_decode_vs_oracle(ctx, orc, pinned, window):
    """Pieces start and end in host memory: encode n coded pieces per object, decode the first m back; windows of
    1 or 2 objects over 7 objects (4-7 windows through 3 slots: every slot refilled behind its previous kernel and
    device-to-host copy), against the oracle and the device-resident batch."""
    import torch

    from rlnc_amd import batch

    k, L, n, m, nobj = 24, 4096 * 5 + 16, 30, 26, 7
    rng = np.random.default_rng(11 + pinned)
    data = [rng.integers(0, 256, k * L - 3, dtype=np.uint8) for _ in range(nobj)]

    def buf(shape, fill=None):
        t = torch.empty(shape, dtype=torch.uint8, pin_memory=pinned)
        if fill is not None:
            t.numpy()[...] = fill
        return t

    src = buf((nobj, k, L), np.stack([orc.pad(x, k) for x in data]))
    co_np = rng.integers(0, 256, (nobj, n, k), dtype=np.uint8)
    co_np[3, 5] = co_np[3, 1] ^ co_np[3, 2]  # a dependent piece among the first m of object 3
    co = buf((nobj, n, k), co_np)
    pieces = buf((nobj, n, k + L), 0)
    p = lambda t: C.c_void_p(t.data_ptr())
    assert ctx.lib.rlnc_encode_host_stream(ctx.h, p(src), k, L, nobj, p(co), n, p(pieces), window) == 0
    hp = pieces.numpy()
    for o in range(nobj):
        assert np.array_equal(hp[o], orc.encode(src.numpy()[o], co_np[o])), o
    decoded = buf((nobj, k, L), 0)
    ps = np.zeros((nobj, m), np.int32)
    os_ = np.zeros(nobj, np.int32)
    dl = np.zeros(nobj, np.uint64)
    assert ctx.lib.rlnc_decode_host_stream(ctx.h, p(pieces), n * (k + L), k, L, m, nobj, p(decoded),
                                           ps.ctypes.data_as(C.POINTER(C.c_int32)),
                                           os_.ctypes.data_as(C.POINTER(C.c_int32)),
                                           dl.ctypes.data_as(C.POINTER(C.c_uint64)), window) == 0
    hd = decoded.numpy()
    for o in range(nobj):
        od = OracleDecoder(L, k)
        assert list(ps[o]) == [od.decode(x) for x in hp[o, :m]], o
        pay = od.padded_payload()
        assert np.array_equal(hd[o, : pay.shape[0]], pay), o
        st, want = od.get_decoded_data()
        assert os_[o] == st, o
        if st == 0:
            assert int(dl[o]) == want.size == data[o].size and np.array_equal(hd[o].reshape(-1)[: dl[o]], data[o])
    # the same bytes as the device-resident batch calls
    dpieces = torch.empty((nobj, n, k + L), dtype=torch.uint8, device="cuda:0")
    batch.encode_batch(src.cuda(), co.cuda(), dpieces, ctx)
    assert np.array_equal(host(dpieces), hp)


def test_host_stream_auto_window_and_errors(ctx, orc):
    import torch

    k, L, n, nobj = 8, 4096, 10, 5
    rng = np.random.default_rng(12)
    src = rng.integers(0, 256, (nobj, k, L), dtype=np.uint8)
    co = rng.integers(0, 256, (nobj, n, k), dtype=np.uint8)
    out = np.zeros((nobj, n, k + L), np.uint8)
    pp = lambda a: a.ctypes.data_as(C.c_void_p)
    assert ctx.lib.rlnc_encode_host_stream(ctx.h, pp(src), k, L, nobj, pp(co), n, pp(out), 0) == 0
    for o in range(nobj):
        assert np.array_equal(out[o], orc.encode(src[o], co[o]))
    assert S[ctx.lib.rlnc_encode_host_stream(ctx.h, pp(src), 0, L, nobj, pp(co), n, pp(out), 0)] == "PieceCountZero"
    assert S[ctx.lib.rlnc_encode_host_stream(ctx.h, pp(src), k, 0, nobj, pp(co), n, pp(out), 0)] == "PieceLengthZero"
    torch.cuda.synchronize()
