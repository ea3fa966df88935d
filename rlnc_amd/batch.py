"""Multi-object, device-resident batch API on torch tensors (torch is plumbing: HBM + streams only).

Layouts (uint8, contiguous, on the context's device):
    src     [obj][k][L]          source pieces (Encoder::new's padded image per object)
    coeffs  [obj][n][k]          coding vectors
    pieces  [obj][n][k+L]        full coded pieces, coeffs ‖ data (encoder.rs:246-248)
    decoded [obj][k][L]          padded payload rows (decoder.rs:141-153)
All launches go to torch's current stream of the tensors' device.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import MatmulDesc
from .context import Context, stream_context
from .errors import check


def _ctx_for(t, ctx: Context | None) -> Context:
    """The context a batch call launches with, on torch's current stream.  Without an explicit ctx each
    (device, stream) pair gets its own default context: a context's workspaces are stream-ordered, so two
    streams sharing one would overwrite each other's in-flight index stream / transform (include/rlnc_hip.h,
    Threading)."""
    import torch

    dev = t.device.index or 0
    if ctx is None:
        ctx = stream_context(dev, torch.cuda.current_stream(dev).cuda_stream)
    else:
        ctx.use_torch_stream()
    if torch.cuda.is_current_stream_capturing():
        ctx.graph_bound = True  # the graph holds its workspace addresses: never evicted (context.stream_context)
    return ctx


def _chk(t, shape=None):
    import torch

    assert t.is_cuda and t.dtype == torch.uint8 and t.is_contiguous(), "uint8 contiguous device tensor required"
    if shape is not None:
        assert tuple(t.shape) == tuple(shape), (tuple(t.shape), shape)


def encode_batch(src, coeffs, out, ctx: Context | None = None) -> None:
    """out[o][i] = coeffs[o][i] ‖ Σ_j coeffs[o][i][j]·src[o][j]  (n coded pieces per object)."""
    nobj, k, L = src.shape
    n = coeffs.shape[1]
    _chk(src)
    _chk(coeffs, (nobj, n, k))
    _chk(out, (nobj, n, k + L))
    ctx = _ctx_for(src, ctx)
    check(ctx.lib.rlnc_encode_batch(ctx.h, C.c_void_p(src.data_ptr()), k, L, nobj, C.c_void_p(coeffs.data_ptr()), n,
                                    C.c_void_p(out.data_ptr())), ctx.lib)


def encode_batch_headers(coeffs, out, ctx: Context | None = None) -> None:
    """The coefficient headers of encode_batch alone: out[o][i][0..k) = coeffs[o][i] (encoder.rs:246-248)."""
    nobj, n, k = coeffs.shape
    _chk(coeffs)
    _chk(out)
    assert out.shape[0] == nobj and out.shape[1] == n and out.shape[2] > k
    ctx = _ctx_for(out, ctx)
    check(ctx.lib.rlnc_encode_batch_headers(ctx.h, C.c_void_p(coeffs.data_ptr()), k, out.shape[2] - k, nobj, n,
                                            C.c_void_p(out.data_ptr())), ctx.lib)


def encode_batch_data(src, coeffs, out, ctx: Context | None = None) -> None:
    """The data part of encode_batch alone: out[o][i][k..) = Σ_j coeffs[o][i][j]·src[o][j]."""
    nobj, k, L = src.shape
    n = coeffs.shape[1]
    _chk(src)
    _chk(coeffs, (nobj, n, k))
    _chk(out, (nobj, n, k + L))
    ctx = _ctx_for(src, ctx)
    check(ctx.lib.rlnc_encode_batch_data(ctx.h, C.c_void_p(src.data_ptr()), k, L, nobj,
                                         C.c_void_p(coeffs.data_ptr()), n, C.c_void_p(out.data_ptr())), ctx.lib)


def encode_plan_bytes(k: int, nobj: int, n: int) -> int:
    """Device bytes of an encode plan buffer (encode_batch_prepare)."""
    from ._lib import load

    return int(load().rlnc_encode_batch_plan_bytes(k, nobj, n))


def encode_batch_prepare(src, coeffs, out, plan, ctx: Context | None = None) -> None:
    """The code-block address stream of encode_batch_data(src, coeffs, out) written ahead into `plan` (a uint8 device
    tensor of encode_plan_bytes bytes) on this context's stream -- e.g. a side stream, so that the encode launch
    itself does not wait for it (encode_batch_data_planned)."""
    nobj, k, L = src.shape
    n = coeffs.shape[1]
    _chk(src)
    _chk(coeffs, (nobj, n, k))
    _chk(out, (nobj, n, k + L))
    _chk(plan)
    ctx = _ctx_for(src, ctx)
    check(ctx.lib.rlnc_encode_batch_prepare(ctx.h, C.c_void_p(src.data_ptr()), k, L, nobj,
                                            C.c_void_p(coeffs.data_ptr()), n, C.c_void_p(out.data_ptr()),
                                            C.c_void_p(plan.data_ptr()), plan.numel()), ctx.lib)


def encode_batch_data_planned(src, coeffs, out, plan, ctx: Context | None = None) -> None:
    """encode_batch_data with the address stream prepared by encode_batch_prepare (same arguments); the caller
    orders this launch after the prepare."""
    nobj, k, L = src.shape
    n = coeffs.shape[1]
    _chk(src)
    _chk(coeffs, (nobj, n, k))
    _chk(out, (nobj, n, k + L))
    ctx = _ctx_for(src, ctx)
    check(ctx.lib.rlnc_encode_batch_data_planned(ctx.h, C.c_void_p(src.data_ptr()), k, L, nobj,
                                                 C.c_void_p(coeffs.data_ptr()), n, C.c_void_p(out.data_ptr()),
                                                 C.c_void_p(plan.data_ptr())), ctx.lib)


def recode_batch(pieces, r, out, k: int, ctx: Context | None = None) -> None:
    """out[o][c] = Σ_i r[o][c][i]·pieces[o][i] (coefficient header and data alike, recoder.rs:122-153)."""
    nobj, n, full = pieces.shape
    count = r.shape[1]
    _chk(pieces)
    _chk(r, (nobj, count, n))
    _chk(out, (nobj, count, full))
    ctx = _ctx_for(pieces, ctx)
    check(ctx.lib.rlnc_recode_batch(ctx.h, C.c_void_p(pieces.data_ptr()), k, full - k, n, nobj,
                                    C.c_void_p(r.data_ptr()), count, C.c_void_p(out.data_ptr())), ctx.lib)


def decode_batch(pieces, k: int, decoded, ctx: Context | None = None):
    """Feed pieces[o][0..m) to a fresh Decoder per object; returns (piece_status[obj][m],
    object_status[obj], data_len[obj]) as numpy arrays (status codes: rlnc_amd.errors.STATUS_NAMES).
    `pieces` may be a view pieces_all[:, :m] of more coded pieces (rows contiguous, objects strided)."""
    import torch

    nobj, m, full = pieces.shape
    L = full - k
    assert pieces.is_cuda and pieces.dtype == torch.uint8
    # strides of size-1 dimensions are arbitrary in torch; only real ones are checked
    obj_stride = pieces.stride(0) if nobj > 1 else m * full
    assert (full == 1 or pieces.stride(2) == 1) and (m == 1 or pieces.stride(1) == full) and obj_stride >= m * full
    _chk(decoded, (nobj, k, L))
    ctx = _ctx_for(pieces, ctx)
    ps = np.zeros((nobj, m), np.int32)
    os_ = np.zeros(nobj, np.int32)
    dl = np.zeros(nobj, np.uint64)
    check(ctx.lib.rlnc_decode_batch(ctx.h, C.c_void_p(pieces.data_ptr()), obj_stride, k, L, m, nobj,
                                    C.c_void_p(decoded.data_ptr()),
                                    ps.ctypes.data_as(C.POINTER(C.c_int32)), os_.ctypes.data_as(C.POINTER(C.c_int32)),
                                    dl.ctypes.data_as(C.POINTER(C.c_uint64))), ctx.lib)
    return ps, os_, dl


def decode_batch_device(pieces, k: int, decoded, piece_status, object_status, data_len, ctx: Context | None = None):
    """Asynchronous decode_batch with device outputs: piece_status int32 [obj][m], object_status int32 [obj],
    data_len int64 [obj] (all device tensors)."""
    import torch

    nobj, m, full = pieces.shape
    L = full - k
    obj_stride = pieces.stride(0) if nobj > 1 else m * full
    assert (m == 1 or pieces.stride(1) == full) and obj_stride >= m * full
    _chk(decoded, (nobj, k, L))
    assert piece_status.dtype == torch.int32 and tuple(piece_status.shape) == (nobj, m)
    assert object_status.dtype == torch.int32 and data_len.dtype == torch.int64
    ctx = _ctx_for(pieces, ctx)
    check(ctx.lib.rlnc_decode_batch_device(ctx.h, C.c_void_p(pieces.data_ptr()), obj_stride, k, L, m, nobj,
                                           C.c_void_p(decoded.data_ptr()), C.c_void_p(piece_status.data_ptr()),
                                           C.c_void_p(object_status.data_ptr()), C.c_void_p(data_len.data_ptr())),
          ctx.lib)


def _pieces_view(pieces, k):
    nobj, m, full = pieces.shape
    obj_stride = pieces.stride(0) if nobj > 1 else m * full
    assert (m == 1 or pieces.stride(1) == full) and obj_stride >= m * full
    return nobj, m, full - k, obj_stride


def decode_batch_eliminate(pieces, k: int, T, piece_status, rank, ctx: Context | None = None):
    """The elimination half of decode_batch_device (reads only the coefficient bytes): T uint8 [obj][k][m],
    piece_status int32 [obj][m], rank int32 [obj] (device tensors), asynchronous on the current stream."""
    import torch

    nobj, m, L, obj_stride = _pieces_view(pieces, k)
    _chk(T, (nobj, k, m))
    assert piece_status.dtype == torch.int32 and tuple(piece_status.shape) == (nobj, m)
    assert rank.dtype == torch.int32 and rank.numel() == nobj
    ctx = _ctx_for(pieces, ctx)
    check(ctx.lib.rlnc_decode_batch_eliminate(ctx.h, C.c_void_p(pieces.data_ptr()), obj_stride, k, L, m, nobj,
                                              C.c_void_p(T.data_ptr()), C.c_void_p(piece_status.data_ptr()),
                                              C.c_void_p(rank.data_ptr())), ctx.lib)


def decode_batch_apply(pieces, k: int, T, rank, decoded, object_status, data_len, ctx: Context | None = None):
    """The data half of decode_batch_device: decoded = T × received data, then the marker scan."""
    import torch

    nobj, m, L, obj_stride = _pieces_view(pieces, k)
    _chk(T, (nobj, k, m))
    _chk(decoded, (nobj, k, L))
    assert object_status.dtype == torch.int32 and data_len.dtype == torch.int64
    ctx = _ctx_for(pieces, ctx)
    check(ctx.lib.rlnc_decode_batch_apply(ctx.h, C.c_void_p(pieces.data_ptr()), obj_stride, k, L, m, nobj,
                                          C.c_void_p(T.data_ptr()), C.c_void_p(rank.data_ptr()),
                                          C.c_void_p(decoded.data_ptr()), C.c_void_p(object_status.data_ptr()),
                                          C.c_void_p(data_len.data_ptr())), ctx.lib)


def decode_apply_plan_bytes(k: int, m: int, nobj: int) -> int:
    """Device bytes of a decode plan buffer (decode_batch_apply_prepare)."""
    from ._lib import load

    return int(load().rlnc_decode_batch_apply_plan_bytes(k, m, nobj))


def decode_batch_apply_prepare(pieces, k: int, T, decoded, plan, ctx: Context | None = None):
    """The code-block address stream of decode_batch_apply(pieces, k, T, ..., decoded) written ahead into `plan` (a
    uint8 device tensor of decode_apply_plan_bytes bytes) on this context's stream, once T is final -- e.g. behind
    decode_batch_eliminate on its side stream, so that the data side does not wait for it
    (decode_batch_apply_planned)."""
    nobj, m, L, obj_stride = _pieces_view(pieces, k)
    _chk(T, (nobj, k, m))
    _chk(decoded, (nobj, k, L))
    _chk(plan)
    ctx = _ctx_for(pieces, ctx)
    check(ctx.lib.rlnc_decode_batch_apply_prepare(ctx.h, C.c_void_p(pieces.data_ptr()), obj_stride, k, L, m, nobj,
                                                  C.c_void_p(T.data_ptr()), C.c_void_p(decoded.data_ptr()),
                                                  C.c_void_p(plan.data_ptr()), plan.numel()), ctx.lib)


def decode_batch_apply_planned(pieces, k: int, T, rank, decoded, object_status, data_len, plan,
                               ctx: Context | None = None):
    """decode_batch_apply with the address stream prepared by decode_batch_apply_prepare (same arguments); the caller
    orders this launch after the prepare."""
    import torch

    nobj, m, L, obj_stride = _pieces_view(pieces, k)
    _chk(T, (nobj, k, m))
    _chk(decoded, (nobj, k, L))
    assert object_status.dtype == torch.int32 and data_len.dtype == torch.int64
    ctx = _ctx_for(pieces, ctx)
    check(ctx.lib.rlnc_decode_batch_apply_planned(ctx.h, C.c_void_p(pieces.data_ptr()), obj_stride, k, L, m, nobj,
                                                  C.c_void_p(T.data_ptr()), C.c_void_p(rank.data_ptr()),
                                                  C.c_void_p(decoded.data_ptr()),
                                                  C.c_void_p(object_status.data_ptr()),
                                                  C.c_void_p(data_len.data_ptr()), C.c_void_p(plan.data_ptr())),
          ctx.lib)


def matmul(coef, inp, out, ctx: Context | None = None) -> None:
    """out[o] = coef[o] ⊗ inp[o] over GF(2^8); coef [obj][n_out][n_in], inp [obj][n_in][W], out [obj][n_out][W]."""
    nobj, n_out, n_in = coef.shape
    W = inp.shape[2]
    _chk(coef)
    _chk(inp, (nobj, n_in, W))
    _chk(out, (nobj, n_out, W))
    ctx = _ctx_for(inp, ctx)
    d = MatmulDesc(inp.data_ptr(), n_in * W, W, coef.data_ptr(), n_out * n_in, n_in, out.data_ptr(), n_out * W, W,
                   None, 0, 0, n_out, n_in, W, nobj)
    check(ctx.lib.rlnc_gf256_matmul(ctx.h, C.byref(d)), ctx.lib)


def mul_vec_by_scalar(vec, scalar: int, ctx: Context | None = None) -> None:
    """gf256_inplace_mul_vec_by_scalar (simd/mod.rs:18-47) on a device vector."""
    _chk(vec)
    ctx = _ctx_for(vec, ctx)
    check(ctx.lib.rlnc_gf256_inplace_mul_vec_by_scalar(ctx.h, C.c_void_p(vec.data_ptr()), vec.numel(), scalar),
          ctx.lib)


def add_vectors(dst, src, ctx: Context | None = None) -> None:
    """gf256_inplace_add_vectors (simd/mod.rs:58-76)."""
    _chk(dst)
    _chk(src, tuple(dst.shape))
    ctx = _ctx_for(dst, ctx)
    check(ctx.lib.rlnc_gf256_inplace_add_vectors(ctx.h, C.c_void_p(dst.data_ptr()), C.c_void_p(src.data_ptr()),
                                                 dst.numel()), ctx.lib)


def mul_vec_by_scalar_then_add_into_vec(dst, src, scalar: int, ctx: Context | None = None) -> None:
    """gf256_mul_vec_by_scalar_then_add_into_vec (simd/mod.rs:89-119)."""
    _chk(dst)
    _chk(src, tuple(dst.shape))
    ctx = _ctx_for(dst, ctx)
    check(ctx.lib.rlnc_gf256_mul_vec_by_scalar_then_add_into_vec(ctx.h, C.c_void_p(dst.data_ptr()),
                                                                 C.c_void_p(src.data_ptr()), dst.numel(), scalar),
          ctx.lib)


# ------------------------------------------------------------------------------------------------------------------
# ragged batches (include/rlnc_hip.h: rlnc_encode_ragged / rlnc_recode_ragged / rlnc_decode_ragged): objects of
# different shapes and buffers, one launch per kernel stage
# ------------------------------------------------------------------------------------------------------------------
def _rows(t):
    """(pointer, row stride) of a 2-D uint8 device view whose rows are contiguous."""
    import torch

    assert t.is_cuda and t.dtype == torch.uint8 and t.dim() == 2 and (t.shape[1] <= 1 or t.stride(1) == 1)
    return t.data_ptr(), (t.stride(0) if t.shape[0] > 1 else t.shape[1])


def encode_ragged(objs, ctx: Context | None = None) -> None:
    """objs: (src [k][L], coeffs [n][k], pieces [n][k+L]) per object -> n coded pieces coeffs ‖ data each."""
    from ._lib import ObjectDesc

    if not objs:
        return
    ctx = _ctx_for(objs[0][0], ctx)
    descs = []
    for src, co, pc in objs:
        k, L = src.shape
        n = co.shape[0]
        assert tuple(co.shape) == (n, k) and tuple(pc.shape) == (n, k + L) and co.is_contiguous()
        sp, ss = _rows(src)
        pp, ps = _rows(pc)
        descs.append(ObjectDesc(sp, ss, co.data_ptr(), pp, ps, k, L, n))
    arr = (ObjectDesc * len(descs))(*descs)
    check(ctx.lib.rlnc_encode_ragged(ctx.h, arr, len(descs)), ctx.lib)


def recode_ragged(objs, ctx: Context | None = None) -> None:
    """objs: (pieces [n][k+L], r [count][n], out [count][k+L], k) per object (recoder.rs:122-153 × count)."""
    from ._lib import RecodeObjDesc

    if not objs:
        return
    ctx = _ctx_for(objs[0][0], ctx)
    descs = []
    for pieces, r, out, k in objs:
        n, full = pieces.shape
        count = r.shape[0]
        assert tuple(r.shape) == (count, n) and r.is_contiguous() and tuple(out.shape) == (count, full)
        pp, ps = _rows(pieces)
        op, os_ = _rows(out)
        descs.append(RecodeObjDesc(pp, ps, r.data_ptr(), op, os_, k, full - k, n, count))
    arr = (RecodeObjDesc * len(descs))(*descs)
    check(ctx.lib.rlnc_recode_ragged(ctx.h, arr, len(descs)), ctx.lib)


def decode_ragged(objs, ctx: Context | None = None):
    """objs: (pieces [m][k+L], k, decoded [k][L]) per object.  Returns device tensors (piece_status int32 [sum m]
    in object order, object_status int32 [count], data_len int64 [count]); asynchronous like decode_batch_device."""
    import torch

    from ._lib import DecodeObjDesc

    dev = objs[0][0].device
    ctx = _ctx_for(objs[0][0], ctx)
    descs = []
    for pieces, k, dec in objs:
        m, full = pieces.shape
        L = full - k
        assert tuple(dec.shape) == (k, L) and dec.is_contiguous()
        pp, ps = _rows(pieces)
        descs.append(DecodeObjDesc(pp, ps, dec.data_ptr(), k, L, m))
    total_m = sum(d.m for d in descs)
    ps_t = torch.empty(total_m, dtype=torch.int32, device=dev)
    os_t = torch.empty(len(descs), dtype=torch.int32, device=dev)
    dl_t = torch.empty(len(descs), dtype=torch.int64, device=dev)
    arr = (DecodeObjDesc * len(descs))(*descs)
    check(ctx.lib.rlnc_decode_ragged(ctx.h, arr, len(descs), C.c_void_p(ps_t.data_ptr()), C.c_void_p(os_t.data_ptr()),
                                     C.c_void_p(dl_t.data_ptr())), ctx.lib)
    return ps_t, os_t, dl_t
