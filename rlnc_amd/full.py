"""rlnc_amd.full — the rlnc::full::{Encoder, Decoder, Recoder} API on the MI355X engine.

Mirrors src/full/{encoder,decoder,recoder}.rs method for method (same names, argument order, getters and
error variants; a Rust ``Err(e)`` is a raised RLNCError ``e``).  Randomness stays with the caller exactly as
in the reference: ``code(rng)`` / ``recode(rng)`` draw the coefficient bytes with ``fill_bytes`` on the host
(encoder.rs:248, recoder.rs:131) and pass them through the C ABI; everything else runs in librlnc_hip.so.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .context import Context, default_context
from .errors import RLNCError, check

__all__ = ["Encoder", "Decoder", "Recoder", "RLNCError", "fill_bytes"]


def fill_bytes(rng, n: int) -> np.ndarray:
    """rng.fill_bytes(n) for the RNGs a Python caller is likely to hold."""
    if n == 0:
        return np.zeros(0, np.uint8)
    if hasattr(rng, "fill_bytes"):
        b = rng.fill_bytes(n)
    elif hasattr(rng, "bytes"):  # numpy Generator / RandomState
        b = rng.bytes(n)
    elif hasattr(rng, "randbytes"):  # random.Random
        b = rng.randbytes(n)
    else:
        raise TypeError("rng must provide fill_bytes(n), bytes(n) or randbytes(n)")
    return np.frombuffer(bytes(b), np.uint8)[:n].copy()


def _u8(x) -> np.ndarray:
    if isinstance(x, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(x), np.uint8)
    return np.ascontiguousarray(np.asarray(x, dtype=np.uint8).reshape(-1))


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data) if a.size else C.c_void_p(0)


class Encoder:
    """rlnc::full::Encoder (encoder.rs:19-270)."""

    def __init__(self, handle, ctx: Context):
        self._h = handle
        self._ctx = ctx
        self._lib = ctx.lib

    @classmethod
    def new(cls, data, piece_count: int, ctx: Context | None = None) -> "Encoder":
        """Encoder::new — encoder.rs:85-106 (pads with the 0x81 marker)."""
        ctx = ctx or default_context()
        d = _u8(data)
        h = C.c_void_p()
        check(ctx.lib.rlnc_encoder_new(ctx.h, _ptr(d), d.size, int(piece_count), C.byref(h)), ctx.lib)
        return cls(h, ctx)

    @classmethod
    def without_padding(cls, data, piece_count: int, ctx: Context | None = None) -> "Encoder":
        """Encoder::without_padding — encoder.rs:50-71."""
        ctx = ctx or default_context()
        d = _u8(data)
        h = C.c_void_p()
        check(ctx.lib.rlnc_encoder_without_padding(ctx.h, _ptr(d), d.size, int(piece_count), C.byref(h)), ctx.lib)
        return cls(h, ctx)

    @classmethod
    def from_device(cls, pieces_dev_ptr: int, piece_count: int, piece_len: int, row_stride: int,
                    ctx: Context | None = None) -> "Encoder":
        ctx = ctx or default_context()
        h = C.c_void_p()
        check(ctx.lib.rlnc_encoder_from_device(ctx.h, C.c_void_p(pieces_dev_ptr), piece_count, piece_len, row_stride,
                                               C.byref(h)), ctx.lib)
        return cls(h, ctx)

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.rlnc_encoder_free(self._h)
            self._h = None

    def clone(self) -> "Encoder":
        """#[derive(Clone)] (encoder.rs:18)."""
        h = C.c_void_p()
        check(self._lib.rlnc_encoder_clone(self._h, C.byref(h)), self._lib)
        return Encoder(h, self._ctx)

    __copy__ = clone

    def get_piece_count(self) -> int:
        return int(self._lib.rlnc_encoder_get_piece_count(self._h))

    def get_piece_byte_len(self) -> int:
        return int(self._lib.rlnc_encoder_get_piece_byte_len(self._h))

    def get_full_coded_piece_byte_len(self) -> int:
        return int(self._lib.rlnc_encoder_get_full_coded_piece_byte_len(self._h))

    def code_with_coding_vector(self, coding_vector, coded_data: np.ndarray) -> None:
        """Encoder::code_with_coding_vector — encoder.rs:128-144 (crate-private in Rust)."""
        cv = _u8(coding_vector)
        assert isinstance(coded_data, np.ndarray) and coded_data.dtype == np.uint8 and coded_data.flags["C_CONTIGUOUS"]
        check(self._lib.rlnc_encoder_code_with_coding_vector(self._h, _ptr(cv), cv.size, _ptr(coded_data),
                                                             coded_data.size), self._lib)

    def code_with_buf(self, rng, full_coded_piece: np.ndarray) -> None:
        """Encoder::code_with_buf — encoder.rs:241-250."""
        assert isinstance(full_coded_piece, np.ndarray) and full_coded_piece.dtype == np.uint8
        if full_coded_piece.size != self.get_full_coded_piece_byte_len():
            raise RLNCError.InvalidOutputBuffer  # checked before drawing, encoder.rs:242-244
        rnd = fill_bytes(rng, self.get_piece_count())
        check(self._lib.rlnc_encoder_code_with_buf(self._h, _ptr(rnd), rnd.size, _ptr(full_coded_piece),
                                                   full_coded_piece.size), self._lib)

    def code(self, rng) -> np.ndarray:
        """Encoder::code — encoder.rs:264-269."""
        out = np.zeros(self.get_full_coded_piece_byte_len(), np.uint8)
        self.code_with_buf(rng, out)
        return out

    def code_batch_device(self, coeffs_dev_ptr: int, n: int, out_dev_ptr: int, out_row_stride: int = 0) -> None:
        """n coded pieces in one launch (device pointers, async on the context stream)."""
        check(self._lib.rlnc_encoder_code_batch_device(self._h, C.c_void_p(coeffs_dev_ptr), n,
                                                       C.c_void_p(out_dev_ptr), out_row_stride), self._lib)


class Recoder:
    """rlnc::full::Recoder (recoder.rs:13-172)."""

    def __init__(self, handle, ctx: Context):
        self._h = handle
        self._ctx = ctx
        self._lib = ctx.lib

    @classmethod
    def new(cls, data, full_coded_piece_byte_len: int, num_pieces_coded_together: int,
            ctx: Context | None = None) -> "Recoder":
        """Recoder::new — recoder.rs:68-108."""
        ctx = ctx or default_context()
        d = _u8(data)
        h = C.c_void_p()
        check(ctx.lib.rlnc_recoder_new(ctx.h, _ptr(d), d.size, int(full_coded_piece_byte_len),
                                       int(num_pieces_coded_together), C.byref(h)), ctx.lib)
        return cls(h, ctx)

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.rlnc_recoder_free(self._h)
            self._h = None

    def clone(self) -> "Recoder":
        """#[derive(Clone)] (recoder.rs:12)."""
        h = C.c_void_p()
        check(self._lib.rlnc_recoder_clone(self._h, C.byref(h)), self._lib)
        return Recoder(h, self._ctx)

    __copy__ = clone

    def get_original_num_pieces_coded_together(self) -> int:
        return int(self._lib.rlnc_recoder_get_original_num_pieces_coded_together(self._h))

    def get_num_pieces_recoded_together(self) -> int:
        return int(self._lib.rlnc_recoder_get_num_pieces_recoded_together(self._h))

    def get_piece_byte_len(self) -> int:
        return int(self._lib.rlnc_recoder_get_piece_byte_len(self._h))

    def get_full_coded_piece_byte_len(self) -> int:
        return int(self._lib.rlnc_recoder_get_full_coded_piece_byte_len(self._h))

    def recode_with_coding_vector(self, r, full_recoded_piece: np.ndarray) -> None:
        """recode_with_buf with the recoding vector given explicitly."""
        rr = _u8(r)
        check(self._lib.rlnc_recoder_recode_with_buf(self._h, _ptr(rr), rr.size, _ptr(full_recoded_piece),
                                                     full_recoded_piece.size), self._lib)

    def recode_with_buf(self, rng, full_recoded_piece: np.ndarray) -> None:
        """Recoder::recode_with_buf — recoder.rs:122-153."""
        assert isinstance(full_recoded_piece, np.ndarray) and full_recoded_piece.dtype == np.uint8
        if full_recoded_piece.size != self.get_full_coded_piece_byte_len():
            raise RLNCError.InvalidOutputBuffer  # recoder.rs:123-125, before drawing
        self.recode_with_coding_vector(fill_bytes(rng, self.get_num_pieces_recoded_together()), full_recoded_piece)

    def recode(self, rng) -> np.ndarray:
        """Recoder::recode — recoder.rs:166-171."""
        out = np.zeros(self.get_full_coded_piece_byte_len(), np.uint8)
        self.recode_with_buf(rng, out)
        return out

    def recode_batch_device(self, r_dev_ptr: int, count: int, out_dev_ptr: int) -> None:
        check(self._lib.rlnc_recoder_recode_batch_device(self._h, C.c_void_p(r_dev_ptr), count,
                                                         C.c_void_p(out_dev_ptr)), self._lib)


class Decoder:
    """rlnc::full::Decoder (decoder.rs:9-178)."""

    def __init__(self, handle, ctx: Context):
        self._h = handle
        self._ctx = ctx
        self._lib = ctx.lib

    @classmethod
    def new(cls, piece_byte_len: int, required_piece_count: int, ctx: Context | None = None) -> "Decoder":
        """Decoder::new(piece_byte_len, required_piece_count) — decoder.rs:65-80."""
        ctx = ctx or default_context()
        h = C.c_void_p()
        check(ctx.lib.rlnc_decoder_new(ctx.h, int(piece_byte_len), int(required_piece_count), C.byref(h)), ctx.lib)
        return cls(h, ctx)

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.rlnc_decoder_free(self._h)
            self._h = None

    def clone(self) -> "Decoder":
        """#[derive(Clone)] (decoder.rs:8): counters, elimination state and received rows."""
        h = C.c_void_p()
        check(self._lib.rlnc_decoder_clone(self._h, C.byref(h)), self._lib)
        return Decoder(h, self._ctx)

    __copy__ = clone

    def decode(self, full_coded_piece) -> None:
        """Decoder::decode — decoder.rs:96-118."""
        p = _u8(full_coded_piece)
        check(self._lib.rlnc_decoder_decode(self._h, _ptr(p), p.size), self._lib)

    def decode_device(self, piece_dev_ptr: int, length: int) -> None:
        check(self._lib.rlnc_decoder_decode_device(self._h, C.c_void_p(piece_dev_ptr), length), self._lib)

    def is_already_decoded(self) -> bool:
        return bool(self._lib.rlnc_decoder_is_already_decoded(self._h))

    def get_num_pieces_coded_together(self) -> int:
        return int(self._lib.rlnc_decoder_get_num_pieces_coded_together(self._h))

    def get_piece_byte_len(self) -> int:
        return int(self._lib.rlnc_decoder_get_piece_byte_len(self._h))

    def get_full_coded_piece_byte_len(self) -> int:
        return int(self._lib.rlnc_decoder_get_full_coded_piece_byte_len(self._h))

    def get_received_piece_count(self) -> int:
        return int(self._lib.rlnc_decoder_get_received_piece_count(self._h))

    def get_useful_piece_count(self) -> int:
        return int(self._lib.rlnc_decoder_get_useful_piece_count(self._h))

    def get_remaining_piece_count(self) -> int:
        return int(self._lib.rlnc_decoder_get_remaining_piece_count(self._h))

    def get_decoded_data(self) -> np.ndarray:
        """Decoder::get_decoded_data — decoder.rs:136-159 (the Python object stays usable)."""
        cap = self.get_num_pieces_coded_together() * self.get_piece_byte_len()
        out = np.empty(cap, np.uint8)
        n = C.c_size_t(0)
        check(self._lib.rlnc_decoder_get_decoded_data(self._h, _ptr(out), cap, C.byref(n)), self._lib)
        return out[: n.value]  # a view: the caller owns it (Vec<u8>), no second pass over the object

    def get_decoded_data_device(self, out_dev_ptr: int, cap: int) -> int:
        n = C.c_size_t(0)
        check(self._lib.rlnc_decoder_get_decoded_data_device(self._h, C.c_void_p(out_dev_ptr), cap, C.byref(n)),
              self._lib)
        return int(n.value)
