"""ctypes binding of oracle/liboracle.so (C restatement of itzmeanjan/rlnc 0.8.5).

TEST INFRASTRUCTURE ONLY — the parity checker and the bench's CPU "port" baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

u8p = C.POINTER(C.c_uint8)
szp = C.POINTER(C.c_size_t)


def build(force: bool = False) -> str:
    """Compile liboracle.so with the committed Makefile (plain gcc)."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    lib = C.CDLL(_LIB_PATH)
    sig = {
        "orc_gf256_tables": (None, [u8p, u8p]),
        "orc_gf256_mul": (C.c_uint8, [C.c_uint8, C.c_uint8]),
        "orc_gf256_inv": (C.c_int, [C.c_uint8]),
        "orc_gf256_nibble_tables": (None, [u8p, u8p]),
        "orc_mul_vec_by_scalar": (None, [u8p, C.c_size_t, C.c_uint8]),
        "orc_add_vectors": (None, [u8p, u8p, C.c_size_t]),
        "orc_mul_vec_by_scalar_then_add_into_vec": (None, [u8p, u8p, C.c_size_t, C.c_uint8]),
        "orc_simd_variant": (C.c_char_p, []),
        "orc_force_scalar": (None, [C.c_int]),
        "orc_piece_byte_len": (C.c_size_t, [C.c_size_t, C.c_size_t]),
        "orc_encoder_pad": (C.c_int, [u8p, C.c_size_t, C.c_size_t, u8p]),
        "orc_code_with_coding_vector": (C.c_int, [u8p, C.c_size_t, C.c_size_t, u8p, C.c_size_t, u8p, C.c_size_t]),
        "orc_code_full_batch": (C.c_int, [u8p, C.c_size_t, C.c_size_t, u8p, C.c_size_t, u8p]),
        "orc_recode_with_vector": (C.c_int, [u8p, C.c_size_t, C.c_size_t, C.c_size_t, u8p, C.c_size_t, u8p, C.c_size_t]),
        "orc_rref": (C.c_size_t, [u8p, C.c_size_t, C.c_size_t, C.c_size_t]),
        "orc_swap_rows": (None, [u8p, C.c_size_t, C.c_size_t, C.c_size_t]),
        "orc_decoder_new": (C.c_void_p, [C.c_size_t, C.c_size_t, C.POINTER(C.c_int)]),
        "orc_decoder_free": (None, [C.c_void_p]),
        "orc_decoder_decode": (C.c_int, [C.c_void_p, u8p, C.c_size_t]),
        "orc_decoder_is_already_decoded": (C.c_int, [C.c_void_p]),
        "orc_decoder_received": (C.c_size_t, [C.c_void_p]),
        "orc_decoder_useful": (C.c_size_t, [C.c_void_p]),
        "orc_decoder_rows": (C.c_size_t, [C.c_void_p]),
        "orc_decoder_matrix": (C.c_void_p, [C.c_void_p]),
        "orc_decoder_get_decoded_data": (C.c_int, [C.c_void_p, u8p, szp]),
        "orc_final_data_len": (C.c_int, [u8p, C.c_size_t, szp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def _p(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(u8p)


def _u8(x) -> np.ndarray:
    return np.ascontiguousarray(np.frombuffer(bytes(x), dtype=np.uint8) if isinstance(x, (bytes, bytearray)) else x, dtype=np.uint8)


class Oracle:
    """Flat-buffer view of the oracle; every method follows the reference function cited in the C file."""

    def __init__(self):
        self.lib = load()

    # field ------------------------------------------------------------------------------------
    def tables(self):
        log = np.zeros(256, np.uint8)
        exp = np.zeros(510, np.uint8)
        self.lib.orc_gf256_tables(_p(log), _p(exp))
        return log, exp

    def nibble_tables(self):
        low = np.zeros((256, 32), np.uint8)
        high = np.zeros((256, 32), np.uint8)
        self.lib.orc_gf256_nibble_tables(_p(low), _p(high))
        return low, high

    def mul(self, a: int, b: int) -> int:
        return int(self.lib.orc_gf256_mul(a, b))

    def inv(self, a: int):
        r = self.lib.orc_gf256_inv(a)
        return None if r < 0 else int(r)

    def mul_table(self) -> np.ndarray:
        """Full 256x256 product table (built from mul_const)."""
        t = np.zeros((256, 256), np.uint8)
        for a in range(256):
            for b in range(256):
                t[a, b] = self.lib.orc_gf256_mul(a, b)
        return t

    def simd_variant(self) -> str:
        return self.lib.orc_simd_variant().decode()

    def force_scalar(self, on: bool):
        self.lib.orc_force_scalar(1 if on else 0)

    # vector primitives --------------------------------------------------------------------------
    def mul_vec_by_scalar(self, vec: np.ndarray, scalar: int) -> np.ndarray:
        v = _u8(vec).copy()
        self.lib.orc_mul_vec_by_scalar(_p(v), v.size, scalar)
        return v

    def add_vectors(self, dst: np.ndarray, src: np.ndarray) -> np.ndarray:
        d = _u8(dst).copy()
        s = _u8(src)
        self.lib.orc_add_vectors(_p(d), _p(s), d.size)
        return d

    def mul_add(self, dst: np.ndarray, src: np.ndarray, scalar: int) -> np.ndarray:
        d = _u8(dst).copy()
        s = _u8(src)
        self.lib.orc_mul_vec_by_scalar_then_add_into_vec(_p(d), _p(s), d.size, scalar)
        return d

    # encoder ------------------------------------------------------------------------------------
    def piece_byte_len(self, data_len: int, k: int) -> int:
        return int(self.lib.orc_piece_byte_len(data_len, k))

    def pad(self, data, k: int) -> np.ndarray:
        d = _u8(data)
        L = self.piece_byte_len(d.size, k)
        out = np.zeros(max(k * L, 1), np.uint8)
        st = self.lib.orc_encoder_pad(_p(d) if d.size else None, d.size, k, _p(out))
        if st:
            raise ValueError(st)
        return out[: k * L].reshape(k, L)

    def encode(self, src: np.ndarray, coeffs: np.ndarray) -> np.ndarray:
        """Full coded pieces (coeffs ‖ Σ c·piece) for each row of coeffs; src is k×L."""
        src = _u8(src)
        k, L = src.shape
        coeffs = _u8(coeffs).reshape(-1, k)
        n = coeffs.shape[0]
        out = np.zeros((n, k + L), np.uint8)
        st = self.lib.orc_code_full_batch(_p(src), k, L, _p(coeffs), n, _p(out))
        if st:
            raise ValueError(st)
        return out

    def code_with_coding_vector(self, src: np.ndarray, cv: np.ndarray, out_len=None):
        src = _u8(src)
        k, L = src.shape
        cv = _u8(cv)
        out = np.zeros(L if out_len is None else max(out_len, 1), np.uint8)
        st = self.lib.orc_code_with_coding_vector(_p(src), k, L, _p(cv) if cv.size else None, cv.size, _p(out),
                                                  L if out_len is None else out_len)
        return st, out

    def recode(self, pieces: np.ndarray, full_len: int, k: int, r: np.ndarray) -> np.ndarray:
        p = _u8(pieces).reshape(-1)
        r = _u8(r)
        out = np.zeros(full_len, np.uint8)
        st = self.lib.orc_recode_with_vector(_p(p), p.size, full_len, k, _p(r), r.size, _p(out), full_len)
        if st:
            raise ValueError(st)
        return out

    # decoder matrix -----------------------------------------------------------------------------
    def rref(self, m: np.ndarray, k: int):
        a = _u8(m).copy()
        rows, cols = a.shape
        r = int(self.lib.orc_rref(_p(a), rows, cols, k))
        return a[:r].copy()

    def swap_rows(self, m: np.ndarray, r1: int, r2: int) -> np.ndarray:
        a = _u8(m).copy()
        self.lib.orc_swap_rows(_p(a), a.shape[1], r1, r2)
        return a

    def final_data_len(self, padded: np.ndarray):
        a = _u8(padded)
        out = C.c_size_t(0)
        st = self.lib.orc_final_data_len(_p(a) if a.size else None, a.size, C.byref(out))
        return st, int(out.value)


class OracleDecoder:
    """Mirror of rlnc::full::Decoder on the C oracle (decoder.rs)."""

    def __init__(self, piece_byte_len: int, required_piece_count: int):
        self.lib = load()
        st = C.c_int(0)
        self.h = self.lib.orc_decoder_new(piece_byte_len, required_piece_count, C.byref(st))
        self.status = st.value
        if not self.h:
            raise ValueError(st.value)
        self.L = piece_byte_len
        self.k = required_piece_count

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.orc_decoder_free(self.h)
            self.h = None

    def decode(self, piece) -> int:
        p = _u8(piece)
        return int(self.lib.orc_decoder_decode(self.h, _p(p) if p.size else None, p.size))

    def is_already_decoded(self) -> bool:
        return bool(self.lib.orc_decoder_is_already_decoded(self.h))

    @property
    def received(self) -> int:
        return int(self.lib.orc_decoder_received(self.h))

    @property
    def useful(self) -> int:
        return int(self.lib.orc_decoder_useful(self.h))

    def matrix(self) -> np.ndarray:
        rows = int(self.lib.orc_decoder_rows(self.h))
        cols = self.k + self.L
        ptr = self.lib.orc_decoder_matrix(self.h)
        buf = (C.c_uint8 * (rows * cols)).from_address(ptr) if rows else b""
        return np.frombuffer(bytes(buf), np.uint8).reshape(rows, cols).copy()

    def get_decoded_data(self):
        out = np.zeros(self.k * self.L, np.uint8)
        n = C.c_size_t(0)
        st = int(self.lib.orc_decoder_get_decoded_data(self.h, _p(out), C.byref(n)))
        return st, out[: n.value].copy() if st == 0 else None

    def padded_payload(self) -> np.ndarray:
        """k×L payload rows in matrix order (get_decoded_data before marker trimming)."""
        m = self.matrix()
        return m[:, self.k:].copy()
