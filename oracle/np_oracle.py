"""Independent numpy restatement of the rlnc 0.8.5 hot path — TEST INFRASTRUCTURE ONLY.

Deliberately shares no code or tables with the C oracle: multiplication is carry-less Russian-peasant
multiplication reduced by 0x11B (the field of src/common/gf256.rs:50-51), not log/exp lookups.  Used to
cross-check oracle/liboracle.so on small cases and to generate the committed golden fixtures.
"""
from __future__ import annotations

import numpy as np

POLY = 0x11B
BOUNDARY_MARKER = 0x81  # src/full/consts.rs:5


def gf_mul_scalar(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= POLY
        b >>= 1
    return r


_MUL = np.array([[gf_mul_scalar(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)
_INV = np.zeros(256, dtype=np.int16)
_INV[0] = -1
for _a in range(1, 256):
    _INV[_a] = int(np.nonzero(_MUL[_a] == 1)[0][0])


def mul_table() -> np.ndarray:
    return _MUL


def gf_inv(a: int):
    return None if a == 0 else int(_INV[a])


def gf_mul_vec(v: np.ndarray, c: int) -> np.ndarray:
    return _MUL[c][v]


def matmul(coef: np.ndarray, src: np.ndarray) -> np.ndarray:
    """Out[i] = XOR_j coef[i,j] * src[j] over GF(2^8) (the batched code_with_coding_vector)."""
    coef = np.asarray(coef, np.uint8)
    src = np.asarray(src, np.uint8)
    out = np.zeros((coef.shape[0], src.shape[1]), np.uint8)
    for i in range(coef.shape[0]):
        for j in range(coef.shape[1]):
            c = int(coef[i, j])
            if c:
                out[i] ^= _MUL[c][src[j]]
    return out


def pad(data: np.ndarray, k: int) -> np.ndarray:
    """Encoder::new padding — encoder.rs:85-106."""
    data = np.asarray(data, np.uint8)
    L = (data.size + 1 + k - 1) // k
    buf = np.zeros(k * L, np.uint8)
    buf[: data.size] = data
    buf[data.size] = BOUNDARY_MARKER
    return buf.reshape(k, L)


def encode(src: np.ndarray, coeffs: np.ndarray) -> np.ndarray:
    coeffs = np.asarray(coeffs, np.uint8).reshape(-1, src.shape[0])
    return np.concatenate([coeffs, matmul(coeffs, src)], axis=1)


def recode(pieces: np.ndarray, k: int, r: np.ndarray) -> np.ndarray:
    """recoder.rs:122-153: coefficients r·C and data r·D — one linear combination of whole pieces."""
    return matmul(np.asarray(r, np.uint8).reshape(1, -1), pieces)[0]


def rref(m: np.ndarray, k: int) -> np.ndarray:
    """DecoderMatrix::rref — decoder_matrix.rs:99-244, diagonal pivots, row ops from column i."""
    m = np.array(m, np.uint8, copy=True)
    rows, cols = m.shape
    boundary = min(rows, cols)
    for i in range(boundary):  # clean_forward :120-166
        if m[i, i] == 0:
            nz = [p for p in range(i + 1, rows) if m[p, i] != 0]
            if not nz:
                continue
            p = nz[0]
            m[[i, p]] = m[[p, i]]
        for j in range(i + 1, rows):
            if m[j, i] == 0:
                continue
            q = int(_MUL[m[j, i], _INV[m[i, i]]])
            m[j, i:] ^= _MUL[q][m[i, i:]]
    for i in reversed(range(boundary)):  # clean_backward :171-215
        if m[i, i] == 0:
            continue
        for j in range(i):
            if m[j, i] == 0:
                continue
            q = int(_MUL[m[j, i], _INV[m[i, i]]])
            m[j, i:] ^= _MUL[q][m[i, i:]]
        if m[i, i] == 1:
            continue
        inv = int(_INV[m[i, i]])
        m[i, i] = 1
        m[i, i + 1:] = _MUL[inv][m[i, i + 1:]]
    keep = [r for r in range(rows) if m[r, :k].any()]  # remove_zero_rows :222-244
    return m[keep]


class Decoder:
    """decoder.rs:9-177 on full rows."""

    def __init__(self, L: int, k: int):
        self.L, self.k = L, k
        self.m = np.zeros((0, k + L), np.uint8)
        self.received = 0
        self.useful = 0

    def is_already_decoded(self) -> bool:
        return self.m.shape[0] == self.k

    def decode(self, piece) -> str:
        piece = np.asarray(piece, np.uint8)
        if self.is_already_decoded():
            return "ReceivedAllPieces"
        if piece.size != self.k + self.L:
            return "InvalidPieceLength"
        before = self.m.shape[0]
        self.m = rref(np.vstack([self.m, piece[None, :]]), self.k)
        self.received += 1
        if self.m.shape[0] == before:
            return "PieceNotUseful"
        self.useful = self.m.shape[0]
        return "Ok"

    def padded_payload(self) -> np.ndarray:
        return self.m[:, self.k:].copy()


def final_data_len(padded: np.ndarray):
    """decoder.rs:162-177. Returns (ok, length)."""
    padded = np.asarray(padded, np.uint8)
    n = padded.size
    last = max(n - 1, 0)
    idx_hits = np.nonzero(padded == BOUNDARY_MARKER)[0]
    idx = int(idx_hits[-1]) if idx_hits.size else 0
    if idx == 0:
        return False, 0
    if padded[idx + 1:].any():
        return False, 0
    return True, idx if last >= 0 else 0
