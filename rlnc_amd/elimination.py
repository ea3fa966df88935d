"""Host-only access to the decoder's exact coefficient elimination (librlnc_hip, no device needed)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .errors import check


class Elimination:
    def __init__(self, k: int, fixed_slots: int = 0):
        self.lib = _lib.load()
        h = C.c_void_p()
        check(self.lib.rlnc_elimination_new(int(k), int(fixed_slots), C.byref(h)), self.lib)
        self.h = h
        self.k = int(k)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.rlnc_elimination_free(self.h)
            self.h = None

    def push(self, coeffs):
        """Returns (status, slot, keep)."""
        c = np.ascontiguousarray(np.asarray(coeffs, np.uint8).reshape(-1)[: self.k])
        assert c.size == self.k
        slot = C.c_int32(-1)
        keep = C.c_int32(0)
        st = self.lib.rlnc_elimination_push(self.h, C.c_void_p(c.ctypes.data), C.byref(slot), C.byref(keep))
        return int(st), int(slot.value), bool(keep.value)

    @property
    def rank(self) -> int:
        return int(self.lib.rlnc_elimination_rank(self.h))

    @property
    def slots(self) -> int:
        return int(self.lib.rlnc_elimination_slots(self.h))

    def transform(self) -> np.ndarray:
        """k × slots (rows beyond rank are zero)."""
        s = self.slots
        T = np.zeros((self.k, s), np.uint8)
        check(self.lib.rlnc_elimination_transform(self.h, C.c_void_p(T.ctypes.data), s), self.lib)
        return T

    def coefficients(self) -> np.ndarray:
        C_ = np.zeros((max(self.rank, 1), self.k), np.uint8)
        check(self.lib.rlnc_elimination_coefficients(self.h, C.c_void_p(C_.ctypes.data)), self.lib)
        return C_[: self.rank]
