"""Device context (device + HIP stream + workspace) of librlnc_hip."""
from __future__ import annotations

import ctypes as C
import threading

from . import _lib
from .errors import RLNCError, check

_tls = threading.local()


class Context:
    """Owns an rlnc_context (one per host thread, like the reference's &mut self types)."""

    def __init__(self, device: int = 0):
        self.lib = _lib.load()
        h = C.c_void_p()
        check(self.lib.rlnc_context_create(int(device), C.byref(h)), self.lib)
        self.h = h
        self.device = int(device)

    def close(self):
        if getattr(self, "h", None):
            self.lib.rlnc_context_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, hip_stream_handle: int):
        """Launch on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream; 0 = null stream)."""
        check(self.lib.rlnc_context_set_stream(self.h, C.c_void_p(hip_stream_handle)), self.lib)

    def use_own_stream(self):
        check(self.lib.rlnc_context_use_own_stream(self.h), self.lib)

    def use_torch_stream(self):
        import torch

        self.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def synchronize(self):
        check(self.lib.rlnc_context_synchronize(self.h), self.lib)

    def set_decode_path(self, path: int = 0):
        """0 auto, 1 host elimination, 2 device elimination, 3 device with the clean state on LDS, 4 device on
        one wave's registers, 5 device blocked clean run (what 0/2 use when k + m <= 256), 6 device, the round-1
        multi-wave register path (all exact; 2-6 exist for A/B)."""
        check(self.lib.rlnc_set_decode_path(self.h, int(path)), self.lib)

    def set_kernel_variant(self, variant: int = 8, max_tile_rows: int = 0):
        """GF(2^8) matmul variant (include/rlnc_hip.h): 7 = bit-sliced, one code block per coefficient, plane
        combinations built once per workgroup and shared through LDS, 6 = the same without sharing,
        5 = bit-sliced with register-indexed XORs, 0 = perm, 1 = nibble (the reference's 4-bit tables,
        ablation), 2 = perm3, 3/4 = wide2/wide4, 8 = as 7 with 64-row tiles of 8 waves above 32 output rows
        (waves 4-7 only read the shared combinations; a barrier every third row; the default), 9 = as 8 with
        column runs (a workgroup walks up to 8 column blocks, one prologue per run).  All are bit-identical."""
        check(self.lib.rlnc_set_kernel_variant(self.h, int(variant), int(max_tile_rows)), self.lib)

    def set_column_run(self, col_run: int = 0):
        """Column blocks per workgroup of variant 9 (0 = automatic)."""
        check(self.lib.rlnc_set_column_run(self.h, int(col_run)), self.lib)


def default_context(device: int = 0) -> Context:
    ctxs = getattr(_tls, "ctxs", None)
    if ctxs is None:
        ctxs = _tls.ctxs = {}
    if device not in ctxs:
        ctxs[device] = Context(device)
    return ctxs[device]


def stream_context(device: int, stream_handle: int) -> Context:
    """This thread's context bound to one HIP stream (created on first use and kept)."""
    ctxs = getattr(_tls, "sctxs", None)
    if ctxs is None:
        ctxs = _tls.sctxs = {}
    key = (device, int(stream_handle or 0))
    c = ctxs.get(key)
    if c is None:
        c = ctxs[key] = Context(device)
        c.set_stream(key[1])
    return c


__all__ = ["Context", "default_context", "stream_context", "RLNCError"]
