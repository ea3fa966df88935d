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
        self.graph_bound = False  # set when a call on it was captured into a HIP graph (batch._ctx_for)

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
        """0 auto, 1 host elimination, 2 device elimination, 5 device blocked clean run (what 0/2 use when
        k + m <= 256; InvalidArgument when it does not apply).  The diagnostic A/B build (make -C rlnc_amd/csrc ab)
        adds 3 (clean state on LDS), 4 (one wave's registers) and 6 (the round-1 multi-wave register path).  All
        are exact."""
        check(self.lib.rlnc_set_decode_path(self.h, int(path)), self.lib)

    def set_kernel_variant(self, variant: int = 8, max_tile_rows: int = 0):
        """GF(2^8) matmul variant (include/rlnc_hip.h): 8 = bit-sliced, one code block per coefficient, plane
        combinations built once per workgroup and shared through LDS, 64-row tiles of 8 waves above 32 output
        rows (the default); 7 = the same with 32-row tiles; 6 = without sharing; 0 = perm; 1 = nibble (the
        reference's 4-bit tables, ablation).  The diagnostic A/B build adds 2-5 and 9.  All are bit-identical."""
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


# Per-thread cap on the stream-bound default contexts.  Each context owns grow-only workspaces, so code rotating
# through torch's stream pool (up to 32 streams per priority) would otherwise keep one full workspace set per stream
# alive.  The least recently used context is closed beyond the cap (its stream is synchronised first, and objects
# built on it keep their own reference) -- unless a HIP graph captured a call on it: the graph holds that context's
# workspace addresses, so it is never evicted.
STREAM_CONTEXTS_PER_THREAD = 4


def stream_context(device: int, stream_handle: int) -> Context:
    """This thread's context bound to one HIP stream (created on first use; at most STREAM_CONTEXTS_PER_THREAD
    are kept per thread, least recently used first out, graph-bound ones never)."""
    from collections import OrderedDict

    ctxs = getattr(_tls, "sctxs", None)
    if ctxs is None:
        ctxs = _tls.sctxs = OrderedDict()
    key = (device, int(stream_handle or 0))
    c = ctxs.get(key)
    if c is None:
        c = ctxs[key] = Context(device)
        c.set_stream(key[1])
    else:
        ctxs.move_to_end(key)
    # closing a context synchronises its streams and frees its workspaces, which a graph capture in progress (torch's
    # default global capture mode) forbids: evict at the next call outside a capture instead
    if len(ctxs) > STREAM_CONTEXTS_PER_THREAD and not _capturing():
        # a context whose own stream is capturing (a global-mode capture on another stream than torch's current one
        # also forbids the synchronisation) is skipped too
        evictable = [k for k, v in ctxs.items() if k != key and not v.graph_bound and not _stream_capturing(k[1])]
        while len(ctxs) > STREAM_CONTEXTS_PER_THREAD and evictable:
            ctxs.pop(evictable.pop(0)).close()
    return c


def _capturing() -> bool:
    try:
        import torch

        return bool(torch.cuda.is_available() and torch.cuda.is_current_stream_capturing())
    except Exception:
        return False


def _stream_capturing(stream_handle: int) -> bool:
    """hipStreamIsCapturing on a raw stream handle, asked through librlnc_hip (rlnc_stream_is_capturing: the HIP
    runtime the library -- and torch -- has loaded, so the handle means the same stream); True when unsure."""
    import ctypes

    try:
        st = ctypes.c_int(1)
        if _lib.load().rlnc_stream_is_capturing(ctypes.c_void_p(stream_handle or None), ctypes.byref(st)) != 0:
            return True
        return st.value != 0
    except Exception:
        return True


def release_stream_contexts() -> None:
    """Close this thread's stream-bound default contexts (except graph-bound ones)."""
    ctxs = getattr(_tls, "sctxs", None) or {}
    for k in [k for k, v in ctxs.items() if not v.graph_bound]:
        ctxs.pop(k).close()


__all__ = ["Context", "default_context", "stream_context", "release_stream_contexts", "RLNCError"]
