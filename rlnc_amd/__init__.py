"""rlnc_amd — MI355X-native (gfx950) engine for the RLNC GF(2^8) hot path of itzmeanjan/rlnc 0.8.5.

The compute lives in librlnc_hip.so (hand-written HIP kernels + C ABI, include/rlnc_hip.h); this package
is the host-side mirror of the reference's public API (rlnc::full::{Encoder, Decoder, Recoder},
rlnc::RLNCError) plus a device-resident batch API.  Importing fails if the HIP library is missing.
"""
from . import _lib

_lib.load()  # fail loudly, no CPU fallback

from .context import Context, default_context  # noqa: E402
from .errors import RLNCError  # noqa: E402
from . import full  # noqa: E402

__all__ = ["Context", "default_context", "RLNCError", "full"]
