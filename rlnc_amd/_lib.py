"""ctypes binding of librlnc_hip.so (the C ABI declared in include/rlnc_hip.h).

There is no fallback: if the HIP library is missing, importing rlnc_amd fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# RLNC_LIB_PATH: diagnostic builds only (scripts/bs_diag.sh); the product is the in-tree library
LIB_PATH = os.environ.get("RLNC_LIB_PATH") or os.path.join(_HERE, "librlnc_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "rlnc_hip.h")

u8p = C.POINTER(C.c_uint8)
i32p = C.POINTER(C.c_int32)
u64p = C.POINTER(C.c_uint64)
szp = C.POINTER(C.c_size_t)
vp = C.c_void_p


class PadDesc(C.Structure):
    _fields_ = [("data", C.c_void_p), ("data_len", C.c_size_t), ("k", C.c_size_t), ("out", C.c_void_p),
                ("out_row_stride", C.c_size_t)]


class ObjectDesc(C.Structure):
    _fields_ = [("src", C.c_void_p), ("src_row_stride", C.c_size_t), ("coeffs", C.c_void_p), ("pieces", C.c_void_p),
                ("piece_row_stride", C.c_size_t), ("k", C.c_size_t), ("L", C.c_size_t), ("n", C.c_size_t)]


class RecodeObjDesc(C.Structure):
    _fields_ = [("pieces", C.c_void_p), ("piece_row_stride", C.c_size_t), ("r", C.c_void_p), ("out", C.c_void_p),
                ("out_row_stride", C.c_size_t), ("k", C.c_size_t), ("L", C.c_size_t), ("n", C.c_size_t),
                ("n_recoded", C.c_size_t)]


class DecodeObjDesc(C.Structure):
    _fields_ = [("pieces", C.c_void_p), ("piece_row_stride", C.c_size_t), ("decoded", C.c_void_p), ("k", C.c_size_t),
                ("L", C.c_size_t), ("m", C.c_size_t)]


class MatmulDesc(C.Structure):
    _fields_ = [
        ("in_", C.c_void_p), ("in_obj_stride", C.c_int64), ("in_row_stride", C.c_int64),
        ("coef", C.c_void_p), ("coef_obj_stride", C.c_int64), ("coef_row_stride", C.c_int64),
        ("out", C.c_void_p), ("out_obj_stride", C.c_int64), ("out_row_stride", C.c_int64),
        ("hdr", C.c_void_p), ("hdr_obj_stride", C.c_int64), ("hdr_row_stride", C.c_int64),
        ("n_out", C.c_int32), ("n_in", C.c_int32), ("width", C.c_int64), ("n_obj", C.c_int32),
    ]


_SIGS = {
    "rlnc_status_name": (C.c_char_p, [C.c_int]),
    "rlnc_status_message": (C.c_char_p, [C.c_int]),
    "rlnc_last_error": (C.c_char_p, []),
    "rlnc_version": (C.c_char_p, []),
    "rlnc_context_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
    "rlnc_context_destroy": (None, [vp]),
    "rlnc_context_set_stream": (C.c_int, [vp, vp]),
    "rlnc_context_use_own_stream": (C.c_int, [vp]),
    "rlnc_context_get_stream": (vp, [vp]),
    "rlnc_context_synchronize": (C.c_int, [vp]),
    "rlnc_context_device": (C.c_int, [vp]),
    "rlnc_device_unaligned_vector_access": (C.c_int, [C.c_int]),
    "rlnc_stream_is_capturing": (C.c_int, [vp, C.POINTER(C.c_int)]),
    "rlnc_gf256_inplace_mul_vec_by_scalar": (C.c_int, [vp, vp, C.c_size_t, C.c_uint8]),
    "rlnc_gf256_inplace_add_vectors": (C.c_int, [vp, vp, vp, C.c_size_t]),
    "rlnc_gf256_mul_vec_by_scalar_then_add_into_vec": (C.c_int, [vp, vp, vp, C.c_size_t, C.c_uint8]),
    "rlnc_gf256_matmul": (C.c_int, [vp, C.POINTER(MatmulDesc)]),
    "rlnc_set_kernel_variant": (C.c_int, [vp, C.c_int, C.c_int]),
    "rlnc_set_column_run": (C.c_int, [vp, C.c_int]),
    "rlnc_set_decode_path": (C.c_int, [vp, C.c_int]),
    "rlnc_encoder_new": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.POINTER(vp)]),
    "rlnc_encoder_without_padding": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.POINTER(vp)]),
    "rlnc_encoder_from_device": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, C.POINTER(vp)]),
    "rlnc_encoder_clone": (C.c_int, [vp, C.POINTER(vp)]),
    "rlnc_encoder_free": (None, [vp]),
    "rlnc_encoder_get_piece_count": (C.c_size_t, [vp]),
    "rlnc_encoder_get_piece_byte_len": (C.c_size_t, [vp]),
    "rlnc_encoder_get_full_coded_piece_byte_len": (C.c_size_t, [vp]),
    "rlnc_encoder_code_with_coding_vector": (C.c_int, [vp, vp, C.c_size_t, vp, C.c_size_t]),
    "rlnc_encoder_code_with_buf": (C.c_int, [vp, vp, C.c_size_t, vp, C.c_size_t]),
    "rlnc_encoder_code_batch_device": (C.c_int, [vp, vp, C.c_size_t, vp, C.c_size_t]),
    "rlnc_recoder_new": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, C.POINTER(vp)]),
    "rlnc_recoder_clone": (C.c_int, [vp, C.POINTER(vp)]),
    "rlnc_recoder_free": (None, [vp]),
    "rlnc_recoder_get_original_num_pieces_coded_together": (C.c_size_t, [vp]),
    "rlnc_recoder_get_num_pieces_recoded_together": (C.c_size_t, [vp]),
    "rlnc_recoder_get_piece_byte_len": (C.c_size_t, [vp]),
    "rlnc_recoder_get_full_coded_piece_byte_len": (C.c_size_t, [vp]),
    "rlnc_recoder_recode_with_buf": (C.c_int, [vp, vp, C.c_size_t, vp, C.c_size_t]),
    "rlnc_recoder_recode_batch_device": (C.c_int, [vp, vp, C.c_size_t, vp]),
    "rlnc_decoder_new": (C.c_int, [vp, C.c_size_t, C.c_size_t, C.POINTER(vp)]),
    "rlnc_decoder_clone": (C.c_int, [vp, C.POINTER(vp)]),
    "rlnc_decoder_free": (None, [vp]),
    "rlnc_decoder_decode": (C.c_int, [vp, vp, C.c_size_t]),
    "rlnc_decoder_decode_device": (C.c_int, [vp, vp, C.c_size_t]),
    "rlnc_decoder_is_already_decoded": (C.c_int, [vp]),
    "rlnc_decoder_get_num_pieces_coded_together": (C.c_size_t, [vp]),
    "rlnc_decoder_get_piece_byte_len": (C.c_size_t, [vp]),
    "rlnc_decoder_get_full_coded_piece_byte_len": (C.c_size_t, [vp]),
    "rlnc_decoder_get_received_piece_count": (C.c_size_t, [vp]),
    "rlnc_decoder_get_useful_piece_count": (C.c_size_t, [vp]),
    "rlnc_decoder_get_remaining_piece_count": (C.c_size_t, [vp]),
    "rlnc_decoder_get_decoded_data": (C.c_int, [vp, vp, C.c_size_t, szp]),
    "rlnc_decoder_get_decoded_data_device": (C.c_int, [vp, vp, C.c_size_t, szp]),
    "rlnc_encode_batch": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, vp, C.c_size_t, vp]),
    "rlnc_encode_batch_data": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, vp, C.c_size_t, vp]),
    "rlnc_encode_batch_headers": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, vp]),
    "rlnc_encode_batch_plan_bytes": (C.c_size_t, [C.c_size_t, C.c_size_t, C.c_size_t]),
    "rlnc_encode_batch_prepare": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, vp, C.c_size_t, vp, vp,
                                            C.c_size_t]),
    "rlnc_encode_batch_data_planned": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, vp, C.c_size_t, vp,
                                                 vp]),
    "rlnc_decode_batch_eliminate": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t,
                                              vp, vp, vp]),
    "rlnc_decode_batch_apply": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, vp,
                                          vp, vp, vp, vp]),
    "rlnc_decode_batch_apply_plan_bytes": (C.c_size_t, [C.c_size_t, C.c_size_t, C.c_size_t]),
    "rlnc_decode_batch_apply_prepare": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t,
                                                  vp, vp, vp, C.c_size_t]),
    "rlnc_decode_batch_apply_planned": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t,
                                                  vp, vp, vp, vp, vp, vp]),
    "rlnc_recode_batch": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, vp, C.c_size_t, vp]),
    "rlnc_decode_batch": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, vp, i32p,
                                    i32p, u64p]),
    "rlnc_decode_batch_device": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, vp,
                                           vp, vp, vp]),
    "rlnc_padded_piece_byte_len": (C.c_size_t, [C.c_size_t, C.c_size_t]),
    "rlnc_pad_device": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, vp, C.c_size_t]),
    "rlnc_pad_batch_device": (C.c_int, [vp, vp, C.c_size_t]),
    "rlnc_encoder_new_device": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.POINTER(vp)]),
    "rlnc_encode_ragged": (C.c_int, [vp, vp, C.c_size_t]),
    "rlnc_recode_ragged": (C.c_int, [vp, vp, C.c_size_t]),
    "rlnc_decode_ragged": (C.c_int, [vp, vp, C.c_size_t, vp, vp, vp]),
    "rlnc_encode_host_stream": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, vp, C.c_size_t, vp,
                                          C.c_size_t]),
    "rlnc_decode_host_stream": (C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, vp,
                                          i32p, i32p, u64p, C.c_size_t]),
    "rlnc_elimination_new": (C.c_int, [C.c_size_t, C.c_size_t, C.POINTER(vp)]),
    "rlnc_elimination_free": (None, [vp]),
    "rlnc_elimination_push": (C.c_int, [vp, vp, i32p, i32p]),
    "rlnc_elimination_rank": (C.c_size_t, [vp]),
    "rlnc_elimination_slots": (C.c_size_t, [vp]),
    "rlnc_elimination_transform": (C.c_int, [vp, vp, C.c_size_t]),
    "rlnc_elimination_coefficients": (C.c_int, [vp, vp]),
}

_lib = None


def load():
    """Load librlnc_hip.so; raises ImportError (never falls back) when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). rlnc_amd has no CPU fallback.")
    try:
        # torch (plumbing for HBM/streams) bundles its own libamdhip64.so.7 — the same SONAME as
        # /opt/rocm's.  Whichever is loaded first serves the whole process; loading torch's first keeps a
        # single HIP runtime (loading ours first leaves torch with no visible GPU).
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def header_symbols(path: str = HEADER_PATH):
    """Function names declared in include/rlnc_hip.h."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rlnc_\w+)\s*\(", txt)))
