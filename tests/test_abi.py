"""CPU: the C-ABI library loads and exports every symbol include/rlnc_hip.h declares; status names and
messages follow src/common/errors.rs; no compute call is made (no GPU here)."""
import ctypes as C

import pytest


def test_library_exports_every_declared_symbol():
    from rlnc_amd import _lib

    lib = _lib.load()
    syms = _lib.header_symbols()
    assert len(syms) >= 50
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # the ctypes signature table covers the whole header (nothing declared is unreachable from Python)
    assert sorted(_lib._SIGS) == syms


def test_library_has_no_undefined_internal_symbols():
    """Every rlnc:: function the engine calls is defined in the library (a shared object links with undefined
    symbols and would only fail when loaded or called)."""
    import shutil
    import subprocess

    from rlnc_amd import _lib

    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    out = subprocess.run([nm, "-D", "--undefined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    undefined = [ln.split()[-1] for ln in out.stdout.splitlines() if "_ZN4rlnc" in ln]
    assert not undefined, undefined


def test_status_names_follow_errors_rs():
    from rlnc_amd import _lib
    from rlnc_amd.errors import STATUS_NAMES, RLNCError

    lib = _lib.load()
    for code, name in enumerate(STATUS_NAMES):
        assert lib.rlnc_status_name(code).decode() == name
        assert str(RLNCError(code)) == lib.rlnc_status_message(code).decode() or code == 0
    assert str(RLNCError.PieceNotUseful) == "Received piece is not useful"  # errors.rs:48
    assert RLNCError(8) == RLNCError.PieceNotUseful and RLNCError(8) != RLNCError.ReceivedAllPieces


def test_null_arguments_are_rejected_not_crashing():
    from rlnc_amd import _lib

    lib = _lib.load()
    assert lib.rlnc_context_create(0, None) == 100
    assert lib.rlnc_context_synchronize(None) == 100
    assert lib.rlnc_gf256_matmul(None, None) == 100
    assert lib.rlnc_elimination_push(None, None, None, None) == 100
    assert lib.rlnc_encoder_get_piece_count(None) == 0
    assert lib.rlnc_decoder_is_already_decoded(None) == 0


def test_no_device_reports_cleanly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    from rlnc_amd import Context
    from rlnc_amd.errors import RLNCError

    with pytest.raises(RLNCError) as ei:
        Context(0)
    assert ei.value == RLNCError.NoDevice


def test_version_string():
    from rlnc_amd import _lib

    assert b"gfx950" in _lib.load().rlnc_version()
