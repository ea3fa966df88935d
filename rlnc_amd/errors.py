"""RLNCError — mirror of rlnc::RLNCError (src/common/errors.rs:3-60) plus engine errors."""
from __future__ import annotations

_NAMES = [
    "Ok", "CodingVectorLengthMismatch", "DataLengthMismatch", "PieceCountZero", "DataLengthZero",
    "PieceLengthZero", "NotEnoughPiecesToRecode", "PieceLengthTooShort", "PieceNotUseful", "ReceivedAllPieces",
    "NotAllPiecesReceivedYet", "InvalidDecodedDataFormat", "InvalidPieceLength", "InvalidOutputBuffer",
]
# Display strings, errors.rs:34-58
_MESSAGES = [
    "Ok", "Coding vector length mismatch", "Data length mismatch", "Piece count is zero", "Data length is zero",
    "Piece length is zero", "Not enough pieces received to recode", "Piece length is too short",
    "Received piece is not useful", "Received all pieces", "Not all pieces are received yet",
    "Invalid decoded data format", "Invalid piece length", "Invalid output buffer",
]
_ENGINE = {100: "InvalidArgument", 101: "DeviceError", 102: "OutOfMemory", 103: "NoDevice"}


class RLNCError(Exception):
    """One RLNCError variant.  Compare with the class attributes: ``err == RLNCError.PieceNotUseful``."""

    def __init__(self, code: int, detail: str = ""):
        self.code = int(code)
        self.name = _NAMES[code] if 0 <= code < len(_NAMES) else _ENGINE.get(code, f"Unknown({code})")
        msg = _MESSAGES[code] if 0 < code < len(_MESSAGES) else self.name
        super().__init__(msg + (f": {detail}" if detail else ""))

    def __eq__(self, other):
        return isinstance(other, RLNCError) and other.code == self.code

    def __hash__(self):
        return hash(self.code)

    def __repr__(self):
        return f"RLNCError::{self.name}"


for _c, _n in enumerate(_NAMES):
    if _c:
        setattr(RLNCError, _n, RLNCError(_c))
for _c, _n in _ENGINE.items():
    setattr(RLNCError, _n, RLNCError(_c))

STATUS_NAMES = list(_NAMES)


def check(status: int, lib=None):
    """Raise RLNCError for a nonzero C-ABI status."""
    if status:
        detail = ""
        if status >= 100 and lib is not None:
            detail = (lib.rlnc_last_error() or b"").decode(errors="replace")
        raise RLNCError(status, detail)
