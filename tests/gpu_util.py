"""Helpers for the -m gpu tests: a vectorised numpy GF(2^8) matmul as the independent CPU checker."""
import os

import numpy as np

from oracle import np_oracle as npo

MUL = npo.mul_table()


def np_matmul(coef: np.ndarray, inp: np.ndarray) -> np.ndarray:
    """out[i] = XOR_j coef[i, j] * inp[j] (independent of the C oracle and of the device kernels)."""
    coef = np.asarray(coef, np.uint8)
    inp = np.asarray(inp, np.uint8)
    out = np.zeros((coef.shape[0], inp.shape[1]), np.uint8)
    for j in range(coef.shape[1]):
        out ^= MUL[coef[:, j]][:, inp[j]]
    return out


def dev(a, device="cuda:0"):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint8)).to(device)


def host(t) -> np.ndarray:
    import torch

    torch.cuda.synchronize()
    return t.cpu().numpy()


# The shipped library carries matmul variants 0, 1, 6, 7, 8 and decode paths 0, 1, 2, 5; the A/B history (variants
# 2-5 and 9, decode paths 3, 4, 6) is in the diagnostic build only (make -C rlnc_amd/csrc ab), which the variant
# tests cover when RLNC_LIB_PATH points at it.
AB_BUILD = os.path.basename(os.environ.get("RLNC_LIB_PATH", "")) == "librlnc_hip_ab.so"
MATMUL_AB_ONLY = {2, 3, 4, 5, 9}
DECODE_AB_ONLY = {3, 4, 6}


def variants(*vals):
    return [v for v in vals if AB_BUILD or v not in MATMUL_AB_ONLY]


def decode_paths(*vals):
    return [v for v in vals if AB_BUILD or v not in DECODE_AB_ONLY]
