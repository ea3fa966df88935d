"""Helpers for the -m gpu tests: a vectorised numpy GF(2^8) matmul as the independent CPU checker."""
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
