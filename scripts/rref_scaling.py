#!/usr/bin/env python3
"""Elimination-kernel cost vs pieces per object (m = 1, 4, 16, 32; k = 32, 16 objects, uniform coefficients):
run under `rocprofv3 --kernel-trace` and read gf_rref_batch_kernel's duration per m (intercept = setup, slope =
per piece).  Decode path via RREF_PATH (2 multi-wave registers, 4 one-wave registers, 3 LDS)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    ctx = rlnc_amd.Context(0)
    ctx.set_decode_path(int(os.environ.get("RREF_PATH", "2")))
    B, k, L = 16, 32, int(os.environ.get("RREF_L", "4096"))
    rng = np.random.default_rng(3)
    src = torch.from_numpy(rng.integers(0, 256, (B, k, L), dtype=np.uint8)).cuda()
    for m in [int(x) for x in os.environ.get("RREF_MS", "1,4,16,32").split(",")]:
        co = torch.from_numpy(rng.integers(0, 256, (B, m, k), dtype=np.uint8)).cuda()
        pieces = torch.empty((B, m, k + L), dtype=torch.uint8, device="cuda")
        batch.encode_batch(src, co, pieces, ctx)
        out = torch.empty((B, k, L), dtype=torch.uint8, device="cuda")
        pst = torch.empty((B, m), dtype=torch.int32, device="cuda")
        ost = torch.empty((B,), dtype=torch.int32, device="cuda")
        dl = torch.empty((B,), dtype=torch.int64, device="cuda")
        for _ in range(5):
            batch.decode_batch_device(pieces, k, out, pst, ost, dl, ctx)
        torch.cuda.synchronize()
        print("m", m, "useful", int((pst == 0).sum()), flush=True)


if __name__ == "__main__":
    main()
