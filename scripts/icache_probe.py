#!/usr/bin/env python3
"""Instruction-cache probe of the bit-sliced jump kernel: the bench's encode launch (32 objects x k = 32 x 1 MiB ->
64 coded pieces, variant 8) timed with coefficients drawn from alphabets of 16, 64, 128 and 256 values.  Every
coefficient selects one of 256 code blocks (136 B each), so the alphabet size sets how much of the 35 KB block table
is hot; the work (XOR3 count per call) is the same.  HIP events, median of 9 launches."""
import json
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
    B, k, n, L = 32, 32, 64, 1 << 20
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty((B, n, k + L), dtype=torch.uint8, device="cuda")
    rng = np.random.default_rng(4)
    for size in (16, 64, 128, 255):
        # a fixed random alphabet of nonzero coefficients (1..255), uniform over it
        alpha = rng.choice(np.arange(1, 256), size, replace=False).astype(np.uint8)
        co = torch.from_numpy(alpha[rng.integers(0, size, (B, n, k))]).cuda()
        ts = []
        for it in range(11):
            a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            batch.encode_batch(src, co, out, ctx)
            b_.record()
            torch.cuda.synchronize()
            if it >= 2:
                ts.append(a.elapsed_time(b_))
        print(json.dumps({"alphabet": size, "hot_block_bytes": size * 136, "encode_ms": round(sorted(ts)[4], 4)}),
              flush=True)


if __name__ == "__main__":
    main()
