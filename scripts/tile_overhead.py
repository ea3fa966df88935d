#!/usr/bin/env python3
"""Per-tile fixed cost of the bit-sliced product kernel: the same 2^36 multiply-adds (32 objects x 64 output rows)
split into tiles of 16 / 32 / 64 / 128 source rows (L shrinks as k grows).  If a tile's prologue (first DMAs,
first sets) and epilogue (transposes + stores) cost `a` and each source row `b`, the launch time is
tiles x (a + k b) / CUs: the fit gives the fraction of the launch that is per-tile overhead.  One JSON line per
shape, HIP events, median of 6 samples of 5 back-to-back calls."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import torch

    import rlnc_amd
    from rlnc_amd import batch
    from bench_configs import timed

    ctx = rlnc_amd.Context(0)
    if os.environ.get("VARIANT"):
        ctx.set_kernel_variant(int(os.environ["VARIANT"]), 0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    B, n = 32, int(os.environ.get("ROWS", "64"))
    for k in (16, 32, 64, 128):
        L = (32 << 20) // k
        src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=g)
        co = torch.randint(0, 256, (B, n, k), dtype=torch.uint8, device=dev, generator=g)
        out = torch.empty((B, n, L), dtype=torch.uint8, device=dev)
        t = timed(lambda: batch.matmul(co, src, out, ctx), 6)
        tiles = B * (L // 4096) * ((n + 63) // 64 if n > 32 else 1)
        print(json.dumps({"k": k, "L": L, "rows": n, "tiles": tiles, "ms": round(t, 4),
                          "T_muladd_per_s": round(B * n * k * L / t / 1e9, 2)}), flush=True)
        del src, co, out


if __name__ == "__main__":
    main()
