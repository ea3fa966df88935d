#!/usr/bin/env python3
"""Products of many small objects (n_out x n_in x W per object, 4,096 objects): the default kernel choice against the
perm kernel (variant 0), HIP events around 5 back-to-back rlnc_gf256_matmul calls, median of 7; outputs compared.
    python scripts/small_products.py   (GPU)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    ctx = rlnc_amd.Context(0)

    def timed(fn):
        ts = []
        for r in range(9):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                fn()
            e1.record()
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(e0.elapsed_time(e1) / 5)
        return sorted(ts)[len(ts) // 2]

    for (B, n, k, W) in ((4096, 4, 4, 4096), (4096, 8, 8, 4096), (4096, 12, 12, 4096), (4096, 16, 16, 4096),
                         (4096, 24, 24, 4096), (4096, 32, 32, 4096), (1024, 8, 8, 16384), (512, 8, 8, 65536)):
        coef = torch.randint(0, 256, (B, n, k), dtype=torch.uint8, device=dev, generator=g)
        inp = torch.randint(0, 256, (B, k, W), dtype=torch.uint8, device=dev, generator=g)
        out = torch.empty((B, n, W), dtype=torch.uint8, device=dev)
        res = {"objects": B, "n_out": n, "n_in": k, "W": W}
        ref = None
        for v in (8, 0):
            ctx.set_kernel_variant(v, 0)
            ms = timed(lambda: batch.matmul(coef, inp, out, ctx))
            res[f"v{v}_ms"] = round(ms, 4)
            res[f"v{v}_T_per_s"] = round(B * n * k * W / ms * 1e-9, 2)
            res[f"v{v}_TBps"] = round(B * (n + k) * W / ms * 1e-9, 2)
            if ref is None:
                ref = out.clone()
            else:
                res["same"] = bool(torch.equal(ref, out))
        ctx.set_kernel_variant(8, 0)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
