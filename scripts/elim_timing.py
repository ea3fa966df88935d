#!/usr/bin/env python3
"""Device elimination (rlnc_decode_batch_eliminate) time per decode path and shape, HIP events on the launch stream,
median of 7 launches after 2 warm-ups; every path's statuses, ranks and T checked equal to path 2's (the round-1
default) on the same pieces.  Shapes: the bench's (32 objects, k = m = 32), configs[4]'s per-GPU share
(512 objects, k = m = 128), configs[0]'s shape batched (4,096 objects, k = m = 16), plus random sparse and
dependent pieces that leave the clean state.  One JSON line per (shape, path).

    ELIM_PATHS=2,5 python scripts/elim_timing.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [  # name, objects, k, m, sparsity, dependent fraction
    ("bench k32", 32, 32, 32, 0.0, 0.0),
    ("configs[4] share k128", 512, 128, 128, 0.0, 0.0),
    ("configs[0] shape k16 x4096", 4096, 16, 16, 0.0, 0.0),
    ("k64 dense", 64, 64, 64, 0.0, 0.0),
    ("k32 sparse 0.7 + dependent", 64, 32, 40, 0.7, 0.1),
    ("k128 sparse 0.9", 64, 128, 128, 0.9, 0.02),
    ("configs[4] share k128, LU (never leaves the clean state)", 512, 128, 128, -1.0, 0.0),
]
if os.environ.get("ELIM_SHAPES") == "small":  # small-k crossover of the one-wave register kernel (path 4)
    SHAPES = [("k8 x4096", 4096, 8, 8, 0.0, 0.0), ("k16 x4096", 4096, 16, 16, 0.0, 0.0),
              ("k16 x512", 512, 16, 16, 0.0, 0.0), ("k16 m24 sparse 0.5 dep", 4096, 16, 24, 0.5, 0.1),
              ("k24 x2048", 2048, 24, 24, 0.0, 0.0), ("k32 x1024", 1024, 32, 32, 0.0, 0.0),
              ("k20 m40 x2048", 2048, 20, 40, 0.2, 0.05), ("k12 x4096", 4096, 12, 12, 0.0, 0.0)]


def gf_mul_table():
    t = np.zeros((256, 256), np.uint8)
    for a in range(256):
        for b in range(256):
            x, y, r = a, b, 0
            while y:
                if y & 1:
                    r ^= x
                x = ((x << 1) ^ 0x11B) if x & 0x80 else x << 1
                y >>= 1
            t[a, b] = r
    return t


def lu_coefficients(rng, k):
    """C = L x U over GF(2^8), L unit lower triangular, U upper triangular with a nonzero diagonal: every leading
    principal minor is nonzero, so the one-piece clean step never meets a zero pivot."""
    MUL = gf_mul_table()
    Lm = np.tril(rng.integers(0, 256, (k, k), dtype=np.uint8), -1) + np.eye(k, dtype=np.uint8)
    U = np.triu(rng.integers(0, 256, (k, k), dtype=np.uint8), 1) + np.diag(rng.integers(1, 256, k, dtype=np.uint8))
    return np.bitwise_xor.reduce(MUL[Lm[:, :, None], U[None, :, :]], axis=1)


def main():
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    ctx = rlnc_amd.Context(0)
    paths = [int(x) for x in os.environ.get("ELIM_PATHS", "6,5").split(",")]
    L = 16  # the elimination reads only the coefficient bytes
    for name, B, k, m, sp, dep in SHAPES:
        rng = np.random.default_rng(k * 7 + m)
        if sp < 0:
            co = np.broadcast_to(lu_coefficients(rng, k), (B, m, k)).copy()
        else:
            co = rng.integers(0, 256, (B, m, k), dtype=np.uint8)
            co[rng.random((B, m, k)) < sp] = 0
        for o in range(B):  # dependent pieces: combinations of two earlier ones (coefficients only matter here)
            for p in range(2, m):
                if rng.random() < dep:
                    a, b = rng.integers(0, p, 2)
                    co[o, p] = co[o, a] ^ co[o, b]
        pieces = torch.zeros((B, m, k + L), dtype=torch.uint8, device="cuda")
        pieces[:, :, :k] = torch.from_numpy(co).cuda()
        ref = None
        for path in paths:
            ctx.set_decode_path(path)
            T = torch.empty((B, k, m), dtype=torch.uint8, device="cuda")
            ps = torch.empty((B, m), dtype=torch.int32, device="cuda")
            rk = torch.empty((B,), dtype=torch.int32, device="cuda")
            ts = []
            for it in range(9):
                a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                batch.decode_batch_eliminate(pieces, k, T, ps, rk, ctx)
                b_.record()
                torch.cuda.synchronize()
                if it >= 2:
                    ts.append(a.elapsed_time(b_))
            out = (T.cpu(), ps.cpu(), rk.cpu())
            if ref is None:
                ref = out
            same = all(torch.equal(x, y) for x, y in zip(out, ref))
            if os.environ.get("ELIM_PROFILE"):  # diagnostic build: statuses 0..7 = phase cycles (wave 0)
                ph = out[1][:, :8].numpy().astype(np.int64)
                print(json.dumps({"shape": name, "phases": "setup step1 step2 step3 close generic - total",
                                  "obj0": ph[0].tolist(), "median": np.median(ph, axis=0).astype(int).tolist(),
                                  "max": ph.max(axis=0).tolist()}), flush=True)
                continue
            print(json.dumps({"shape": name, "objects": B, "k": k, "m": m, "path": path,
                              "ms": round(sorted(ts)[len(ts) // 2], 4), "full_rank": int((out[2] == k).sum()),
                              "same_as_first_path": same}), flush=True)
    ctx.set_decode_path(0)


if __name__ == "__main__":
    main()
