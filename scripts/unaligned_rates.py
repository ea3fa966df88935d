#!/usr/bin/env python3
"""Rates of the batch API on shapes whose rows are not 16-byte aligned (k or L not a multiple of 16: the coded
piece's data starts at byte k of a (k + L)-byte row), against an aligned shape of the same size.  HIP events around
5 back-to-back calls, median of 7; decode outputs checked against the source.
    python scripts/unaligned_rates.py   (GPU)
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
    g.manual_seed(9)
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

    shapes = [(16, 32, 1 << 20, 64), (16, 30, 1 << 20, 60), (16, 32, (1 << 20) + 5, 64), (16, 33, 1 << 20, 1),
              (16, 32, 1 << 20, 1), (256, 24, 65536, 24), (256, 32, 65536, 32), (4096, 8, 4096, 8), (64, 100, 10007, 100)]
    for (B, k, L, n) in shapes:
        src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=g)
        coeffs = torch.randint(0, 256, (B, n, k), dtype=torch.uint8, device=dev, generator=g)
        pieces = torch.empty((B, n, k + L), dtype=torch.uint8, device=dev)
        enc = timed(lambda: batch.encode_batch(src, coeffs, pieces, ctx))
        res = {"objects": B, "k": k, "L": L, "coded": n, "encode_ms": round(enc, 4),
               "encode_T_per_s": round(B * n * k * L / enc * 1e-9, 2)}
        if n >= k:
            rec = pieces[:, :k]
            dec = torch.empty((B, k, L), dtype=torch.uint8, device=dev)
            ps = torch.empty((B, k), dtype=torch.int32, device=dev)
            os_ = torch.empty(B, dtype=torch.int32, device=dev)
            dl = torch.empty(B, dtype=torch.int64, device=dev)
            d = timed(lambda: batch.decode_batch_device(rec, k, dec, ps, os_, dl, ctx))
            full = (ps != 8).all(dim=1)  # no PieceNotUseful (status 8): rank k from the first k pieces
            res.update({"decode_ms": round(d, 4), "decode_T_per_s": round(B * k * k * L / d * 1e-9, 2),
                        "verified": bool(torch.equal(dec[full], src[full]))})
        print(json.dumps(res), flush=True)
        del src, pieces


if __name__ == "__main__":
    main()
