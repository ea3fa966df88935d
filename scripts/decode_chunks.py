#!/usr/bin/env python3
"""Batch-decode rates of small and mid-size objects: one rlnc_decode_batch_device call per sample, HIP events
around 5 back-to-back calls, median of 7; prints ms and a digest of every output so that runs can be compared.
Round 3 used it for the A/B of a chunked decode (an A/B-build knob RLNC_DECODE_CHUNKS = C that eliminated chunk
c + 1 on a side stream beside chunk c's T x data product): bit-identical and 12-50 % slower on every shape
(profiles/r03_decode_chunks_ab.jsonl), so the knob was removed.
    python scripts/decode_chunks.py   (GPU)
"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    dev = torch.device("cuda", 0)
    ctx = rlnc_amd.Context(0)
    for (B, k, L) in ((4096, 16, 4096), (4096, 8, 4096), (2048, 32, 4096), (1024, 16, 16384), (16, 32, 1 << 20)):
        g = torch.Generator(device=dev)
        g.manual_seed(B + k + L)
        m = k
        src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=g)
        coeffs = torch.randint(0, 256, (B, m, k), dtype=torch.uint8, device=dev, generator=g)
        pieces = torch.empty((B, m, k + L), dtype=torch.uint8, device=dev)
        batch.encode_batch(src, coeffs, pieces, ctx)
        dec = torch.empty((B, k, L), dtype=torch.uint8, device=dev)
        ps = torch.empty((B, m), dtype=torch.int32, device=dev)
        os_ = torch.empty(B, dtype=torch.int32, device=dev)
        dl = torch.empty(B, dtype=torch.int64, device=dev)
        ts = []
        for r in range(9):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                batch.decode_batch_device(pieces, k, dec, ps, os_, dl, ctx)
            e1.record()
            torch.cuda.synchronize()
            if r >= 2:
                ts.append(e0.elapsed_time(e1) / 5)
        h = hashlib.sha1()
        for t in (dec, ps, os_, dl):
            h.update(t.cpu().numpy().tobytes())
        full = (os_ == 0).cpu()
        ok = bool(torch.equal(dec[full.to(dev)], src[full.to(dev)]))
        ms = sorted(ts)[len(ts) // 2]
        print(json.dumps({"chunks": int(os.environ.get("RLNC_DECODE_CHUNKS", "1")), "objects": B, "k": k, "L": L,
                          "ms": round(ms, 4), "T_per_s": round(B * k * m * L / ms * 1e-9, 2),
                          "full_rank_decoded": ok, "digest": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
