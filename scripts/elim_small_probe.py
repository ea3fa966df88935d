#!/usr/bin/env python3
"""Drives the many-small-objects elimination alone (configs[0] shape: 4,096 objects x k = 16, 16 received pieces)
REPS times, for rocprofv3 PMC passes (scripts/archive/r05_pmc_elim.sh) and HIP-event timing (printed, median of 5 x 10)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    B, k, L, m = int(os.environ.get("OBJS", "4096")), int(os.environ.get("K", "16")), 4096, 16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=g)
    co = torch.randint(0, 256, (B, m, k), dtype=torch.uint8, device=dev, generator=g)
    pieces = torch.empty((B, m, k + L), dtype=torch.uint8, device=dev)
    ctx = rlnc_amd.Context(0)
    batch.encode_batch(src, co, pieces, ctx)
    T = torch.empty((B, k, m), dtype=torch.uint8, device=dev)
    pst = torch.empty((B, m), dtype=torch.int32, device=dev)
    rank = torch.empty(B, dtype=torch.int32, device=dev)
    ts = []
    for r in range(int(os.environ.get("REPS", "5"))):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            batch.decode_batch_eliminate(pieces, k, T, pst, rank, ctx)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 10)
    print(json.dumps({"what": "eliminate", "objects": B, "k": k, "m": m, "ms": round(sorted(ts)[len(ts) // 2], 4),
                      "full_rank": int((rank == k).sum())}), flush=True)


if __name__ == "__main__":
    main()
