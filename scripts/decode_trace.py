#!/usr/bin/env python3
"""configs[4]'s per-GPU decode (512 objects, k = 128 x 64 KiB, decode from the 128 coded pieces) three times, for
`rocprofv3 --kernel-trace` timelines of the pipelined device decode (elimination chunks on the aux stream beside the
T x data products); prints the HIP-event time of each call."""
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
    B, k, L = int(os.environ.get("DT_OBJECTS", "512")), 128, 1 << 16
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device="cuda", generator=g)
    co = torch.randint(0, 256, (B, k, k), dtype=torch.uint8, device="cuda", generator=g)
    pieces = torch.empty((B, k, k + L), dtype=torch.uint8, device="cuda")
    batch.encode_batch(src, co, pieces, ctx)
    out = torch.empty((B, k, L), dtype=torch.uint8, device="cuda")
    pst = torch.empty((B, k), dtype=torch.int32, device="cuda")
    ost = torch.empty((B,), dtype=torch.int32, device="cuda")
    dl = torch.empty((B,), dtype=torch.int64, device="cuda")
    for _ in range(3):
        a, b_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        batch.decode_batch_device(pieces, k, out, pst, ost, dl, ctx)
        b_.record()
        torch.cuda.synchronize()
        print("decode ms", round(a.elapsed_time(b_), 4), flush=True)
    ok = bool(torch.equal(out[ost == 0], src[ost == 0]))
    print("verified", ok, "full rank", int((ost == 0).sum()))


if __name__ == "__main__":
    main()
