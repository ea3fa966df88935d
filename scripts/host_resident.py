#!/usr/bin/env python3
"""Host-resident rate (BASELINE.json north_star: "pieces start and end in host memory ... the rate including
pinned hipMemcpyAsync to and from the device is also measured and recorded in DESIGN.md").

Same workload as bench.py (per object: encode k=32 × 1 MiB → 64 coded pieces, decode from the first 32), but
every object's source starts in pinned host memory and its coded pieces and decoded data end there:
    H2D source (32 MiB) → encode → D2H 64 coded pieces (64 MiB)
    H2D 32 received pieces (32 MiB) → decode → D2H decoded data (32 MiB)
Objects are pipelined over two HIP streams (copies of one object overlap the kernels of the other).
Reports GiB/s in bench.py's counters plus the raw pinned H2D / D2H bandwidth.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--objects", type=int, default=16)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench
    import rlnc_amd
    from rlnc_amd import batch

    k, L, n, m, B = 32, 1 << 20, 64, 32, args.objects
    dev = torch.device("cuda", 0)
    # pinned host buffers
    src_h = torch.randint(0, 256, (B, k, L), dtype=torch.uint8).pin_memory()
    co_h = torch.from_numpy(np.random.default_rng(1).integers(0, 256, (B, n, k), dtype=np.uint8)).pin_memory()
    coded_h = torch.empty((B, n, k + L), dtype=torch.uint8).pin_memory()
    dec_h = torch.empty((B, k, L), dtype=torch.uint8).pin_memory()
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    ctxs = [rlnc_amd.Context(0) for _ in range(2)]
    bufs = []
    for _ in range(2):
        bufs.append(dict(src=torch.empty((1, k, L), dtype=torch.uint8, device=dev),
                         co=torch.empty((1, n, k), dtype=torch.uint8, device=dev),
                         pieces=torch.empty((1, n, k + L), dtype=torch.uint8, device=dev),
                         recv=torch.empty((1, m, k + L), dtype=torch.uint8, device=dev),
                         dec=torch.empty((1, k, L), dtype=torch.uint8, device=dev),
                         ps=torch.empty((1, m), dtype=torch.int32, device=dev),
                         os=torch.empty(1, dtype=torch.int32, device=dev),
                         dl=torch.empty(1, dtype=torch.int64, device=dev)))

    def step():
        for o in range(B):
            s, c, b = streams[o % 2], ctxs[o % 2], bufs[o % 2]
            with torch.cuda.stream(s):
                b["src"].copy_(src_h[o:o + 1], non_blocking=True)
                b["co"].copy_(co_h[o:o + 1], non_blocking=True)
                batch.encode_batch(b["src"], b["co"], b["pieces"], c)
                coded_h[o:o + 1].copy_(b["pieces"], non_blocking=True)
                # the receiver side: 32 coded pieces arrive from host memory
                b["recv"].copy_(coded_h[o:o + 1, :m], non_blocking=True)
                batch.decode_batch_device(b["recv"], k, b["dec"], b["ps"], b["os"], b["dl"], c)
                dec_h[o:o + 1].copy_(b["dec"], non_blocking=True)

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.steps
    ok = bool(torch.equal(dec_h[B - 1], src_h[B - 1]))

    # raw pinned bandwidth
    big_h = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    big_d = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    big_d.copy_(big_h, non_blocking=True)
    torch.cuda.synchronize()
    h2d = (1 << 30) / (time.perf_counter() - t) / 1e9
    t = time.perf_counter()
    big_h.copy_(big_d, non_blocking=True)
    torch.cuda.synchronize()
    d2h = (1 << 30) / (time.perf_counter() - t) / 1e9
    moved = B * (k * L + n * (k + L) + m * (k + L) + k * L)
    print(json.dumps({
        "metric": "host-resident RLNC encode+decode GiB/s (pinned hipMemcpyAsync in and out), k=32 x 1 MiB",
        "value": round(bench.step_bytes(B, k, L, n) / el / 2**30, 2), "unit": "GiB/s",
        "ms_per_step": round(el * 1e3, 3), "objects": B, "pcie_bytes_per_step": moved,
        "pcie_GBps_effective": round(moved / el / 1e9, 2), "pinned_h2d_GBps": round(h2d, 2),
        "pinned_d2h_GBps": round(d2h, 2), "verified": ok,
        "roundtrip_goodput_GiBps": round(B * k * L / el / 2**30, 3)}))


if __name__ == "__main__":
    main()
