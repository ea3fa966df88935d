#!/usr/bin/env python3
"""Ragged receiver batches on one MI355X: 256 objects of 8 shapes decoded (and recoded) in one rlnc_decode_ragged /
rlnc_recode_ragged call, against the same objects decoded shape group by shape group with rlnc_decode_batch_device
(one call per shape).  Prints one JSON line (HIP-event times, median of 7 calls after 3 warm-ups, outputs checked
equal between the two paths).  Run it under `rocprofv3 --kernel-trace --stats` to count the launches per stage."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rlnc_amd  # noqa: E402
from rlnc_amd import batch  # noqa: E402

SHAPES = [(16, 4096, 16), (16, 8192, 18), (32, 16384, 32), (32, 65536, 34), (64, 16384, 64), (64, 4096 * 6, 66),
          (128, 8192, 128), (128, 65536, 130)]  # (k, L, m): 32 objects each


def median_ms(fn, reps=7, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def main():
    ctx = rlnc_amd.Context(0)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    groups = []
    for k, L, m in SHAPES:
        B = 32
        src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device="cuda", generator=gen)
        co = torch.randint(0, 256, (B, m, k), dtype=torch.uint8, device="cuda", generator=gen)
        pieces = torch.empty((B, m, k + L), dtype=torch.uint8, device="cuda")
        batch.encode_batch(src, co, pieces, ctx)
        groups.append(dict(k=k, L=L, m=m, B=B, src=src, pieces=pieces,
                           dec_r=torch.zeros((B, k, L), dtype=torch.uint8, device="cuda"),
                           dec_g=torch.zeros((B, k, L), dtype=torch.uint8, device="cuda"),
                           ps=torch.empty((B, m), dtype=torch.int32, device="cuda"),
                           os=torch.empty(B, dtype=torch.int32, device="cuda"),
                           dl=torch.empty(B, dtype=torch.int64, device="cuda")))
    objs = [(g["pieces"][o], g["k"], g["dec_r"][o]) for g in groups for o in range(g["B"])]
    rng = np.random.default_rng(1)
    objs = [objs[i] for i in rng.permutation(len(objs))]  # shapes interleaved

    def ragged():
        batch.decode_ragged(objs, ctx)

    def grouped():
        for g in groups:
            batch.decode_batch_device(g["pieces"], g["k"], g["dec_g"], g["ps"], g["os"], g["dl"], ctx)

    t_r = median_ms(ragged)
    t_g = median_ms(grouped)
    torch.cuda.synchronize()
    ok = all(torch.equal(g["dec_r"], g["dec_g"]) and torch.equal(g["dec_r"], g["src"]) for g in groups)
    ma = sum(g["B"] * g["k"] * g["m"] * g["L"] for g in groups)  # T x data multiply-adds
    # recode: every object recodes 8 pieces from its m received ones
    robjs, rkeep = [], []
    for g in groups:
        for o in range(g["B"]):
            r = torch.randint(0, 256, (8, g["m"]), dtype=torch.uint8, device="cuda", generator=gen)
            out = torch.empty((8, g["k"] + g["L"]), dtype=torch.uint8, device="cuda")
            robjs.append((g["pieces"][o], r, out, g["k"]))
    t_rec = median_ms(lambda: batch.recode_ragged(robjs, ctx))
    rma = sum(8 * g["m"] * (g["k"] + g["L"]) * g["B"] for g in groups)
    print(json.dumps({
        "what": "rlnc_decode_ragged over 256 objects of 8 shapes vs rlnc_decode_batch_device per shape group",
        "shapes": SHAPES, "objects": len(objs),
        "ragged_decode_ms": round(t_r, 4), "grouped_decode_ms": round(t_g, 4),
        "ragged_decode_T_ma_per_s": round(ma / (t_r * 1e-3) / 1e12, 2),
        "grouped_decode_T_ma_per_s": round(ma / (t_g * 1e-3) / 1e12, 2),
        "ragged_recode_ms": round(t_rec, 4), "ragged_recode_T_ma_per_s": round(rma / (t_rec * 1e-3) / 1e12, 2),
        "verified": bool(ok)}), flush=True)


if __name__ == "__main__":
    main()
