#!/usr/bin/env python3
"""Interleaved in-process A/B of GF(2^8) matmul kernel configurations (cdna_hip_programming.md §5.4 rule 24).

Times the encode launch of the bench workload (16 objects × k=32 × 1 MiB → 64 coded pieces) and the decode
T × D launch shape (32 × 32) for each (variant, tile) configuration, N rounds, HIP events on the launch
stream.  Prints one JSON line per configuration with median/min ms and GF multiply-add rate.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--objects", type=int, default=16)
    ap.add_argument("--configs", default="0:0,0:16,0:8,1:0")
    ap.add_argument("--fill", default="random", choices=["random", "zero", "ones"],
                    help="source bytes (zero/ones: the data-dependent power/clock check of MI355X_MICROARCH.md)")
    args = ap.parse_args()
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    ctx = rlnc_amd.Context(0)
    B, k, L, n = args.objects, 32, 1 << 20, 64
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device="cuda", generator=g)
    if args.fill != "random":
        src.fill_(0 if args.fill == "zero" else 0xFF)
    co = torch.randint(0, 256, (B, n, k), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty((B, n, k + L), dtype=torch.uint8, device="cuda")
    T = torch.randint(0, 256, (B, k, k), dtype=torch.uint8, device="cuda", generator=g)
    dec = torch.empty((B, k, L), dtype=torch.uint8, device="cuda")
    configs = [tuple(int(x) for x in c.split(":")) for c in args.configs.split(",")]
    res = {c: {"enc": [], "dec": []} for c in configs}
    ref_enc = ref_dec = None
    for r in range(args.rounds + 1):
        for c in configs:
            ctx.set_kernel_variant(*c)
            for name, fn in (("enc", lambda: batch.encode_batch(src, co, out, ctx)),
                             ("dec", lambda: batch.matmul(T, src, dec, ctx))):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                if r:
                    res[c][name].append(e0.elapsed_time(e1))
            if r == 0:  # all configurations must agree bit for bit
                if ref_enc is None:
                    ref_enc, ref_dec = out.clone(), dec.clone()
                elif not os.environ.get("RLNC_DIAG"):
                    assert torch.equal(out, ref_enc) and torch.equal(dec, ref_dec), c
    for c in configs:
        line = {"variant": ["perm", "nibble", "perm3", "wide2", "wide4", "bitsliced", "bitsliced-jump",
                            "bitsliced-jump-shared", "bitsliced-jump-shared-8w", "bitsliced-jump-run"][c[0]],
                "tile_rows": c[1]}
        for name, ma in (("enc", B * n * k * L), ("dec", B * k * k * L)):
            v = sorted(res[c][name])
            line[name + "_ms_med"] = round(v[len(v) // 2], 4)
            line[name + "_ms_min"] = round(v[0], 4)
            line[name + "_Tma_s"] = round(ma / (v[len(v) // 2] * 1e-3) / 1e12, 2)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
