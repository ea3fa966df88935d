#!/usr/bin/env python3
"""HBM roofline of the single-pass encode: n coded pieces (n = 1, 2, 4, 8) from k = 32 source pieces x 1 MiB,
16 objects (512 MiB of source, > the 256 MiB Infinity Cache), one launch; reports the HBM read rate of the
source (k*L bytes per object, read once) and the total compulsory traffic rate against the 8 TB/s peak.
HIP events on the launch stream, median of N rounds, results checked against a CPU product on one column slice."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def mul_table():
    """GF(2^8) products (0x11B), Russian-peasant: a local check, independent of the library."""
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


def np_matmul(co, src, MUL):
    out = np.zeros((co.shape[0], src.shape[1]), np.uint8)
    for i in range(co.shape[0]):
        for j in range(co.shape[1]):
            out[i] ^= MUL[co[i, j]][src[j]]
    return out


def main():
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    ctx = rlnc_amd.Context(0)
    MUL = mul_table()
    B, k, L = int(os.environ.get("HBM_OBJECTS", "16")), 32, 1 << 20
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device="cuda", generator=g)
    for n in [int(x) for x in os.environ.get("HBM_NS", "1,2,4,8").split(",")]:
        for variant in [int(x) for x in os.environ.get("HBM_VARIANTS", "6,0").split(",")]:
            ctx.set_kernel_variant(variant, 0)
            co = torch.randint(0, 256, (B, n, k), dtype=torch.uint8, device="cuda", generator=g)
            out = torch.empty((B, n, k + L), dtype=torch.uint8, device="cuda")
            ts = []
            for r in range(12):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                batch.encode_batch(src, co, out, ctx)
                e1.record()
                torch.cuda.synchronize()
                if r >= 2:
                    ts.append(e0.elapsed_time(e1))
            ms = sorted(ts)[len(ts) // 2]
            o = 3
            want = np_matmul(co[o].cpu().numpy(), src[o, :, :4096].cpu().numpy(), MUL)
            ok = np.array_equal(out[o, :, k:k + 4096].cpu().numpy(), want)
            if variant != 0:  # the whole output against the perm kernel (variant 0, independent code)
                ref = torch.empty_like(out)
                ctx.set_kernel_variant(0, 0)
                batch.encode_batch(src, co, ref, ctx)
                ctx.set_kernel_variant(variant, 0)
                ok = ok and bool(torch.equal(ref, out))
            read = B * (k * L + n * k)
            write = B * n * (k + L)
            print(json.dumps({"n_coded": n, "variant": variant, "ms": round(ms, 4),
                              "source_read_TBps": round(read / ms / 1e9, 3),
                              "read_frac_of_8TBps": round(read / ms / 1e9 / 8.0, 3),
                              "compulsory_TBps": round((read + write) / ms / 1e9, 3), "ok": ok}), flush=True)
    ctx.set_kernel_variant(6, 0)


if __name__ == "__main__":
    main()
