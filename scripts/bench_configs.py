#!/usr/bin/env python3
"""Device-resident rates of every BASELINE.json config on one MI355X (the bench line measures configs[1]+[2]):

  encode  configs[1]: 32 x 1 MiB -> 64 coded pieces, 16 objects per launch
  decode  configs[2]: Gaussian RREF + T x data on 32 received pieces x (32 + 1 MiB), 16 objects
  recode  configs[3]: 64 coded pieces x (64 + 256 KiB) -> 64 recoded pieces, 16 objects
  batch   configs[4]: per GPU 512 of the 4096 objects (the 8-GPU sharding), k = 128 x 64 KiB: encode 128 coded
                      pieces + decode from the first 128, one launch each for all 512 objects
  round1  configs[0] at device scale: 16 x 4 KiB source pieces, encode 16 + decode 16, 4096 objects

GiB/s in the reference's own counters (benches/full_rlnc_*.rs): encode (kL + k + L) per coded
piece, decode k(k + L) per object, recode (n + 1)(k + L) per recoded piece.  HIP events around the launches on
the launch stream (5 back-to-back calls per sample), median of ROUNDS; every config's outputs are checked (decode: recovered source; recode:
decodes back).  One JSON line per config.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GIB = float(1 << 30)


def timed(fn, rounds, reps=5):
    """Median over `rounds` of the mean time of `reps` back-to-back calls (steady clocks: a lone call after an
    idle gap runs ~15 % slower while the GPU clock ramps up)."""
    import torch

    ts = []
    for r in range(rounds + 2):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        if r >= 2:
            ts.append(a.elapsed_time(b) / reps)
    return sorted(ts)[len(ts) // 2]


def main():
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    rounds = int(os.environ.get("ROUNDS", "6"))
    ctx = rlnc_amd.Context(0)
    if os.environ.get("VARIANT"):  # A/B: another matmul kernel variant (default: the context's)
        ctx.set_kernel_variant(int(os.environ["VARIANT"]), 0)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(11)

    def rnd(*shape):
        return torch.randint(0, 256, shape, dtype=torch.uint8, device=dev, generator=g)

    def enc_dec(name, B, k, L, n, m):
        src, co = rnd(B, k, L), rnd(B, n, k)
        pieces = torch.empty((B, n, k + L), dtype=torch.uint8, device=dev)
        dec = torch.empty((B, k, L), dtype=torch.uint8, device=dev)
        pst = torch.empty((B, m), dtype=torch.int32, device=dev)
        ost = torch.empty((B,), dtype=torch.int32, device=dev)
        dl = torch.empty((B,), dtype=torch.int64, device=dev)
        t_enc = timed(lambda: batch.encode_batch(src, co, pieces, ctx), rounds)
        t_dec = timed(lambda: batch.decode_batch_device(pieces[:, :m], k, dec, pst, ost, dl, ctx), rounds)
        full_rank = (pst == 0).sum(1) == k
        ok = bool(torch.equal(dec[full_rank], src[full_rank])) and bool(full_rank.any())
        enc_b = B * n * (k * L + k + L)
        dec_b = B * k * (k + L)
        return {"config": name, "objects": B, "k": k, "piece_bytes": L, "coded": n, "decoded_from": m,
                "encode_ms": round(t_enc, 4), "encode_GiBps": round(enc_b / t_enc / 1e-3 / GIB, 1),
                "encode_T_muladd_per_s": round(B * n * k * L / t_enc / 1e9, 2),
                "decode_ms": round(t_dec, 4), "decode_GiBps": round(dec_b / t_dec / 1e-3 / GIB, 1),
                "decode_T_muladd_per_s": round(B * k * k * L / t_dec / 1e9, 2),
                "roundtrip_GiBps": round((enc_b + dec_b) / (t_enc + t_dec) / 1e-3 / GIB, 1),
                "full_rank_objects": int(full_rank.sum()), "verified": ok}

    def recode(out):  # configs[3]: recoder over 64 coded pieces (k = 64, L = 256 KiB) -> 64 recoded pieces
        B, k, L, n, cnt = 16, 64, 1 << 18, 64, 64
        src, co, r = rnd(B, k, L), rnd(B, n, k), rnd(B, cnt, n)
        pieces = torch.empty((B, n, k + L), dtype=torch.uint8, device=dev)
        batch.encode_batch(src, co, pieces, ctx)
        rec = torch.empty((B, cnt, k + L), dtype=torch.uint8, device=dev)
        t_rec = timed(lambda: batch.recode_batch(pieces, r, rec, k, ctx), rounds)
        dec = torch.empty((B, k, L), dtype=torch.uint8, device=dev)
        pst = torch.empty((B, cnt), dtype=torch.int32, device=dev)
        ost = torch.empty((B,), dtype=torch.int32, device=dev)
        dl = torch.empty((B,), dtype=torch.int64, device=dev)
        batch.decode_batch_device(rec, k, dec, pst, ost, dl, ctx)
        torch.cuda.synchronize()
        fr = (pst == 0).sum(1) == k
        rec_b = B * cnt * (n + 1) * (k + L)
        out.append({"config": "configs[3] recode", "objects": B, "k": k, "piece_bytes": L, "received": n,
                    "recoded": cnt, "recode_ms": round(t_rec, 4),
                    "recode_GiBps": round(rec_b / t_rec / 1e-3 / GIB, 1),
                    "recode_T_muladd_per_s": round(B * cnt * n * (k + L) / t_rec / 1e9, 2),
                    "verified": bool(torch.equal(dec[fr], src[fr])) and bool(fr.any())})

    only = os.environ.get("CONFIGS")  # a subset, e.g. CONFIGS=0 or CONFIGS=1,3 (profiling runs)
    want = (lambda c: only is None or c in only.split(","))
    out = []
    if want("1"):
        out.append(enc_dec("configs[1]+[2] (bench)", 16, 32, 1 << 20, 64, 32))
    if want("3"):
        recode(out)
    if want("4"):
        out.append(enc_dec("configs[4] batch (512 of 4096 objects per GPU)", 512, 128, 1 << 16, 128, 128))
    if want("0"):
        out.append(enc_dec("configs[0] shape at device scale", 4096, 16, 4096, 16, 16))
    for line in out:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
