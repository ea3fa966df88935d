#!/usr/bin/env python3
"""Ragged receiver batches on one MI355X: 256 objects of 8 shapes decoded (and recoded) in one rlnc_decode_ragged /
rlnc_recode_ragged call, against the same objects decoded shape group by shape group with rlnc_decode_batch_device
(one call per shape).  Prints one JSON line (HIP-event times, median of 7 calls after 3 warm-ups, outputs checked
equal between the two paths).  Run it under `rocprofv3 --kernel-trace --stats` to count the launches per stage."""
import json
import time
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
    # the same calls through the C ABI with the descriptor tables built once (what a native caller pays: the
    # Python wrapper above builds 256 ctypes descriptors per call)
    import ctypes as C

    from rlnc_amd._lib import DecodeObjDesc, RecodeObjDesc

    rarr = (RecodeObjDesc * len(robjs))(*[RecodeObjDesc(p.data_ptr(), p.shape[1], r.data_ptr(), o.data_ptr(),
                                                        o.shape[1], k, p.shape[1] - k, p.shape[0], r.shape[0])
                                          for p, r, o, k in robjs])
    darr = (DecodeObjDesc * len(objs))(*[DecodeObjDesc(p.data_ptr(), p.shape[1], d.data_ptr(), k, p.shape[1] - k,
                                                       p.shape[0]) for p, k, d in objs])
    total_m = sum(p.shape[0] for p, _, _ in objs)
    ps_t = torch.empty(total_m, dtype=torch.int32, device="cuda")
    os_t = torch.empty(len(objs), dtype=torch.int32, device="cuda")
    dl_t = torch.empty(len(objs), dtype=torch.int64, device="cuda")

    def rec_abi():
        assert ctx.lib.rlnc_recode_ragged(ctx.h, rarr, len(robjs)) == 0

    def dec_abi():
        assert ctx.lib.rlnc_decode_ragged(ctx.h, darr, len(objs), C.c_void_p(ps_t.data_ptr()),
                                          C.c_void_p(os_t.data_ptr()), C.c_void_p(dl_t.data_ptr())) == 0

    ctx.use_torch_stream()
    t_rec_abi = median_ms(rec_abi)
    t_dec_abi = median_ms(dec_abi)

    def host_ms(fn, reps=9):  # host time of the (asynchronous) call alone: descriptor checks, table upload, launches
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t0) * 1e3)
        torch.cuda.synchronize()
        return sorted(ts)[reps // 2]

    h_rec, h_dec = host_ms(rec_abi), host_ms(dec_abi)
    torch.cuda.synchronize()
    ok = ok and all(torch.equal(g["dec_r"], g["src"]) for g in groups)
    print(json.dumps({
        "what": "rlnc_decode_ragged over 256 objects of 8 shapes vs rlnc_decode_batch_device per shape group",
        "shapes": SHAPES, "objects": len(objs),
        "ragged_decode_ms": round(t_r, 4), "grouped_decode_ms": round(t_g, 4),
        "ragged_decode_T_ma_per_s": round(ma / (t_r * 1e-3) / 1e12, 2),
        "grouped_decode_T_ma_per_s": round(ma / (t_g * 1e-3) / 1e12, 2),
        "ragged_recode_ms": round(t_rec, 4), "ragged_recode_T_ma_per_s": round(rma / (t_rec * 1e-3) / 1e12, 2),
        "abi_decode_ms": round(t_dec_abi, 4), "abi_decode_T_ma_per_s": round(ma / (t_dec_abi * 1e-3) / 1e12, 2),
        "abi_recode_host_ms": round(h_rec, 4), "abi_decode_host_ms": round(h_dec, 4),
        "abi_recode_ms": round(t_rec_abi, 4), "abi_recode_T_ma_per_s": round(rma / (t_rec_abi * 1e-3) / 1e12, 2),
        "verified": bool(ok)}), flush=True)


if __name__ == "__main__":
    main()
