#!/usr/bin/env python3
"""configs[0]-shape decode (4,096 objects x k = 16 x 4 KiB, 16 received pieces each): can the elimination hide behind
the HBM-bound T x data product?  Measures, with HIP events (median of ROUNDS samples of 5 back-to-back calls):
  * the whole decode (rlnc_decode_batch_device), the elimination alone, the product + scan alone;
  * the product on CU-masked streams (hipExtStreamCreateWithCUMask) of N CUs, two mask layouts;
  * the elimination on CU-masked streams of E CUs;
  * the chunked overlap: chunk c + 1's elimination on E CUs beside chunk c's product on the other 256 - E.
One JSON line per measurement.  Every overlapped run's decoded objects are compared with the plain decode.
    python3 scripts/cfg0_overlap.py > gpurun_out/cfg0_overlap.jsonl
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    rounds = int(os.environ.get("ROUNDS", "6"))
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]

    def masked(cus):
        words = (ncu + 31) // 32
        arr = (ctypes.c_uint32 * words)()
        for i in cus:
            arr[i // 32] |= 1 << (i % 32)
        s = ctypes.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, arr) == 0
        return torch.cuda.ExternalStream(s.value, device=dev)

    def layout(n, kind, first=True):
        """n CUs: 'lo' = CUs 0..n-1 (or the top n), 'mod' = n / ncu of every 8-CU group (spread over CU ids)."""
        if kind == "lo":
            return list(range(n)) if first else list(range(ncu - n, ncu))
        per = n * 8 // ncu
        sel = [i for i in range(ncu) if (i % 8) < per] if first else [i for i in range(ncu) if (i % 8) >= 8 - per]
        return sel

    def complement(sel):
        s = set(sel)
        return [i for i in range(ncu) if i not in s]

    def timed(fn, reps=5):
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

    B, k, L, m = 4096, 16, 4096, 16
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=g)
    co = torch.randint(0, 256, (B, m, k), dtype=torch.uint8, device=dev, generator=g)
    pieces = torch.empty((B, m, k + L), dtype=torch.uint8, device=dev)
    ctx = rlnc_amd.Context(0)
    batch.encode_batch(src, co, pieces, ctx)
    dec = torch.empty((B, k, L), dtype=torch.uint8, device=dev)
    pst = torch.empty((B, m), dtype=torch.int32, device=dev)
    ost = torch.empty(B, dtype=torch.int32, device=dev)
    dl = torch.empty(B, dtype=torch.int64, device=dev)
    T = torch.empty((B, k, m), dtype=torch.uint8, device=dev)
    rank = torch.empty(B, dtype=torch.int32, device=dev)

    def emit(**kw):
        print(json.dumps(kw), flush=True)

    t_full = timed(lambda: batch.decode_batch_device(pieces, k, dec, pst, ost, dl, ctx))
    ref = dec.clone()
    ref_pst = pst.clone()
    emit(what="decode_batch_device", ms=round(t_full, 4), T_ma_per_s=round(B * k * k * L / t_full / 1e9, 2))
    t_el = timed(lambda: batch.decode_batch_eliminate(pieces, k, T, pst, rank, ctx))
    emit(what="eliminate", ms=round(t_el, 4))
    t_ap = timed(lambda: batch.decode_batch_apply(pieces, k, T, rank, dec, ost, dl, ctx))
    emit(what="apply (product + scan, offset launch included)", ms=round(t_ap, 4))
    assert torch.equal(dec, ref)

    ctxs = {}

    def ctx_for(stream):
        if stream not in ctxs:
            c = rlnc_amd.Context(0)
            ctxs[stream] = c
        return ctxs[stream]

    # the product on CU-masked streams
    for kind in ("lo", "mod"):
        for n in (256, 224, 192, 160, 128):
            if n > ncu:
                continue
            s = masked(layout(n, kind))
            c = ctx_for(s)
            with torch.cuda.stream(s):
                t = timed(lambda: batch.decode_batch_apply(pieces, k, T, rank, dec, ost, dl, c))
            emit(what="apply on masked stream", layout=kind, cus=n, ms=round(t, 4))
        for e in (32, 64, 96, 128):
            s = masked(layout(e, kind))
            c = ctx_for(s)
            with torch.cuda.stream(s):
                t = timed(lambda: batch.decode_batch_eliminate(pieces, k, T, pst, rank, c))
            emit(what="eliminate on masked stream", layout=kind, cus=e, ms=round(t, 4))

    # chunked overlap: elimination of chunk c+1 (stream A, E CUs) beside the product of chunk c (stream B, the rest)
    for kind in ("lo", "mod"):
        for e in (32, 64, 96, 128):
            sel = layout(e, kind)
            sa, sb = masked(sel), masked(complement(sel))
            ca, cb = ctx_for(sa), ctx_for(sb)
            for C in (2, 4, 8):
                per = B // C
                evs = [torch.cuda.Event() for _ in range(C)]
                done = torch.cuda.Event()

                def run():
                    cur = torch.cuda.current_stream()
                    ev0 = torch.cuda.Event()
                    ev0.record(cur)
                    sa.wait_event(ev0)
                    sb.wait_event(ev0)
                    for c in range(C):
                        sl = slice(c * per, (c + 1) * per)
                        with torch.cuda.stream(sa):
                            batch.decode_batch_eliminate(pieces[sl], k, T[sl], pst[sl], rank[sl], ca)
                            evs[c].record(sa)
                        with torch.cuda.stream(sb):
                            sb.wait_event(evs[c])
                            batch.decode_batch_apply(pieces[sl], k, T[sl], rank[sl], dec[sl], ost[sl], dl[sl], cb)
                    done.record(sb)
                    cur.wait_event(done)

                dec.zero_()
                t = timed(run)
                ok = bool(torch.equal(dec, ref)) and bool(torch.equal(pst, ref_pst))
                emit(what="chunked overlap", layout=kind, elim_cus=e, chunks=C, ms=round(t, 4),
                     T_ma_per_s=round(B * k * k * L / t / 1e9, 2), verified=ok)


if __name__ == "__main__":
    main()
