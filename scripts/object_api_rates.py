#!/usr/bin/env python3
"""The drop-in object API (rlnc::full::{Encoder, Decoder, Recoder} over host buffers, through the C ABI) at the
reference's own bench shapes (benches/full_rlnc_{encoder,decoder,recoder}.rs: Encoder::new over 2^20..2^25 random
bytes with k = 16..256, so L = ceil((len + 1) / k) is odd), timed per call like divan: the median of N calls, GiB/s in
the reference's byte counters.  Every call is synchronous and moves its piece across PCIe (pageable numpy buffers),
as a Rust caller's Vec<u8> would.  Beside each line: the published EPYC 9R14 single-thread number where BASELINE.md
has one.

    python scripts/object_api_rates.py   (GPU)
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GIB = float(1 << 30)
# BASELINE.md §1 (EPYC 9R14, single thread): encode_zero_alloc, decode (whole object), recode zero-alloc
PUBLISHED = {("encode", 1 << 25, 32): 27.01, ("decode", 1 << 25, 32): 631.3 / 1024, ("encode", 1 << 24, 128): 38.84,
             ("decode", 1 << 24, 128): 279.5 / 1024, ("recode", 1 << 24, 64): 38.14}


def med(ts):
    return sorted(ts)[len(ts) // 2]


def main():
    import rlnc_amd
    from rlnc_amd.full import Decoder, Encoder, Recoder

    ctx = rlnc_amd.Context(0)
    rng = np.random.default_rng(1)
    out = []
    for (size, k) in ((1 << 20, 16), (1 << 20, 32), (1 << 20, 128), (1 << 24, 32), (1 << 24, 128), (1 << 25, 32),
                      (1 << 25, 256)):
        data = rng.integers(0, 256, size, dtype=np.uint8)
        enc = Encoder.new(data, k, ctx)
        L, full = enc.get_piece_byte_len(), enc.get_full_coded_piece_byte_len()
        buf = np.zeros(full, np.uint8)
        n = max(8, min(64, int(2e8 // full)))
        ts = []
        for i in range(n + 2):
            t0 = time.perf_counter()
            enc.code_with_buf(rng, buf)
            if i >= 2:
                ts.append(time.perf_counter() - t0)
        t = med(ts)
        counter = k * L + full  # benches/full_rlnc_encoder.rs:111-113
        rec = {"op": "encode (code_with_buf)", "data_bytes": size, "k": k, "L": L, "calls": n, "us_per_call": round(t * 1e6, 1),
               "GiBps": round(counter / t / GIB, 2), "published_epyc_GiBps": PUBLISHED.get(("encode", size, k))}
        print(json.dumps(rec), flush=True)
        # decode: k + 2 coded pieces (a dependent one possible), whole object incl. get_decoded_data
        pieces = [enc.code(rng) for _ in range(k + 2)]
        reps = 3 if size >= (1 << 24) else 5
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            dec = Decoder.new(L, k, ctx)
            for p in pieces:
                if dec.is_already_decoded():
                    break
                try:
                    dec.decode(p)
                except Exception:
                    pass
            got = dec.get_decoded_data()
            ts.append(time.perf_counter() - t0)
        assert np.array_equal(got, data), "decode mismatch"
        t = med(ts)
        counter = k * full  # benches/full_rlnc_decoder.rs:118
        print(json.dumps({"op": "decode (k decode() + get_decoded_data)", "data_bytes": size, "k": k, "L": L,
                          "ms_per_object": round(t * 1e3, 2), "GiBps": round(counter / t / GIB, 3),
                          "published_epyc_GiBps": PUBLISHED.get(("decode", size, k))}), flush=True)
        del enc, pieces
    # recode: 16 MB / k = 64, recoding 32 received pieces (benches/full_rlnc_recoder.rs)
    size, k, nrec = 1 << 24, 64, 32
    data = rng.integers(0, 256, size, dtype=np.uint8)
    enc = Encoder.new(data, k, ctx)
    full = enc.get_full_coded_piece_byte_len()
    received = np.concatenate([enc.code(rng) for _ in range(nrec)])
    r = Recoder.new(received, full, k, ctx)
    buf = np.zeros(full, np.uint8)
    ts = []
    for i in range(34):
        t0 = time.perf_counter()
        r.recode_with_buf(rng, buf)
        if i >= 2:
            ts.append(time.perf_counter() - t0)
    t = med(ts)
    counter = (nrec + 1) * full  # benches/full_rlnc_recoder.rs:137-142
    print(json.dumps({"op": "recode (recode_with_buf)", "data_bytes": size, "k": k, "received": nrec,
                      "us_per_call": round(t * 1e6, 1), "GiBps": round(counter / t / GIB, 2),
                      "published_epyc_GiBps": PUBLISHED.get(("recode", size, k))}), flush=True)


if __name__ == "__main__":
    main()
