#!/usr/bin/env python3
"""Where a whole-object decode through the drop-in object API spends its time (GPU): Decoder::new, each
Decoder::decode call (first / median / last), Decoder::get_decoded_data, at the reference bench shapes
(benches/full_rlnc_decoder.rs: Encoder::new over 1-32 MiB, k = 16..256).  Medians over 5 objects, microseconds.

    python scripts/decode_call_profile.py   (GPU)
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import rlnc_amd
    from rlnc_amd.full import Decoder, Encoder

    ctx = rlnc_amd.Context(0)
    rng = np.random.default_rng(3)
    for size, k in ((1 << 20, 16), (1 << 20, 32), (1 << 20, 128), (1 << 24, 32), (1 << 25, 32)):
        data = rng.integers(0, 256, size, dtype=np.uint8)
        enc = Encoder.new(data, k, ctx)
        L = enc.get_piece_byte_len()
        if "--after-encode" in sys.argv:  # as object_api_rates.py: code_with_buf calls first
            buf = np.zeros(enc.get_full_coded_piece_byte_len(), np.uint8)
            for _ in range(66):
                enc.code_with_buf(rng, buf)
        pieces = [enc.code(rng) for _ in range(k + 2)]
        rows = []
        for rep in range(6):
            t0 = time.perf_counter()
            dec = Decoder.new(L, k, ctx)
            t1 = time.perf_counter()
            calls = []
            for p in pieces:
                if dec.is_already_decoded():
                    break
                c0 = time.perf_counter()
                try:
                    dec.decode(p)
                except Exception:
                    pass
                calls.append(time.perf_counter() - c0)
            t2 = time.perf_counter()
            got = dec.get_decoded_data()
            t3 = time.perf_counter()
            del dec
            t4 = time.perf_counter()
            if rep:
                rows.append((t1 - t0, calls[0], sorted(calls)[len(calls) // 2], calls[-1], sum(calls), t3 - t2, t4 - t3,
                             t3 - t0))
        assert np.array_equal(got, data)
        med = [sorted(r[i] for r in rows)[len(rows) // 2] * 1e6 for i in range(8)]
        print(json.dumps({"data_bytes": size, "k": k, "L": L, "new_us": round(med[0], 1),
                          "decode_first_us": round(med[1], 1), "decode_median_us": round(med[2], 1),
                          "decode_last_us": round(med[3], 1), "decode_sum_us": round(med[4], 1),
                          "get_decoded_data_us": round(med[5], 1), "free_us": round(med[6], 1),
                          "object_us": round(med[7], 1), "object_us_each": [round(r[7] * 1e6) for r in rows],
                          "get_us_each": [round(r[5] * 1e6) for r in rows], "sum_us_each": [round(r[4] * 1e6) for r in rows]}),
              flush=True)


if __name__ == "__main__":
    main()
