#!/usr/bin/env python3
"""Per-call timeline of the object API (for rocprofv3 --runtime-trace --kernel-trace --memory-copy-trace): 40
Encoder::code_with_buf calls at two shapes (1 MiB / k = 32: L = 32,769; 32 MiB / k = 32: L = 1,048,577) and 40
Recoder::recode_with_buf calls, host wall time per call printed.
    rocprofv3 --runtime-trace --kernel-trace --memory-copy-trace -d gpurun_out/objtrace -o run -- python3 scripts/object_api_trace.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import rlnc_amd
    from rlnc_amd.full import Encoder, Recoder

    ctx = rlnc_amd.Context(0)
    rng = np.random.default_rng(2)
    for size, k in ((1 << 20, 32), (1 << 25, 32)):
        enc = Encoder.new(rng.integers(0, 256, size, dtype=np.uint8), k, ctx)
        buf = np.zeros(enc.get_full_coded_piece_byte_len(), np.uint8)
        ts = []
        for _ in range(40):
            t0 = time.perf_counter()
            enc.code_with_buf(rng, buf)
            ts.append(time.perf_counter() - t0)
        print(f"encode size={size} k={k} median_us={1e6 * sorted(ts)[20]:.1f}", flush=True)
    enc = Encoder.new(rng.integers(0, 256, 1 << 24, dtype=np.uint8), 64, ctx)
    full = enc.get_full_coded_piece_byte_len()
    r = Recoder.new(np.concatenate([enc.code(rng) for _ in range(32)]), full, 64, ctx)
    buf = np.zeros(full, np.uint8)
    ts = []
    for _ in range(40):
        t0 = time.perf_counter()
        r.recode_with_buf(rng, buf)
        ts.append(time.perf_counter() - t0)
    print(f"recode median_us={1e6 * sorted(ts)[20]:.1f}", flush=True)


if __name__ == "__main__":
    main()
