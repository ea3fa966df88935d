#!/usr/bin/env python3
"""Where the time of the many-small-objects elimination goes (rref.hip gf_rref_small_kernel): a diagnostic build
(-DRLNC_RREF_PROFILE, loaded through RLNC_LIB_PATH) turns statuses 0-7 into per-wave cycle counts -- 0 between
pieces, 2 forward, 3 normalise, 4 backward (reg_run), 5 setup (table copy, header staging), 6 entry to outputs
in shader cycles, 7 the same in 10 ns ticks -- and the rank into the wave's entry tick (100 MHz).  Prints the
median/max per phase, the spread of entry ticks across the grid, and the kernel's event time."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    ctx = rlnc_amd.Context(0)
    for B, k, m in [(4096, 16, 16), (4096, 8, 8), (2048, 16, 16)]:
        rng = np.random.default_rng(k)
        pieces = torch.zeros((B, m, k + 16), dtype=torch.uint8, device="cuda")
        pieces[:, :, :k] = torch.from_numpy(rng.integers(0, 256, (B, m, k), dtype=np.uint8)).cuda()
        T = torch.empty((B, k, m), dtype=torch.uint8, device="cuda")
        ps = torch.empty((B, m), dtype=torch.int32, device="cuda")
        rk = torch.empty((B,), dtype=torch.int32, device="cuda")
        ts = []
        for it in range(7):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            batch.decode_batch_eliminate(pieces, k, T, ps, rk, ctx)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ph = ps.cpu().numpy()[:, :8].astype(np.int64)
        entry = rk.cpu().numpy().astype(np.int64)
        entry -= entry.min()
        end = entry + ph[:, 7]
        print(json.dumps({"objects": B, "k": k, "m": m, "event_ms": round(sorted(ts)[3], 4),
                          "phases": "between forward normalise backward setup entry_to_out_cycles entry_to_out_10ns",
                          "median": [int(x) for x in np.median(ph[:, [0, 2, 3, 4, 5, 6, 7]], axis=0)],
                          "max": [int(x) for x in ph[:, [0, 2, 3, 4, 5, 6, 7]].max(axis=0)],
                          "entry_spread_10ns": [int(x) for x in np.percentile(entry, [0, 50, 90, 100])],
                          "last_end_10ns": int(end.max())}), flush=True)


if __name__ == "__main__":
    main()
