#!/usr/bin/env python3
"""Cost of the device elimination (gf_rref_batch_kernel) by coefficient structure.

Decodes 16 objects (k = 32, first 32 coded pieces, L = 64 KiB so the T × D product is small) whose coding
vectors are (a) unit upper triangular — every piece keeps the matrix a clean RREF, (b) uniform random (the
bench), (c) uniform random but with piece 1 of every object a multiple of piece 0 shifted so that its
reduced diagonal is zero (every object leaves the clean path at piece 1).  Prints the median decode time per
case (HIP events); the differences are the elimination kernel's.
"""
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
    B, k, L, m = 16, 32, 1 << 16, 32
    rng = np.random.default_rng(7)
    src = torch.from_numpy(rng.integers(0, 256, (B, k, L), dtype=np.uint8)).cuda()
    cases = {}
    tri = np.zeros((B, m, k), np.uint8)
    for o in range(B):
        for r in range(m):
            tri[o, r, r] = 1
            tri[o, r, r + 1:] = rng.integers(0, 256, k - r - 1)
    cases["clean_upper_triangular"] = tri
    cases["random"] = rng.integers(0, 256, (B, m, k), dtype=np.uint8)
    dirty = rng.integers(0, 256, (B, m, k), dtype=np.uint8)
    dirty[:, 0, :] = 0
    dirty[:, 0, 0] = 1
    dirty[:, 0, 2:] = rng.integers(0, 256, (B, k - 2))
    dirty[:, 1, :] = 0
    dirty[:, 1, 2] = 5  # reduced by row 0 (column 0 is zero) -> diagonal M[1][1] = 0, column 2 nonzero: kept
    cases["dirty_from_piece_1"] = dirty
    # 2 registers (multi-wave initial clean run), 3 LDS clean state, 4 registers on one wave
    paths = [int(x) for x in os.environ.get("RREF_PATHS", "2,4,3").split(",")]
    for (name, co), path in [(c, p) for c in cases.items() for p in paths]:
        ctx.set_decode_path(path)
        pieces = torch.empty((B, m, k + L), dtype=torch.uint8, device="cuda")
        batch.encode_batch(src, torch.from_numpy(co).cuda(), pieces, ctx)
        out = torch.empty((B, k, L), dtype=torch.uint8, device="cuda")
        pst = torch.empty((B, m), dtype=torch.int32, device="cuda")
        ost = torch.empty((B,), dtype=torch.int32, device="cuda")
        dl = torch.empty((B,), dtype=torch.int64, device="cuda")
        times = []
        for r in range(12):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            batch.decode_batch_device(pieces, k, out, pst, ost, dl, ctx)
            e1.record()
            torch.cuda.synchronize()
            if r >= 2:
                times.append(e0.elapsed_time(e1))
        times.sort()
        line = {"case": name, "decode_path": path, "decode_ms_med": round(times[len(times) // 2], 4), "decode_ms_min": round(times[0], 4)}
        if os.environ.get("RLNC_RREF_PROFILE"):  # diagnostic library: cycles per piece / setup (object 0..2)
            line["phase_cycles_obj0_1"] = pst[:2, :8].cpu().tolist()
            ent = pst[:, 4].cpu().numpy().astype(np.int64)
            line["entry_ticks_10ns_rel"] = (ent - ent.min()).tolist()  # when each object's workgroup started
            line["phase_names"] = "row_init spare_copy forward normalise backward generic is_clean status"
        else:
            line["object_status"] = ost.cpu().tolist()
            line["useful_pieces"] = (pst == 0).sum(1).cpu().tolist()
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
