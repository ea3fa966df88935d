#!/usr/bin/env python3
"""Timeline of the many-small-objects elimination (configs[0] shape) from per-wave timestamps: run with the
diagnostic build (RLNC_LIB_PATH=rlnc_amd/librlnc_hip_ab.so), which takes RLNC_SMALL_PROF=<hex device address> and
writes wall-clock stamps (s_memrealtime, 100 MHz) at wave start, after the table copy, after the header staging,
after the pieces and at the end, plus the CU id.  Prints percentiles of each phase and of the start / end times."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import rlnc_amd
    from rlnc_amd import batch

    B, k, L, m = int(os.environ.get("OBJS", "4096")), 16, 4096, 16
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=g)
    co = torch.randint(0, 256, (B, m, k), dtype=torch.uint8, device=dev, generator=g)
    pieces = torch.empty((B, m, k + L), dtype=torch.uint8, device=dev)
    ctx = rlnc_amd.Context(0)
    batch.encode_batch(src, co, pieces, ctx)
    T = torch.empty((B, k, m), dtype=torch.uint8, device=dev)
    pst = torch.empty((B, m), dtype=torch.int32, device=dev)
    rank = torch.empty(B, dtype=torch.int32, device=dev)
    for _ in range(5):
        batch.decode_batch_eliminate(pieces, k, T, pst, rank, ctx)
    prof = torch.zeros((B, 8), dtype=torch.int64, device=dev)
    os.environ["RLNC_SMALL_PROF"] = "%x" % prof.data_ptr()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    batch.decode_batch_eliminate(pieces, k, T, pst, rank, ctx)
    b.record()
    torch.cuda.synchronize()
    del os.environ["RLNC_SMALL_PROF"]
    ms = a.elapsed_time(b)
    P = prof.cpu().numpy().astype(np.float64)
    t0 = P[:, 0].min()
    us = (P[:, :5] - t0) / 100.0  # 100 MHz -> us
    pct = lambda x: [round(float(np.percentile(x, q)), 2) for q in (0, 10, 50, 90, 100)]
    out = {"event_ms": round(ms, 4), "objects": B, "percentiles": "0/10/50/90/100",
           "start_us": pct(us[:, 0]), "end_us": pct(us[:, 4]),
           "table_copy_us": pct(us[:, 1] - us[:, 0]), "headers_us": pct(us[:, 2] - us[:, 1]),
           "pieces_us": pct(us[:, 3] - us[:, 2]), "outputs_us": pct(us[:, 4] - us[:, 3]),
           "wave_life_us": pct(us[:, 4] - us[:, 0]),
           "distinct_cu_ids": int(len(np.unique(prof.cpu().numpy()[:, 5] >> 32)))}
    dirty = (prof.cpu().numpy()[:, 5] & 0xFFFFFFFF).astype(np.int64)
    rows = prof.cpu().numpy()[:, 6]
    life = us[:, 4] - us[:, 0]
    out["objects_with_dirty_pieces"] = int((dirty > 0).sum())
    out["dirty_pieces_total"] = int(dirty.sum())
    out["life_us_clean_objects"] = pct(life[dirty == 0]) if (dirty == 0).any() else None
    out["life_us_dirty_objects"] = pct(life[dirty > 0]) if (dirty > 0).any() else None
    out["rank_deficient_objects"] = int((rows < k).sum())
    cu = (prof.cpu().numpy()[:, 5] >> 32).astype(np.int64)
    ids, counts = np.unique(cu, return_counts=True)
    out["objects_per_cu_hist"] = {int(c): int(n) for c, n in zip(*np.unique(counts, return_counts=True))}
    per_cu = dict(zip(ids.tolist(), counts.tolist()))
    by_count = {}
    for i in range(B):
        by_count.setdefault(per_cu[int(cu[i])], []).append(life[i])
    out["life_us_median_by_cu_load"] = {int(c): round(float(np.median(v)), 2) for c, v in sorted(by_count.items())}
    # the slowest 20 objects: (life us, dirty pieces, rows, cu)
    idx = np.argsort(-life)[:20]
    out["slowest"] = [[round(float(life[i]), 2), int(dirty[i]), int(rows[i]), int(prof.cpu().numpy()[i, 5] >> 32)]
                      for i in idx]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
