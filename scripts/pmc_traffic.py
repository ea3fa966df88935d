#!/usr/bin/env python3
"""Turn scripts/pmc_bench.sh's summary (per kernel/grid, FETCH_SIZE x2 gfx950 correction applied) into
profiles/pmc_traffic.json: HBM bytes per launch of the bench's dominant kernel, keyed by kernel variant and
shape (objects = grid threads / (2 row tiles x 256 column blocks x 256 threads)), which bench.py reports as roofline.traffic when the configuration matches."""
import json
import sys

summary, variant, kernel, grid, out = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
for line in open(summary):
    d = json.loads(line)
    if kernel in d["kernel"] and d["grid"] == grid:
        rec = {"variant": variant, "kernel": d["kernel"], "grid": grid, "objects": grid // (2 * 256 * 256), "k": 32,
               "piece_bytes": 1 << 20, "coded": 64, "hbm_read_bytes": d["hbm_read_bytes"],
               "hbm_write_bytes": d["hbm_write_bytes"], "source": summary}
        try:
            table = json.load(open(out))
        except FileNotFoundError:
            table = {}
        table[variant] = rec
        json.dump(table, open(out, "w"), indent=1)
        print(json.dumps(rec))
        break
else:
    sys.exit(f"no {kernel}@{grid} in {summary}")
