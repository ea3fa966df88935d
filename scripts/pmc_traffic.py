#!/usr/bin/env python3
"""Turn scripts/pmc_bench.sh's summary (per kernel/grid, FETCH_SIZE x2 gfx950 correction applied) into
profiles/pmc_traffic.json: HBM bytes per launch of one of the bench's kernels, keyed by name (the encode's kernel
variant, or "decode:<variant>" for the decode's T x data product), with the bench shape it was measured on, which
bench.py reports as roofline.traffic / roofline_decode.traffic when the configuration matches.

    python3 scripts/pmc_traffic.py SUMMARY KEY KERNEL GRID OUT [THREADS_PER_OBJECT]

THREADS_PER_OBJECT: grid threads of one object (default 131072: the encode's 64-row tile of 512 threads per 4 KiB
column block, 256 column blocks; the decode's 32-row product: 256 threads x 256 column blocks = 65536)."""
import json
import sys

summary, key, kernel, grid, out = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
per_obj = int(sys.argv[6]) if len(sys.argv) > 6 else 2 * 256 * 256
for line in open(summary):
    d = json.loads(line)
    if kernel in d["kernel"] and d["grid"] == grid:
        rec = {"variant": key, "kernel": d["kernel"], "grid": grid, "objects": grid // per_obj, "k": 32,
               "piece_bytes": 1 << 20, "coded": 64, "hbm_read_bytes": d["hbm_read_bytes"],
               "hbm_write_bytes": d["hbm_write_bytes"], "source": summary}
        try:
            table = json.load(open(out))
        except FileNotFoundError:
            table = {}
        table[key] = rec
        json.dump(table, open(out, "w"), indent=1)
        print(json.dumps(rec))
        break
else:
    sys.exit(f"no {kernel}@{grid} in {summary}")
