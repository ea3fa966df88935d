#!/usr/bin/env python3
"""Summarise object-API grid runs (scripts/object_api_bench.cpp output, one JSONL file per box run): per bench and
shape the median over runs, the min-max spread, and the reference's EPYC 9R14 median.
    python3 scripts/objgrid_table.py profiles/r05_object_api_grid_*.jsonl"""
import json
import statistics
import sys
from collections import defaultdict


def main(paths):
    rows = defaultdict(list)
    epyc = {}
    for p in paths:
        for ln in open(p):
            if not ln.startswith("{"):
                continue
            r = json.loads(ln)
            key = (r["bench"], r["data_bytes"], r["k"])
            t = r["decode_total_median_us"] if r["bench"] == "decode" else r["median_us"]
            rows[key].append(t)
            epyc[key] = r["epyc_median_us"]
            if r["bench"] == "decode":
                rows[("get_decoded_data",) + key[1:]].append(r["get_decoded_data_median_us"])
    order = ["encode_zero_alloc", "encode", "recode_zero_alloc", "recode", "decode", "get_decoded_data"]
    for b in order:
        for key in sorted(k for k in rows if k[0] == b):
            v = rows[key]
            e = epyc.get(key)
            print(json.dumps({"bench": b, "MB": key[1] >> 20, "k": key[2], "runs": len(v),
                              "median_us": round(statistics.median(v), 2), "min_us": round(min(v), 2),
                              "max_us": round(max(v), 2), "epyc_median_us": e,
                              "median_vs_epyc": round(statistics.median(v) / e, 3) if e else None}))


if __name__ == "__main__":
    main(sys.argv[1:])
