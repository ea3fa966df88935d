#!/usr/bin/env python3
"""Per-launch durations of one kernel from a rocprofv3 rocpd database (rocprofv3 --kernel-trace), each with the
time it ran beside other kernels (other streams) and which: explains a spread of durations (e.g. bench.py's
decode-side elimination, gf_rref_block_kernel, which runs on its own stream beside the next launch group's encode).
Usage: launch_overlap.py run_results.db --match gf_rref_block_kernel [--grid N] > overlap.csv"""
import argparse
import re
import sqlite3
import statistics


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("rlnc::", "")
    return re.sub(r"\(.*", "", name)[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", required=True)
    ap.add_argument("--grid", type=int, default=0, help="only launches of this grid_x (work-items)")
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute("select name, grid_x, start, end from kernels order by start").fetchall()
    ks = [(short(n), g, s, e) for n, g, s, e in rows]
    t0 = ks[0][2] if ks else 0
    print("launch,start_us,duration_us,overlapped_us,overlap_frac,beside")
    alone, shared = [], []
    for i, (n, g, s, e) in enumerate(ks):
        if a.match not in n or (a.grid and g != a.grid):
            continue
        ov, names = 0, set()
        for n2, g2, s2, e2 in ks:
            if (n2, g2, s2, e2) == (n, g, s, e) or e2 <= s or s2 >= e:
                continue
            ov += min(e, e2) - max(s, s2)
            names.add(n2)
        d = (e - s) / 1e3
        frac = min(1.0, ov / (e - s)) if e > s else 0.0
        (shared if frac > 0.5 else alone).append(d)
        print(f"{i},{(s - t0) / 1e3:.1f},{d:.2f},{ov / 1e3:.2f},{frac:.2f},\"{' | '.join(sorted(names))}\"")
    for lab, v in (("alone (overlap <= 50 %)", alone), ("beside other kernels (> 50 %)", shared)):
        if v:
            print(f"# {lab}: {len(v)} launches, median {statistics.median(v):.2f} us, min {min(v):.2f}, max {max(v):.2f}")


if __name__ == "__main__":
    main()
