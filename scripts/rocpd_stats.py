#!/usr/bin/env python3
"""Per-(kernel, grid) duration statistics from a rocprofv3 rocpd database (the default output of
`rocprofv3 --kernel-trace --stats` on ROCm 7.2), as CSV: the encode and decode launches share kernel names, so the
grid size separates them.  Usage: rocpd_stats.py run_results.db [--match SUBSTR] > stats.csv"""
import argparse
import re
import sqlite3
import statistics


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*", "", name)  # drop the argument list
    return name.replace("rlnc::", "")[:120]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, grid_x, grid_y, grid_z, workgroup_x, duration from kernels").fetchall()
    groups = {}
    for name, gx, gy, gz, wx, dur in rows:
        if a.match and a.match not in name:
            continue
        groups.setdefault((short(name), gx, gy, gz, wx), []).append(dur / 1e3)  # ns -> us
    print("kernel,grid_x,grid_y,grid_z,workgroup,calls,total_us,avg_us,median_us,min_us,max_us")
    for (n, gx, gy, gz, wx), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"\"{n}\",{gx},{gy},{gz},{wx},{len(d)},{sum(d):.1f},{sum(d) / len(d):.2f},{statistics.median(d):.2f},"
              f"{min(d):.2f},{max(d):.2f}")


if __name__ == "__main__":
    main()
