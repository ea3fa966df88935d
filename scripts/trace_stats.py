#!/usr/bin/env python3
"""Per-(kernel, grid) launch statistics from a rocprofv3 --kernel-trace CSV.  rocprofv3 --stats groups by kernel name,
and the encode (grid 2,097,152 at the bench shape) and decode (1,048,576) launches of the matmul share one name; this
splits them so the bench line's roofline.kernel_ms can be checked against the encode launches alone.
    python3 scripts/trace_stats.py gpurun_out/prof/run_kernel_trace.csv > profiles/..._by_grid.csv"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    launches = defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        launches[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "grid_threads", "calls", "avg_us", "median_us", "min_us", "max_us"])
    for (name, grid), d in sorted(launches.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, grid, len(d), round(statistics.mean(d), 2), round(statistics.median(d), 2),
                    round(min(d), 2), round(max(d), 2)])


if __name__ == "__main__":
    main()
