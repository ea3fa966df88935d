#!/usr/bin/env python3
"""Step timeline of a rocprofv3 --kernel-trace CSV (the bench's rlnc kernels): per launch, start offset and
duration in µs from the first kernel of the last N launches; shows how steps overlap under --pipeline 2.
    python3 scripts/timeline.py gpurun_out/prof_p2/run_kernel_trace.csv [N]"""
import csv
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = [r for r in csv.DictReader(open(path)) if "rlnc" in r["Kernel_Name"] and "stream_kernel" not in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("void ", "").replace("rlnc::(anonymous namespace)::", "").split("(")[0]
        print(f"{name:45s} grid {int(r['Grid_Size_X']):8d}  start {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us")


if __name__ == "__main__":
    main()
