"""Summarise gpurun_out/piece_ab.txt (scripts/archive/r04_piece_ab.sh) one line per row."""
import json
import sys

for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/piece_ab.txt"):
    line = line.strip()
    if line.startswith("=="):
        print(line)
        continue
    try:
        d = json.loads(line)
    except Exception:
        continue
    if "piece_trace" in d:
        print("   trace", d["piece_trace"])
    elif "median_us" in d:
        print("   %-18s k=%-4d %7.2f us  epyc %7.2f" % (d["bench"], d["k"], d["median_us"], d["epyc_median_us"]))
