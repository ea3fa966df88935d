#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output per kernel (mean counter value per dispatch)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "?")
        short = name.split("(")[0][-60:]
        acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        short = row["Kernel_Name"].split("(")[0][-60:]
        durs[short].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
for k, cs in acc.items():
    if "rlnc" not in k and "gf_" not in k:
        continue
    print(k)
    d = durs.get(k, [])
    if d:
        print(f"   duration_ns(mean, profiled) = {sum(d)/len(d):.0f}  n={len(d)}")
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v)/len(v):.4g}   (n={len(v)})")
