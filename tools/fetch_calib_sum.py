#!/usr/bin/env python3
"""FETCH_SIZE per dispatch of tools/fetch_calib (rocprofv3 --pmc FETCH_SIZE) against the known
128-B line counts the probe prints: the factor FETCH_SIZE x 1024 / line bytes per access shape.
usage: fetch_calib_sum.py <counter_collection.csv> <probe stdout>"""
import csv
import re
import sys
from collections import defaultdict

per, name = defaultdict(float), {}
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] == "FETCH_SIZE":
        per[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        name[int(r["Dispatch_Id"])] = r["Kernel_Name"]
known = [(m.group(1), float(m.group(2))) for m in
         (re.match(r"(\S+)\s+lines\s+\S+\s+line_bytes\s+(\S+)", l) for l in open(sys.argv[2])) if m]
disp = sorted(d for d in per if "fill" not in name[d].lower())
disp = disp[-len(known):]
print("shape        line_bytes        FETCH_SIZE*1KiB   ratio (FETCH/line bytes)")
for (k, lb), d in zip(known, disp):
    fb = per[d] * 1024.0
    print(f"{k:11s} {lb:16.0f} {fb:18.0f}   {fb / lb:.3f}    [{name[d][:40]}]")
