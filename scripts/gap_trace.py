#!/usr/bin/env python3
"""Kernel durations and the gaps between consecutive kernels of the last steps in a
rocprofv3 kernel trace (usage: gap_trace.py <run_kernel_trace.csv> [n])"""
import csv
import sys

tr = list(csv.DictReader(open(sys.argv[1])))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
prev = None
for r in tr[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    print(f"gap {gap:6.2f} us  dur {(e - s) / 1000:6.2f} us  {r['Kernel_Name'][:70]}")
    prev = e
