#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of bench.py: per-kernel mean duration and the
idle gap before each kernel within a training step (steady-state steps only).
usage: python scripts/trace_summary.py gpurun_out/prof/run_kernel_trace.csv [out.md]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:60]
names = [short(r["Kernel_Name"]) for r in rows]
# steady state: the last 60% of the dispatches
start = int(len(rows) * 0.4)
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
for i in range(start, len(rows)):
    r = rows[i]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[names[i]].append((e - s) / 1e3)
    if i > 0:
        gap[names[i]].append((s - int(rows[i - 1]["End_Timestamp"])) / 1e3)
lines = ["| kernel | calls | mean us | mean gap before (us) |", "|---|---:|---:|---:|"]
tot = 0.0
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    g = gap[k]
    lines.append(f"| `{k}` | {len(v)} | {sum(v)/len(v):.1f} | {sum(g)/max(1,len(g)):.1f} |")
    tot += sum(v)
out = "\n".join(lines)
print(out)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(out + "\n")
