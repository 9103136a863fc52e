#!/usr/bin/env python3
"""Per-kernel durations and the idle gap before each launch, from a rocprofv3
kernel trace (run_kernel_trace.csv): averaged per kernel name over the last
N steps.  usage: trace_gaps.py TRACE_CSV [names_per_step]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "jwv::" in r["Kernel_Name"]]
dur, gap = collections.defaultdict(list), collections.defaultdict(list)
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = r["Kernel_Name"].split("(")[0].replace("void jwv::", "")[:60]
    dur[k].append((e - s) / 1e3)
    if prev is not None and 0 <= s - prev < 50_000:
        gap[k].append((s - prev) / 1e3)
    prev = e
for k in dur:
    g = gap.get(k, [])
    print("%-62s dur %7.2f us  gap-before %6.2f us  (n=%d)"
          % (k, sum(dur[k]) / len(dur[k]), sum(g) / len(g) if g else 0.0, len(dur[k])))
