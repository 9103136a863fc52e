#!/usr/bin/env python3
"""Per-(kernel, grid) dispatch durations from a rocprofv3 kernel-trace CSV dir."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
fs = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
rows = list(csv.DictReader(open(fs[0])))
agg = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    short = name.split("(")[0].replace("void ", "")[:90]
    grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    agg[(short, grid)].append(dur)
tot = 0.0
for (k, g), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    tot += sum(v)
    print("%-90s grid=%-8s n=%-4d med=%8.2f us  min=%8.2f  sum=%9.1f" % (k, g, len(v), v[len(v) // 2], v[0], sum(v)))
print("total %.1f us" % tot)

# timeline of the last few jwv dispatches: start offset, duration, gap to previous end
jw = sorted((r for r in rows if "jwv" in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
if jw:
    tail = jw[-int(sys.argv[2]) if len(sys.argv) > 2 else -12:]
    t0 = int(tail[0]["Start_Timestamp"])
    prev = None
    print("timeline (last %d jwv dispatches):" % len(tail))
    for r in tail:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000.0 if prev is not None else 0.0
        g = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        print("  +%9.2f us  dur %8.2f  gap %6.2f  grid=%-8s %s" % ((s - t0) / 1000.0, (e - s) / 1000.0, gap, g,
                                                                r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]))
        prev = e
