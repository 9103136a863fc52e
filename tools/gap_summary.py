#!/usr/bin/env python3
"""Gap between each big<...> dispatch's end and the next dispatch's start."""
import collections, csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
agg = collections.defaultdict(lambda: ([], []))
for a, b in zip(rows, rows[1:]):
    if "big" not in a["Kernel_Name"]:
        continue
    k = a["Kernel_Name"].split("(")[0].replace("void ", "")
    d = (int(a["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e3
    gap = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    agg[k][0].append(d); agg[k][1].append(gap)
for k, (d, g) in agg.items():
    d.sort(); g.sort()
    print("%-28s dur med %7.2f us   gap med %6.2f us  (min %6.2f)" % (k, d[len(d) // 2], g[len(g) // 2], g[0]))
