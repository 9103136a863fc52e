#!/usr/bin/env python3
"""Mean counter value per kernel kind over all rocprofv3 counter_collection CSVs in a dir."""
import csv, glob, os, re, sys
from collections import defaultdict
d = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        m = re.search(r"jwv::(\w+)<([^>]*)>", name) or re.search(r"(copy_axis_kernel)", name)
        if not m:
            continue
        k = m.group(1) + ("<%s>" % m.group(2)[:20] if m.lastindex and m.lastindex > 1 else "")
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in sorted(vals.items()):
    print("==", k)
    for c, v in sorted(cs.items()):
        print("   %-34s %16.4g" % (c, sum(v) / len(v)))
