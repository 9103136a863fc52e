#!/usr/bin/env python3
"""Summarise bench JSON lines and rocprofv3 kernel stats under a gpurun_out dir."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in sorted(glob.glob(os.path.join(d, "bench_*.json"))):
    try:
        r = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:
        print(os.path.basename(f), "unreadable", e)
        continue
    rf = r["roofline"]
    print("%-26s %.4g samples/s  %.4f ms/step  %7.1f GB/s  dom=%s %.1f us %.0f GB/s (%.1f%%)  err=%.2g"
          % (os.path.basename(f), r["value"], r["ms_per_step"], r["hbm_gbps"], rf["kernel"],
             rf["avg_launch_us"], rf["achieved"], 100 * rf["frac"], r["roundtrip_max_abs_err"]))
    for k, v in r.get("kernels", r.get("kernels_profiled_pass", {})).items():
        print("    %-16s n=%-4d avg %9.2f us  %7.1f GB/s" % (k, v["launches"], v["avg_us"], v["GBps"]))
    if r.get("batched_wpt_strong"):
        print("    wpt strong:", r["batched_wpt_strong"])
    if r.get("cpu_baseline"):
        print("    cpu:", r["cpu_baseline"])
for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)):
    print("==", f)
    for row in csv.DictReader(open(f)):
        name = row["Name"]
        if "jwv" not in name:
            continue
        print("  %6s calls avg %10.1f ns min %10s max %10s  %s" % (row["Calls"], float(row["AverageNs"]),
              row["MinNs"], row["MaxNs"], name.split("(")[0][:90]))
