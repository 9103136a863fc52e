#!/usr/bin/env python3
"""Parse two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate passes as
MI355X_MICROARCH.md §rocprofv3 requires) into HBM bytes per launch per kernel.

Correction (MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7): counter
values are KB; FETCH_SIZE under-reports wide streaming reads on gfx950, and
other access widths are uncalibrated.  We therefore calibrate both counters on
the copy_axis kernel of the same run, whose bytes are known exactly (8 B per
lane loads/stores like our FWT kernels): factor = known / counted.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [calib_bytes_each_way]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

KINDS = ["fwt_fwd_tile", "fwt_fwd_res", "fwt_rev_tile", "fwt_rev_res", "wpt_fwd_tile",
         "wpt_fwd_res", "wpt_rev_tile", "wpt_rev_res", "modwt_fwd_tile", "modwt_fwd_level",
         "modwt_inv_tile", "modwt_inv_level", "fwt_rev_head", "fwt_fwd_chain", "fwt_rev_chain",
         "copy_axis_kernel"]
# tiled FWT passes: the launch over the full-length axis keeps the kind's name,
# passes over intermediate approximations (smaller grids) become "<kind>_deep"
# (the split capi.cpp's profiler uses).
DEEP_SPLIT = ("fwt_fwd_tile", "fwt_rev_tile")


def kind_of(name):
    for k in KINDS:
        if k in name:
            m = re.search(r"Lb([01])E", name)
            mode = {"0": "exact", "1": "fma"}.get(m.group(1)) if m else "exact"
            return k.replace("_kernel", ""), mode
    return None, None


def read(dirpath, counter):
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k, mode = kind_of(row.get("Kernel_Name", ""))
                if k:
                    vals[(k, mode, int(row.get("Grid_Size") or 0))].append(float(row["Counter_Value"]))
    out = defaultdict(list)
    for (k, mode, grid), vs in vals.items():
        grids = [g for (k2, m2, g) in vals if k2 == k and m2 == mode]
        if k in DEEP_SPLIT and grid < max(grids):
            k = k + "_deep"
        out[(k, mode)].extend(vs)
    return out


def main():
    fdir, wdir, out = sys.argv[1:4]
    calib = float(sys.argv[4]) if len(sys.argv) > 4 else 8.0 * (1 << 24)
    fetch = read(fdir, "FETCH_SIZE")
    write = read(wdir, "WRITE_SIZE")
    cf = [v for (k, _), vs in fetch.items() if k == "copy_axis" for v in vs]
    cw = [v for (k, _), vs in write.items() if k == "copy_axis" for v in vs]
    f_fac = calib / (1024.0 * (sum(cf) / len(cf))) if cf else 2.0
    w_fac = calib / (1024.0 * (sum(cw) / len(cw))) if cw else 1.0
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes)",
           "calibration": {"kernel": "copy_axis", "known_bytes_each_way": calib,
                           "fetch_factor": f_fac, "write_factor": w_fac,
                           "note": "bytes = counter_KB * 1024 * factor"},
           "kernels": {}}
    for key in sorted(set(fetch) | set(write)):
        k, mode = key
        fv = fetch.get(key, [])
        wv = write.get(key, [])
        fb = (sum(fv) / len(fv)) * 1024.0 * f_fac if fv else None
        wb = (sum(wv) / len(wv)) * 1024.0 * w_fac if wv else None
        res["kernels"]["%s/%s" % (k, mode)] = {
            "launches": max(len(fv), len(wv)),
            "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
            "hbm_bytes_per_launch": (fb or 0.0) + (wb or 0.0) if fb is not None and wb is not None else None,
            "raw_fetch_kb_mean": (sum(fv) / len(fv)) if fv else None,
            "raw_write_kb_mean": (sum(wv) / len(wv)) if wv else None}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
