#!/usr/bin/env python3
"""Parse two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate passes as
MI355X_MICROARCH.md §rocprofv3 requires) into HBM bytes per launch, per
(workload, planner kernel kind, math mode).

Attribution: the driver ran with JWV_LAUNCH_LOG=1, so the library printed one
line per launch ("JWV_LAUNCH <kind> <algorithmic bytes>") in launch order; the
jwv dispatches of each counter pass, in dispatch order, are paired with those
lines one to one (the same deterministic launch sequence).  Keys therefore
follow capi.cpp's kinds exactly (e.g. fwt_fwd_tile = every full-length tile
pass of that workload, rows and column slabs alike), never another workload's.

Correction (MI355X_MICROARCH.md §HBM): counter values are KB; FETCH_SIZE
reports half the bytes of a wide streaming read on gfx950.  Both counters are
calibrated on the copy_axis launches of the same run, whose bytes are known
exactly: factor = known / counted (expect 2.0 for FETCH, 1.0 for WRITE).

usage: pmc_traffic.py WORKLOAD MATH FETCH_DIR FETCH_LOG WRITE_DIR WRITE_LOG OUT.json
"""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

CALIB_BYTES = 8.0 * (1 << 24)  # copy_axis: 2^24 doubles each way


def launches(logfile):
    out = []
    for line in open(logfile, errors="replace"):
        if line.startswith("JWV_LAUNCH "):
            _, kind, b = line.split()[:3]
            out.append((kind, float(b)))
    return out


def dispatches(dirpath, counter):
    files = glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True)
    rows = {}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r.get("Counter_Name") != counter or "jwv::" not in r.get("Kernel_Name", ""):
                    continue
                key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                ent = rows.setdefault(key, [name, 0.0])
                ent[1] += float(r["Counter_Value"])  # summed over XCD/instance rows
    return [rows[k] for k in sorted(rows)]


def attribute(dirpath, counter, logfile):
    disp = dispatches(dirpath, counter)
    lau = launches(logfile)
    if len(disp) != len(lau):
        raise SystemExit("%s: %d jwv dispatches vs %d logged launches" % (counter, len(disp), len(lau)))
    per = defaultdict(lambda: {"kb": [], "alg": [], "inst": set()})
    for (name, kb), (kind, alg) in zip(disp, lau):
        e = per[kind]
        e["kb"].append(kb)
        e["alg"].append(alg)
        e["inst"].add(name)
    return per


def lib_record():
    """Digest of the library the counter passes loaded (JWAVE_AMD_LIB or the
    in-tree build): bench.py's build.lib_sha256 of the same file."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.environ.get("JWAVE_AMD_LIB") or os.path.join(root, "jwave_amd", "lib", "libjwave_hip.so")
    h = hashlib.sha256()
    with open(lib, "rb") as fh:
        for blk in iter(lambda: fh.read(1 << 20), b""):
            h.update(blk)
    return {"lib": os.path.relpath(lib, root), "lib_sha256": h.hexdigest()[:16]}


def main():
    workload, math, fdir, flog, wdir, wlog, out = sys.argv[1:8]
    fetch = attribute(fdir, "FETCH_SIZE", flog)
    write = attribute(wdir, "WRITE_SIZE", wlog)
    cf, cw = fetch.pop("copy_axis", None), write.pop("copy_axis", None)
    f_fac = CALIB_BYTES / (1024.0 * sum(cf["kb"]) / len(cf["kb"])) if cf else 2.0
    w_fac = CALIB_BYTES / (1024.0 * sum(cw["kb"]) / len(cw["kb"])) if cw else 1.0
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), "
                     "dispatches attributed by the library's launch log",
           "workload": workload, "math": math, "build": lib_record(),
           "calibration": {"kernel": "copy_axis", "known_bytes_each_way": CALIB_BYTES,
                           "fetch_factor": f_fac, "write_factor": w_fac,
                           "note": "bytes = counter_KB * 1024 * factor"},
           "kernels": {}}
    for kind in sorted(set(fetch) | set(write)):
        fv = fetch.get(kind, {"kb": []})["kb"]
        wv = write.get(kind, {"kb": []})["kb"]
        fb = sum(fv) / len(fv) * 1024.0 * f_fac if fv else None
        wb = sum(wv) / len(wv) * 1024.0 * w_fac if wv else None
        alg = fetch.get(kind) or write.get(kind)
        algb = sum(alg["alg"]) / len(alg["alg"])
        res["kernels"]["%s:%s/%s" % (workload, kind, math)] = {
            "launches": max(len(fv), len(wv)),
            "instances": sorted((fetch.get(kind) or write.get(kind))["inst"]),
            "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
            "hbm_bytes_per_launch": fb + wb if fb is not None and wb is not None else None,
            "algorithmic_bytes_per_launch": algb,
            "traffic_over_algorithmic": (fb + wb) / algb if fb is not None and wb is not None
            and algb else None}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
