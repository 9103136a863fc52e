#!/usr/bin/env python3
"""Does the gfx950 FETCH_SIZE correction (x2, MI355X_MICROARCH.md §HBM:
FETCH_SIZE reports half the bytes of a wide streaming read) hold for small,
cache-resident footprints?  (VERDICT r04, config-2 fused tail: 1.79x
algorithmic with the x2 correction at a 2 MiB footprint.)

drive : run under `rocprofv3 --pmc FETCH_SIZE` (then WRITE_SIZE): for every
        footprint F (doubles), REPS times: a producer copy that writes the
        F-double source (as the tail's source is written by the launch before
        it), then the measured copy_axis of that source; then REPS config-2
        steps (fwd tile, fused tail, rev head, rev tile).
parse : pmc_footprint.py parse FETCH_DIR WRITE_DIR -> per footprint the raw
        counter bytes of the measured copy over its known bytes, and the same
        for the config-2 kernels (raw and x2-corrected fetch).
"""
import csv
import ctypes
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = [1 << 15, 1 << 18, 1 << 21, 1 << 23, 1 << 25, 1 << 26, 1 << 27]
REPS = 3


def drive():
    import numpy as np
    import torch
    import jwave_amd as jw
    from jwave_amd import _lib as L
    from jwave_amd.transforms import _TapsHolder
    lib = L.lib()
    ctx = jw.Context(0, "exact")
    ctx.set_stream(None)
    t = _TapsHolder.of(jw.by_class("Daubechies4"))
    p = lambda a: ctypes.c_void_p(a.data_ptr())  # noqa: E731
    big = torch.from_numpy(np.random.default_rng(1).random(SIZES[-1])).cuda()
    for n in SIZES:
        xs = torch.empty(n, dtype=torch.float64, device="cuda")
        ys = torch.empty_like(xs)
        for _ in range(REPS):
            assert lib.jwv_fwt_fwd_f64_dev(p(big), p(xs), n, 0, t, ctx.handle) == 0  # producer
            assert lib.jwv_fwt_fwd_f64_dev(p(xs), p(ys), n, 0, t, ctx.handle) == 0  # measured
        torch.cuda.synchronize()
        del xs, ys
    n = 1 << 24
    x = torch.from_numpy(np.random.default_rng(2).random(n)).cuda()
    y, z = torch.empty_like(x), torch.empty_like(x)
    for _ in range(REPS):
        assert lib.jwv_fwt_fwd_f64_dev(p(x), p(y), n, 24, t, ctx.handle) == 0
        assert lib.jwv_fwt_rev_f64_dev(p(y), p(z), n, 24, t, ctx.handle) == 0
    torch.cuda.synchronize()
    print("pmc footprint driver done", flush=True)


def dispatches(dirpath, counter):
    rows = {}
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter or "jwv::" not in r.get("Kernel_Name", ""):
                continue
            key = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            ent = rows.setdefault(key, [r["Kernel_Name"].split("(")[0].replace("void jwv::", ""), 0.0])
            ent[1] += float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def parse(fdir, wdir):
    out = {"note": "raw = counter KB * 1024 / known bytes of the measured copy (read F*8, write "
                   "F*8); the x2 FETCH correction assumes raw fetch = 0.5", "copy": [], "config2": {}}
    f, w = dispatches(fdir, "FETCH_SIZE"), dispatches(wdir, "WRITE_SIZE")
    assert len(f) == len(w), (len(f), len(w))
    i = 0
    for n in SIZES:
        fr, wr = [], []
        for _ in range(REPS):
            i += 1  # producer
            fr.append(f[i][1] * 1024 / (8.0 * n))
            wr.append(w[i][1] * 1024 / (8.0 * n))
            i += 1
        out["copy"].append({"doubles": n, "bytes_each_way": 8 * n,
                            "raw_fetch_over_known": round(sum(fr) / REPS, 4),
                            "raw_write_over_known": round(sum(wr) / REPS, 4)})
    acc = defaultdict(lambda: [0.0, 0.0, 0])
    for (name, fk), (_, wk) in zip(f[i:], w[i:]):
        a = acc[name.split("<")[0]]
        a[0] += fk * 1024
        a[1] += wk * 1024
        a[2] += 1
    alg = {"fwt_fwd_tile1": 16.0 * (1 << 24), "fwt_fwd_tail1": 16.0 * (1 << 18),
           "fwt_rev_head1": 16.0 * (1 << 19), "fwt_rev_tile1": 16.0 * (1 << 24)}
    for k, (fb, wb, c) in acc.items():
        fb, wb = fb / c, wb / c
        a = alg.get(k)
        out["config2"][k] = {"launches": c, "raw_fetch_bytes": fb, "write_bytes": wb,
                             "algorithmic_bytes": a,
                             "raw_over_alg": a and round((fb + wb) / a, 3),
                             "fetch_x2_over_alg": a and round((2 * fb + wb) / a, 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "parse":
        parse(sys.argv[2], sys.argv[3])
    else:
        drive()
