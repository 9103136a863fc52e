#!/usr/bin/env python3
"""Pageable host-entry A/B of two library builds with raw ctypes (no jwave_amd
import, so builds with different symbol sets load alike): config 2 (D4,
N = 2^24, full depth) forward + reverse on pageable numpy arrays, ms/step.
usage: host_entry_ab.py LIB REPS"""
import ctypes
import json
import sys
import time

import numpy as np

lib = ctypes.CDLL(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
D = ctypes.c_double


class Taps(ctypes.Structure):
    _fields_ = [("L", ctypes.c_int32), ("tw", ctypes.c_int32)] + \
               [(k, ctypes.POINTER(D)) for k in ("lo", "hi", "lo_r", "hi_r")] + [("sc", D)]


taps = json.load(open("jwave_amd/data/taps.json"))
w = taps["wavelets"]["Daubechies4"]
arr = {k: (D * len(w[k]))(*w[k]) for k in ("lo", "hi", "lo_r", "hi_r")}
t = Taps(len(w["lo"]), 2, arr["lo"], arr["hi"], arr["lo_r"], arr["hi_r"], 1.0)
ctx = ctypes.c_void_p()
assert lib.jwv_ctx_create(0, ctypes.byref(ctx)) == 0
n = 1 << 24
x = np.random.default_rng(7).random(n)
y, z = np.empty(n), np.empty(n)
dp = ctypes.POINTER(D)


def step():
    assert lib.jwv_fwt_fwd_f64(x.ctypes.data_as(dp), y.ctypes.data_as(dp), ctypes.c_int64(n), 24,
                               ctypes.byref(t), ctx) == 0
    assert lib.jwv_fwt_rev_f64(y.ctypes.data_as(dp), z.ctypes.data_as(dp), ctypes.c_int64(n), 24,
                               ctypes.byref(t), ctx) == 0


step()
t0 = time.perf_counter()
for _ in range(reps):
    step()
ms = (time.perf_counter() - t0) / reps * 1e3
print(json.dumps({"lib": sys.argv[1], "pageable_ms_per_step": round(ms, 3),
                  "max_err": float(np.abs(z - x).max())}))
