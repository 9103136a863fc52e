#!/usr/bin/env python3
"""Workload run under `rocprofv3 --pmc ...` to price HBM traffic per kernel.

1. calibration: a level-0 FWT of 2^24 doubles = the copy_axis kernel, whose
   bytes are known exactly (read 128 MiB + write 128 MiB, 8 B per lane — the
   access width our FWT kernels use), to calibrate FETCH_SIZE/WRITE_SIZE on
   gfx950 (MI355X_MICROARCH.md §HBM: FETCH_SIZE under-reports wide streams).
2. the bench workload: config 2 (D4, N=2^24, full depth) forward + reverse.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import jwave_amd as jw  # noqa: E402
from jwave_amd import _lib as L  # noqa: E402
from jwave_amd.transforms import _TapsHolder  # noqa: E402


def main():
    math = sys.argv[1] if len(sys.argv) > 1 else "exact"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    lib = L.lib()
    ctx = jw.Context(0, math)
    ctx.set_stream(None)
    n = 1 << 24
    w = jw.by_class("Daubechies4")
    t = _TapsHolder.of(w)
    x = torch.from_numpy(np.random.default_rng(1).random(n)).cuda()
    y = torch.empty_like(x)
    xr = torch.empty_like(x)
    p = lambda a: ctypes.c_void_p(a.data_ptr())  # noqa: E731
    torch.cuda.synchronize()
    for _ in range(reps):
        assert lib.jwv_fwt_fwd_f64_dev(p(x), p(y), n, 0, t, ctx.handle) == 0  # copy_axis
    for _ in range(reps):
        assert lib.jwv_fwt_fwd_f64_dev(p(x), p(y), n, 24, t, ctx.handle) == 0
        assert lib.jwv_fwt_rev_f64_dev(p(y), p(xr), n, 24, t, ctx.handle) == 0
    torch.cuda.synchronize()
    print("pmc driver done", float((xr - x).abs().max()))


if __name__ == "__main__":
    main()
