#!/usr/bin/env python3
"""Workload run under `rocprofv3 --pmc ...` to price HBM traffic per kernel.

usage: pmc_driver.py WORKLOAD MATH REPS     (WORKLOAD: fwt1d fwt2d wpt modwt)

1. calibration: a level-0 FWT of 2^24 doubles = the copy_axis kernel, whose
   bytes are known exactly (read 128 MiB + write 128 MiB) — MI355X_MICROARCH.md
   §HBM: FETCH_SIZE reports half the bytes of a wide streaming read on gfx950;
   the copy measures that factor in the same run.
2. REPS steps of the bench workload (bench.setup: same shapes and data).
Run with JWV_LAUNCH_LOG=1: the library prints one line per launch (its kernel
kind) in launch order; tools/pmc_traffic.py pairs them with the dispatches.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import jwave_amd as jw  # noqa: E402
import bench  # noqa: E402
from jwave_amd import _lib as L  # noqa: E402
from jwave_amd.transforms import _TapsHolder  # noqa: E402


def main():
    workload = sys.argv[1] if len(sys.argv) > 1 else "fwt1d"
    math = sys.argv[2] if len(sys.argv) > 2 else "exact"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    lib = L.lib()
    ctx = jw.Context(0, math)
    ctx.set_stream(None)
    n = 1 << 24
    t = _TapsHolder.of(jw.by_class("Daubechies4"))
    x = torch.from_numpy(np.random.default_rng(1).random(n)).cuda()
    y = torch.empty_like(x)
    p = lambda a: ctypes.c_void_p(a.data_ptr())  # noqa: E731
    torch.cuda.synchronize()
    for _ in range(reps):
        assert lib.jwv_fwt_fwd_f64_dev(p(x), p(y), n, 0, t, ctx.handle) == 0  # copy_axis
    torch.cuda.synchronize()
    del x, y
    args = bench.parse(["--workload", workload, "--math", math])
    d = bench.Dist(1, False)
    W = bench.setup(args, d)
    for _ in range(reps):
        W["step"]()
    torch.cuda.synchronize()
    print("pmc driver done", workload, math, W["check"](), flush=True)


if __name__ == "__main__":
    main()
