#!/usr/bin/env python3
"""Per-kernel timings (hipEvents via the C ABI profile hook) for a matrix of
operations/sizes; for iterating on kernels.  usage: microbench.py [case ...]"""
import ctypes
import json
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import jwave_amd as jw  # noqa: E402
from jwave_amd import _lib as L  # noqa: E402
from jwave_amd.transforms import _TapsHolder  # noqa: E402

CASES = {
    # name: (op, wavelet, batch, n, level)
    "fwt_d4_2^24": ("fwt", "Daubechies4", 1, 1 << 24, 24),
    "fwt_d4_4096": ("fwt", "Daubechies4", 1, 4096, 12),
    "fwt_d4_2^18": ("fwt", "Daubechies4", 1, 1 << 18, 18),
    "fwt_d4_2^20": ("fwt", "Daubechies4", 1, 1 << 20, 20),
    "fwt_d4_2^22": ("fwt", "Daubechies4", 1, 1 << 22, 22),
    "fwt_d4_b64x65536": ("fwt", "Daubechies4", 64, 1 << 16, 16),
    "fwt_d8_rows8192": ("fwt", "Daubechies8", 8192, 8192, 13),
    "wpt_s8_b512x65536": ("wpt", "Symlet8", 512, 1 << 16, 6),
    "modwt_d4_1e7": ("modwt", "Daubechies4", 1, 10_000_000, 8),
}


def run(name, math, reps=20):
    op, wn, b, n, lev = CASES[name]
    lib = L.lib()
    ctx = jw.Context(0, math)
    ctx.set_stream(None)
    t = _TapsHolder.of(jw.by_class(wn))
    x = torch.rand(b * n, dtype=torch.float64, device="cuda")
    p = lambda a: ctypes.c_void_p(a.data_ptr())  # noqa: E731
    if op == "modwt":
        y = torch.empty((lev + 1) * n, dtype=torch.float64, device="cuda")
        fm, im = lib.jwv_modwt_fwd_f64_dev, lib.jwv_modwt_inv_f64_dev
        f = lambda xi, yo, b_, n_, ld, lv, t_, h_: fm(xi, yo, n_, lv, t_, h_)  # noqa: E731
        r = lambda yi, zo, b_, n_, ld, lv, t_, h_: im(yi, zo, n_, lv, t_, h_)  # noqa: E731
    else:
        y = torch.empty_like(x)
        f = getattr(lib, "jwv_%s_fwd_batch_f64_dev" % op)
        r = getattr(lib, "jwv_%s_rev_batch_f64_dev" % op)
    z = torch.empty_like(x)
    for _ in range(3):
        assert f(p(x), p(y), b, n, n, lev, t, ctx.handle) == 0
        assert r(p(y), p(z), b, n, n, lev, t, ctx.handle) == 0
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    for _ in range(reps):
        assert f(p(x), p(y), b, n, n, lev, t, ctx.handle) == 0
        assert r(p(y), p(z), b, n, n, lev, t, ctx.handle) == 0
    torch.cuda.synchronize()
    step_us = (time.perf_counter() - t0) / reps * 1e6
    ctx.profile(True)
    for _ in range(reps):
        assert f(p(x), p(y), b, n, n, lev, t, ctx.handle) == 0
        assert r(p(y), p(z), b, n, n, lev, t, ctx.handle) == 0
    prof = ctx.profile_read()
    ctx.profile(False)
    out = {k: round(v["total_ms"] * 1e3 / reps, 2) for k, v in prof.items()}
    out["sum_us_per_fwd+rev"] = round(sum(out.values()), 2)
    err = float((z - x).abs().max())
    print(json.dumps({"case": name, "math": math, "step_us_no_events": round(step_us, 2),
                      "us_per_call": out, "err": err}), flush=True)


if __name__ == "__main__":
    names = [a for a in sys.argv[1:] if a in CASES] or list(CASES)
    maths = [a for a in sys.argv[1:] if a in ("exact", "fma")] or ["exact"]
    for m in maths:
        for nm in names:
            run(nm, m)
