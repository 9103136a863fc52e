#!/usr/bin/env python3
"""Regenerate tests/golden/golden.json — the golden vectors of SURVEY §8c.

Inputs are java.util.Random(seed).nextDouble() streams (the reference tests'
generator, PropertyBasedTest.java:47), produced bit-exactly by the oracle.
Outputs come from the CPU oracle (oracle/jwave_oracle.c), cross-checked bit for
bit by tests/numpy_restatement.py.  Small outputs are stored whole (as hex
doubles); large ones as SHA-256 of their little-endian bytes plus samples.
The Java reference itself cannot run in this image (no JDK), so these vectors
are pinned to it through the KATs in test_oracle.py.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle  # noqa: E402
import jwave_amd.wavelets as W  # noqa: E402


def enc(a):
    a = np.ascontiguousarray(np.asarray(a, dtype="<f8"))
    rec = {"shape": list(a.shape), "sha256": hashlib.sha256(a.tobytes()).hexdigest()}
    if a.size <= 4096:
        rec["hex"] = [float(v).hex() for v in a.ravel()]
    else:
        idx = np.linspace(0, a.size - 1, 17).astype(int)
        rec["samples"] = {str(int(i)): float(a.ravel()[i]).hex() for i in idx}
    return rec


def cases():
    out = []
    # config 1: Haar1, N=1024, forward+reverse full depth
    x = oracle.java_random_doubles(42, 1024)
    w = W.by_class("Haar1")
    y = oracle.fwt_forward(w, x, 10)
    out.append(dict(name="cfg1_haar1_fwt_1024", wavelet="Haar1", op="fwt", seed=42, n=1024,
                    level=10, forward=enc(y), roundtrip=enc(oracle.fwt_reverse(w, y, 10))))
    # Daubechies4 full depth at several sizes
    w = W.by_class("Daubechies4")
    for n in (8, 1024, 65536):
        x = oracle.java_random_doubles(42, n)
        lev = n.bit_length() - 1
        y = oracle.fwt_forward(w, x, lev)
        out.append(dict(name="d4_fwt_%d" % n, wavelet="Daubechies4", op="fwt", seed=42, n=n,
                        level=lev, forward=enc(y), roundtrip=enc(oracle.fwt_reverse(w, y, lev))))
    # Daubechies8 2-D 64x64 full levels
    w = W.by_class("Daubechies8")
    x = oracle.java_random_doubles(42, 64 * 64).reshape(64, 64)
    y = oracle.transform_2d("fwt", True, w, x, 6, 6)
    out.append(dict(name="d8_fwt2d_64x64", wavelet="Daubechies8", op="fwt2d", seed=42,
                    shape=[64, 64], levels=[6, 6], forward=enc(y),
                    roundtrip=enc(oracle.transform_2d("fwt", False, w, y, 6, 6))))
    # Symlet8 WPT 6 levels, N=4096, batch 4 (seed 42+b)
    w = W.by_class("Symlet8")
    x = np.stack([oracle.java_random_doubles(42 + b, 4096) for b in range(4)])
    y = oracle.batch("wpt", True, w, x, 6)
    out.append(dict(name="sym8_wpt_4x4096_l6", wavelet="Symlet8", op="wpt_batch", seed=42,
                    batch=4, n=4096, level=6, forward=enc(y),
                    roundtrip=enc(oracle.batch("wpt", False, w, y, 6))))
    # MODWT Daubechies4 J=8 at N=1000 (non power of two), DIRECT semantics
    w = W.by_class("Daubechies4")
    x = oracle.java_random_doubles(42, 1000)
    c = oracle.modwt_forward(w, x, 8, sparse=False)
    out.append(dict(name="d4_modwt_1000_j8", wavelet="Daubechies4", op="modwt", seed=42, n=1000,
                    level=8, forward=enc(c), roundtrip=enc(oracle.modwt_inverse(w, c, sparse=False))))
    return out


if __name__ == "__main__":
    data = {"generator": "tests/golden/make_golden.py", "cases": cases()}
    with open(os.path.join(HERE, "golden.json"), "w") as fh:
        json.dump(data, fh, indent=0)
    print("wrote %d cases" % len(data["cases"]))
