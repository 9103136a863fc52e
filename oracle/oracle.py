"""ctypes front-end of the CPU restatement in ``oracle/jwave_oracle.c``.

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s cpu_baseline leg as the checker / CPU baseline.  The product
path (``jwave_amd``) never imports this module.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libjwave_oracle.so")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)


class _Taps(ctypes.Structure):
    _fields_ = [("L", ctypes.c_int), ("tw", ctypes.c_int),
                ("lo", _dp), ("hi", _dp), ("lo_r", _dp), ("hi_r", _dp),
                ("reverse_scale", ctypes.c_double)]


def build(force=False):
    srcs = [os.path.join(_HERE, f) for f in ("jwave_oracle.c", "jwave_oracle_par.c", "Makefile")]
    if force or not os.path.exists(_LIB_PATH) or \
            any(os.path.getmtime(_LIB_PATH) < os.path.getmtime(s) for s in srcs):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        alt = os.environ.get("JWAVE_ORACLE_LIB")  # tools/sanitize.sh: ASan/UBSan build
        if not alt:
            build()
        _lib = ctypes.CDLL(alt or _LIB_PATH)
        i64, c_int = ctypes.c_int64, ctypes.c_int
        tp = ctypes.POINTER(_Taps)
        for name in ("orc_fwt_forward", "orc_fwt_reverse", "orc_wpt_forward", "orc_wpt_reverse"):
            getattr(_lib, name).argtypes = [tp, _dp, _dp, c_int, c_int]
        _lib.orc_batch.argtypes = [c_int, c_int, tp, _dp, _dp, c_int, c_int, i64, c_int]
        for name in ("orc_2d_forward", "orc_2d_reverse"):
            getattr(_lib, name).argtypes = [c_int, tp, _dp, _dp, c_int, c_int, c_int, c_int]
        for name in ("orc_3d_forward", "orc_3d_reverse"):
            getattr(_lib, name).argtypes = [c_int, tp, _dp, _dp] + [c_int] * 6
        _lib.orc_2d_par.argtypes = [c_int, c_int, tp, _dp, _dp] + [c_int] * 5
        _lib.orc_batch_par.argtypes = [c_int, c_int, tp, _dp, _dp, c_int, c_int, i64, c_int, c_int]
        _lib.orc_modwt_forward.argtypes = [tp, _dp, _dp, c_int, c_int, c_int]
        _lib.orc_modwt_inverse.argtypes = [tp, _dp, _dp, c_int, c_int, c_int]
        _lib.orc_modwt_filters.argtypes = [tp, _dp, _dp]
        _lib.orc_wavelet_forward.argtypes = [tp, _dp, _dp, c_int]
        _lib.orc_wavelet_reverse.argtypes = [tp, _dp, _dp, c_int]
        _lib.orc_java_random_doubles.argtypes = [i64, _dp, i64]
        _lib.orc_get_exponent.argtypes = [ctypes.c_double]
        _lib.orc_get_exponent.restype = c_int
    return _lib


def _ptr(a):
    return a.ctypes.data_as(_dp)


class OracleTaps:
    """Keeps the numpy tap arrays alive next to the ctypes struct."""

    def __init__(self, wavelet):
        self.arrs = [np.ascontiguousarray(np.asarray(v, dtype=np.float64))
                     for v in (wavelet.lo, wavelet.hi, wavelet.lo_r, wavelet.hi_r)]
        self.s = _Taps(wavelet.mother_wavelength, wavelet.transform_wavelength,
                       *[_ptr(a) for a in self.arrs], wavelet.reverse_scale)

    def ref(self):
        return ctypes.byref(self.s)


def _f64(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64))


class OracleError(Exception):
    pass


def _check(rc):
    if rc != 0:
        raise OracleError("oracle status %d" % rc)


def java_random_doubles(seed, n):
    out = np.empty(int(n), dtype=np.float64)
    lib().orc_java_random_doubles(int(seed), _ptr(out), int(n))
    return out


def fwt_forward(wavelet, x, level):
    x = _f64(x); y = np.empty_like(x); t = OracleTaps(wavelet)
    _check(lib().orc_fwt_forward(t.ref(), _ptr(x), _ptr(y), x.size, int(level)))
    return y


def fwt_reverse(wavelet, y, level):
    y = _f64(y); x = np.empty_like(y); t = OracleTaps(wavelet)
    _check(lib().orc_fwt_reverse(t.ref(), _ptr(y), _ptr(x), y.size, int(level)))
    return x


def wpt_forward(wavelet, x, level):
    x = _f64(x); y = np.empty_like(x); t = OracleTaps(wavelet)
    _check(lib().orc_wpt_forward(t.ref(), _ptr(x), _ptr(y), x.size, int(level)))
    return y


def wpt_reverse(wavelet, y, level):
    y = _f64(y); x = np.empty_like(y); t = OracleTaps(wavelet)
    _check(lib().orc_wpt_reverse(t.ref(), _ptr(y), _ptr(x), y.size, int(level)))
    return x


_KIND = {"fwt": 0, "wpt": 1}


def batch(kind, forward, wavelet, x, level):
    x = _f64(x); y = np.empty_like(x); t = OracleTaps(wavelet)
    b, n = x.shape
    _check(lib().orc_batch(_KIND[kind], int(forward), t.ref(), _ptr(x), _ptr(y), b, n, n, int(level)))
    return y


def batch_par(kind, forward, wavelet, x, level, nthreads):
    """Signal-level parallel batch (ParallelizationOpportunityTest.java:80-98)."""
    x = _f64(x); y = np.empty_like(x); t = OracleTaps(wavelet)
    b, n = x.shape
    _check(lib().orc_batch_par(_KIND[kind], int(forward), t.ref(), _ptr(x), _ptr(y), b, n, n,
                               int(level), int(nthreads)))
    return y


def transform_2d_par(kind, forward, wavelet, x, lvl_m, lvl_n, nthreads):
    """ParallelTransform 2-D (ParallelTransform.java:70-126): rows, join, columns."""
    x = _f64(x); y = np.empty_like(x); t = OracleTaps(wavelet)
    r, c = x.shape
    _check(lib().orc_2d_par(_KIND[kind], int(forward), t.ref(), _ptr(x), _ptr(y), r, c,
                            int(lvl_m), int(lvl_n), int(nthreads)))
    return y


def transform_2d(kind, forward, wavelet, x, lvl_m, lvl_n):
    x = _f64(x); y = np.empty_like(x); t = OracleTaps(wavelet)
    r, c = x.shape
    fn = lib().orc_2d_forward if forward else lib().orc_2d_reverse
    _check(fn(_KIND[kind], t.ref(), _ptr(x), _ptr(y), r, c, int(lvl_m), int(lvl_n)))
    return y


def transform_3d(kind, forward, wavelet, x, lvl_p, lvl_q, lvl_r):
    x = _f64(x); y = np.empty_like(x); t = OracleTaps(wavelet)
    p, q, r = x.shape
    fn = lib().orc_3d_forward if forward else lib().orc_3d_reverse
    _check(fn(_KIND[kind], t.ref(), _ptr(x), _ptr(y), p, q, r, int(lvl_p), int(lvl_q), int(lvl_r)))
    return y


def modwt_forward(wavelet, x, J, sparse=True):
    x = _f64(x); n = x.size
    out = np.empty((J + 1, n), dtype=np.float64); t = OracleTaps(wavelet)
    _check(lib().orc_modwt_forward(t.ref(), _ptr(x), _ptr(out), n, int(J), int(sparse)))
    return out


def modwt_inverse(wavelet, coeffs, sparse=True):
    c = _f64(coeffs); J = c.shape[0] - 1; n = c.shape[1]
    x = np.empty(n, dtype=np.float64); t = OracleTaps(wavelet)
    _check(lib().orc_modwt_inverse(t.ref(), _ptr(c), _ptr(x), n, int(J), int(sparse)))
    return x


def modwt_filters(wavelet):
    L = wavelet.mother_wavelength
    g = np.empty(L); h = np.empty(L); t = OracleTaps(wavelet)
    lib().orc_modwt_filters(t.ref(), _ptr(g), _ptr(h))
    return g, h


def compress_magnitude(x, threshold):
    """CompressorMagnitude(threshold).compress(x) -> (y, magnitude)."""
    x = _f64(x); y = np.empty_like(x)
    f = lib().orc_compress_magnitude
    f.restype = ctypes.c_double
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_double]
    mag = f(_ptr(x), _ptr(y), x.size, float(threshold))
    return y, mag
