"""ctypes binding of libjwave_hip.so (the C ABI declared in include/jwave_hip.h).

The library is the only compute path: there is no CPU fallback.  If the
shared object is missing or fails to load, ``lib()`` raises ``JWaveError``.
"""
import ctypes
import os
import re
import threading

from .exceptions import JWaveError

HERE = os.path.dirname(os.path.abspath(__file__))
# JWAVE_AMD_LIB: an alternative build of the same library (tools/sanitize.sh
# points it at the ASan/UBSan host build); default: the in-tree build.
LIB_PATH = os.environ.get("JWAVE_AMD_LIB") or os.path.join(HERE, "lib", "libjwave_hip.so")
HEADER = os.path.join(HERE, "..", "include", "jwave_hip.h")

JWV_OK = 0
JWV_ERR_FAILURE = 1
JWV_ERR_ILLEGAL_ARGUMENT = 2
JWV_ERR_DEVICE = 3
JWV_ERR_BAD_CALL = 4
JWV_MATH_EXACT = 0
JWV_MATH_FMA = 1
JWV_PLAN_CHAIN_REV = 1
JWV_PLAN_CHAIN_FWD = 2
JWV_PLAN_REV_HEAD = 4
JWV_PLAN_FWD_TAIL = 8
JWV_TRANSFORM_FWT = 0
JWV_TRANSFORM_WPT = 1

_dp = ctypes.c_void_p  # device or host double*
_i64 = ctypes.c_int64
_int = ctypes.c_int


class Taps(ctypes.Structure):
    _fields_ = [("mother_wavelength", ctypes.c_int32),
                ("transform_wavelength", ctypes.c_int32),
                ("lo", ctypes.POINTER(ctypes.c_double)),
                ("hi", ctypes.POINTER(ctypes.c_double)),
                ("lo_r", ctypes.POINTER(ctypes.c_double)),
                ("hi_r", ctypes.POINTER(ctypes.c_double)),
                ("reverse_scale", ctypes.c_double)]


_TP = ctypes.POINTER(Taps)


class KernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_int64),
                ("total_ms", ctypes.c_double), ("bytes", ctypes.c_double)]

_CTX = ctypes.c_void_p

# name -> argtypes (restype int unless listed in _RESTYPES)
_SIGS = {
    "jwv_version": [],
    "jwv_ctx_create": [_int, ctypes.POINTER(ctypes.c_void_p)],
    "jwv_ctx_destroy": [_CTX],
    "jwv_last_error": [_CTX],
    "jwv_ctx_set_stream": [_CTX, ctypes.c_void_p],
    "jwv_ctx_reset_stream": [_CTX],
    "jwv_ctx_get_stream": [_CTX],
    "jwv_ctx_set_math": [_CTX, _int],
    "jwv_ctx_set_plan": [_CTX, _int],
    "jwv_ctx_synchronize": [_CTX],
    "jwv_ctx_set_poll_limit": [_CTX, ctypes.c_uint],
    "jwv_ctx_trim": [_CTX],
    "jwv_host_alloc": [_CTX, _i64, ctypes.POINTER(ctypes.c_void_p)],
    "jwv_host_free": [_CTX, ctypes.c_void_p],
    "jwv_ctx_stage_stats": [_CTX, ctypes.POINTER(ctypes.c_double), _int],
    "jwv_host_copy_threads": [],
    "jwv_modwt_fwd_ld_f64_dev": [_dp, _dp, _i64, _i64, _int, _TP, _CTX],
    "jwv_modwt_inv_ld_f64_dev": [_dp, _i64, _dp, _i64, _int, _TP, _CTX],
    "jwv_ctx_profile_enable": [_CTX, _int],
    "jwv_ctx_profile_select": [_CTX, ctypes.c_char_p],
    "jwv_ctx_profile_read": [_CTX, ctypes.POINTER(KernelStat), _int, ctypes.POINTER(_int)],
    "jwv_modwt_filters": [_TP, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)],
}
for _n in ("fwt_fwd", "fwt_rev", "wpt_fwd", "wpt_rev"):
    for _s in ("", "_dev"):
        _SIGS["jwv_%s_f64%s" % (_n, _s)] = [_dp, _dp, _i64, _int, _TP, _CTX]
        _SIGS["jwv_%s_batch_f64%s" % (_n, _s)] = [_dp, _dp, _i64, _i64, _i64, _int, _TP, _CTX]
for _n in ("fwt2d_fwd", "fwt2d_rev"):
    for _s in ("", "_dev"):
        _SIGS["jwv_%s_f64%s" % (_n, _s)] = [_dp, _dp, _i64, _i64, _int, _int, _TP, _CTX]
for _n in ("wpt2d_fwd", "wpt2d_rev"):
    for _s in ("", "_dev"):
        _SIGS["jwv_%s_f64%s" % (_n, _s)] = [_dp, _dp, _i64, _i64, _int, _int, _TP, _CTX]
for _n in ("fwt3d_fwd", "fwt3d_rev"):
    for _s in ("", "_dev"):
        _SIGS["jwv_%s_f64%s" % (_n, _s)] = [_dp, _dp, _i64, _i64, _i64, _int, _int, _int, _TP, _CTX]
for _s in ("", "_dev"):
    _SIGS["jwv_fwt3d_rev_pt_f64%s" % _s] = [_dp, _dp, _i64, _i64, _i64, _int, _int, _int, _TP,
                                            _CTX]
for _n in ("wpt3d_fwd", "wpt3d_rev", "wpt3d_rev_pt"):
    _SIGS["jwv_%s_f64" % _n] = [_dp, _dp, _i64, _i64, _i64, _int, _int, _int, _TP, _CTX]
for _n in ("fwt_axis_fwd", "fwt_axis_rev", "wpt_axis_fwd", "wpt_axis_rev"):
    _SIGS["jwv_%s_f64_dev" % _n] = [_dp, _dp, _i64, _i64, _i64, _int, _TP, _CTX]
for _s in ("", "_dev"):
    _SIGS["jwv_compress_magnitude_f64%s" % _s] = [_dp, _dp, _i64, ctypes.c_double,
                                                  ctypes.POINTER(ctypes.c_double), _CTX]
    _SIGS["jwv_fwt_denoise_f64%s" % _s] = [_dp, _dp, _i64, _int, ctypes.c_double, _TP, _CTX]
for _s in ("", "_dev"):
    _SIGS["jwv_aed_fwd_f64%s" % _s] = [_dp, _dp, _i64, _int, _TP, _CTX]
    _SIGS["jwv_aed_rev_f64%s" % _s] = [_dp, _dp, _i64, _int, _TP, _CTX]
    _SIGS["jwv_decompose_f64%s" % _s] = [_dp, _dp, _i64, _int, _TP, _CTX]
for _n in ("modwt_fwd", "modwt_inv"):
    for _s in ("", "_dev"):
        _SIGS["jwv_%s_f64%s" % (_n, _s)] = [_dp, _dp, _i64, _int, _TP, _CTX]
for _n in ("fwd", "rev"):
    _SIGS["jwv_fwt_rows_seg_%s_f64_dev" % _n] = [_dp, _dp, _i64, _i64, _int, _i64, _TP, _CTX]

_MCTX = ctypes.c_void_p
_SIGS.update({
    "jwv_mctx_create": [ctypes.POINTER(_int), _int, ctypes.POINTER(ctypes.c_void_p)],
    "jwv_mctx_destroy": [_MCTX],
    "jwv_mctx_last_error": [_MCTX],
    "jwv_mctx_size": [_MCTX],
    "jwv_mctx_ctx": [_MCTX, _int],
    "jwv_mctx_set_math": [_MCTX, _int],
    "jwv_batch_split": [_i64, _int, _int, ctypes.POINTER(_i64), ctypes.POINTER(_i64)],
})
for _n in ("fwt_fwd", "fwt_rev", "wpt_fwd", "wpt_rev"):
    _SIGS["jwv_m_%s_batch_f64" % _n] = [_dp, _dp, _i64, _i64, _i64, _int, _TP, _MCTX]
for _n in ("fwt2d_fwd", "fwt2d_rev", "wpt2d_fwd", "wpt2d_rev"):
    _SIGS["jwv_m_%s_f64" % _n] = [_dp, _dp, _i64, _i64, _int, _int, _TP, _MCTX]
for _n in ("modwt_fwd", "modwt_inv"):
    _SIGS["jwv_%s_batch_f64" % _n] = [_dp, _dp, _i64, _i64, _int, _TP, _CTX]
    _SIGS["jwv_m_%s_batch_f64" % _n] = [_dp, _dp, _i64, _i64, _int, _TP, _MCTX]

_RESTYPES = {"jwv_last_error": ctypes.c_char_p, "jwv_ctx_get_stream": ctypes.c_void_p,
             "jwv_mctx_last_error": ctypes.c_char_p, "jwv_mctx_ctx": ctypes.c_void_p}

_lib = None
_lock = threading.Lock()


def hip_runtimes_mapped():
    """Paths of libamdhip64 copies mapped into this process (expect exactly one)."""
    out = set()
    try:
        with open("/proc/self/maps") as fh:
            for line in fh:
                if "libamdhip64" in line:
                    out.add(line.split()[-1])
    except OSError:
        pass
    return sorted(out)


def header_symbols():
    """Function names declared in include/jwave_hip.h."""
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(jwv_[a-z0-9_]+)\s*\(", txt)))


def provenance():
    """The in-tree library's build record (lib/libjwave_hip.so.json) and
    whether it matches the sources of this tree."""
    from . import _build
    s = _build.stamp() or {}
    return {"sources_sha256": s.get("sources_sha256", "")[:16],
            "lib_sha256": s.get("lib_sha256", "")[:16], "hipcc": s.get("hipcc"),
            "built_utc": s.get("built_utc"), "matches_sources": not _build.stale()}


def lib(path=None):
    """Load libjwave_hip.so (building it first if the sources are newer)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        # One HIP runtime per process: torch bundles its own libamdhip64.so
        # (SONAME libamdhip64.so.7, the same SONAME as /opt/rocm's).  If torch
        # is loaded first, the dynamic linker binds our NEEDED entry to torch's
        # copy; loaded the other way round, two runtimes would fight over the
        # device ("No HIP GPUs are available" in torch).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if os.environ.get("JWAVE_AMD_NO_BUILD") != "1" and not os.environ.get("JWAVE_AMD_LIB"):
            try:
                from . import _build
                if _build.stale():
                    _build.build()
            except Exception as e:  # build tools missing: fall through to load
                if not os.path.exists(p):
                    raise JWaveError("libjwave_hip.so missing and build failed: %s" % e)
        if not os.path.exists(p):
            raise JWaveError("libjwave_hip.so not found at %s (run __graft_entry__.build())" % p)
        if not path and not os.environ.get("JWAVE_AMD_LIB"):
            from . import _build
            if _build.stale():
                raise JWaveError("libjwave_hip.so at %s was not built from these sources "
                                 "(provenance %s); run __graft_entry__.build()"
                                 % (p, _build.STAMP))
        try:
            L = ctypes.CDLL(p)
        except OSError as e:
            raise JWaveError("cannot load %s: %s" % (p, e))
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = L
        return _lib
