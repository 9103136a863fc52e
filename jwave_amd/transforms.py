"""Host mirror of JWave's operator surface over libjwave_hip.so.

Same names, argument meaning and error behaviour as the reference classes:
  Transform (facade)            jwave/Transform.java:43-512
  BasicTransform (operator SPI) jwave/transforms/BasicTransform.java:42-699
  WaveletTransform              jwave/transforms/WaveletTransform.java:34-183
  FastWaveletTransform          jwave/transforms/FastWaveletTransform.java:39-154
  WaveletPacketTransform        jwave/transforms/WaveletPacketTransform.java:40-193
  MODWTTransform                jwave/transforms/MODWTTransform.java:104-913
Validation happens here first, with the reference's exception types and
messages (as the JNI shim does); every transform then runs on the
GPU through the C ABI.  There is no CPU compute path.

Arrays: numpy float64 arrays use the host-pointer entry points (copy in,
compute, copy out).  torch float64 CUDA tensors use the ``_dev`` entry points
on torch's current stream (no host round trip).
"""
import ctypes
import threading

import numpy as np

from . import _lib as L
from .exceptions import JWaveError, JWaveException, JWaveFailure
from .wavelets import Wavelet

MAX_DECOMPOSITION_LEVEL = 13  # MODWTTransform.java:111

_BINARY_MSG = ("given array length is not 2^p | p E N ... = 1, 2, 4, 8, 16, 32, .. "
               "please use the Ancient Egyptian Decomposition for any other array length!")


def is_binary(n):
    """MathToolKit.isBinary (tools/MathToolKit.java:185-188)."""
    n = int(n)
    return n > 0 and (n & (n - 1)) == 0


def get_exponent(n):
    """MathToolKit.getExponent for powers of two (tools/MathToolKit.java:202-206)."""
    n = int(n)
    return n.bit_length() - 1 if n > 0 else 0


# ----------------------------------------------------------------- context
class Context:
    """A jwv_ctx: one device, one stream, a math mode ("exact" | "fma")."""

    def __init__(self, device=0, math="exact"):
        self._lib = L.lib()
        h = ctypes.c_void_p()
        rc = self._lib.jwv_ctx_create(int(device), ctypes.byref(h))
        if rc != 0:
            raise JWaveError(self._lib.jwv_last_error(None).decode())
        self.handle = h
        self.device = int(device)
        self.set_math(math)

    def set_math(self, math):
        mode = {"exact": L.JWV_MATH_EXACT, "fma": L.JWV_MATH_FMA}[math]
        self._check(self._lib.jwv_ctx_set_math(self.handle, mode))
        self.math = math

    def set_plan(self, flags=None):
        """Pass plan for long single 1-D FWT signals (jwv_ctx_set_plan): a set
        of {"rev_head", "fwd_tail", "chain_rev", "chain_fwd"}, empty = the
        multi-launch plan, None = the default.  Results are bit-identical under
        every plan."""
        if flags is None:
            flags = {"rev_head", "fwd_tail"}
        bits = {"chain_rev": L.JWV_PLAN_CHAIN_REV, "chain_fwd": L.JWV_PLAN_CHAIN_FWD,
                "rev_head": L.JWV_PLAN_REV_HEAD, "fwd_tail": L.JWV_PLAN_FWD_TAIL}
        self._check(self._lib.jwv_ctx_set_plan(self.handle, sum(bits[f] for f in set(flags))))

    def set_poll_limit(self, spins=0):
        """Diagnostic: bound of each in-kernel wait (chained reverse plan) in
        polls; 0 = the default.  A tiny bound forces the timeout error path."""
        self._check(self._lib.jwv_ctx_set_poll_limit(self.handle, int(spins)))

    def set_stream(self, stream_handle):
        self._check(self._lib.jwv_ctx_set_stream(self.handle, stream_handle))

    def reset_stream(self):
        """Back to the context's own stream (ordered after the current one)."""
        self._check(self._lib.jwv_ctx_reset_stream(self.handle))

    def synchronize(self):
        self._check(self._lib.jwv_ctx_synchronize(self.handle))

    def profile(self, on=True):
        """Record hipEvents around every kernel launch (see jwv_ctx_profile_enable)."""
        self._check(self._lib.jwv_ctx_profile_enable(self.handle, 1 if on else 0))

    def profile_select(self, kind=None):
        """Restrict profiling events to one kernel kind (None = all)."""
        self._check(self._lib.jwv_ctx_profile_select(self.handle, kind.encode() if kind else None))

    def profile_read(self):
        """-> {kind: {"launches", "total_ms", "bytes"}} since the last read (synchronises)."""
        arr = (L.KernelStat * 32)()
        n = ctypes.c_int(0)
        self._check(self._lib.jwv_ctx_profile_read(self.handle, arr, 32, ctypes.byref(n)))
        return {arr[i].name.decode(): {"launches": int(arr[i].launches),
                                       "total_ms": float(arr[i].total_ms),
                                       "bytes": float(arr[i].bytes)} for i in range(n.value)}

    def trim(self):
        self._check(self._lib.jwv_ctx_trim(self.handle))

    def close(self):
        if getattr(self, "handle", None):
            self._lib.jwv_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc == 0:
            return
        msg = (self._lib.jwv_last_error(self.handle) or b"").decode()
        if rc == L.JWV_ERR_FAILURE:
            raise JWaveFailure(msg)
        if rc == L.JWV_ERR_ILLEGAL_ARGUMENT:
            raise ValueError(msg)  # IllegalArgumentException
        raise JWaveError(msg)


def _raise_for(rc, msg):
    if rc == L.JWV_ERR_FAILURE:
        raise JWaveFailure(msg)
    if rc == L.JWV_ERR_ILLEGAL_ARGUMENT:
        raise ValueError(msg)  # IllegalArgumentException
    raise JWaveError(msg)


def batch_split(batch, n_devices, i):
    """(start, count) of device i's contiguous block of a batch spread over
    n_devices (jwv_batch_split: start = floor(batch*i/n))."""
    lib = L.lib()
    s, c = ctypes.c_int64(0), ctypes.c_int64(0)
    rc = lib.jwv_batch_split(int(batch), int(n_devices), int(i), ctypes.byref(s), ctypes.byref(c))
    if rc != 0:
        _raise_for(rc, (lib.jwv_last_error(None) or b"").decode())
    return s.value, c.value


class MultiContext:
    """A jwv_mctx: one context per listed device.  Batched host arrays are
    split into contiguous blocks of signals, one per device, transformed
    concurrently (each device over its own PCIe link, no collective) and
    returned as one array -- the executor-over-signals batch of
    src/test/java/jwave/ParallelizationOpportunityTest.java:80-98 over the
    node's GPUs.  Results equal the single-device batched call."""

    def __init__(self, devices=(0,), math="exact"):
        self._lib = L.lib()
        devs = [int(d) for d in devices]
        arr = (ctypes.c_int * len(devs))(*devs)
        h = ctypes.c_void_p()
        rc = self._lib.jwv_mctx_create(arr, len(devs), ctypes.byref(h))
        if rc != 0:
            _raise_for(rc, (self._lib.jwv_mctx_last_error(None) or b"").decode())
        self.handle = h
        self.devices = devs
        mode = {"exact": L.JWV_MATH_EXACT, "fma": L.JWV_MATH_FMA}[math]
        self._check(self._lib.jwv_mctx_set_math(self.handle, mode))
        self.math = math

    def _check(self, rc):
        if rc != 0:
            _raise_for(rc, (self._lib.jwv_mctx_last_error(self.handle) or b"").decode())

    def batch(self, x, wavelet, level, forward=True, kind="fwt"):
        """Every row of the host array x (batch x n) transformed with `level`."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        if x.ndim != 2:
            raise JWaveFailure("MultiContext.batch: a 2-D array of signals is required")
        b, n = x.shape
        y = np.empty_like(x)
        name = "jwv_m_%s_%s_batch_f64" % (kind, "fwd" if forward else "rev")
        t = _TapsHolder.of(wavelet)
        self._check(getattr(self._lib, name)(x.ctypes.data, y.ctypes.data, b, n, n, int(level),
                                             t, self.handle))
        return y

    def transform_2d(self, x, wavelet, lvl_m, lvl_n, forward=True, kind="fwt"):
        """ParallelTransform.forward / reverse(double[][], lvlM, lvlN) of the host
        matrix x over the devices: row blocks, one device-to-device exchange,
        column slabs (jwv_m_fwt2d_*); the single-device entry's bits."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        if x.ndim != 2:
            raise JWaveFailure("MultiContext.transform_2d: a 2-D array is required")
        rows, cols = x.shape
        y = np.empty_like(x)
        name = "jwv_m_%s2d_%s_f64" % (kind, "fwd" if forward else "rev")
        self._check(getattr(self._lib, name)(x.ctypes.data, y.ctypes.data, rows, cols,
                                             int(lvl_m), int(lvl_n), _TapsHolder.of(wavelet),
                                             self.handle))
        return y

    def modwt_forward(self, x, wavelet, J):
        """forwardMODWT of every row of x (batch x n) -> [batch][J+1][n]."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        if x.ndim != 2:
            raise JWaveFailure("MultiContext.modwt_forward: a 2-D array of signals is required")
        b, n = x.shape
        c = np.empty((b, int(J) + 1, n))
        self._check(self._lib.jwv_m_modwt_fwd_batch_f64(x.ctypes.data, c.ctypes.data, b, n,
                                                        int(J), _TapsHolder.of(wavelet),
                                                        self.handle))
        return c

    def modwt_inverse(self, c, wavelet):
        """inverseMODWT of every [J+1][n] block of c ([batch][J+1][n])."""
        c = np.ascontiguousarray(c, dtype=np.float64)
        if c.ndim != 3:
            raise JWaveFailure("MultiContext.modwt_inverse: [batch][J+1][n] coefficients required")
        b, J1, n = c.shape
        x = np.empty((b, n))
        self._check(self._lib.jwv_m_modwt_inv_batch_f64(c.ctypes.data, x.ctypes.data, b, n,
                                                        J1 - 1, _TapsHolder.of(wavelet),
                                                        self.handle))
        return x

    def close(self):
        if getattr(self, "handle", None):
            self._lib.jwv_mctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_tls = threading.local()


def default_context(device=0):
    ctxs = getattr(_tls, "ctxs", None)
    if ctxs is None:
        ctxs = _tls.ctxs = {}
    if device not in ctxs:
        ctxs[device] = Context(device)
    return ctxs[device]


class _TapsHolder:
    """Keeps numpy tap arrays alive next to the jwv_taps struct."""
    _cache = {}

    def __init__(self, w):
        dp = ctypes.POINTER(ctypes.c_double)
        self.arrs = [np.ascontiguousarray(np.asarray(v, dtype=np.float64))
                     for v in (w.lo, w.hi, w.lo_r, w.hi_r)]
        self.s = L.Taps(w.mother_wavelength, w.transform_wavelength,
                        *[a.ctypes.data_as(dp) for a in self.arrs], w.reverse_scale)

    @classmethod
    def of(cls, w):
        key = id(w)
        ent = cls._cache.get(key)
        if ent is None or ent[0] is not w:
            ent = (w, cls(w))
            cls._cache[key] = ent
        return ctypes.byref(ent[1].s)


def _is_torch(x):
    return type(x).__module__.startswith("torch")


def _is_complex(x):
    if _is_torch(x):
        return x.is_complex()
    return np.iscomplexobj(x)


def _prep(x, ctx):
    """-> (ptr, keepalive, is_device, like) for an input array."""
    if _is_torch(x):
        import torch
        if not x.is_cuda:
            x = x.detach().numpy()
        else:
            if x.dtype != torch.float64:
                raise JWaveFailure("device arrays must be float64")
            x = x.contiguous()
            ctx.set_stream(torch.cuda.current_stream(x.device).cuda_stream)
            return ctypes.c_void_p(x.data_ptr()), x, True
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    return ctypes.c_void_p(a.ctypes.data), a, False


def _empty(like, shape, dev):
    if dev:
        import torch
        return torch.empty(shape, dtype=torch.float64, device=like.device)
    return np.empty(shape, dtype=np.float64)


def _ptr(out, dev):
    return ctypes.c_void_p(out.data_ptr() if dev else out.ctypes.data)


# --------------------------------------------------------- functional layer
def _ctx_for(ctx, x):
    """The caller's context, else this thread's default context on x's device
    (a cuda:N tensor runs on device N; host arrays on device 0)."""
    if ctx is not None:
        return ctx
    if _is_torch(x) and x.is_cuda:
        return default_context(x.device.index or 0)
    return default_context()


def _run(fn_host, fn_dev, ctx, x, out_shape, args):
    ctx = _ctx_for(ctx, x)
    px, keep, dev = _prep(x, ctx)
    out = _empty(keep, out_shape, dev)
    lib = L.lib()
    fn = getattr(lib, fn_dev if dev else fn_host)
    ctx._check(fn(px, _ptr(out, dev), *args, ctx.handle))
    return out


def fwt_forward(x, wavelet, level, ctx=None, kind="fwt"):
    """Forward FWT/WPT of one signal (1-D) or a batch of signals (2-D array, one per row)."""
    shape = tuple(x.shape)
    t = _TapsHolder.of(wavelet)
    if len(shape) == 1:
        return _run("jwv_%s_fwd_f64" % kind, "jwv_%s_fwd_f64_dev" % kind, ctx, x, shape,
                    (shape[0], int(level), t))
    b, n = shape
    return _run("jwv_%s_fwd_batch_f64" % kind, "jwv_%s_fwd_batch_f64_dev" % kind, ctx, x, shape,
                (b, n, n, int(level), t))


def fwt_reverse(y, wavelet, level, ctx=None, kind="fwt"):
    shape = tuple(y.shape)
    t = _TapsHolder.of(wavelet)
    if len(shape) == 1:
        return _run("jwv_%s_rev_f64" % kind, "jwv_%s_rev_f64_dev" % kind, ctx, y, shape,
                    (shape[0], int(level), t))
    b, n = shape
    return _run("jwv_%s_rev_batch_f64" % kind, "jwv_%s_rev_batch_f64_dev" % kind, ctx, y, shape,
                (b, n, n, int(level), t))


def wpt_forward(x, wavelet, level, ctx=None):
    return fwt_forward(x, wavelet, level, ctx, kind="wpt")


def wpt_reverse(y, wavelet, level, ctx=None):
    return fwt_reverse(y, wavelet, level, ctx, kind="wpt")


def transform_2d(x, wavelet, lvl_m, lvl_n, forward=True, ctx=None, kind="fwt"):
    r, c = x.shape
    d = "fwd" if forward else "rev"
    return _run("jwv_%s2d_%s_f64" % (kind, d), "jwv_%s2d_%s_f64_dev" % (kind, d), ctx, x,
                (r, c), (r, c, int(lvl_m), int(lvl_n), _TapsHolder.of(wavelet)))


def transform_3d(x, wavelet, lvl_p, lvl_q, lvl_r, forward=True, ctx=None, kind="fwt",
                 pt_order=False):
    """3-D transform (BasicTransform.java:509-659).  pt_order: the reverse in
    ParallelTransform's order, P axis first (jwv_*3d_rev_pt_f64)."""
    p, q, r = x.shape
    d = "fwd" if forward else ("rev_pt" if pt_order else "rev")
    dev_name = "jwv_%s3d_%s_f64_dev" % (kind, d) if kind == "fwt" else None
    if _is_torch(x) and getattr(x, "is_cuda", False) and dev_name is None:
        raise JWaveError("device 3-D packet transform is not exported")
    return _run("jwv_%s3d_%s_f64" % (kind, d), dev_name, ctx, x, (p, q, r),
                (p, q, r, int(lvl_p), int(lvl_q), int(lvl_r), _TapsHolder.of(wavelet)))


def transform_axis(x, wavelet, level, axis_len_dim=1, forward=True, ctx=None, kind="fwt"):
    """FWT/WPT of every line along one dimension of a contiguous device array
    (the per-dimension pass of BasicTransform.java:369-395).  x: float64 CUDA
    tensor; the transformed dimension is `axis_len_dim`, everything before it
    is `outer`, everything after it is `inner`."""
    if not (_is_torch(x) and x.is_cuda):
        raise JWaveError("transform_axis takes a float64 device tensor")
    shape = tuple(x.shape)
    outer = int(np.prod(shape[:axis_len_dim], dtype=np.int64))
    ln = int(shape[axis_len_dim])
    inner = int(np.prod(shape[axis_len_dim + 1:], dtype=np.int64))
    d = "fwd" if forward else "rev"
    return _run(None, "jwv_%s_axis_%s_f64_dev" % (kind, d), ctx, x, shape,
                (outer, ln, inner, int(level), _TapsHolder.of(wavelet)))


def fwt_rows_to_chunks(x, wavelet, level, seg, ctx=None):
    """Forward FWT of every row of the device matrix x [rows][cols], result in
    the sharded 2-D transform's all-to-all layout [cols/seg][rows][seg]
    (chunk j = columns [j seg, (j+1) seg)); jwv_fwt_rows_seg_fwd_f64_dev.
    Values are those of fwt_forward(x) (BasicTransform.java:369-378)."""
    if not (_is_torch(x) and x.is_cuda and x.dim() == 2):
        raise JWaveError("fwt_rows_to_chunks takes a [rows][cols] float64 device tensor")
    rows, cols = (int(v) for v in x.shape)
    seg = int(seg)
    if seg < 2 or (seg & (seg - 1)) or cols % seg:
        raise JWaveError("fwt_rows_to_chunks: seg must be a power of two >= 2 dividing cols "
                         "(%d, %d)" % (seg, cols))
    return _run(None, "jwv_fwt_rows_seg_fwd_f64_dev", ctx, x, (cols // seg, rows, seg),
                (rows, cols, int(level), seg, _TapsHolder.of(wavelet)))


def fwt_chunks_to_rows(y, wavelet, level, ctx=None):
    """Reverse of fwt_rows_to_chunks: y [cols/seg][rows][seg] (chunked
    coefficient rows) -> [rows][cols]; jwv_fwt_rows_seg_rev_f64_dev.  Values
    are those of fwt_reverse on the plain rows (BasicTransform.java:461-470)."""
    if not (_is_torch(y) and y.is_cuda and y.dim() == 3):
        raise JWaveError("fwt_chunks_to_rows takes a [chunks][rows][seg] float64 device tensor")
    nch, rows, seg = (int(v) for v in y.shape)
    return _run(None, "jwv_fwt_rows_seg_rev_f64_dev", ctx, y, (rows, nch * seg),
                (rows, nch * seg, int(level), seg, _TapsHolder.of(wavelet)))


def modwt_forward(x, wavelet, J, ctx=None):
    if not _is_torch(x):
        x = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    n = x.shape[0]
    return _run("jwv_modwt_fwd_f64", "jwv_modwt_fwd_f64_dev", ctx, x, (int(J) + 1, n),
                (n, int(J), _TapsHolder.of(wavelet)))


def modwt_inverse(coeffs, wavelet, ctx=None):
    J = coeffs.shape[0] - 1
    n = coeffs.shape[1]
    return _run("jwv_modwt_inv_f64", "jwv_modwt_inv_f64_dev", ctx, coeffs, (n,),
                (n, int(J), _TapsHolder.of(wavelet)))


def _check_ld(name, c, x):
    """The _ld entries address c by raw pointer and row stride (in doubles) and
    x as n contiguous doubles: both must be float64 tensors on one device, x
    contiguous, c with unit column stride."""
    import torch
    if not (_is_torch(x) and x.is_cuda and _is_torch(c) and c.is_cuda):
        raise JWaveError("%s takes float64 device tensors" % name)
    if c.dtype != torch.float64 or x.dtype != torch.float64:
        raise JWaveError("%s takes float64 device tensors (got %s, %s)" % (name, c.dtype, x.dtype))
    if c.device != x.device:
        raise JWaveError("%s: c and x on different devices (%s, %s)" % (name, c.device, x.device))
    if not x.is_contiguous():
        raise JWaveError("%s: x must be contiguous" % name)
    if c.dim() != 2 or c.stride(1) != 1:
        raise JWaveError("%s: c must be a 2-D matrix with unit column stride" % name)


def modwt_forward_ld(x, c, n, J, wavelet, ctx=None):
    """forwardMODWT of the device signal x[:n] into the rows of the device
    matrix c (row stride c.stride(0) >= n), columns [0, n)
    (jwv_modwt_fwd_ld_f64_dev)."""
    _check_ld("modwt_forward_ld", c, x)
    if c.shape[0] != J + 1 or c.shape[1] < n or x.numel() < n:
        raise JWaveError("modwt_forward_ld: c must be [J+1][>= n] with unit column stride")
    ctx = _ctx_for(ctx, x)
    ctx.set_stream(__import__("torch").cuda.current_stream(x.device).cuda_stream)
    ctx._check(L.lib().jwv_modwt_fwd_ld_f64_dev(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(c.data_ptr()), c.stride(0),
                                                int(n), int(J), _TapsHolder.of(wavelet),
                                                ctx.handle))


def modwt_inverse_ld(c, col0, n, x, wavelet, ctx=None):
    """inverseMODWT of the columns [col0, col0 + n) of the device matrix c
    ([J+1] rows at stride c.stride(0)) into the device vector x[:n]
    (jwv_modwt_inv_ld_f64_dev)."""
    _check_ld("modwt_inverse_ld", c, x)
    if col0 < 0 or col0 + n > c.shape[1] or x.numel() < n:
        raise JWaveError("modwt_inverse_ld: columns out of range")
    ctx = _ctx_for(ctx, x)
    ctx.set_stream(__import__("torch").cuda.current_stream(x.device).cuda_stream)
    J = c.shape[0] - 1
    ctx._check(L.lib().jwv_modwt_inv_ld_f64_dev(ctypes.c_void_p(c.data_ptr() + 8 * col0),
                                                c.stride(0), ctypes.c_void_p(x.data_ptr()),
                                                int(n), int(J), _TapsHolder.of(wavelet),
                                                ctx.handle))


def _transform_id(kind):
    return {"fwt": L.JWV_TRANSFORM_FWT, "wpt": L.JWV_TRANSFORM_WPT}[kind]


def aed_transform(x, wavelet, kind, forward, ctx=None):
    """AncientEgyptianDecomposition(FWT | WPT).forward / reverse of an array
    of any length >= 1 (jwv_aed_*: AncientEgyptianDecomposition.java:97-184)."""
    if not _is_torch(x):
        x = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    n = int(x.shape[0])
    d = "fwd" if forward else "rev"
    return _run("jwv_aed_%s_f64" % d, "jwv_aed_%s_f64_dev" % d, ctx, x, (n,),
                (n, _transform_id(kind), _TapsHolder.of(wavelet)))


def decompose(x, wavelet, kind="fwt", ctx=None):
    """WaveletTransform.decompose (WaveletTransform.java:136-145): a
    (log2 n + 1) x n matrix, row p = forward(x, p); one native call."""
    if not _is_torch(x):
        x = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    n = int(x.shape[0])
    rows = (n.bit_length() if n > 0 else 1)  # log2 n + 1 for powers of two
    return _run("jwv_decompose_f64", "jwv_decompose_f64_dev", ctx, x, (rows, n),
                (n, _transform_id(kind), _TapsHolder.of(wavelet)))


def compress_magnitude(x, threshold=1.0, ctx=None):
    """CompressorMagnitude(threshold).compress(x) on the GPU -> (y, magnitude)
    (compressions/CompressorMagnitude.java:73-84).  The kept/zeroed decisions
    equal Java's for every input; the magnitude is a tree sum (last bits may
    differ from Java's) unless a coefficient lies within its n*eps band of the
    cut, in which case it is Java's left-to-right sum (launch_compress.hip)."""
    ctx = _ctx_for(ctx, x)
    n = int(x.shape[0])
    mag = ctypes.c_double(0.0)
    y = _run("jwv_compress_magnitude_f64", "jwv_compress_magnitude_f64_dev", ctx, x, (n,),
             (n, float(threshold), ctypes.byref(mag)))
    return y, mag.value


def fwt_denoise(x, wavelet, level, threshold=1.0, ctx=None):
    """forward(level) -> CompressorMagnitude(threshold) -> reverse(level), on
    the device (the Transform + Compressor denoising sequence)."""
    n = int(x.shape[0])
    return _run("jwv_fwt_denoise_f64", "jwv_fwt_denoise_f64_dev", ctx, x, (n,),
                (n, int(level), float(threshold), _TapsHolder.of(wavelet)))


class CompressorMagnitude:
    """jwave.compressions.CompressorMagnitude (CompressorMagnitude.java:35-136),
    1-D on the GPU."""

    def __init__(self, threshold=1.0, ctx=None):
        if threshold <= 0.0:  # Compressor.java:66-80: reported, default used
            threshold = 1.0
        self._threshold = float(threshold)
        self._magnitude = 0.0
        self._ctx = ctx

    def compress(self, arr):
        y, self._magnitude = compress_magnitude(arr, self._threshold, self._ctx)
        return y

    @staticmethod
    def calcCompressionRate(arr):  # noqa: N802 — Compressor.java:152-166
        a = np.asarray(arr.cpu() if _is_torch(arr) else arr)
        zeros = int(np.count_nonzero(a == 0.0))
        return zeros / a.shape[0] * 100.0 if zeros else 0.0


def modwt_filters(wavelet):
    g = np.empty(wavelet.mother_wavelength)
    h = np.empty(wavelet.mother_wavelength)
    dp = ctypes.POINTER(ctypes.c_double)
    rc = L.lib().jwv_modwt_filters(_TapsHolder.of(wavelet), g.ctypes.data_as(dp),
                                   h.ctypes.data_as(dp))
    if rc:
        raise JWaveError(L.lib().jwv_last_error(None).decode())
    return g, h


# ------------------------------------------------------ operator-class mirror
class BasicTransform:
    """jwave.transforms.BasicTransform (BasicTransform.java:42): 1-D/2-D/3-D
    forward/reverse overloads dispatch on the array rank."""

    kind = None  # "fwt" | "wpt"

    def __init__(self, wavelet=None, ctx=None):
        self._wavelet = wavelet
        self._ctx = ctx
        self._name = None

    def getName(self):  # noqa: N802
        return self._name

    def getWavelet(self):  # noqa: N802
        if self._wavelet is None:
            raise JWaveFailure("BasicTransform#getWavelet - not available")
        return self._wavelet

    # -- overload dispatch --------------------------------------------------
    def forward(self, a, *levels):
        if _is_complex(a):
            return self._complex(a, True)
        nd = len(np.shape(a)) if not _is_torch(a) else a.dim()
        if nd == 1:
            return self.forward_1d(a, *levels)
        if nd == 2:
            return self.forward_2d(a, *levels)
        if nd == 3:
            return self.forward_3d(a, *levels)
        raise JWaveFailure("unsupported array rank %d" % nd)

    def reverse(self, a, *levels):
        if _is_complex(a):
            return self._complex(a, False)
        nd = len(np.shape(a)) if not _is_torch(a) else a.dim()
        if nd == 1:
            return self.reverse_1d(a, *levels)
        if nd == 2:
            return self.reverse_2d(a, *levels)
        if nd == 3:
            return self.reverse_3d(a, *levels)
        raise JWaveFailure("unsupported array rank %d" % nd)

    # -- Complex[]: BasicTransform.java:257-322 -----------------------------
    def _complex(self, a, fwd):
        """forward/reverse(Complex[]): real and imaginary parts interleaved
        {r0, i0, r1, i1, ..} into one real array of 2n, transformed at full
        depth (the single-argument forward/reverse), then split again."""
        if _is_torch(a):
            import torch
            bulk = torch.view_as_real(a.contiguous()).reshape(-1).to(torch.float64).contiguous()
            out = self.forward_1d(bulk) if fwd else self.reverse_1d(bulk)
            return torch.view_as_complex(out.reshape(-1, 2).contiguous())
        z = np.asarray(a, dtype=np.complex128)
        bulk = np.empty(2 * z.shape[0])
        bulk[0::2], bulk[1::2] = z.real, z.imag
        out = np.asarray(self.forward_1d(bulk) if fwd else self.reverse_1d(bulk))
        return out[0::2] + 1j * out[1::2]

    # -- 2-D: BasicTransform.java:336-474 ----------------------------------
    def forward_2d(self, m, lvl_m=None, lvl_n=None):
        r, c = m.shape
        if lvl_m is None:
            lvl_m, lvl_n = get_exponent(r), get_exponent(c)
        self._check_1d(c, lvl_n, True)
        self._check_1d(r, lvl_m, True)
        return transform_2d(m, self._wavelet, lvl_m, lvl_n, True, self._ctx, self.kind)

    def reverse_2d(self, m, lvl_m=None, lvl_n=None):
        r, c = m.shape
        if lvl_m is None:
            lvl_m, lvl_n = get_exponent(r), get_exponent(c)
        self._check_1d(r, lvl_m, False)
        self._check_1d(c, lvl_n, False)
        return transform_2d(m, self._wavelet, lvl_m, lvl_n, False, self._ctx, self.kind)

    # -- 3-D: BasicTransform.java:487-659 ----------------------------------
    def forward_3d(self, s, lvl_p=None, lvl_q=None, lvl_r=None):
        p, q, r = s.shape
        if lvl_p is None:
            lvl_p, lvl_q, lvl_r = get_exponent(p), get_exponent(q), get_exponent(r)
        self._check_1d(r, lvl_q, True)
        self._check_1d(q, lvl_p, True)
        self._check_1d(p, lvl_r, True)
        return transform_3d(s, self._wavelet, lvl_p, lvl_q, lvl_r, True, self._ctx, self.kind)

    def reverse_3d(self, s, lvl_p=None, lvl_q=None, lvl_r=None):
        p, q, r = s.shape
        if lvl_p is None:
            lvl_p, lvl_q, lvl_r = get_exponent(p), get_exponent(q), get_exponent(r)
        self._check_1d(q, lvl_p, False)
        self._check_1d(r, lvl_q, False)
        self._check_1d(p, lvl_r, False)
        return transform_3d(s, self._wavelet, lvl_p, lvl_q, lvl_r, False, self._ctx, self.kind)

    def _check_1d(self, n, level, fwd):
        raise NotImplementedError


class WaveletTransform(BasicTransform):
    """jwave.transforms.WaveletTransform (WaveletTransform.java:34-183)."""

    _who = "WaveletTransform"

    def forward_1d(self, arr, level=None):
        n = arr.shape[0]
        if level is None:  # WaveletTransform.forward(double[]) :77-88
            if not is_binary(n):
                raise JWaveFailure("WaveletTransform#forward - " + _BINARY_MSG)
            level = get_exponent(n)
        self._check_1d(n, level, True)
        return fwt_forward(arr, self._wavelet, level, self._ctx, self.kind)

    def reverse_1d(self, arr, level=None):
        n = arr.shape[0]
        if level is None:  # :101-112
            if not is_binary(n):
                raise JWaveFailure("WaveletTransform#reverse - " + _BINARY_MSG)
            level = get_exponent(n)
        self._check_1d(n, level, False)
        return fwt_reverse(arr, self._wavelet, level, self._ctx, self.kind)

    def forward_batch(self, signals, level=None, mctx=None):
        """Batched 1-D forward: one row per independent signal (one native
        call; with a MultiContext, host rows split over its devices)."""
        n = signals.shape[1]
        level = get_exponent(n) if level is None else level
        self._check_1d(n, level, True)
        if mctx is not None:
            return mctx.batch(signals, self._wavelet, level, True, self.kind)
        return fwt_forward(signals, self._wavelet, level, self._ctx, self.kind)

    def reverse_batch(self, coeffs, level=None, mctx=None):
        n = coeffs.shape[1]
        level = get_exponent(n) if level is None else level
        self._check_1d(n, level, False)
        if mctx is not None:
            return mctx.batch(coeffs, self._wavelet, level, False, self.kind)
        return fwt_reverse(coeffs, self._wavelet, level, self._ctx, self.kind)

    # WaveletTransform.decompose / recompose (:136-182)
    def decompose(self, arr):
        """All levels at once: row p = forward(arr, p), p = 0..log2 n, one
        native call (jwv_decompose_f64).  Transforms without a native
        decompose (MODWT) run the reference loop itself, row p = the first n
        values of forward(arr, p) (:136-145); for MODWT that raises at p = 0
        exactly as the reference does (forwardMODWT rejects level 0,
        MODWTTransform.java:257-260)."""
        if self.kind in ("fwt", "wpt"):
            return decompose(arr, self._wavelet, self.kind, self._ctx)
        a = np.asarray(arr, dtype=np.float64)
        n = len(a)
        if not is_binary(n):
            raise JWaveFailure("BasicTransform#calcExponent - given number is not binary: "
                               "2^p | pEN .. = 1, 2, 4, 8, 16, 32, .. ")
        return np.stack([np.asarray(self.forward_1d(a, p))[:n] for p in range(get_exponent(n) + 1)])

    def recompose(self, mat, level=None):
        if level is None:
            level = len(mat) - 1
        if level < 0 or level >= len(mat):
            raise JWaveFailure("WaveletTransform#recompose - given level is out of range")
        return self.reverse_1d(np.asarray(mat[level]), level)


class FastWaveletTransform(WaveletTransform):
    """FastWaveletTransform.java:39-154 — Mallat pyramid on the GPU."""

    kind = "fwt"

    def __init__(self, wavelet, ctx=None):
        super().__init__(wavelet, ctx)
        self._name = "Fast Wavelet Transform"

    def _check_1d(self, n, level, fwd):
        who = "FastWaveletTransform#%s - " % ("forward" if fwd else "reverse")
        if not is_binary(n):  # :74-78 / :122-126
            raise JWaveFailure(who + _BINARY_MSG)
        if level < 0 or level > get_exponent(n):  # :80-83 / :128-131
            raise JWaveFailure(who + "given level is out of range for given array")


class InPlaceFastWaveletTransform(FastWaveletTransform):
    """InPlaceFastWaveletTransform.java:33-121: forwardInPlace / reverseInPlace
    overwrite the caller's array (numpy array or torch tensor) with the result
    and return that same object.  Each is one native call; the array is
    written only after the call succeeded, so a failing call leaves it as it
    was (the reference copies back after super.forward returned).  forward /
    reverse stay out of place (:106-121)."""

    @staticmethod
    def _store(arr, out):
        if _is_torch(arr):
            arr.copy_(out)
        else:
            arr[...] = out
        return arr

    def forwardInPlace(self, arrTime, level=None):  # noqa: N802,N803 (reference names)
        # forwardInPlace(a) = super.forward(a): WaveletTransform.forward(double[])
        # (:77-88) checks the length with its own message, then maximal level
        return self._store(arrTime, self.forward_1d(arrTime, level))

    def reverseInPlace(self, arrHilb, level=None):  # noqa: N802,N803
        return self._store(arrHilb, self.reverse_1d(arrHilb, level))


class WaveletPacketTransform(WaveletTransform):
    """WaveletPacketTransform.java:40-193 — full packet tree on the GPU."""

    kind = "wpt"

    def __init__(self, wavelet, ctx=None):
        super().__init__(wavelet, ctx)
        self._name = "Wavelet Packet Transform"

    def _check_1d(self, n, level, fwd):
        if not is_binary(n):  # :76-79
            raise JWaveFailure(_BINARY_MSG)
        if level < 0 or level > get_exponent(n):  # :81-84
            raise JWaveFailure("WaveletPacketTransform#%s - given level is out of range for given"
                               " array" % ("forward" if fwd else "reverse"))


class PooledWaveletPacketTransform(WaveletPacketTransform):
    """PooledWaveletPacketTransform.java:24-127: same math; forward rejects level 0 (:29)."""

    def _check_1d(self, n, level, fwd):
        if fwd:
            if not is_binary(n):
                raise JWaveFailure("PooledWaveletPacketTransform#forward - array length is not 2^p")
            if level <= 0 or level > get_exponent(n):
                raise JWaveFailure("PooledWaveletPacketTransform#forward - invalid level")
            return
        super()._check_1d(n, level, fwd)


class ParallelWaveletPacketTransform(WaveletPacketTransform):
    """ParallelWaveletPacketTransform.java: same math as the sequential WPT."""


def _check_modwt_levels(n, J):
    """MODWTTransform.forwardMODWT's checks, in the reference's order
    (MODWTTransform.java:257-282); n = 0 skips the theoretical-limit check
    (empty input returns J+1 empty rows)."""
    if J < 1:
        raise ValueError("MODWTTransform#forwardMODWT - decomposition level must be at least 1,"
                         " requested: %d" % J)
    if J > MAX_DECOMPOSITION_LEVEL:
        raise ValueError("MODWTTransform#forwardMODWT - maximum supported decomposition level"
                         " is %d, requested: %d" % (MAX_DECOMPOSITION_LEVEL, J))
    if n > 0:
        theo = int(n).bit_length() - 1
        if J > theo:
            raise ValueError("Decomposition level %d exceeds theoretical limit %d for signal length"
                             " %d" % (J, theo, n))


def _zeros_like_input(a, n):
    if _is_torch(a):
        import torch
        return torch.zeros(n, dtype=torch.float64, device=a.device)
    return np.zeros(n)


class MODWTTransform(WaveletTransform):
    """MODWTTransform.java:104-913 (DIRECT convolution semantics)."""

    kind = None

    def __init__(self, wavelet, ctx=None):
        super().__init__(wavelet, ctx)
        self._name = "MODWT"

    @staticmethod
    def getMaxDecompositionLevel():  # noqa: N802
        return MAX_DECOMPOSITION_LEVEL

    def forwardMODWT(self, data, maxLevel):  # noqa: N802,N803 — :256-306
        if data is None or len(data) == 0:
            _check_modwt_levels(0, maxLevel)
            return np.zeros((maxLevel + 1, 0))
        _check_modwt_levels(len(data), maxLevel)
        return modwt_forward(data, self._wavelet, maxLevel, self._ctx)

    def inverseMODWT(self, coefficients):  # noqa: N802 — :337-375
        if coefficients is None or len(coefficients) <= 1:
            return np.zeros(0)
        if _is_torch(coefficients):
            return modwt_inverse(coefficients, self._wavelet, self._ctx)
        c = np.ascontiguousarray(np.asarray(coefficients, dtype=np.float64))
        return modwt_inverse(c, self._wavelet, self._ctx)

    # flattened pow-2 API: forward/reverse(double[], int) :389-443 and the
    # single-argument forward/reverse(double[]) :854-912
    def forward_1d(self, arr, level=None):
        n = len(arr)
        if n == 0:
            return _zeros_like_input(arr, 0)
        if level is None:  # :854-870: calcExponent, then forwardMODWT at full depth
            if not is_binary(n):
                raise JWaveFailure("BasicTransform#calcExponent - given number is not binary: "
                                   "2^p | pEN .. = 1, 2, 4, 8, 16, 32, .. ")
            level = get_exponent(n)
        else:  # :389-404
            if not is_binary(n):
                raise JWaveFailure("MODWTTransform#forward - given array length is not 2^p | p E N"
                                   " ... = 1, 2, 4, 8, 16, 32, .. ")
            if level < 0 or level > get_exponent(n):
                raise JWaveFailure("MODWTTransform#forward - given level is out of range for given"
                                   " array")
            if level > MAX_DECOMPOSITION_LEVEL:
                raise JWaveFailure("MODWTTransform#forward - maximum supported decomposition level"
                                   " is %d, requested: %d" % (MAX_DECOMPOSITION_LEVEL, level))
        # [W_1 .. W_J, V_J] rows of N, flattened (:406-416)
        return self.forwardMODWT(arr, level).reshape(-1)

    def reverse_1d(self, arr, level=None):
        total = len(arr)
        if total == 0:
            return _zeros_like_input(arr, 0)
        if level is None:
            # :880-902: the first N (ascending) with N | total, N = 2^p and
            # total/N - 1 <= p; ambiguous by design (N=16,J=1 reads as N=8,J=3,
            # SURVEY Appendix A.6) — reproduced, not "fixed".  Only powers of
            # two can pass isBinary, so they are the only candidates tried.
            n = levels = 0
            p = 0
            while (1 << p) <= total:
                t = 1 << p
                if total % t == 0 and 0 <= total // t - 1 <= p:
                    n, levels = t, total // t - 1
                    break
                p += 1
            if n == 0:
                raise JWaveFailure("MODWTTransform#reverse - Invalid flattened coefficient array "
                                   "length. Cannot determine original signal dimensions.")
            level = levels
        else:  # :419-443
            n = total // (level + 1)
            if not is_binary(n):
                raise JWaveFailure("MODWTTransform#reverse - Invalid coefficient array for given "
                                   "level")
            if total != n * (level + 1):
                raise JWaveFailure("MODWTTransform#reverse - Coefficient array length does not "
                                   "match expected size for given level")
        return self.inverseMODWT(arr.reshape(level + 1, n) if _is_torch(arr)
                                 else np.asarray(arr, dtype=np.float64).reshape(level + 1, n))

    def _check_1d(self, n, level, fwd):
        pass


def decompose_number(number, block_size=None):
    """MathToolKit.decompose(int) (tools/MathToolKit.java:57-80): the powers
    of the ancient Egyptian decomposition, largest first (42 -> [5, 3, 1]);
    with block_size (:97-138): full blocks of block_size first (entries are
    the block size itself, as in the reference), then the decomposition of
    the rest."""
    number = int(number)
    if block_size is not None:
        block_size = int(block_size)
        if not is_binary(block_size):
            raise JWaveFailure("given block size is not 2^p|p={1,2,3,4,..}. "
                               "block size shold be e. g.: 4, 8, 16, 32, ..")
        if number < block_size:
            raise JWaveFailure("Given blockSize is greater than the given number "
                               "to be split by it")
        nb = number // block_size
        rest = number - nb * block_size
        return [block_size] * nb + decompose_number(rest)
    if number < 1:
        raise JWaveFailure("the supported number for decomposition is smaller than one")
    out = []
    cur = number
    while cur >= 1:
        p = cur.bit_length() - 1
        out.append(p)
        cur -= 1 << p
    return out


class AncientEgyptianDecomposition(BasicTransform):
    """jwave.transforms.AncientEgyptianDecomposition (AncientEgyptianDecomposition.java:47-184):
    an array of arbitrary length is split into sub-arrays of the powers of
    two of its length (largest first, MathToolKit.decompose); each goes
    through the wrapped transform's full-depth forward / reverse (one native
    call per sub-array, on the GPU) and lands at its original offset."""

    def __init__(self, basic_transform, initial_wavelet_space_size=0):
        super().__init__(basic_transform.getWavelet() if basic_transform._wavelet else None,
                         basic_transform._ctx)
        self._basic = basic_transform
        self._name = "Ancient Egyptian Decomposition"

    def _run(self, a, fwd):
        n = a.shape[0]
        if getattr(self._basic, "kind", None) in ("fwt", "wpt"):
            # one native call: every piece <= 8192 in one varlen launch
            return aed_transform(a, self._basic.getWavelet(), self._basic.kind, fwd,
                                 self._basic._ctx)
        if _is_torch(a):
            import torch
            out = torch.empty_like(a)
        else:
            a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
            out = np.empty_like(a)
        off = 0
        for p in decompose_number(n):
            m = 1 << p
            sub = a[off:off + m]
            out[off:off + m] = self._basic.forward_1d(sub) if fwd else self._basic.reverse_1d(sub)
            off += m
        return out

    def forward_1d(self, arr, level=None):
        return self._run(arr, True)

    def reverse_1d(self, arr, level=None):
        return self._run(arr, False)


class ParallelTransform(BasicTransform):
    """jwave.transforms.ParallelTransform (ParallelTransform.java:23-403) over
    a GPU transform.  The reference forks row / column / line tasks that call
    the wrapped transform once per line (RowTransformTask :247-263,
    ColumnTransformTask :307-330, Space3DTransformTask :380-397): wrapped
    around a GPU transform that would be one native call per line.  Here every
    2-D / 3-D call is ONE native call with the reference's result:

    * 1-D, 2-D and the 3-D forward: the wrapped transform's own methods
      (rows with lvlN then columns with lvlM; slices then the P axis) -- the
      same order the ForkJoin tasks use, so the same doubles;
    * 3-D reverse: the P axis FIRST, then each slice's 2-D reverse
      (ParallelTransform.java:183-216), which BasicTransform does the other
      way round (slices first): jwv_*3d_rev_pt_f64.

    Errors carry the reference's prefixes ("Error in parallel 2D forward
    transform: ..."), for matrices the reference runs in parallel (both
    dimensions >= MIN_PARALLEL_SIZE = 16; smaller 2-D inputs go straight to
    the wrapped transform, as :73-76 do)."""

    MIN_PARALLEL_SIZE = 16

    def __init__(self, transform, parallelism=None):
        super().__init__(transform._wavelet, transform._ctx)
        self._transform = transform
        self._parallelism = parallelism
        self.kind = transform.kind
        # ParallelTransform never sets _name: getName() is null
        # (BasicTransform.java:56-58, 69-71)
        self._name = None

    def _check_1d(self, n, level, fwd):
        return self._transform._check_1d(n, level, fwd)

    def forward_1d(self, arr, *levels):
        return self._transform.forward_1d(arr, *levels)

    def reverse_1d(self, arr, *levels):
        return self._transform.reverse_1d(arr, *levels)

    def _par(self, what, fn, *args):
        # The reference's tasks wrap the JWaveException in a RuntimeException
        # (ParallelTransform.java:259-269), whose message is the cause's
        # Throwable.toString(): "jwave.exceptions.JWaveFailure: <msg>".  When
        # the failing task ran on a pool worker, ForkJoinTask may re-wrap it
        # once more ("java.lang.RuntimeException: ..."); which task fails first
        # is scheduling-dependent, so that extra prefix is not reproduced
        # (parity unpinned, tests/test_parallel_transform.py).
        try:
            return fn(*args)
        except JWaveException as e:
            raise JWaveException("Error in parallel %s transform: jwave.exceptions.%s: %s"
                                 % (what, type(e).__name__, e.getMessage()))

    def forward_2d(self, m, lvl_m=None, lvl_n=None):
        r, c = m.shape
        if r < self.MIN_PARALLEL_SIZE or c < self.MIN_PARALLEL_SIZE:
            return self._transform.forward_2d(m, lvl_m, lvl_n)
        return self._par("2D forward", self._transform.forward_2d, m, lvl_m, lvl_n)

    def reverse_2d(self, m, lvl_m=None, lvl_n=None):
        r, c = m.shape
        if r < self.MIN_PARALLEL_SIZE or c < self.MIN_PARALLEL_SIZE:
            return self._transform.reverse_2d(m, lvl_m, lvl_n)
        return self._par("2D reverse", self._transform.reverse_2d, m, lvl_m, lvl_n)

    def forward_3d(self, s, lvl_p=None, lvl_q=None, lvl_r=None):
        return self._par("3D forward", self._transform.forward_3d, s, lvl_p, lvl_q, lvl_r)

    def reverse_3d(self, s, lvl_p=None, lvl_q=None, lvl_r=None):
        def run():
            p, q, r = s.shape
            lp, lq, lr = lvl_p, lvl_q, lvl_r
            if lp is None:
                lp, lq, lr = get_exponent(p), get_exponent(q), get_exponent(r)
            self._check_1d(p, lr, False)  # the P-axis task runs first (:191)
            self._check_1d(q, lp, False)
            self._check_1d(r, lq, False)
            return transform_3d(s, self._wavelet, lp, lq, lr, False, self._ctx, self.kind,
                                pt_order=True)
        return self._par("3D reverse", run)

    def shutdown(self):
        """ParallelTransform.shutdown (:399-401): no pool to stop here."""


class Transform:
    """Final facade (Transform.java:43-512): delegates to a BasicTransform and,
    like the reference (:81-90), prints a JWaveException and returns None."""

    def __init__(self, transform):
        if transform is None:
            raise JWaveFailure("Transform - no transform given")
        self._transform = transform

    def _safe(self, fn, *a):
        try:
            return fn(*a)
        except JWaveException as e:
            print("%s: %s" % (type(e).__name__, e.getMessage()))
            return None

    def forward(self, a, *levels):
        return self._safe(self._transform.forward, a, *levels)

    def reverse(self, a, *levels):
        return self._safe(self._transform.reverse, a, *levels)

    def decompose(self, a):
        return self._safe(self._transform.decompose, a)

    def recompose(self, m, level=None):
        return self._safe(self._transform.recompose, m, level)

    def getWavelet(self):  # noqa: N802
        return self._safe(self._transform.getWavelet)

    def getBasicTransform(self):  # noqa: N802
        return self._transform
