"""The JNI shim (java/native/jwave_hip_jni.c) executed without a JVM.

The image has no JDK, so the shim is compiled (tests/jni/Makefile) against a
JNI test double (tests/jni/jni.h + fake_jvm.c: Java arrays with bounds and a
pending-exception state) and driven through ctypes exactly as HipNative's
natives would be called (HipNative.java:92-124):

* CPU: linked against a C-ABI test double (tests/jni/fake_capi.c) that records
  every call: argument and array-length marshaling of each native, the taps,
  status passthrough, the exceptions the shim raises before any GPU work
  (short arrays, bad taps), per-thread pinned staging reuse across two
  threads, and the pageable path above the 64 MiB pin cap;
* CPU: linked against the real libjwave_hip.so with no device: every symbol
  resolves and ctxCreate reports JWV_ERR_DEVICE with a message;
* GPU: the same shim on the real library: Transform.forward(double[])'s
  drop-in path (Transform.java:81-90 -> HipFastWaveletTransform ->
  HipNative.transform1d) is bit-identical to the oracle, and the reference's
  level error reaches Java as status 1 (JWaveFailure) + lastError text.
"""
import ctypes
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "tests", "jni")
sys.path.insert(0, ROOT)

STAGE_FAIL = -100
D = ctypes.c_double
P = ctypes.c_void_p
I = ctypes.c_int32
J = ctypes.c_int64
B = ctypes.c_uint8


def _build():
    r = subprocess.run(["make", "-s", "-C", JNI, "build/libjni_fake.so"], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr


class FcCall(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 48), ("a", J * 6), ("L", I), ("tw", I),
                ("scale", D), ("lo0", D), ("hi0", D), ("lor0", D), ("hirL", D),
                ("nin", J), ("nout", J), ("xin", P)]


def _declare(lib):
    lib.fj_env.restype = P
    lib.fj_darray.restype = P
    lib.fj_darray.argtypes = [I, P]
    lib.fj_larray.restype = P
    lib.fj_larray.argtypes = [I]
    lib.fj_data.restype = P
    lib.fj_data.argtypes = [P]
    lib.fj_string.restype = ctypes.c_char_p
    lib.fj_string.argtypes = [P]
    lib.fj_free.argtypes = [P]
    lib.fj_exception.restype = ctypes.c_char_p
    lib.fj_exception_msg.restype = ctypes.c_char_p
    taps = [I, I, D, P, P, P, P]
    lib.Java_jwave_amd_HipNative_ctxCreate.argtypes = [P, P, I, P]
    lib.Java_jwave_amd_HipNative_lastError.argtypes = [P, P, J]
    lib.Java_jwave_amd_HipNative_lastError.restype = P
    lib.Java_jwave_amd_HipNative_transform1d.argtypes = [P, P, J, I, B, P, P, I] + taps
    lib.Java_jwave_amd_HipNative_transformBatch.argtypes = [P, P, J, I, B, P, P, I, I, I] + taps
    lib.Java_jwave_amd_HipNative_transform2d.argtypes = [P, P, J, I, B, P, P, I, I, I, I] + taps
    lib.Java_jwave_amd_HipNative_transform3d.argtypes = ([P, P, J, I, B, P, P, I, I, I, I, I, I]
                                                         + taps)
    lib.Java_jwave_amd_HipNative_transform3dPt.argtypes = ([P, P, J, I, P, P, I, I, I, I, I, I]
                                                           + taps)
    lib.Java_jwave_amd_HipNative_modwt.argtypes = [P, P, J, B, P, P, I, I, I, I, P, P, P, P]
    lib.Java_jwave_amd_HipNative_aed.argtypes = [P, P, J, I, B, P, P] + taps
    lib.Java_jwave_amd_HipNative_decompose.argtypes = [P, P, J, I, P, P] + taps
    lib.fj_iarray.restype = P
    lib.fj_iarray.argtypes = [I, P]
    lib.Java_jwave_amd_HipNative_mctxCreate.argtypes = [P, P, P, P]
    lib.Java_jwave_amd_HipNative_mctxLastError.argtypes = [P, P, J]
    lib.Java_jwave_amd_HipNative_mctxLastError.restype = P
    lib.Java_jwave_amd_HipNative_transformBatchMulti.argtypes = ([P, P, J, I, B, P, P, I, I, I]
                                                                 + taps)
    lib.Java_jwave_amd_HipNative_transform2dMulti.argtypes = ([P, P, J, I, B, P, P, I, I, I, I]
                                                              + taps)
    mtaps = [I, I, P, P, P, P]
    lib.Java_jwave_amd_HipNative_modwtBatchMulti.argtypes = [P, P, J, B, P, P, I, I, I] + mtaps
    lib.Java_jwave_amd_HipNative_modwtBatch.argtypes = [P, P, J, B, P, P, I, I, I] + mtaps
    for f in ("transform1d", "transformBatch", "transform2d", "transform3d", "transform3dPt",
              "modwt", "aed",
              "decompose", "ctxCreate", "mctxCreate", "transformBatchMulti",
              "transform2dMulti", "modwtBatchMulti", "modwtBatch"):
        getattr(lib, "Java_jwave_amd_HipNative_" + f).restype = I
    return lib


class Jvm:
    """Java-side view of one shim build: arrays, the pending exception and
    HipNative's natives with their Java argument lists."""

    def __init__(self, path, fake_capi):
        self.lib = _declare(ctypes.CDLL(path))
        self.env = self.lib.fj_env()
        self.fake = fake_capi
        if fake_capi:
            self.lib.fc_last.restype = ctypes.POINTER(FcCall)
            for f in ("fc_allocs", "fc_frees", "fc_live_bytes", "fc_thread_allocs",
                      "fc_thread_frees"):
                getattr(self.lib, f).restype = ctypes.c_long
            self.lib.fc_set_rc.argtypes = [I]
        self._keep = []

    def darray(self, a):
        a = np.ascontiguousarray(a, dtype=np.float64)
        h = self.lib.fj_darray(len(a), a.ctypes.data)
        self._keep.append(h)
        return h

    def empty(self, n):
        h = self.lib.fj_darray(n, None)
        self._keep.append(h)
        return h

    def read(self, h, n):
        return np.ctypeslib.as_array(ctypes.cast(self.lib.fj_data(h), ctypes.POINTER(D)),
                                     shape=(n,)).copy()

    def exception(self):
        return self.lib.fj_exception().decode(), self.lib.fj_exception_msg().decode()

    def clear(self):
        self.lib.fj_clear()

    def taps(self, w, L=None, scale=None):
        L = w.mother_wavelength if L is None else L
        arrs = [self.darray(np.asarray(v, dtype=np.float64)) for v in (w.lo, w.hi, w.lo_r, w.hi_r)]
        return [L, w.transform_wavelength, w.reverse_scale if scale is None else scale] + arrs

    def native(self, name, *args):
        return getattr(self.lib, "Java_jwave_amd_HipNative_" + name)(self.env, None, *args)

    def last(self):
        return self.lib.fc_last().contents

    def free_all(self):
        for h in self._keep:
            self.lib.fj_free(h)
        self._keep = []


@pytest.fixture(scope="module")
def jvm():
    _build()
    j = Jvm(os.path.join(JNI, "build", "libjni_fake.so"), True)
    yield j
    j.free_all()


@pytest.fixture(autouse=True)
def _clear(request):
    if "jvm" in request.fixturenames:
        request.getfixturevalue("jvm").clear()
        request.getfixturevalue("jvm").lib.fc_set_rc(0)


def _w(name="Daubechies4"):
    from jwave_amd import wavelets
    return wavelets.by_class(name)


def _ctx(jvm):
    h = jvm.lib.fj_larray(1)
    assert jvm.native("ctxCreate", 0, h) == 0
    v = ctypes.cast(jvm.lib.fj_data(h), ctypes.POINTER(ctypes.c_int64))[0]
    jvm.lib.fj_free(h)
    return v


def test_transform1d_marshaling(jvm):
    w = _w("Daubechies4")
    ctx = _ctx(jvm)
    x = np.arange(1024, dtype=np.float64)
    for kind, fwd, name, k in [(0, 1, b"jwv_fwt_fwd_f64", 1), (0, 0, b"jwv_fwt_rev_f64", 2),
                               (1, 1, b"jwv_wpt_fwd_f64", 3), (1, 0, b"jwv_wpt_rev_f64", 4)]:
        jx, jy = jvm.darray(x), jvm.empty(1024)
        rc = jvm.native("transform1d", ctx, kind, fwd, jx, jy, 7, *jvm.taps(w))
        assert rc == 0 and jvm.exception()[0] == ""
        c = jvm.last()
        assert c.name == name and c.a[0] == 1024 and c.a[1] == 7
        assert (c.L, c.tw, c.scale) == (8, w.transform_wavelength, 1.0)
        assert (c.lo0, c.hi0, c.lor0, c.hirL) == (w.lo[0], w.hi[0], w.lo_r[0], w.hi_r[7])
        assert np.array_equal(jvm.read(jy, 1024), 2 * x + k)


def test_batch_2d_3d_aed_decompose_marshaling(jvm):
    w = _w("Haar1")
    ctx = _ctx(jvm)
    x = np.random.default_rng(1).standard_normal(4 * 64)
    jx, jy = jvm.darray(x), jvm.empty(256)
    assert jvm.native("transformBatch", ctx, 1, 1, jx, jy, 4, 64, 3, *jvm.taps(w)) == 0
    c = jvm.last()
    assert c.name == b"jwv_wpt_fwd_batch_f64" and list(c.a[:4]) == [4, 64, 64, 3]
    assert np.array_equal(jvm.read(jy, 256), 2 * x + 7)
    jy = jvm.empty(256)
    assert jvm.native("transform2d", ctx, 0, 0, jx, jy, 16, 16, 2, 3, *jvm.taps(w)) == 0
    c = jvm.last()
    assert c.name == b"jwv_fwt2d_rev_f64" and list(c.a[:4]) == [16, 16, 2, 3]
    assert np.array_equal(jvm.read(jy, 256), 2 * x + 10)
    jy = jvm.empty(256)
    assert jvm.native("transform3d", ctx, 1, 1, jx, jy, 4, 8, 8, 1, 2, 3, *jvm.taps(w)) == 0
    c = jvm.last()
    assert c.name == b"jwv_wpt3d_fwd_f64" and list(c.a) == [4, 8, 8, 1, 2, 3]
    for kind, name, k in [(0, b"jwv_fwt3d_rev_pt_f64", 22), (1, b"jwv_wpt3d_rev_pt_f64", 23)]:
        jy = jvm.empty(256)
        assert jvm.native("transform3dPt", ctx, kind, jx, jy, 4, 8, 8, 1, 2, 3, *jvm.taps(w)) == 0
        c = jvm.last()
        assert c.name == name and list(c.a) == [4, 8, 8, 1, 2, 3]
        assert np.array_equal(jvm.read(jy, 256), 2 * x + k)
    jx7, jy7 = jvm.darray(x[:7]), jvm.empty(7)
    assert jvm.native("aed", ctx, 1, 0, jx7, jy7, *jvm.taps(w)) == 0
    c = jvm.last()
    assert c.name == b"jwv_aed_rev_f64" and list(c.a[:2]) == [7, 1]
    assert np.array_equal(jvm.read(jy7, 7), 2 * x[:7] + 20)
    j64, jm = jvm.darray(x[:64]), jvm.empty(7 * 64)
    assert jvm.native("decompose", ctx, 0, j64, jm, *jvm.taps(w)) == 0
    c = jvm.last()
    assert c.name == b"jwv_decompose_f64" and c.nout == 7 * 64
    assert np.array_equal(jvm.read(jm, 7 * 64), 2 * np.tile(x[:64], 7) + 21)


def test_modwt_marshaling_and_bounds(jvm):
    w = _w("Daubechies4")
    ctx = _ctx(jvm)
    n, Jl = 100, 3
    x = np.random.default_rng(2).standard_normal(n)
    jx, jwv = jvm.darray(x), jvm.empty((Jl + 1) * n)
    tp = jvm.taps(w)[:2] + jvm.taps(w)[3:]  # modwt takes no scale
    assert jvm.native("modwt", ctx, 1, jx, jwv, n, Jl, *tp) == 0
    c = jvm.last()
    assert c.name == b"jwv_modwt_fwd_f64" and c.nin == n and c.nout == (Jl + 1) * n
    assert np.array_equal(jvm.read(jwv, (Jl + 1) * n), 2 * np.tile(x, Jl + 1) + 17)
    jr = jvm.empty(n)
    assert jvm.native("modwt", ctx, 0, jr, jwv, n, Jl, *tp) == 0
    assert jvm.last().name == b"jwv_modwt_inv_f64" and jvm.last().nin == (Jl + 1) * n
    # output too short: exception pending before any C-ABI call
    jvm.lib.fc_last().contents.name = b"none"
    short = jvm.empty((Jl + 1) * n - 1)
    assert jvm.native("modwt", ctx, 1, jx, short, n, Jl, *tp) == STAGE_FAIL
    assert jvm.exception()[0] == "java/lang/ArrayIndexOutOfBoundsException"
    assert jvm.last().name == b"none"
    jvm.clear()
    # input too short (the inverse reads (J+1)*n): the region read throws
    assert jvm.native("modwt", ctx, 0, jr, short, n, Jl, *tp) == STAGE_FAIL
    exc, msg = jvm.exception()
    assert exc == "java/lang/ArrayIndexOutOfBoundsException" and "out of bounds" in msg
    assert jvm.last().name == b"none"


def test_bad_taps_throw_before_any_call(jvm):
    w = _w("Daubechies4")
    ctx = _ctx(jvm)
    jvm.lib.fc_last().contents.name = b"none"
    jx, jy = jvm.darray(np.ones(64)), jvm.empty(64)
    for L in (0, -1, 65):
        jvm.clear()
        assert jvm.native("transform1d", ctx, 0, 1, jx, jy, 2, *jvm.taps(w, L=L)) == STAGE_FAIL
        assert jvm.exception()[0] == "java/lang/IllegalArgumentException"
    jvm.clear()  # tap arrays shorter than L
    assert jvm.native("transform1d", ctx, 0, 1, jx, jy, 2, *jvm.taps(w, L=12)) == STAGE_FAIL
    assert jvm.exception()[0] == "java/lang/ArrayIndexOutOfBoundsException"
    assert jvm.last().name == b"none"
    assert np.array_equal(jvm.read(jy, 64), np.zeros(64))


def test_status_passthrough_leaves_output_untouched(jvm):
    w = _w("Haar1")
    ctx = _ctx(jvm)
    jx, jy = jvm.darray(np.ones(32)), jvm.darray(np.full(32, 5.0))
    for rc in (1, 2, 3, 4):  # FAILURE, ILLEGAL_ARGUMENT, DEVICE, BAD_CALL -> HipNative.check
        jvm.lib.fc_set_rc(rc)
        assert jvm.native("transform1d", ctx, 0, 1, jx, jy, 5, *jvm.taps(w)) == rc
        assert jvm.exception()[0] == ""
        assert np.array_equal(jvm.read(jy, 32), np.full(32, 5.0))
    jvm.lib.fc_set_rc(0)
    msg = jvm.lib.fj_string(jvm.native("lastError", ctx))
    assert msg == b"fake error text"


def test_in_place_same_array(jvm):
    """HipInPlaceFastWaveletTransform.forwardInPlace / reverseInPlace pass the
    caller's array as both input and output (InPlaceFastWaveletTransform.java:70-120):
    the shim stages the input before the call, so the result lands in that
    array; a failing call leaves it untouched (the reference copies back only
    after super.forward returned)."""
    w = _w("Daubechies4")
    ctx = _ctx(jvm)
    x = np.linspace(-1.0, 1.0, 512)
    ja = jvm.darray(x)
    assert jvm.native("transform1d", ctx, 0, 1, ja, ja, 9, *jvm.taps(w)) == 0
    c = jvm.last()
    assert c.name == b"jwv_fwt_fwd_f64" and c.a[0] == 512 and c.a[1] == 9
    assert np.array_equal(jvm.read(ja, 512), 2 * x + 1)
    assert jvm.native("transform1d", ctx, 0, 0, ja, ja, 9, *jvm.taps(w)) == 0
    assert np.array_equal(jvm.read(ja, 512), 2 * (2 * x + 1) + 2)
    before = jvm.read(ja, 512)
    jvm.lib.fc_set_rc(1)
    assert jvm.native("transform1d", ctx, 0, 1, ja, ja, 20, *jvm.taps(w)) == 1
    jvm.lib.fc_set_rc(0)
    assert np.array_equal(jvm.read(ja, 512), before)


def test_multi_device_batch_marshaling(jvm):
    """HipWaveletPacketTransform.forwardBatch under -Djwave.hip.devices=0,1,2
    (HipNative.mctx): mctxCreate passes the device list, transformBatchMulti
    stages the packed batch once and calls the multi-device entry with the
    batch geometry; its status passes through and a failure leaves the output
    untouched."""
    jvm.lib.fc_mctx_devices.argtypes = [P]
    devs = (ctypes.c_int32 * 3)(0, 1, 2)
    jd = jvm.lib.fj_iarray(3, ctypes.cast(devs, P))
    h = jvm.lib.fj_larray(1)
    assert jvm.native("mctxCreate", jd, h) == 0
    m = ctypes.cast(jvm.lib.fj_data(h), ctypes.POINTER(ctypes.c_int64))[0]
    got = (ctypes.c_int32 * 16)()
    assert jvm.lib.fc_mctx_devices(ctypes.cast(got, P)) == 3 and list(got[:3]) == [0, 1, 2]
    w = _w("Symlet8")
    x = np.arange(6 * 256, dtype=np.float64)
    for kind, fwd, name, k in [(0, 1, b"jwv_m_fwt_fwd_batch_f64", 30),
                               (0, 0, b"jwv_m_fwt_rev_batch_f64", 31),
                               (1, 1, b"jwv_m_wpt_fwd_batch_f64", 32),
                               (1, 0, b"jwv_m_wpt_rev_batch_f64", 33)]:
        jx, jy = jvm.darray(x), jvm.empty(x.size)
        assert jvm.native("transformBatchMulti", m, kind, fwd, jx, jy, 6, 256, 5,
                          *jvm.taps(w)) == 0
        c = jvm.last()
        assert c.name == name and list(c.a[:5]) == [6, 256, 256, 5, 3]
        assert np.array_equal(jvm.read(jy, x.size), 2 * x + k)
    jy = jvm.empty(x.size)
    jvm.lib.fc_set_rc(3)
    assert jvm.native("transformBatchMulti", m, 1, 1, jvm.darray(x), jy, 6, 256, 5,
                      *jvm.taps(w)) == 3
    jvm.lib.fc_set_rc(0)
    assert not jvm.read(jy, x.size).any()
    msg = jvm.native("mctxLastError", m)
    assert jvm.lib.fj_string(msg) == b"fake multi error text"
    jvm.lib.fj_free(jd)
    jvm.lib.fj_free(h)


def test_multi_device_2d_and_modwt_marshaling(jvm):
    """HipNative.run2d / modwtForwardBatch under -Djwave.hip.devices
    (HipParallelTransform 2-D, HipMODWTTransform.forwardMODWT(double[][], J)):
    transform2dMulti passes the matrix geometry and levels to
    jwv_m_{fwt,wpt}2d_*, modwtBatchMulti / modwtBatch the batch, length and
    level to the MODWT batch entries, with (J+1)-row coefficient blocks; a
    failing status leaves the output untouched."""
    devs = (ctypes.c_int32 * 2)(0, 1)
    jd = jvm.lib.fj_iarray(2, ctypes.cast(devs, P))
    h = jvm.lib.fj_larray(1)
    assert jvm.native("mctxCreate", jd, h) == 0
    m = ctypes.cast(jvm.lib.fj_data(h), ctypes.POINTER(ctypes.c_int64))[0]
    w = _w("Daubechies8")
    x = np.arange(64 * 32, dtype=np.float64)
    for kind, fwd, name, k in [(0, 1, b"jwv_m_fwt2d_fwd_f64", 34), (0, 0, b"jwv_m_fwt2d_rev_f64", 35),
                               (1, 1, b"jwv_m_wpt2d_fwd_f64", 36), (1, 0, b"jwv_m_wpt2d_rev_f64", 37)]:
        jx, jy = jvm.darray(x), jvm.empty(x.size)
        assert jvm.native("transform2dMulti", m, kind, fwd, jx, jy, 64, 32, 6, 5,
                          *jvm.taps(w)) == 0
        c = jvm.last()
        assert c.name == name and list(c.a[:5]) == [64, 32, 6, 5, 2]
        assert np.array_equal(jvm.read(jy, x.size), 2 * x + k)
    # MODWT batches: 3 signals of 100, J = 4 -> 3 x 5 x 100 coefficients
    wd = _w("Daubechies4")
    tap = jvm.taps(wd)
    mtap = tap[:2] + tap[3:]  # the MODWT natives take no reverse scale
    xs = np.arange(300, dtype=np.float64)
    cw = jvm.empty(1500)
    assert jvm.native("modwtBatchMulti", m, 1, jvm.darray(xs), cw, 3, 100, 4, *mtap) == 0
    c = jvm.last()
    assert c.name == b"jwv_m_modwt_fwd_batch_f64" and list(c.a[:4]) == [3, 100, 4, 2]
    assert c.nin == 300 and c.nout == 1500
    coef = np.arange(1500, dtype=np.float64)
    jx = jvm.empty(300)
    assert jvm.native("modwtBatchMulti", m, 0, jx, jvm.darray(coef), 3, 100, 4, *mtap) == 0
    c = jvm.last()
    assert c.name == b"jwv_m_modwt_inv_batch_f64" and c.nin == 1500 and c.nout == 300
    assert np.array_equal(jvm.read(jx, 300), 2 * coef[:300] + 39)
    ctx = _ctx(jvm)
    assert jvm.native("modwtBatch", ctx, 1, jvm.darray(xs), jvm.empty(1500), 3, 100, 4, *mtap) == 0
    assert jvm.last().name == b"jwv_modwt_fwd_batch_f64"
    jvm.lib.fc_set_rc(2)
    jy = jvm.empty(x.size)
    assert jvm.native("transform2dMulti", m, 0, 1, jvm.darray(x), jy, 64, 32, 6, 5,
                      *jvm.taps(w)) == 2
    jvm.lib.fc_set_rc(0)
    assert not jvm.read(jy, x.size).any()
    jvm.lib.fj_free(jd)
    jvm.lib.fj_free(h)


def test_staging_per_thread_reuse_and_cap(jvm):
    w = _w("Haar1")
    ctx = _ctx(jvm)
    tp = jvm.taps(w)
    res = {}

    def worker(tag, sizes):
        counts = []
        for n in sizes:
            jx, jy = jvm.darray(np.ones(n)), jvm.empty(n)
            assert jvm.native("transform1d", ctx, 0, 1, jx, jy, 1, *tp) == 0
            assert np.array_equal(jvm.read(jy, n), np.full(n, 3.0))
            counts.append(jvm.lib.fc_thread_allocs())
        res[tag] = counts

    frees0 = jvm.lib.fc_frees()
    a = threading.Thread(target=worker, args=("a", [1000, 500, 1000, 4000, 100]))
    b = threading.Thread(target=worker, args=("b", [2000, 2000]))
    a.start(); b.start(); a.join(); b.join()
    # two pinned buffers per thread on its first call, reused while they fit,
    # regrown (free + alloc) only when a larger array comes
    assert res["a"] == [2, 2, 2, 4, 4]
    assert res["b"] == [2, 2]
    # thread exit frees every thread's staging (4 of a's, 2 of them already at
    # the regrow, + b's 2).  Python's join() returns before the OS thread runs
    # its pthread key destructors, so wait for them briefly.
    for _ in range(200):
        if jvm.lib.fc_frees() - frees0 == 6:
            break
        time.sleep(0.01)
    assert jvm.lib.fc_frees() - frees0 == 6
    # above the 64 MiB pin cap: pageable memory of the call, nothing pinned
    n = (64 << 20) // 8 + 1
    res.clear()
    t = threading.Thread(target=worker, args=("c", [n, 100]))
    t.start(); t.join()
    assert res["c"] == [0, 2]


def test_real_library_links_and_reports_no_device():
    r = subprocess.run(["make", "-s", "-C", JNI, "build/libjni_real.so"], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    code = (
        "import ctypes,sys;sys.path.insert(0,%r);from tests.test_jni_shim import Jvm;"
        "j=Jvm(%r,False);h=j.lib.fj_larray(1);rc=j.native('ctxCreate',0,h);"
        "print(rc, j.lib.fj_string(j.native('lastError',0)).decode())"
        % (ROOT, os.path.join(JNI, "build", "libjni_real.so")))
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    rc, msg = out.stdout.split(" ", 1)
    assert int(rc) == 3 and "no HIP device" in msg  # JWV_ERR_DEVICE -> JWaveError in check()


@pytest.mark.gpu
def test_real_library_drop_in_path_gpu():
    """HipFastWaveletTransform.forward/reverse(double[]) and HipMODWTTransform
    through the shim on the GPU: bit-identical to the oracle; the reference's
    level error arrives as FAILURE (JWaveFailure) + its message."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    so = os.path.join(JNI, "build", "libjni_real.so")
    if not os.path.exists(so):  # normally built by __graft_entry__.build()
        subprocess.run(["make", "-s", "-C", JNI, "build/libjni_real.so"], check=True)
    j = Jvm(so, False)
    h = j.lib.fj_larray(1)
    assert j.native("ctxCreate", 0, h) == 0
    ctx = ctypes.cast(j.lib.fj_data(h), ctypes.POINTER(ctypes.c_int64))[0]
    assert ctx != 0
    w = _w("Daubechies4")
    n = 1 << 16
    x = oracle.java_random_doubles(42, n)
    jx, jy, jr = j.darray(x), j.empty(n), j.empty(n)
    assert j.native("transform1d", ctx, 0, 1, jx, jy, 16, *j.taps(w)) == 0
    y = j.read(jy, n)
    assert np.array_equal(y, oracle.fwt_forward(w, x, 16))
    assert j.native("transform1d", ctx, 0, 0, jy, jr, 16, *j.taps(w)) == 0
    assert np.array_equal(j.read(jr, n), oracle.fwt_reverse(w, y, 16))
    m, Jl = 1000, 4
    jm, jwv = j.darray(x[:m]), j.empty((Jl + 1) * m)
    tp = j.taps(w)[:2] + j.taps(w)[3:]
    assert j.native("modwt", ctx, 1, jm, jwv, m, Jl, *tp) == 0
    assert np.array_equal(j.read(jwv, (Jl + 1) * m).reshape(Jl + 1, m),
                          oracle.modwt_forward(w, x[:m], Jl))
    # level beyond log2 n: FastWaveletTransform.java:80-83's JWaveFailure
    assert j.native("transform1d", ctx, 0, 1, jx, jy, 17, *j.taps(w)) == 1
    assert j.lib.fj_string(j.native("lastError", ctx))
    j.free_all()
