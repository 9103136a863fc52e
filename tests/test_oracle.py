"""CPU tests: the oracle against the reference's own KATs / fixtures, against an
independent numpy restatement, and against the committed golden vectors; the
filter-bank data; the host mirror's validation; the C ABI exports.

No GPU needed (the native library is loaded but no compute call is made).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
import numpy_restatement as npr
import jwave_amd as jw
from jwave_amd import _lib
from jwave_amd.wavelets import WaveletBuilder

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CREATE2ARR = WaveletBuilder.create2arr()


def load_vec(name):
    return np.loadtxt(os.path.join(GOLDEN, name))


# ----------------------------------------------------------- taps / fixtures
def test_haar_taps_fixture():
    """CrossValidationTest.testHaarWaveletCoefficients (CrossValidationTest.java:159-184)."""
    w = jw.by_class("Haar1")
    np.testing.assert_allclose(w.getScalingDeComposition(), load_vec("filter_haar_dec_lo.txt"), atol=1e-10)
    np.testing.assert_allclose(w.getWaveletDeComposition(), load_vec("filter_haar_dec_hi.txt"), atol=1e-10)
    np.testing.assert_allclose(w.getScalingReConstruction(), load_vec("filter_haar_rec_lo.txt"), atol=1e-10)


def test_db2_fixture_matches_daubechies2():
    """filter_db4_dec_lo.txt is PyWavelets' db2 == JWave Daubechies2 (4 taps)."""
    np.testing.assert_allclose(jw.by_class("Daubechies2").lo, load_vec("filter_db4_dec_lo.txt"), atol=1e-12)


@pytest.mark.parametrize("w", CREATE2ARR, ids=lambda w: w.name)
def test_filter_bank_shape(w):
    L = w.mother_wavelength
    assert len(w.lo) == len(w.hi) == len(w.lo_r) == len(w.hi_r) == L
    assert w.transform_wavelength == 2


def test_config_wavelets_orthonormal_to_tap_precision():
    # the reference taps are orthonormal only to ~1e-12
    for cls, bound in (("Haar1", 1e-15), ("Daubechies4", 1e-12), ("Daubechies8", 3e-12),
                       ("Symlet8", 1e-12)):
        w = jw.by_class(cls)
        assert abs(sum(c * c for c in w.lo) - 1.0) < bound


def test_builder_refusals():
    for name in ("Battle 23", "CDF 5/3", "CDF 9/7"):
        with pytest.raises(jw.JWaveFailure, match="odd number of coefficients"):
            WaveletBuilder.create(name)
    with pytest.raises(jw.JWaveFailure, match="unknown type of wavelet"):
        WaveletBuilder.create("Nope 7")
    assert len(CREATE2ARR) == 52


# ----------------------------------------------------------------- KATs
def test_haar_level1_kat():
    """CrossValidationTest.testHaarTransformWithReference (:187-211), tol 1e-10."""
    x = load_vec("haar_simple_input.txt")
    y = oracle.fwt_forward(jw.by_class("Haar1"), x, 1)
    np.testing.assert_allclose(y[:4], load_vec("haar_level1_approx_manual.txt"), atol=1e-10)
    np.testing.assert_allclose(y[4:], load_vec("haar_level1_detail_manual.txt"), atol=1e-10)


def test_modwt_haar_kat():
    """MODWTTransformTest.testKnownValuesWithHaar (MODWTTransformTest.java:39-72)."""
    c = oracle.modwt_forward(jw.by_class("Haar1"), np.arange(1.0, 9.0), 1, sparse=False)
    np.testing.assert_allclose(c[0], [-3.5] + [0.5] * 7, atol=1e-9)
    np.testing.assert_allclose(c[1], [4.5, 1.5, 2.5, 3.5, 4.5, 5.5, 6.5, 7.5], atol=1e-9)
    g, h = oracle.modwt_filters(jw.by_class("Haar1"))
    np.testing.assert_allclose(g, [0.5, 0.5], atol=1e-15)
    np.testing.assert_allclose(h, [0.5, -0.5], atol=1e-15)


def _stepping_expect(n, p):
    e = np.zeros(n)
    e[: n >> p] = 2.0 ** (p / 2.0)
    return e


@pytest.mark.parametrize("w", CREATE2ARR, ids=lambda w: w.name)
def test_stepping_kat(w):
    """SteppingTest.testStepping (SteppingTest.java:37-315): constant signals,
    FWT and WPT, level-p energy 2^(p/2) in the first N/2^p slots, delta 1e-8."""
    for n in (4, 64):
        x = np.ones(n)
        for p in range(0, n.bit_length()):
            y = oracle.fwt_forward(w, x, p)
            np.testing.assert_allclose(y, _stepping_expect(n, p), atol=1e-8)
            np.testing.assert_allclose(oracle.fwt_reverse(w, y, p), x, atol=1e-8)
            yw = oracle.wpt_forward(w, x, p)
            np.testing.assert_allclose(yw, _stepping_expect(n, p), atol=1e-8)
            np.testing.assert_allclose(oracle.wpt_reverse(w, yw, p), x, atol=1e-8)


def _decompose_oracle(w, x):
    """WaveletTransform.decompose (WaveletTransform.java:136-145) on the oracle:
    row p = forward(x, p), p = 0..log2 n."""
    return np.stack([oracle.fwt_forward(w, x, p) for p in range(len(x).bit_length())])


@pytest.mark.parametrize("w", CREATE2ARR, ids=lambda w: w.name)
def test_decompose_kat(w):
    """DecomposeTest.testDecompose (DecomposeTest.java:30-170): constant
    signals of 4 and 64 give the orthonormal pyramid (row p: 2^(p/2) in the
    first n/2^p slots), delta 1e-8; recompose (WaveletTransform.java:173-182:
    reverse(row level, level)) from every level returns the signal."""
    for n in (4, 64):
        x = np.ones(n)
        mat = _decompose_oracle(w, x)
        exp = np.stack([_stepping_expect(n, p) for p in range(n.bit_length())])
        np.testing.assert_allclose(mat, exp, atol=1e-8)
        for lev in range(mat.shape[0]):
            np.testing.assert_allclose(oracle.fwt_reverse(w, mat[lev], lev), x, atol=1e-8)


def test_modwt_flattened_host_logic(monkeypatch):
    """MODWTTransform's flattened API host logic (MODWTTransform.java:389-443,
    854-912) without a device: validation messages, and the auto-level
    reverse(double[]) search — the first N = 2^p with total/N - 1 <= p,
    including the reference's ambiguity (N=16, J=1 is read as N=8, J=3)."""
    m = jw.MODWTTransform(jw.by_class("Haar1"))
    seen = []
    monkeypatch.setattr(m, "inverseMODWT", lambda c: seen.append(np.asarray(c).shape) or "ok")
    assert m.reverse(np.zeros(32)) == "ok" and seen[-1] == (4, 8)      # N=8, J=3
    assert m.reverse(np.zeros(16 * 2)) == "ok" and seen[-1] == (4, 8)  # N=16,J=1 -> N=8,J=3
    assert m.reverse(np.zeros(1024 * 5)) == "ok" and seen[-1] == (10, 512)  # 512 x 10 fits first
    assert m.reverse(np.zeros(2)) == "ok" and seen[-1] == (1, 2)       # N=2, J=0
    with pytest.raises(jw.JWaveFailure, match="Cannot determine original signal dimensions"):
        m.reverse(np.zeros(7))
    with pytest.raises(jw.JWaveFailure, match="Invalid coefficient array for given level"):
        m.reverse(np.zeros(15), 2)
    with pytest.raises(jw.JWaveFailure, match="does not match expected size"):
        m.reverse(np.zeros(17), 1)
    with pytest.raises(jw.JWaveFailure, match="calcExponent"):
        m.forward(np.zeros(10))
    with pytest.raises(jw.JWaveFailure, match=r"MODWTTransform#forward - given array length"):
        m.forward(np.zeros(10), 2)
    with pytest.raises(jw.JWaveFailure, match="out of range"):
        m.forward(np.zeros(8), 5)
    with pytest.raises(jw.JWaveFailure, match="maximum supported decomposition level is 13"):
        m.forward(np.zeros(1 << 14), 14)
    with pytest.raises(ValueError, match="maximum supported decomposition level is 13"):
        m.forward(np.zeros(1 << 14))  # full depth 14 > 13: forwardMODWT's IllegalArgumentException
    with pytest.raises(ValueError, match="at least 1"):
        m.forward(np.zeros(8), 0)
    # WaveletTransform.decompose (WaveletTransform.java:136-145) is inherited
    # by MODWTTransform: its row 0 is forward(arr, 0), which forwardMODWT
    # rejects (MODWTTransform.java:257-260) -- IllegalArgumentException, not a
    # lookup error of the native decompose
    with pytest.raises(ValueError, match="at least 1"):
        m.decompose(np.zeros(8))
    with pytest.raises(jw.JWaveFailure, match="calcExponent"):
        m.decompose(np.zeros(6))


@pytest.mark.parametrize("w", CREATE2ARR[:20] + CREATE2ARR[25:32], ids=lambda w: w.name)
def test_general_roundtrip(w):
    """GeneralTest.testExample (GeneralTest.java:36-80): fixed 8-vector round trip."""
    x = np.array([1., 2., 3., 4., 5., 6., 7., 8.])
    y = oracle.fwt_forward(w, x, 3)
    np.testing.assert_allclose(oracle.fwt_reverse(w, y, 3), x, atol=1e-6)


def test_property_linearity_energy():
    """PropertyBasedTest (PropertyBasedTest.java:138-382) on the oracle, Random(42)."""
    for cls in ("Haar1", "Daubechies4", "Symlet4"):
        w = jw.by_class(cls)
        x = oracle.java_random_doubles(42, 256)
        z = oracle.java_random_doubles(43, 256)
        a = 3.25
        fx, fz = oracle.fwt_forward(w, x, 8), oracle.fwt_forward(w, z, 8)
        np.testing.assert_allclose(oracle.fwt_forward(w, a * x + z, 8), a * fx + fz, atol=1e-8)
        assert abs(np.dot(fx, fx) - np.dot(x, x)) < 1e-8 * np.dot(x, x)


def test_java_random_matches_reference_algorithm():
    """java.util.Random(42).nextDouble() first values (the LCG of the JDK spec)."""
    v = oracle.java_random_doubles(42, 3)
    assert v[0] == 0.7275636800328681 and v[1] == 0.6832234717598454 and v[2] == 0.30871945533265976


# ------------------------------------------------- oracle vs numpy (bitwise)
@pytest.mark.parametrize("cls", ["Haar1", "Daubechies4", "Daubechies8", "Symlet8", "Coiflet1",
                                 "Haar1Orthogonal", "CDF53", "Battle23", "BiOrthogonal35",
                                 "DiscreteMeyer"])
def test_oracle_equals_numpy_restatement(cls):
    w = jw.by_class(cls)
    for n in (2, 8, 64, 512):
        x = oracle.java_random_doubles(n, n)
        for lev in range(0, n.bit_length()):
            y = oracle.fwt_forward(w, x, lev)
            assert np.array_equal(y, npr.fwt_forward(w, x, lev))
            assert np.array_equal(oracle.fwt_reverse(w, y, lev), npr.fwt_reverse(w, y, lev))
            yw = oracle.wpt_forward(w, x, lev)
            assert np.array_equal(yw, npr.wpt_forward(w, x, lev))
            assert np.array_equal(oracle.wpt_reverse(w, yw, lev), npr.wpt_reverse(w, yw, lev))


@pytest.mark.parametrize("cls", ["Haar1", "Daubechies4", "Symlet8", "CDF53"])
def test_oracle_modwt_equals_numpy(cls):
    w = jw.by_class(cls)
    for n, J in ((8, 3), (100, 5), (1000, 8), (37, 2)):
        x = oracle.java_random_doubles(7, n)
        c = oracle.modwt_forward(w, x, J, sparse=False)
        assert np.array_equal(c, oracle.modwt_forward(w, x, J, sparse=True))
        assert np.array_equal(c, npr.modwt_forward(w, x, J))
        assert np.array_equal(oracle.modwt_inverse(w, c), npr.modwt_inverse(w, c))
    assert np.array_equal(np.stack(oracle.modwt_filters(w)), np.stack(npr.modwt_filters(w)))


NONFINITE = (np.inf, -np.inf, np.nan)


def assert_nan_bits(got, ref, what=""):
    """NaN at the same positions and every other value bit for bit (NaN
    payloads and signs are not compared: the JVM's NaN is not specified)."""
    got = np.ascontiguousarray(got, dtype=np.float64).ravel()
    ref = np.ascontiguousarray(ref, dtype=np.float64).ravel()
    gn, rn = np.isnan(got), np.isnan(ref)
    bad = np.flatnonzero(gn != rn)
    assert bad.size == 0, "%s: NaN positions differ at %d places, first %d (got %r ref %r)" % (
        what, bad.size, bad[0], got[bad[0]], ref[bad[0]])
    gb, rb = got[~rn].view(np.int64), ref[~rn].view(np.int64)
    bad = np.flatnonzero(gb != rb)
    assert bad.size == 0, "%s: %d values differ in their bits" % (what, bad.size)


@pytest.mark.parametrize("cls", ["Haar1", "Daubechies4", "Symlet8", "CDF53"])
def test_oracle_modwt_nonfinite_sparse_equals_direct(cls):
    """MODWTTransform.java:677-716 multiplies every zero tap of the upsampled
    filter too, so a +-inf / NaN sample at a zero tap of an output's window
    makes that output NaN.  The oracle's sparse path (real taps plus the
    zero-tap NaN rule) must equal the as-written DIRECT loops bit for bit,
    NaN positions included, and so must the numpy restatement of the DIRECT
    loops; windows longer than N (wrapping several times) included."""
    w = jw.by_class(cls)
    rng = np.random.default_rng(3)
    more_nan = 0
    for n, J in ((8, 3), (37, 2), (37, 5), (100, 5), (300, 6), (1000, 8)):
        for trial in range(4):
            x = oracle.java_random_doubles(11 + trial, n)
            k = int(rng.integers(1, 4))
            x[rng.choice(n, size=k, replace=False)] = rng.choice(NONFINITE, size=k)
            cd = oracle.modwt_forward(w, x, J, sparse=False)
            assert_nan_bits(oracle.modwt_forward(w, x, J, sparse=True), cd, "fwd n=%d J=%d" % (n, J))
            assert_nan_bits(npr.modwt_forward_dense(w, x, J), cd, "numpy fwd n=%d J=%d" % (n, J))
            with np.errstate(invalid="ignore", over="ignore"):
                more_nan += int(np.isnan(cd).sum() > np.isnan(npr.modwt_forward(w, x, J)).sum())
            c = oracle.modwt_forward(w, oracle.java_random_doubles(5, n), J)
            c[rng.integers(0, J + 1, k), rng.integers(0, n, k)] = rng.choice(NONFINITE, size=k)
            xd = oracle.modwt_inverse(w, c, sparse=False)
            assert_nan_bits(oracle.modwt_inverse(w, c, sparse=True), xd, "inv n=%d J=%d" % (n, J))
            assert_nan_bits(npr.modwt_inverse_dense(w, c), xd, "numpy inv n=%d J=%d" % (n, J))
    # the rule is not vacuous: the zero taps add NaNs the real-tap sums lack
    assert more_nan > 0


def test_oracle_modwt_overflow_sparse_equals_direct():
    """Finite input whose sums overflow: inf from one level meets the next
    level's zero taps (NaN in Java), exactly as an inf input would."""
    w = jw.by_class("Daubechies4")
    g, _ = oracle.modwt_filters(w)
    x = oracle.java_random_doubles(3, 500)
    x[100 - np.arange(len(g))] = np.sign(g) * 1.7e308  # V_1[100] = sum |g| * 1.7e308
    assert np.abs(g).sum() * 1.7e308 > np.finfo(np.float64).max
    cd = oracle.modwt_forward(w, x, 6, sparse=False)
    assert np.isinf(cd[0:6]).any() and np.isnan(cd).any()
    assert np.isfinite(x).all()
    assert_nan_bits(oracle.modwt_forward(w, x, 6, sparse=True), cd, "overflow fwd")


def test_oracle_2d_3d_equal_loops():
    """2-D/3-D oracle == explicit per-line loops of the 1-D oracle (BasicTransform.java:361-659)."""
    w = jw.by_class("Daubechies4")
    x = oracle.java_random_doubles(5, 16 * 32).reshape(16, 32)
    y = np.array([oracle.fwt_forward(w, r, 3) for r in x])
    y = np.array([oracle.fwt_forward(w, c, 2) for c in y.T]).T
    assert np.array_equal(oracle.transform_2d("fwt", True, w, x, 2, 3), y)
    s = oracle.java_random_doubles(6, 4 * 8 * 16).reshape(4, 8, 16)
    ref = np.stack([oracle.transform_2d("fwt", True, w, s[i], 3, 4) for i in range(4)])
    ref = np.apply_along_axis(lambda v: oracle.fwt_forward(w, v, 2), 0, ref)
    assert np.array_equal(oracle.transform_3d("fwt", True, w, s, 3, 4, 2), ref)


# --------------------------------------------------------------- golden vectors
def _check(rec, a):
    a = np.ascontiguousarray(np.asarray(a, dtype="<f8"))
    assert list(a.shape) == rec["shape"]
    assert hashlib.sha256(a.tobytes()).hexdigest() == rec["sha256"]
    if "hex" in rec:
        assert [float(v).hex() for v in a.ravel()] == rec["hex"]


def test_golden_vectors():
    data = json.load(open(os.path.join(GOLDEN, "golden.json")))
    for case in data["cases"]:
        w = jw.by_class(case["wavelet"])
        op = case["op"]
        if op == "fwt":
            x = oracle.java_random_doubles(case["seed"], case["n"])
            y = oracle.fwt_forward(w, x, case["level"])
            _check(case["forward"], y)
            _check(case["roundtrip"], oracle.fwt_reverse(w, y, case["level"]))
        elif op == "fwt2d":
            r, c = case["shape"]
            x = oracle.java_random_doubles(case["seed"], r * c).reshape(r, c)
            y = oracle.transform_2d("fwt", True, w, x, *case["levels"])
            _check(case["forward"], y)
            _check(case["roundtrip"], oracle.transform_2d("fwt", False, w, y, *case["levels"]))
        elif op == "wpt_batch":
            x = np.stack([oracle.java_random_doubles(case["seed"] + b, case["n"])
                          for b in range(case["batch"])])
            y = oracle.batch("wpt", True, w, x, case["level"])
            _check(case["forward"], y)
            _check(case["roundtrip"], oracle.batch("wpt", False, w, y, case["level"]))
        elif op == "modwt":
            x = oracle.java_random_doubles(case["seed"], case["n"])
            c = oracle.modwt_forward(w, x, case["level"])
            _check(case["forward"], c)
            _check(case["roundtrip"], oracle.modwt_inverse(w, c))


# ----------------------------------------------------------- host mirror (no GPU)
def test_mirror_validation_messages():
    w = jw.by_class("Daubechies4")
    fwt = jw.FastWaveletTransform(w)
    with pytest.raises(jw.JWaveFailure, match=r"^FastWaveletTransform#forward - given array length"):
        fwt.forward(np.zeros(12), 2)
    with pytest.raises(jw.JWaveFailure, match=r"^FastWaveletTransform#reverse - given level is out"):
        fwt.reverse(np.zeros(16), 5)
    with pytest.raises(jw.JWaveFailure, match=r"^WaveletTransform#forward - given array length"):
        fwt.forward(np.zeros(12))
    wpt = jw.WaveletPacketTransform(w)
    with pytest.raises(jw.JWaveFailure, match=r"^WaveletPacketTransform#forward - given level"):
        wpt.forward(np.zeros(16), 7)
    with pytest.raises(jw.JWaveFailure, match="invalid level"):
        jw.PooledWaveletPacketTransform(w).forward(np.zeros(16), 0)
    m = jw.MODWTTransform(w)
    with pytest.raises(ValueError, match="at least 1"):
        m.forwardMODWT(np.zeros(8), 0)
    with pytest.raises(ValueError, match="maximum supported decomposition level is 13"):
        m.forwardMODWT(np.zeros(8), 14)
    with pytest.raises(ValueError, match="exceeds theoretical limit 3 for signal length 10"):
        m.forwardMODWT(np.zeros(10), 4)
    assert m.forwardMODWT(np.zeros(0), 3).shape == (4, 0)
    assert m.inverseMODWT(np.zeros((1, 5))).shape == (0,)
    # the facade prints and returns None (Transform.java:81-90)
    assert jw.Transform(fwt).forward(np.zeros(12), 1) is None


# ------------------------------------------------------------------- C ABI
def test_abi_exports_every_header_symbol():
    lib = _lib.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 40
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert lib.jwv_version() >= 100


def test_abi_no_device_reports_error():
    """Without a GPU the library loads and refuses a context loudly (no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import ctypes
    lib = _lib.lib()
    h = ctypes.c_void_p()
    assert lib.jwv_ctx_create(0, ctypes.byref(h)) == _lib.JWV_ERR_DEVICE
    assert b"device" in lib.jwv_last_error(None)
    with pytest.raises(jw.JWaveError):
        jw.Context(0)


def test_abi_modwt_filters_host_only():
    g, h = jw.modwt_filters(jw.by_class("Daubechies4"))
    go, ho = oracle.modwt_filters(jw.by_class("Daubechies4"))
    assert np.array_equal(g, go) and np.array_equal(h, ho)


def test_decompose_number_ancient_egyptian():
    """MathToolKit.decompose (tools/MathToolKit.java:57-80, :97-138): powers
    largest first; the blocked form returns the block size itself for the
    blocks (reference behaviour, see its Javadoc example 127 / 32)."""
    import jwave_amd as jw
    assert jw.decompose_number(42) == [5, 3, 1]        # Javadoc: 42 = 2^5 + 2^3 + 2^1
    assert jw.decompose_number(1) == [0]
    assert jw.decompose_number(1024) == [10]
    assert jw.decompose_number(127, 32) == [32, 32, 32, 4, 3, 2, 1, 0]
    for n in (3, 7, 1000, 65535, 10 ** 7):
        ps = jw.decompose_number(n)
        assert sum(1 << p for p in ps) == n and ps == sorted(ps, reverse=True)
    with pytest.raises(jw.JWaveFailure, match="smaller than one"):
        jw.decompose_number(0)
    with pytest.raises(jw.JWaveFailure, match="block size is not 2"):
        jw.decompose_number(100, 24)
    with pytest.raises(jw.JWaveFailure, match="greater than the given number"):
        jw.decompose_number(10, 16)


def _tree_sum(a, np_, rb=256):
    """launch_compress.hip's fixed two-level tree, restated: grid-stride
    per-thread sums, a block halving tree, then the same over the partials."""
    def block(vals):
        red = list(vals) + [0.0] * (rb - len(vals))
        s = rb // 2
        while s:
            for i in range(s):
                red[i] = red[i] + red[i + s]
            s //= 2
        return red[0]
    n = len(a)
    partial = []
    for b in range(np_):
        th = []
        for t in range(rb):
            s = 0.0
            for i in range(b * rb + t, n, np_ * rb):
                s += float(a[i])
            th.append(s)
        partial.append(block(th))
    th = []
    for t in range(rb):
        s = 0.0
        for i in range(t, np_, rb):
            s += partial[i]
        th.append(s)
    return block(th)


@pytest.mark.parametrize("n,seed,scale", [(1000, 1, 1.0), (4099, 2, 1e-300), (6000, 3, 1e300),
                                          (2048, 4, 1.0)])
def test_compress_band_contains_java_cut(n, seed, scale):
    """The n*eps band of launch_compress.hip around the tree sum always holds
    Java's left-to-right cut (CompressorMagnitude.java:78-82), so a coefficient
    outside [cut_lo, cut_hi) is decided as Java decides it."""
    rng = np.random.default_rng(seed)
    a = np.abs(rng.standard_normal(n) * rng.choice([1.0, 1e8, 1e-8], n)) * scale
    np_ = max(1, min(1024, (n + 2047) // 2048))
    tot = _tree_sum(a, np_)
    s_j = 0.0
    for v in a:
        s_j += float(v)
    rel = 2.0 * (n + 64.0) * 2.0 ** -53 * 1.01
    band = tot * rel + (n + 1.0) * 2.0 ** -1074
    lo = max(float(np.nextafter(tot - band, 0.0)), 0.0)
    hi = float(np.nextafter(tot + band, np.inf))
    for thr in (1.0, 0.37, 2.5):
        cut = lambda s: (s / float(n)) * thr
        if np.isfinite(hi):
            assert cut(lo) <= cut(s_j) <= cut(hi)
