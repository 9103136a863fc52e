"""GPU parity: libjwave_hip.so (through the C ABI) vs the CPU oracle.

Bar: EXACT math is bit-identical to the oracle (which evaluates the Java loops
in the Java order without FMA).  FMA math: |diff| <= 1e-12 * max(1, max|ref|)
(BASELINE.md parity gates).  Round trips are additionally compared with the
input.  Sizes cover both kernel shapes (resident <= 8192 per signal, tiled
above), wrap-around at every level, tiny levels (h < L), odd / long / scaled
banks and non power-of-two MODWT lengths.
"""
import numpy as np
import pytest

import oracle
import jwave_amd as jw
from jwave_amd import transforms as T

pytestmark = pytest.mark.gpu

FMA_TOL = 1e-12

# config wavelets + the generic-kernel cases (odd L, long L, scaled, tw=8, biorthogonal)
WAVELETS = ["Haar1", "Daubechies2", "Daubechies4", "Daubechies8", "Symlet8", "Coiflet1",
            "Daubechies20", "Haar1Orthogonal", "BiOrthogonal13", "BiOrthogonal35", "CDF53",
            "Battle23", "DiscreteMeyer", "Legendre3", "Symlet2"]


def rnd(n, seed=42):
    return oracle.java_random_doubles(seed, n)


def assert_exact(got, ref, what=""):
    got = np.asarray(got)
    if not np.array_equal(got, ref):
        d = np.abs(got - ref)
        i = int(np.argmax(d))
        raise AssertionError("%s not bit-exact: max|diff|=%g at %d (got %r ref %r)"
                             % (what, d.max(), i, got.flat[i], ref.flat[i]))


def assert_close(got, ref, what=""):
    got = np.asarray(got)
    tol = FMA_TOL * max(1.0, float(np.abs(ref).max()) if ref.size else 1.0)
    d = float(np.abs(got - ref).max()) if ref.size else 0.0
    assert d <= tol, "%s: max|diff| %g > %g" % (what, d, tol)


def levels_for(n, w):
    full = int(n).bit_length() - 1
    return sorted({0, 1, full // 2, full})


# ------------------------------------------------------------------ 1-D FWT
@pytest.mark.parametrize("wname", WAVELETS)
def test_fwt_small_all_levels(ctx, wname):
    w = jw.by_class(wname)
    for n in (1, 2, 4, 8, 16, 32, 64, 256, 1024):
        x = rnd(n, 7 + n)
        for lev in range(0, int(n).bit_length()):
            y = T.fwt_forward(x, w, lev, ctx)
            assert_exact(y, oracle.fwt_forward(w, x, lev), "%s fwd n=%d l=%d" % (wname, n, lev))
            xr = T.fwt_reverse(y, w, lev, ctx)
            assert_exact(xr, oracle.fwt_reverse(w, np.asarray(y), lev),
                         "%s rev n=%d l=%d" % (wname, n, lev))


@pytest.mark.parametrize("wname", WAVELETS)
@pytest.mark.parametrize("n", [8192, 16384, 1 << 16, 1 << 18])
def test_fwt_large(ctx, wname, n):
    w = jw.by_class(wname)
    x = rnd(n, n)
    for lev in levels_for(n, w):
        y = T.fwt_forward(x, w, lev, ctx)
        yr = oracle.fwt_forward(w, x, lev)
        assert_exact(y, yr, "%s fwd n=%d l=%d" % (wname, n, lev))
        xr = T.fwt_reverse(yr, w, lev, ctx)
        assert_exact(xr, oracle.fwt_reverse(w, yr, lev), "%s rev n=%d l=%d" % (wname, n, lev))


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Daubechies8", "Symlet8", "Coiflet1"])
def test_fwt_fma_mode(ctx_fma, wname):
    w = jw.by_class(wname)
    for n in (64, 4096, 1 << 15, 1 << 17):
        x = rnd(n, 3)
        lev = int(n).bit_length() - 1
        yr = oracle.fwt_forward(w, x, lev)
        assert_close(T.fwt_forward(x, w, lev, ctx_fma), yr, "fma fwd %s %d" % (wname, n))
        assert_close(T.fwt_reverse(yr, w, lev, ctx_fma), oracle.fwt_reverse(w, yr, lev),
                     "fma rev %s %d" % (wname, n))


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Symlet8", "Coiflet1"])
def test_fwt_batch(ctx, wname):
    w = jw.by_class(wname)
    for b, n in ((5, 64), (3, 8192), (2, 32768)):
        x = np.stack([rnd(n, 100 + i) for i in range(b)])
        for lev in (1, int(n).bit_length() - 1):
            y = T.fwt_forward(x, w, lev, ctx)
            yr = oracle.batch("fwt", True, w, x, lev)
            assert_exact(y, yr, "batch fwd")
            assert_exact(T.fwt_reverse(yr, w, lev, ctx), oracle.batch("fwt", False, w, yr, lev),
                         "batch rev")


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies2", "Daubechies4", "Daubechies8", "Symlet8"])
@pytest.mark.parametrize("n", [1 << 18, 1 << 20, 1 << 21])
def test_fwt_chain(ctx, wname, n):
    """Pass plans for long single signals (fwt1_chain.hpp: reverse head,
    whole-direction chains, multi-launch): every level count that switches roles
    on or off (forward chain from 13 levels, reverse chain when the resident
    part fits), each call twice in a row so a counter or flag left behind by
    the first would corrupt the second."""
    w = jw.by_class(wname)
    x = rnd(n, n + 1)
    full = n.bit_length() - 1
    try:
        for plan in ({"rev_head"}, {"rev_head", "fwd_tail"}, {"chain_rev", "chain_fwd"}, set()):
            ctx.set_plan(plan)
            for lev in sorted({12, 13, 14, 15, full - 1, full}):
                yr = oracle.fwt_forward(w, x, lev)
                tag = "%s n=%d l=%d plan=%s" % (wname, n, lev, sorted(plan))
                for rep in range(2):
                    assert_exact(T.fwt_forward(x, w, lev, ctx), yr, "fwd %s #%d" % (tag, rep))
                xr = oracle.fwt_reverse(w, yr, lev)
                for rep in range(2):
                    assert_exact(T.fwt_reverse(yr, w, lev, ctx), xr, "rev %s #%d" % (tag, rep))
            ctx.synchronize()  # raises if a chained wait timed out
    finally:
        ctx.set_plan()


def test_chain_wait_timeout_is_an_error(ctx):
    """A bounded in-kernel wait that gives up must fail the call
    (JWV_ERR_DEVICE -> JWaveError), never return rc = 0 with invalid data
    (the error contract of Transform.java:83-89 / SURVEY 8b).  A poll bound of
    one forces the timeout in the chained reverse; the default plan has no
    inter-workgroup wait at all and stays bit-exact under the same bound."""
    w = jw.by_class("Daubechies4")
    n = 1 << 20
    x = rnd(n, 5)
    y = oracle.fwt_forward(w, x, 20)
    xr = oracle.fwt_reverse(w, y, 20)
    try:
        ctx.set_poll_limit(1)
        ctx.set_plan({"chain_rev"})
        with pytest.raises(jw.JWaveError, match="timed out"):
            T.fwt_reverse(y, w, 20, ctx)
        ctx.set_plan()  # default: reverse head, no wait -> unaffected by the bound
        assert_exact(T.fwt_reverse(y, w, 20, ctx), xr, "rev head under poll bound 1")
    finally:
        ctx.set_poll_limit(0)
        ctx.set_plan()
    ctx.set_plan({"chain_rev"})
    try:
        assert_exact(T.fwt_reverse(y, w, 20, ctx), xr, "chained rev after the timeout")
    finally:
        ctx.set_plan()


def test_dev_entry_rejects_foreign_pointers(ctx):
    """_dev entry points accept only device memory of the context's device."""
    import ctypes
    from jwave_amd import _lib as L
    w = jw.by_class("Daubechies4")
    t = T._TapsHolder.of(w)
    lib = L.lib()
    host = np.zeros(64)
    hp = ctypes.c_void_p(host.ctypes.data)
    rc = lib.jwv_fwt_fwd_f64_dev(hp, hp, 64, 6, t, ctx.handle)
    assert rc == L.JWV_ERR_BAD_CALL
    assert b"host pointer" in lib.jwv_last_error(ctx.handle) or \
        b"not a HIP device pointer" in lib.jwv_last_error(ctx.handle)


# north_star gate: the forward -> reverse round trip matches the Java
# reference's round trip within 1e-12 max-abs on the same inputs.  EXACT math
# is bit-identical (0); FMA math is held to the gate itself.
RT_GATE = 1e-12


def test_fwt_config2_full_size(ctx, ctx_fma):
    """Config 2: Daubechies4, N = 2^24, full depth — exact vs oracle, and the
    round trip vs the input (reported bound from the taps' precision).  FMA:
    round trip within RT_GATE of the oracle's (Java-order) round trip."""
    w = jw.by_class("Daubechies4")
    n = 1 << 24
    x = rnd(n, 42)
    y = T.fwt_forward(x, w, 24, ctx)
    yr = oracle.fwt_forward(w, x, 24)
    assert_exact(y, yr, "D4 2^24 fwd")
    xr = T.fwt_reverse(y, w, 24, ctx)
    xr_ref = oracle.fwt_reverse(w, yr, 24)
    assert_exact(xr, xr_ref, "D4 2^24 rev")
    assert np.abs(xr - x).max() < 1e-11
    rt = T.fwt_reverse(T.fwt_forward(x, w, 24, ctx_fma), w, 24, ctx_fma)
    assert np.abs(rt - xr_ref).max() <= RT_GATE


# ------------------------------------------------------------------ WPT
@pytest.mark.parametrize("wname", WAVELETS)
def test_wpt_small(ctx, wname):
    w = jw.by_class(wname)
    for n in (2, 4, 16, 64, 1024, 8192):
        x = rnd(n, 11 + n)
        for lev in levels_for(n, w):
            y = T.wpt_forward(x, w, lev, ctx)
            yr = oracle.wpt_forward(w, x, lev)
            assert_exact(y, yr, "%s wpt fwd n=%d l=%d" % (wname, n, lev))
            assert_exact(T.wpt_reverse(yr, w, lev, ctx), oracle.wpt_reverse(w, yr, lev),
                         "%s wpt rev n=%d l=%d" % (wname, n, lev))


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Symlet8", "Coiflet1", "Battle23"])
@pytest.mark.parametrize("n", [16384, 1 << 16, 1 << 17])
def test_wpt_large(ctx, wname, n):
    w = jw.by_class(wname)
    x = rnd(n, 5)
    full = int(n).bit_length() - 1
    for lev in (1, 6, 8, full):
        y = T.wpt_forward(x, w, lev, ctx)
        yr = oracle.wpt_forward(w, x, lev)
        assert_exact(y, yr, "%s wpt fwd n=%d l=%d" % (wname, n, lev))
        assert_exact(T.wpt_reverse(yr, w, lev, ctx), oracle.wpt_reverse(w, yr, lev),
                     "%s wpt rev n=%d l=%d" % (wname, n, lev))


def test_wpt_config4_shape(ctx, ctx_fma):
    """Config 4 shape (Symlet8, 6 levels, N=65536) on a small batch; FMA too."""
    w = jw.by_class("Symlet8")
    x = np.stack([rnd(1 << 16, 42 + i) for i in range(4)])
    yr = oracle.batch("wpt", True, w, x, 6)
    assert_exact(T.wpt_forward(x, w, 6, ctx), yr, "wpt cfg4 fwd")
    xr_ref = oracle.batch("wpt", False, w, yr, 6)
    assert_exact(T.wpt_reverse(yr, w, 6, ctx), xr_ref, "wpt cfg4 rev")
    assert_close(T.wpt_forward(x, w, 6, ctx_fma), yr, "wpt cfg4 fwd fma")
    assert_close(T.wpt_reverse(yr, w, 6, ctx_fma), xr_ref, "wpt cfg4 rev fma")


def assert_bits(got, ref, what=""):
    """Bit-for-bit, signed zeros included (np.array_equal has -0.0 == +0.0)."""
    got = np.ascontiguousarray(np.asarray(got, dtype=np.float64))
    ref = np.ascontiguousarray(ref)
    gb, rb = got.view(np.int64), ref.view(np.int64)
    bad = np.flatnonzero(gb != rb)
    assert bad.size == 0, "%s: %d values differ in their bits, first at %d (got %r ref %r)" % (
        what, bad.size, bad[0], got.flat[bad[0]], ref.flat[bad[0]])


@pytest.mark.parametrize("wname", ["Symlet8", "Daubechies4", "Haar1", "Coiflet1", "Daubechies8"])
def test_wpt_signed_zeros(ctx, wname):
    """The WPT tiles' LDS-only levels start each sum at its first product
    (fwt_kernels.hpp, ZS): values identical, a zero's sign possibly not, until
    the level that writes HBM starts from +0.0 again.  Inputs with runs of
    +0.0 / -0.0 and isolated values make many outputs exact zeros of both
    product signs; every output must match Java's bits, zero signs included."""
    w = jw.by_class(wname)
    rng = np.random.default_rng(7)
    n, B = 1 << 16, 3
    x = np.stack([rnd(n, 31 + i) for i in range(B)])
    z = rng.random((B, n))
    x[z < 0.45] = 0.0
    x[(z >= 0.45) & (z < 0.75)] = -0.0
    for b in range(B):
        for s0 in rng.integers(0, n - 4096, 8):
            x[b, s0:s0 + int(rng.integers(64, 4096))] = -0.0 if s0 & 1 else 0.0
    for lev in (1, 3, 6, 9):
        yr = oracle.batch("wpt", True, w, x, lev)
        assert_bits(T.wpt_forward(x, w, lev, ctx), yr, "%s wpt fwd l=%d" % (wname, lev))
        # coefficients with signed-zero runs for the reverse
        yz = yr.copy()
        yz[z < 0.3] = -0.0
        assert_bits(T.wpt_reverse(yz, w, lev, ctx), oracle.batch("wpt", False, w, yz, lev),
                    "%s wpt rev l=%d" % (wname, lev))


@pytest.mark.parametrize("n,J", [(1 << 16, 8), (100003, 8), (50000, 5)])
def test_modwt_signed_zeros(ctx, n, J):
    """The MODWT inverse's LDS-only levels start each sum at its first
    product (modwt1_kernels.hpp, JWV_MOD_NZS): inputs with +0.0 / -0.0 runs
    (zero outputs of both product signs) must still give Java's bits at every
    output, zero signs included, forward and inverse."""
    w = jw.by_class("Daubechies4")
    rng = np.random.default_rng(11)
    x = rnd(n, 77)
    z = rng.random(n)
    x[z < 0.4] = 0.0
    x[(z >= 0.4) & (z < 0.7)] = -0.0
    for s0 in rng.integers(0, n - 3000, 6):
        x[s0:s0 + int(rng.integers(300, 3000))] = -0.0 if s0 & 1 else 0.0
    c_ref = oracle.modwt_forward(w, x, J)
    assert_bits(T.modwt_forward(x, w, J, ctx), c_ref, "modwt fwd n=%d J=%d" % (n, J))
    cz = c_ref.copy()
    cz[:, rng.random(n) < 0.3] = -0.0
    assert_bits(T.modwt_inverse(cz, w, ctx), oracle.modwt_inverse(w, cz), "modwt inv n=%d J=%d" % (n, J))


@pytest.mark.parametrize("B", [3, 64, 97])
def test_wpt_batch_runs(ctx, B):
    """Batches whose rows the streamed kernels share out in runs of tiles
    that start and end inside rows: every row exact."""
    w = jw.by_class("Symlet8")
    x = np.stack([rnd(1 << 16, 900 + i) for i in range(B)])
    yr = oracle.batch("wpt", True, w, x, 6)
    assert_exact(T.wpt_forward(x, w, 6, ctx), yr, "wpt batch %d fwd" % B)
    assert_exact(T.wpt_reverse(yr, w, 6, ctx), oracle.batch("wpt", False, w, yr, 6),
                 "wpt batch %d rev" % B)


def test_wpt_config4_full_batch(ctx, ctx_fma):
    """Config 4 at its full shape in ONE call per direction: 4096 Symlet8
    signals x 65536, 6 levels (WaveletPacketTransform.java:73-191 per signal),
    2 GiB per buffer.  Sampled signals -- first, last, both sides of the
    signal-2048 midpoint (byte offset 2^30) and the last signal (ending at
    byte 2^31) -- are bit-exact against the oracle in EXACT math.  FMA math:
    the round trip's absolute error against the oracle's EXACT round trip is
    <= 1e-12 (the north_star gate), on the sampled signals and, against the
    input, on the whole batch."""
    import torch
    B, n, lev = 4096, 1 << 16, 6
    w = jw.by_class("Symlet8")
    gen = torch.Generator(device="cuda:0").manual_seed(4096)
    x = torch.rand(B, n, dtype=torch.float64, device="cuda:0", generator=gen)
    sample = [0, 1, 777, 2047, 2048, 2049, 3333, 4094, 4095]
    xs = x[sample].cpu().numpy()
    y = T.wpt_forward(x, w, lev, ctx)
    ys_ref = oracle.batch("wpt", True, w, xs, lev)
    assert_exact(y[sample].cpu().numpy(), ys_ref, "wpt cfg4 full batch fwd")
    xr = T.wpt_reverse(y, w, lev, ctx)
    xrs_ref = oracle.batch("wpt", False, w, ys_ref, lev)
    assert_exact(xr[sample].cpu().numpy(), xrs_ref, "wpt cfg4 full batch rev")
    del xr, y
    yf = T.wpt_forward(x, w, lev, ctx_fma)
    xrf = T.wpt_reverse(yf, w, lev, ctx_fma)
    del yf
    rt_vs_exact = float(np.abs(xrf[sample].cpu().numpy() - xrs_ref).max())
    rt_vs_input = float((xrf - x).abs().max().item())
    assert rt_vs_exact <= 1e-12, "FMA round trip vs EXACT round trip: %g" % rt_vs_exact
    assert rt_vs_input <= 1e-12, "FMA round trip vs input: %g" % rt_vs_input
    torch.cuda.synchronize()


# ------------------------------------------------------------------ 2-D / 3-D
@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Daubechies8", "Coiflet1", "Battle23"])
@pytest.mark.parametrize("shape", [(2, 2), (8, 4), (64, 64), (256, 32), (32, 256), (2048, 16),
                                   (16, 16384), (4096, 64)])
def test_fwt2d(ctx, wname, shape):
    w = jw.by_class(wname)
    r, c = shape
    x = rnd(r * c, r + c).reshape(r, c)
    for lm, ln in ((r.bit_length() - 1, c.bit_length() - 1), (1, 1), (0, c.bit_length() - 1)):
        y = T.transform_2d(x, w, lm, ln, True, ctx)
        yr = oracle.transform_2d("fwt", True, w, x, lm, ln)
        assert_exact(y, yr, "2d fwd %s %s" % (wname, shape))
        assert_exact(T.transform_2d(yr, w, lm, ln, False, ctx),
                     oracle.transform_2d("fwt", False, w, yr, lm, ln), "2d rev")


@pytest.mark.parametrize("wname", ["Daubechies4", "Daubechies8"])
@pytest.mark.parametrize("shape", [(64, 8192), (128, 4096), (64, 4096), (256, 16384)])
def test_fwt2d_rowcap(ctx, ctx_fma, wname, shape):
    """The row pass of >= 64 rows longer than 2048 samples (capi.cpp fwt_res_cap):
    fwt_fwd_tile1 passes down to a 2048-sample resident tail forward, the fwt1
    tiled reverse above a short resident head.  Config 3 takes this branch.
    Full and partial levels; EXACT bit-exact, FMA within 1e-12*max|c|."""
    w = jw.by_class(wname)
    r, c = shape
    x = rnd(r * c, r ^ c).reshape(r, c)
    fm, fn = r.bit_length() - 1, c.bit_length() - 1
    for lm, ln in ((fm, fn), (2, fn - 1), (fm, 3), (0, fn)):
        yr = oracle.transform_2d("fwt", True, w, x, lm, ln)
        assert_exact(T.transform_2d(x, w, lm, ln, True, ctx), yr,
                     "2d fwd %s %s l=(%d,%d)" % (wname, shape, lm, ln))
        xr = oracle.transform_2d("fwt", False, w, yr, lm, ln)
        assert_exact(T.transform_2d(yr, w, lm, ln, False, ctx), xr,
                     "2d rev %s %s l=(%d,%d)" % (wname, shape, lm, ln))
        if (lm, ln) == (fm, fn):
            assert_close(T.transform_2d(x, w, lm, ln, True, ctx_fma), yr, "2d fwd fma")
            assert_close(T.transform_2d(yr, w, lm, ln, False, ctx_fma), xr, "2d rev fma")


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies2", "Daubechies4", "Daubechies8"])
@pytest.mark.parametrize("shape", [(2048, 2048), (512, 8192), (1024, 4096), (8192, 512),
                                   (4096, 1024)])
def test_fwt2d_overlapped_schedule(ctx, ctx_fma, wname, shape):
    """Matrices of >= 2^22 elements take the overlapped 2-D schedule
    (capi.cpp body_2d_fwt): row / column resident passes on side streams
    beside the tile passes of independent column groups.  Every column runs
    its serial plan, so the result must stay bit-exact at full and partial
    levels on both axes (partial levels move or remove the resident passes
    and the group [0, hr))."""
    w = jw.by_class(wname)
    r, c = shape
    x = rnd(r * c, r + 3 * c).reshape(r, c)
    fm, fn = r.bit_length() - 1, c.bit_length() - 1
    for lm, ln in ((fm, fn), (3, fn), (fm, 2), (0, fn), (fm, 0), (fm - 1, fn - 3)):
        yr = oracle.transform_2d("fwt", True, w, x, lm, ln)
        assert_exact(T.transform_2d(x, w, lm, ln, True, ctx), yr,
                     "2d fwd %s %s l=(%d,%d)" % (wname, shape, lm, ln))
        xr = oracle.transform_2d("fwt", False, w, yr, lm, ln)
        assert_exact(T.transform_2d(yr, w, lm, ln, False, ctx), xr,
                     "2d rev %s %s l=(%d,%d)" % (wname, shape, lm, ln))
        if (lm, ln) == (fm, fn) and wname == "Daubechies8":
            assert_close(T.transform_2d(x, w, lm, ln, True, ctx_fma), yr, "2d fwd fma")
            assert_close(T.transform_2d(yr, w, lm, ln, False, ctx_fma), xr, "2d rev fma")


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Daubechies8", "Symlet8", "Coiflet1",
                                   "BiOrthogonal35", "Daubechies20"])
@pytest.mark.parametrize("shape", [(64, 8192, 1024), (32, 8192, 2048), (16, 65536, 8192),
                                   (8, 4096, 4096), (64, 16384, 16384), (8, 8192, 512),
                                   (3, 2048, 256), (1, 8192, 1024), (40, 32768, 1024)])
def test_fwt_rows_chunked(ctx, ctx_fma, wname, shape):
    """jwv_fwt_rows_seg_{fwd,rev}_f64_dev (the sharded 2-D transform's row
    passes): values of the plain batched row FWT, laid out [cols/seg][rows][seg].
    seg >= 1024 with >= 2 rows on the fast banks runs the row kernels with
    chunked addressing (no copy launch); short chunks, one row and the generic
    banks take the plain pass + one packing copy (as do partial levels whose
    approximation prefix outgrows the first chunk).  Full and partial levels."""
    import torch
    w = jw.by_class(wname)
    rows, cols, seg = shape
    x = rnd(rows * cols, rows + 5 * cols + seg).reshape(rows, cols)
    xd = torch.from_numpy(x).cuda()
    full = cols.bit_length() - 1
    fast = wname in ("Haar1", "Daubechies4", "Daubechies8", "Symlet8")  # static-L banks

    def chunk(a):
        return np.ascontiguousarray(a.reshape(rows, cols // seg, seg).transpose(1, 0, 2))

    for lev in sorted({0, 1, 5, full - 3, full}):
        yr = oracle.batch("fwt", True, w, x, lev)
        ctx.profile(True)
        y = T.fwt_rows_to_chunks(xd, w, lev, seg, ctx)
        prof = ctx.profile_read()
        ctx.profile(False)
        assert tuple(y.shape) == (cols // seg, rows, seg)
        assert_exact(y.cpu().numpy(), chunk(yr), "seg fwd %s %s l=%d" % (wname, shape, lev))
        if fast and rows >= 2 and seg >= 1024 and lev == full and cols > 8192:
            assert "copy_axis" not in prof, "seg fwd packed with a copy: %s" % sorted(prof)
        xr = oracle.batch("fwt", False, w, yr, lev)
        yd = torch.from_numpy(chunk(yr)).cuda()
        ctx.profile(True)
        got = T.fwt_chunks_to_rows(yd, w, lev, ctx)
        prof = ctx.profile_read()
        ctx.profile(False)
        assert_exact(got.cpu().numpy(), xr, "seg rev %s %s l=%d" % (wname, shape, lev))
        if fast and rows >= 2 and seg >= 1024 and lev == full and cols > 8192:
            assert "copy_axis" not in prof, "seg rev unpacked with a copy: %s" % sorted(prof)
        if lev == full and wname == "Daubechies8":
            assert_close(T.fwt_rows_to_chunks(xd, w, lev, seg, ctx_fma).cpu().numpy(), chunk(yr),
                         "seg fwd fma")
            assert_close(T.fwt_chunks_to_rows(yd, w, lev, ctx_fma).cpu().numpy(), xr,
                         "seg rev fma")


def test_fwt_rows_chunked_errors(ctx):
    import torch
    w = jw.by_class("Daubechies4")
    xd = torch.zeros((4, 4096), dtype=torch.float64, device="cuda")
    with pytest.raises(jw.JWaveError):
        T.fwt_rows_to_chunks(xd, w, 12, 1, ctx)           # seg < 2
    with pytest.raises(jw.JWaveError):
        T.fwt_rows_to_chunks(xd, w, 12, 3000, ctx)        # does not divide cols
    with pytest.raises(jw.JWaveError):
        T.fwt_rows_to_chunks(xd[:, :3000].contiguous(), w, 3, 1000, ctx)  # not 2^p
    with pytest.raises(jw.JWaveFailure, match="level is out of range"):
        T.fwt_rows_to_chunks(xd, w, 13, 1024, ctx)        # the reference's own check


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies2", "Daubechies4", "Daubechies8", "Symlet8"])
def test_fwt_batch_rowcap(ctx, wname):
    """Batched 1-D FWT, 64 signals x 8192 (>= 64 rows, > 2048 samples: the
    row-cap branch), and 100 x 4096 (not a multiple of 8 rows), all levels
    the planner treats differently."""
    w = jw.by_class(wname)
    for b, n in ((64, 8192), (100, 4096)):
        x = rnd(b * n, b + n).reshape(b, n)
        full = n.bit_length() - 1
        for lev in (1, 2, 6, 9, full - 1, full):
            yr = oracle.batch("fwt", True, w, x, lev)
            assert_exact(T.fwt_forward(x, w, lev, ctx), yr, "batch fwd %d x %d l=%d" % (b, n, lev))
            assert_exact(T.fwt_reverse(yr, w, lev, ctx), oracle.batch("fwt", False, w, yr, lev),
                         "batch rev %d x %d l=%d" % (b, n, lev))


@pytest.mark.parametrize("wname", ["Daubechies4", "Daubechies8"])
def test_3d_long_lines(ctx, wname):
    """3-D block whose innermost lines exceed 2048 samples with >= 64 of them
    (the row-cap branch inside the slice 2-D pass), plus strided axes."""
    w = jw.by_class(wname)
    shape = (4, 16, 4096)
    p, q, r = shape
    x = rnd(p * q * r, 23).reshape(shape)
    for lp, lq, lr in ((4, 12, 2), (2, 9, 1)):
        yr = oracle.transform_3d("fwt", True, w, x, lp, lq, lr)
        assert_exact(T.transform_3d(x, w, lp, lq, lr, True, ctx), yr, "3d fwd")
        assert_exact(T.transform_3d(yr, w, lp, lq, lr, False, ctx),
                     oracle.transform_3d("fwt", False, w, yr, lp, lq, lr), "3d rev")


@pytest.mark.parametrize("wname", ["Daubechies4", "Daubechies8", "Symlet8", "Coiflet1"])
def test_fwt2d_column_tail(ctx, ctx_fma, wname):
    """The column passes' resident tails over 1024 rows (fwt_colres.hpp,
    compile-time geometry, 8-column slabs: fwt_fwd_cres8 / fwt_rev_cres8) at
    every level count, both directions: matrices of 1024 rows (the tails from
    level 0 / up to the full size) and 8192 rows (beside the tile passes),
    slab counts that are and are not whole XCD pairs."""
    w = jw.by_class(wname)
    for r, c in ((1024, 64), (1024, 256), (8192, 32)):
        x = rnd(r * c, r + c).reshape(r, c)
        for lm in range(1, r.bit_length()):
            ln = 3
            yr = oracle.transform_2d("fwt", True, w, x, lm, ln)
            assert_exact(T.transform_2d(x, w, lm, ln, True, ctx), yr,
                         "%s col tail %dx%d lm=%d" % (wname, r, c, lm))
            assert_close(T.transform_2d(x, w, lm, ln, True, ctx_fma), yr,
                         "%s col tail fma %dx%d lm=%d" % (wname, r, c, lm))
            xr = oracle.transform_2d("fwt", False, w, yr, lm, ln)
            assert_exact(T.transform_2d(yr, w, lm, ln, False, ctx), xr,
                         "%s col tail rev %dx%d lm=%d" % (wname, r, c, lm))
            assert_close(T.transform_2d(yr, w, lm, ln, False, ctx_fma), xr,
                         "%s col tail rev fma %dx%d lm=%d" % (wname, r, c, lm))


@pytest.mark.parametrize("wname", ["Daubechies4", "Daubechies8", "Coiflet1"])
def test_fwt2d_row_tail(ctx, ctx_fma, wname):
    """The row passes' reverse resident tail over 1024-sample row tops
    (fwt_rev_rres8: 8 rows per block, compile-time levels) at every level
    count: rows of 1024 (the tail up to the full row) and 8192 samples (under
    the tile pass); a batch of 72 signals (a partial last block)."""
    w = jw.by_class(wname)
    for r, c in ((64, 1024), (64, 8192)):
        x = rnd(r * c, 7 * r + c).reshape(r, c)
        for ln in range(1, c.bit_length()):
            lm = 1 if ln % 3 == 0 else 0
            yr = oracle.transform_2d("fwt", True, w, x, lm, ln)
            xr = oracle.transform_2d("fwt", False, w, yr, lm, ln)
            assert_exact(T.transform_2d(yr, w, lm, ln, False, ctx), xr,
                         "%s row tail rev %dx%d ln=%d" % (wname, r, c, ln))
            assert_close(T.transform_2d(yr, w, lm, ln, False, ctx_fma), xr,
                         "%s row tail rev fma %dx%d ln=%d" % (wname, r, c, ln))
    # a batch of 72 signals (2-D shapes are powers of two): partial last block
    x = np.stack([rnd(1024, 300 + i) for i in range(72)])
    for lev in (1, 4, 10):
        yr = oracle.batch("fwt", True, w, x, lev)
        assert_exact(T.fwt_reverse(yr, w, lev, ctx), oracle.batch("fwt", False, w, yr, lev),
                     "%s row tail rev batch 72 lev=%d" % (wname, lev))


def test_fwt2d_config3_full_size(ctx, ctx_fma):
    """Config 3 at full size: Daubechies8, 8192 x 8192, levels 13 x 13
    (BasicTransform.java:361-474), both directions bit-exact vs the oracle in
    EXACT mode and within 1e-12*max|c| in FMA mode; round trip vs the input."""
    w = jw.by_class("Daubechies8")
    n = 8192
    x = rnd(n * n, 42).reshape(n, n)
    yr = oracle.transform_2d("fwt", True, w, x, 13, 13)
    y = T.transform_2d(x, w, 13, 13, True, ctx)
    assert_exact(y, yr, "config 3 fwd")
    assert_close(T.transform_2d(x, w, 13, 13, True, ctx_fma), yr, "config 3 fwd fma")
    del y
    xr = oracle.transform_2d("fwt", False, w, yr, 13, 13)
    got = T.transform_2d(yr, w, 13, 13, False, ctx)
    assert_exact(got, xr, "config 3 rev")
    assert_close(T.transform_2d(yr, w, 13, 13, False, ctx_fma), xr, "config 3 rev fma")
    assert np.abs(got - x).max() < 1e-10
    del got
    rt = T.transform_2d(T.transform_2d(x, w, 13, 13, True, ctx_fma), w, 13, 13, False, ctx_fma)
    d = float(np.abs(rt - xr).max())
    assert d <= RT_GATE, "config 3 FMA round trip vs oracle round trip: %g" % d


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Symlet8"])
def test_wpt2d(ctx, wname):
    w = jw.by_class(wname)
    x = rnd(64 * 128, 9).reshape(64, 128)
    y = T.transform_2d(x, w, 6, 7, True, ctx, kind="wpt")
    yr = oracle.transform_2d("wpt", True, w, x, 6, 7)
    assert_exact(y, yr, "wpt2d fwd")
    assert_exact(T.transform_2d(yr, w, 6, 7, False, ctx, kind="wpt"),
                 oracle.transform_2d("wpt", False, w, yr, 6, 7), "wpt2d rev")


@pytest.mark.parametrize("kind", ["fwt", "wpt"])
@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Daubechies8"])
@pytest.mark.parametrize("shape", [(2, 4, 8), (16, 32, 64), (8, 8, 8), (64, 16, 2048)])
def test_3d(ctx, kind, wname, shape):
    """3-D BasicTransform.forward/reverse (BasicTransform.java:487-659) for the
    FWT and for the packet transform (jwv_wpt3d_*, the Java plugin's 3-D WPT
    route) against the oracle's restatement, every axis at full depth."""
    w = jw.by_class(wname)
    p, q, r = shape
    x = rnd(p * q * r, 17).reshape(shape)
    # levels as the reference applies them: (lvlP on Q, lvlQ on R, lvlR on P)
    lp, lq, lr = q.bit_length() - 1, r.bit_length() - 1, p.bit_length() - 1
    y = T.transform_3d(x, w, lp, lq, lr, True, ctx, kind=kind)
    yr = oracle.transform_3d(kind, True, w, x, lp, lq, lr)
    assert_exact(y, yr, "%s 3d fwd" % kind)
    assert_exact(T.transform_3d(yr, w, lp, lq, lr, False, ctx, kind=kind),
                 oracle.transform_3d(kind, False, w, yr, lp, lq, lr), "%s 3d rev" % kind)
    if kind == "wpt":  # partial depth on every axis as well
        y = T.transform_3d(x, w, lp // 2, lq // 2, lr // 2, True, ctx, kind=kind)
        assert_exact(y, oracle.transform_3d(kind, True, w, x, lp // 2, lq // 2, lr // 2),
                     "wpt 3d fwd partial")


# ------------------------------------------------------------------ MODWT
@pytest.mark.parametrize("wname", ["Haar1", "Daubechies2", "Daubechies4", "Daubechies8",
                                   "Symlet8", "Coiflet1", "Daubechies20", "CDF53"])
def test_modwt(ctx, wname):
    w = jw.by_class(wname)
    for n in (2, 3, 8, 100, 288, 500, 1000, 4097, 12345):
        x = rnd(n, n)
        for J in sorted({1, min(4, n.bit_length() - 1), min(8, n.bit_length() - 1)}):
            c = T.modwt_forward(x, w, J, ctx)
            cr = oracle.modwt_forward(w, x, J)
            assert_exact(c, cr, "%s modwt fwd n=%d J=%d" % (wname, n, J))
            xr = T.modwt_inverse(cr, w, ctx)
            assert_exact(xr, oracle.modwt_inverse(w, cr), "%s modwt inv n=%d J=%d" % (wname, n, J))


def test_modwt_deep_levels(ctx):
    """Levels whose halo exceeds one tile run per level (J up to 13)."""
    w = jw.by_class("Daubechies4")
    n = 20000
    x = rnd(n, 1)
    for J in (10, 13):
        c = T.modwt_forward(x, w, J, ctx)
        cr = oracle.modwt_forward(w, x, J)
        assert_exact(c, cr, "modwt J=%d" % J)
        assert_exact(T.modwt_inverse(cr, w, ctx), oracle.modwt_inverse(w, cr), "imodwt J=%d" % J)


def test_modwt_config5_full_size(ctx, ctx_fma):
    """Config 5: Daubechies4, J=8, N=10^7 — exact vs oracle; round trip."""
    w = jw.by_class("Daubechies4")
    n = 10_000_000
    x = rnd(n, 42)
    c = T.modwt_forward(x, w, 8, ctx)
    cr = oracle.modwt_forward(w, x, 8)
    assert_exact(c, cr, "modwt 1e7")
    xr = T.modwt_inverse(c, w, ctx)
    assert_exact(xr, oracle.modwt_inverse(w, cr), "imodwt 1e7")
    assert np.abs(xr - x).max() < 1e-10
    cf = T.modwt_forward(x, w, 8, ctx_fma)
    assert_close(cf, cr, "modwt fma")
    d = float(np.abs(T.modwt_inverse(cf, w, ctx_fma) - oracle.modwt_inverse(w, cr)).max())
    assert d <= RT_GATE, "config 5 FMA round trip vs oracle round trip: %g" % d


@pytest.mark.parametrize("n", [5_634, 5_636, 5_638, 6_146, 1_000_002, 1_000_003, 2_097_152,
                               3_333_331])
def test_modwt_chunked_sizes(ctx, n):
    """J = 8, Daubechies4.  Even N take the streamed forward (modwt_stream.hpp,
    1024-sample tiles walked left to right with carried halos, one chunk per
    resident block); its minimum is N = 2 (XP + Wn(1)) = 2 (1786 + 1032) =
    5636, where the prologue and the first tile's wrap are tightest (5634:
    the tile kernel; 5638, 6146: one and a few tiles past the minimum, ragged
    last tile; 1_000_002: many chunks, ragged last tile).  Odd N take the tile
    kernel.  The inverse is the tile kernel at every N."""
    w = jw.by_class("Daubechies4")
    x = rnd(n, 5)
    cr = oracle.modwt_forward(w, x, 8)
    assert_exact(T.modwt_forward(x, w, 8, ctx), cr, "modwt n=%d" % n)
    assert_exact(T.modwt_inverse(cr, w, ctx), oracle.modwt_inverse(w, cr), "imodwt n=%d" % n)


def test_modwt_direct_vs_sparse_oracle():
    """The oracle's zero-tap-skipping loop equals the as-written DIRECT loop bit for bit."""
    w = jw.by_class("Daubechies4")
    x = rnd(300, 3)
    assert_exact(oracle.modwt_forward(w, x, 5, sparse=True), oracle.modwt_forward(w, x, 5, sparse=False))


# ------------------------------------------------------------------ non-finite input
NONFINITE = (np.inf, -np.inf, np.nan)


def assert_nan_bits(got, ref, what=""):
    """NaN at the same positions and every other value bit for bit (NaN
    payloads are not compared: Java's NaN is the JVM's, the GPU's is its
    canonical quiet NaN)."""
    got = np.ascontiguousarray(np.asarray(got), dtype=np.float64).ravel()
    ref = np.ascontiguousarray(ref, dtype=np.float64).ravel()
    gn, rn = np.isnan(got), np.isnan(ref)
    bad = np.flatnonzero(gn != rn)
    assert bad.size == 0, "%s: NaN positions differ at %d places, first %d (got %r ref %r)" % (
        what, bad.size, bad[0], got[bad[0]], ref[bad[0]])
    gb, rb = got[~rn].view(np.int64), ref[~rn].view(np.int64)
    bad = np.flatnonzero(gb != rb)
    assert bad.size == 0, "%s: %d values differ in their bits, first at %d" % (what, bad.size, bad[0])


def assert_nan_close(got, ref, what=""):
    """FMA mode: the same NaN and +-inf positions, the rest within the gate."""
    got = np.asarray(got, dtype=np.float64).ravel()
    ref = np.asarray(ref, dtype=np.float64).ravel()
    assert np.array_equal(np.isnan(got), np.isnan(ref)), what + ": NaN positions"
    assert np.array_equal(np.isposinf(got), np.isposinf(ref)), what + ": +inf positions"
    assert np.array_equal(np.isneginf(got), np.isneginf(ref)), what + ": -inf positions"
    m = np.isfinite(ref)
    assert_close(got[m], ref[m], what)


def _edges(n, tiles=(1024, 2048, 4096, 8192)):
    """Positions at and around the tile edges of every MODWT kernel geometry,
    the wrap (0, n-1) and the middle."""
    p = {0, 1, n - 1, n - 2, n // 2}
    for t in tiles:
        for k in range(1, min(n // t, 3) + 1):
            p.update((k * t - 1, k * t))
    return sorted(q for q in p if 0 <= q < n)


def _inject(x, pos, rng):
    x = x.copy()
    pos = np.asarray(pos)
    x[..., pos] = rng.choice(NONFINITE, size=x[..., pos].shape)
    return x


@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Daubechies8", "Symlet8", "CDF53",
                                   "Daubechies20"])
def test_modwt_nonfinite(ctx, wname):
    """MODWTTransform.java:677-716 multiplies every zero tap of the upsampled
    filter: +-inf / NaN at a zero tap of an output's window gives NaN there,
    which the real-tap sums alone would miss (modwt_nonfinite.hpp).  One to
    three non-finite values at tile edges, across the wrap and in the middle,
    for every kernel form (streamed forward, compile-time and runtime tiles,
    deep one-level kernels), forward and inverse, against the oracle (its
    sparse path follows the same rule; test_oracle pins it to the DIRECT
    loops)."""
    w = jw.by_class(wname)
    rng = np.random.default_rng(17)
    for n in (8, 100, 1000, 4097, 5636, 12345, 20000):
        full = n.bit_length() - 1
        for J in sorted({1, 2, min(5, full), min(8, full), min(13, full) if n >= 20000 else 1}):
            edges = _edges(n)
            for trial in range(3):
                pos = rng.choice(edges, size=int(rng.integers(1, 4)), replace=False)
                x = _inject(rnd(n, n + trial), pos, rng)
                cr = oracle.modwt_forward(w, x, J)
                assert_nan_bits(T.modwt_forward(x, w, J, ctx), cr, "%s fwd n=%d J=%d" % (wname, n, J))
                c = oracle.modwt_forward(w, rnd(n, 3 + trial), J)
                rows = rng.integers(0, J + 1, len(pos))
                c[rows, pos] = rng.choice(NONFINITE, size=len(pos))
                assert_nan_bits(T.modwt_inverse(c, w, ctx), oracle.modwt_inverse(w, c),
                                "%s inv n=%d J=%d" % (wname, n, J))


@pytest.mark.parametrize("J", [2, 8, 13])
def test_modwt_nonfinite_direct(ctx, J):
    """The GPU against the oracle's as-written DIRECT loops (sparse=False, every
    zero tap multiplied) at J = 2, 8 and 13: +inf, -inf and NaN at a tile
    edge, across the wrap and in the middle, forward and inverse."""
    w = jw.by_class("Daubechies4")
    n = 20000
    x = rnd(n, 91)
    x[[0, 1023, 1024, n // 2]] = [np.nan, np.inf, -np.inf, np.nan]
    x[n - 1] = np.inf
    cd = oracle.modwt_forward(w, x, J, sparse=False)
    assert_nan_bits(T.modwt_forward(x, w, J, ctx), cd, "fwd J=%d" % J)
    c = oracle.modwt_forward(w, rnd(n, 92), J)
    c[0, 2047] = np.inf
    c[J, 2048] = -np.inf
    c[J // 2, n - 1] = np.nan
    assert_nan_bits(T.modwt_inverse(c, w, ctx), oracle.modwt_inverse(w, c, sparse=False), "inv J=%d" % J)


def test_modwt_nonfinite_config5(ctx, ctx_fma):
    """Config 5 (Daubechies4, J = 8, N = 10^7): non-finite samples at streamed
    tile and chunk edges, across the wrap and inside, forward and inverse;
    EXACT bit for bit (NaN positions) against the oracle, FMA with the same
    NaN / inf positions."""
    w = jw.by_class("Daubechies4")
    n = 10_000_000
    rng = np.random.default_rng(23)
    pos = [0, 1, 1023, 1024, 2047, 2048, 13 * 1024, 4_999_999, 5_000_000, 7_777_777, n - 2, n - 1]
    x = _inject(rnd(n, 42), pos, rng)
    cr = oracle.modwt_forward(w, x, 8)
    assert_nan_bits(T.modwt_forward(x, w, 8, ctx), cr, "modwt 1e7 fwd")
    assert_nan_close(T.modwt_forward(x, w, 8, ctx_fma), cr, "modwt 1e7 fwd fma")
    c = oracle.modwt_forward(w, rnd(n, 43), 8)
    c[rng.integers(0, 9, len(pos)), pos] = rng.choice(NONFINITE, size=len(pos))
    xr = oracle.modwt_inverse(w, c)
    assert_nan_bits(T.modwt_inverse(c, w, ctx), xr, "modwt 1e7 inv")
    assert_nan_close(T.modwt_inverse(c, w, ctx_fma), xr, "modwt 1e7 inv fma")


def test_modwt_nonfinite_overflow_and_all_nan(ctx):
    """Finite input whose level-1 sum overflows (inf meets level 2's zero
    taps), and an all-NaN signal (every block repairs)."""
    w = jw.by_class("Daubechies4")
    g, _ = oracle.modwt_filters(w)
    n = 100_000
    x = rnd(n, 5)
    x[50_000 - np.arange(len(g))] = np.sign(g) * 1.7e308
    assert np.isfinite(x).all()
    cr = oracle.modwt_forward(w, x, 8)
    assert np.isnan(cr).any()
    assert_nan_bits(T.modwt_forward(x, w, 8, ctx), cr, "overflow fwd")
    x = np.full(n, np.nan)
    assert np.isnan(np.asarray(T.modwt_forward(x, w, 8, ctx))).all()
    assert np.isnan(np.asarray(T.modwt_inverse(np.full((9, n), np.nan), w, ctx))).all()


@pytest.mark.parametrize("wname", ["Daubechies4", "Symlet8", "Haar1", "CDF53"])
def test_fwt_wpt_nonfinite(ctx, wname):
    """FWT / WPT have no zero taps (Wavelet.java:236-303), so the kernels'
    sums already meet +-inf / NaN in Java's order: same NaN and inf positions
    and bits as the oracle, forward and reverse, resident and tiled sizes."""
    w = jw.by_class(wname)
    rng = np.random.default_rng(29)
    for n in (1024, 1 << 16):
        pos = _edges(n)
        x = _inject(rnd(n, 9), rng.choice(pos, size=3, replace=False), rng)
        for lev in (1, 4, n.bit_length() - 1):
            assert_nan_bits(T.fwt_forward(x, w, lev, ctx), oracle.fwt_forward(w, x, lev),
                            "%s fwt fwd n=%d l=%d" % (wname, n, lev))
            assert_nan_bits(T.fwt_reverse(x, w, lev, ctx), oracle.fwt_reverse(w, x, lev),
                            "%s fwt rev n=%d l=%d" % (wname, n, lev))
            if lev <= 9:
                assert_nan_bits(T.wpt_forward(x, w, lev, ctx), oracle.wpt_forward(w, x, lev),
                                "%s wpt fwd n=%d l=%d" % (wname, n, lev))
                assert_nan_bits(T.wpt_reverse(x, w, lev, ctx), oracle.wpt_reverse(w, x, lev),
                                "%s wpt rev n=%d l=%d" % (wname, n, lev))


# ------------------------------------------------------------------ KATs on GPU
def test_haar_kat_gpu(ctx):
    """CrossValidationTest.testHaarTransformWithReference (CrossValidationTest.java:187-211)."""
    import os
    g = os.path.join(os.path.dirname(__file__), "golden")
    x = np.loadtxt(os.path.join(g, "haar_simple_input.txt"))
    a = np.loadtxt(os.path.join(g, "haar_level1_approx_manual.txt"))
    d = np.loadtxt(os.path.join(g, "haar_level1_detail_manual.txt"))
    y = T.fwt_forward(x, jw.by_class("Haar1"), 1, ctx)
    assert np.abs(y[:4] - a).max() < 1e-10 and np.abs(y[4:] - d).max() < 1e-10


def test_modwt_haar_kat_gpu(ctx):
    """MODWTTransformTest.testKnownValuesWithHaar (MODWTTransformTest.java:39-72)."""
    x = np.arange(1.0, 9.0)
    c = T.modwt_forward(x, jw.by_class("Haar1"), 1, ctx)
    assert np.abs(c[0] - np.array([-3.5] + [0.5] * 7)).max() < 1e-9
    assert np.abs(c[1] - np.array([4.5, 1.5, 2.5, 3.5, 4.5, 5.5, 6.5, 7.5])).max() < 1e-9


# ------------------------------------------------------------------ C ABI errors
def test_native_validation_messages(ctx):
    w = jw.by_class("Daubechies4")
    with pytest.raises(jw.JWaveFailure, match="FastWaveletTransform#forward - given array length"):
        T.fwt_forward(np.zeros(12), w, 1, ctx)
    with pytest.raises(jw.JWaveFailure, match="given level is out of range"):
        T.fwt_forward(np.zeros(16), w, 5, ctx)
    with pytest.raises(jw.JWaveFailure, match="WaveletPacketTransform#reverse"):
        T.wpt_reverse(np.zeros(16), w, -1, ctx)
    with pytest.raises(ValueError, match="theoretical limit 3"):
        T.modwt_forward(np.zeros(10), w, 4, ctx)
    with pytest.raises(ValueError, match="maximum supported decomposition level is 13"):
        T.modwt_forward(np.zeros(1 << 15), w, 14, ctx)


def test_single_hip_runtime(ctx):
    """torch and libjwave_hip.so share one HIP runtime in the process."""
    import torch
    from jwave_amd import _lib
    assert torch.cuda.is_available()
    maps = _lib.hip_runtimes_mapped()
    assert len(maps) == 1, maps


def test_device_tensors_and_stream(ctx):
    """torch CUDA tensors go through the _dev entry points on torch's stream."""
    import torch
    w = jw.by_class("Daubechies4")
    x = rnd(1 << 16, 4)
    xt = torch.from_numpy(x).cuda()
    y = T.fwt_forward(xt, w, 16, ctx)
    xr = T.fwt_reverse(y, w, 16, ctx)
    torch.cuda.synchronize()
    yr = oracle.fwt_forward(w, x, 16)
    assert_exact(y.cpu().numpy(), yr, "dev fwd")
    assert_exact(xr.cpu().numpy(), oracle.fwt_reverse(w, yr, 16), "dev rev")


def test_alternating_streams_one_context(ctx):
    """Two torch streams, one context, no host sync between the calls: each
    stream switch (jwv_ctx_set_stream) makes the new stream wait for the old
    one's work, so the fused forward tail's arrival counter and the shared
    workspace stay ordered (config-2 plan at 2^20 and 2^22)."""
    import torch
    w = jw.by_class("Daubechies4")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    try:
        _alternate(ctx, w, s1, s2)
    finally:
        ctx.reset_stream()  # before s1 / s2 go away
        torch.cuda.synchronize()


def _alternate(ctx, w, s1, s2):
    import torch
    for n in (1 << 20, 1 << 22):
        lev = n.bit_length() - 1
        xs = [rnd(n, 50 + i) for i in range(6)]
        xt = [torch.from_numpy(x).cuda() for x in xs]
        torch.cuda.synchronize()
        ys, rs = [], []
        for i, x in enumerate(xt):
            with torch.cuda.stream(s1 if i % 2 == 0 else s2):
                y = T.fwt_forward(x, w, lev, ctx)
                ys.append(y)
                rs.append(T.fwt_reverse(y, w, lev, ctx))
        torch.cuda.synchronize()
        for i, x in enumerate(xs):
            yr = oracle.fwt_forward(w, x, lev)
            assert_exact(ys[i].cpu().numpy(), yr, "stream-alternating fwd n=%d #%d" % (n, i))
            assert_exact(rs[i].cpu().numpy(), oracle.fwt_reverse(w, yr, lev),
                         "stream-alternating rev n=%d #%d" % (n, i))


def test_facade_and_classes(ctx):
    """SteppingTest-style use of the operator mirror (SteppingTest.java:55-80)."""
    for w in jw.WaveletBuilder.create2arr():
        t = jw.Transform(jw.FastWaveletTransform(w, ctx))
        x = np.ones(4)
        s2 = np.sqrt(2.0)
        np.testing.assert_allclose(t.forward(x, 0), [1, 1, 1, 1], atol=1e-8)
        np.testing.assert_allclose(t.forward(x, 1), [s2, s2, 0, 0], atol=1e-8)
        np.testing.assert_allclose(t.forward(x, 2), [2, 0, 0, 0], atol=1e-8)
        for lev in (0, 1, 2):
            np.testing.assert_allclose(t.reverse(t.forward(x, lev), lev), x, atol=1e-8)
    assert jw.Transform(jw.FastWaveletTransform(jw.by_class("Haar1"), ctx)).forward(np.ones(3)) is None


def test_in_place_fwt(ctx):
    """InPlaceFastWaveletTransform (InPlaceFastWaveletTransform.java:70-120):
    forwardInPlace / reverseInPlace return the caller's own array holding the
    result, bit-identical to the oracle, for numpy arrays and device tensors,
    at the maximal and a given level; a failing call (level out of range,
    non-power-of-two length) raises the reference's message and leaves the
    array untouched; forward / reverse stay out of place."""
    import torch
    w = jw.by_class("Daubechies4")
    t = jw.InPlaceFastWaveletTransform(w, ctx)
    for n, lev in ((1 << 14, None), (1 << 14, 5), (1 << 20, None), (2, None)):
        x = rnd(n, n + 1)
        full = n.bit_length() - 1 if lev is None else lev
        yr = oracle.fwt_forward(w, x, full)
        a = x.copy()
        assert t.forwardInPlace(a, lev) is a
        assert_exact(a, yr, "in-place fwd n=%d" % n)
        assert t.reverseInPlace(a, lev) is a
        assert_exact(a, oracle.fwt_reverse(w, yr, full), "in-place rev n=%d" % n)
        d = torch.from_numpy(x.copy()).cuda()
        assert t.forwardInPlace(d, lev) is d
        torch.cuda.synchronize()
        assert_exact(d.cpu().numpy(), yr, "in-place fwd tensor n=%d" % n)
    x = rnd(1024, 5)
    a = x.copy()
    with pytest.raises(jw.JWaveFailure, match="^FastWaveletTransform#forward - given level is out"):
        t.forwardInPlace(a, 11)
    assert np.array_equal(a, x)
    with pytest.raises(jw.JWaveFailure, match="^WaveletTransform#reverse - given array length"):
        t.reverseInPlace(np.ones(12))
    y = t.forward(x)
    assert y is not x and np.array_equal(x, rnd(1024, 5))
    assert_exact(y, oracle.fwt_forward(w, x, 10), "out-of-place forward")


@pytest.mark.parametrize("kind,wname,R,cw,lev", [
    ("fwt", "Daubechies4", 1024, 24, 10), ("fwt", "Symlet8", 16384, 8, 14),
    ("fwt", "Haar1", 64, 3, 6), ("fwt", "Daubechies8", 32768, 16, 7),
    ("wpt", "Symlet8", 4096, 8, 6), ("wpt", "Daubechies4", 256, 5, 8)])
def test_axis_columns(ctx, kind, wname, R, cw, lev):
    """jwv_{fwt,wpt}_axis_*_dev on a [R][cw] column slab (the sharded 2-D
    column pass) vs the oracle on the transposed lines, both directions."""
    import torch
    w = jw.by_class(wname)
    x = rnd(R * cw, seed=7).reshape(R, cw)
    ref = oracle.batch(kind, True, w, np.ascontiguousarray(x.T), lev).T
    xd = torch.from_numpy(x).cuda()
    y = T.transform_axis(xd, w, lev, 0, True, ctx, kind=kind)
    assert_exact(y.cpu().numpy(), ref, "%s axis fwd" % kind)
    back = oracle.batch(kind, False, w, np.ascontiguousarray(ref.T), lev).T
    xr = T.transform_axis(y, w, lev, 0, False, ctx, kind=kind)
    assert_exact(xr.cpu().numpy(), back, "%s axis rev" % kind)
    # rows of a 3-D block: middle axis of [2][R][cw]
    x3 = torch.stack([xd, xd.flip(0)])
    y3 = T.transform_axis(x3, w, lev, 1, True, ctx, kind=kind)
    assert_exact(y3[0].cpu().numpy(), ref, "%s axis fwd 3d" % kind)


@pytest.mark.parametrize("kind", ["fwt", "wpt"])
@pytest.mark.parametrize("wname,n", [("Daubechies4", 1000), ("Haar1", 127), ("Symlet8", 70000),
                                     ("Daubechies8", 1), ("Daubechies2", 3),
                                     ("Coiflet1", 8191), ("Haar1Orthogonal", 24577),
                                     ("Daubechies20", 12345), ("Daubechies4", (1 << 20) + 8191)])
def test_ancient_egyptian_decomposition(ctx, kind, wname, n):
    """AncientEgyptianDecomposition over the native FWT / WPT
    (AncientEgyptianDecomposition.java:97-184) through jwv_aed_*: every
    power-of-two sub-array through the full-depth forward/reverse — the pieces
    up to 8192 in ONE varlen launch, larger ones on their own plans — bit-exact
    vs the oracle applied to the same sub-arrays; numpy and device tensors."""
    import torch
    w = jw.by_class(wname)
    basic = jw.FastWaveletTransform(w, ctx) if kind == "fwt" else jw.WaveletPacketTransform(w, ctx)
    aed = jw.AncientEgyptianDecomposition(basic)
    fwd = oracle.fwt_forward if kind == "fwt" else oracle.wpt_forward
    rev = oracle.fwt_reverse if kind == "fwt" else oracle.wpt_reverse
    x = rnd(n, seed=11)
    ref = np.empty(n)
    off = 0
    for p in jw.decompose_number(n):
        m = 1 << p
        ref[off:off + m] = fwd(w, x[off:off + m], p)
        off += m
    y = aed.forward(x)
    assert_exact(y, ref, "aed %s fwd" % kind)
    back = np.empty(n)
    off = 0
    for p in jw.decompose_number(n):
        m = 1 << p
        back[off:off + m] = rev(w, ref[off:off + m], p)
        off += m
    assert_exact(aed.reverse(ref), back, "aed %s rev" % kind)
    yd = aed.forward(torch.from_numpy(x).cuda())
    assert_exact(yd.cpu().numpy(), ref, "aed %s fwd device" % kind)


def test_aed_one_varlen_launch(ctx):
    """n = 2^20 + 8191: the 2^20 piece on its pass plan, the 13 pieces of
    8191 = 4096 + .. + 1 in ONE launch (not 13)."""
    w = jw.by_class("Daubechies4")
    x = rnd((1 << 20) + 8191, seed=3)
    ctx.profile(True)
    try:
        T.aed_transform(x, w, "fwt", True, ctx)
        prof = ctx.profile_read()
    finally:
        ctx.profile(False)
    assert prof["aed_varlen"]["launches"] == 1
    with pytest.raises(jw.JWaveFailure, match="smaller than one"):
        T.aed_transform(np.zeros(0), w, "fwt", True, ctx)


# ------------------------------------------------------- decompose / recompose
@pytest.mark.parametrize("kind", ["fwt", "wpt"])
@pytest.mark.parametrize("wname", ["Haar1", "Daubechies4", "Symlet8", "Coiflet1", "Daubechies20",
                                   "Haar1Orthogonal", "BiOrthogonal35", "CDF53"])
def test_decompose_recompose(ctx, kind, wname):
    """WaveletTransform.decompose / recompose (WaveletTransform.java:136-182)
    in one native call (jwv_decompose_f64): row p == forward(x, p) of the
    oracle, bit-exact, for every level; recompose(mat, level) from every
    level == the oracle's reverse(row, level)."""
    w = jw.by_class(wname)
    fwd = oracle.fwt_forward if kind == "fwt" else oracle.wpt_forward
    rev = oracle.fwt_reverse if kind == "fwt" else oracle.wpt_reverse
    t = jw.FastWaveletTransform(w, ctx) if kind == "fwt" else jw.WaveletPacketTransform(w, ctx)
    for n in (1, 2, 4, 64, 1024, 1 << 15):
        x = rnd(n, seed=n + 5)
        mat = t.decompose(x)
        assert mat.shape == (n.bit_length(), n)
        for p in range(n.bit_length()):
            ref = fwd(w, x, p)
            assert_exact(mat[p], ref, "%s %s decompose n=%d row %d" % (kind, wname, n, p))
            assert_exact(t.recompose(mat, p), rev(w, ref, p),
                         "%s %s recompose n=%d level %d" % (kind, wname, n, p))
        assert_exact(t.recompose(mat), rev(w, mat[-1], n.bit_length() - 1), "recompose()")


def test_decompose_kat_gpu(ctx):
    """DecomposeTest.testDecompose (DecomposeTest.java:30-170) on the GPU for
    every create2arr wavelet: constant signals of 4 and 64, the expected
    orthonormal pyramids (delta 1e-8), recompose from every level."""
    s2 = np.sqrt(2.0)
    exp4 = np.array([[1, 1, 1, 1], [s2, s2, 0, 0], [2, 0, 0, 0]], dtype=float)
    exp64 = np.zeros((7, 64))
    for p in range(7):
        m = 64 >> p
        exp64[p, :m] = 2.0 ** (p / 2.0)
    exp64[0] = 1.0
    for w in jw.WaveletBuilder.create2arr():
        t = jw.Transform(jw.FastWaveletTransform(w, ctx))
        for x, exp in ((np.ones(4), exp4), (np.ones(64), exp64)):
            mat = t.decompose(x)
            np.testing.assert_allclose(mat, exp, atol=1e-8, err_msg=w.name)
            np.testing.assert_allclose(t.recompose(mat), x, atol=1e-8, err_msg=w.name)
            for lev in range(mat.shape[0]):
                np.testing.assert_allclose(t.recompose(mat, lev), x, atol=1e-8, err_msg=w.name)
    with pytest.raises(jw.JWaveFailure, match="calcExponent"):
        jw.FastWaveletTransform(jw.by_class("Haar1"), ctx).decompose(np.ones(12))


# ------------------------------------------------------- flattened MODWT API
def test_modwt_flattened_interface(ctx):
    """MODWT1DInterfaceTest (MODWT1DInterfaceTest.java:22-136) through the
    native path, plus bit-exactness vs the oracle: forward(x) / forward(x,
    level) flatten [W_1..W_J, V_J]; reverse(flat, level) and the auto-level
    reverse(flat) (MODWTTransform.java:389-443, 854-912)."""
    haar, d4 = jw.by_class("Haar1"), jw.by_class("Daubechies4")
    m = jw.MODWTTransform(haar, ctx)
    sig8 = np.arange(1.0, 9.0)
    flat = m.forward(sig8)
    assert flat.shape == (8 * 4,)
    assert_exact(flat, oracle.modwt_forward(haar, sig8, 3).reshape(-1), "flat fwd")
    assert_exact(m.reverse(flat), oracle.modwt_inverse(haar, flat.reshape(4, 8)), "auto rev")
    np.testing.assert_allclose(m.reverse(flat), sig8, atol=1e-10)
    sig64 = np.sin(2 * np.pi * np.arange(64) / 16.0)
    for level in range(1, 7):
        f = m.forward(sig64, level)
        assert f.shape == (64 * (level + 1),)
        assert_exact(f, oracle.modwt_forward(haar, sig64, level).reshape(-1), "lvl %d" % level)
    md = jw.MODWTTransform(d4, ctx)
    sig128 = np.cos(2 * np.pi * np.arange(128) / 32.0) + 0.5 * np.sin(2 * np.pi * np.arange(128) / 8.0)
    for level in range(1, 6):
        f = md.forward(sig128, level)
        r = md.reverse(f, level)
        assert_exact(r, oracle.modwt_inverse(d4, f.reshape(level + 1, 128)), "rev lvl %d" % level)
        np.testing.assert_allclose(r, sig128, atol=1e-10)
    c2 = m.forwardMODWT(sig8, 2)
    assert_exact(m.forward(sig8, 2), np.asarray(c2).reshape(-1), "1D vs 2D interface")
    # the reference's ambiguous auto-level guess is reproduced: N=16, J=1 reads as N=8, J=3
    sig16 = rnd(16, seed=2)
    f16 = m.forward(sig16, 1)
    assert_exact(m.reverse(f16), oracle.modwt_inverse(haar, f16.reshape(4, 8)), "ambiguous")
    with pytest.raises(jw.JWaveFailure, match="2\\^p"):
        m.forward(np.zeros(10))
    with pytest.raises(jw.JWaveFailure, match="out of range"):
        m.forward(np.zeros(8), 5)
    with pytest.raises(jw.JWaveFailure, match="does not match|Invalid coefficient array"):
        m.reverse(np.zeros(15), 2)
    assert m.forward(np.zeros(0)).shape == (0,) and m.reverse(np.zeros(0)).shape == (0,)


def test_modwt_flattened_device_tensors(ctx):
    import torch
    d4 = jw.by_class("Daubechies4")
    md = jw.MODWTTransform(d4, ctx)
    x = rnd(256, seed=9)
    xd = torch.from_numpy(x).cuda()
    f = md.forward(xd, 4)
    assert isinstance(f, torch.Tensor) and f.is_cuda and f.shape == (5 * 256,)
    assert_exact(f.cpu().numpy(), oracle.modwt_forward(d4, x, 4).reshape(-1), "dev flat fwd")
    r = md.reverse(f)  # auto: 1280 = 256 x 5 -> first fit N=256, J=4
    assert isinstance(r, torch.Tensor)
    assert_exact(r.cpu().numpy(), oracle.modwt_inverse(d4, oracle.modwt_forward(d4, x, 4)), "dev auto")


# ------------------------------------------------------------- reentrancy
def test_c_abi_reentrancy_threads():
    """Every C-ABI entry is reentrant: two threads with a context
    each, and two threads sharing one context (its mutex serialises them),
    hammer FWT / WPT / MODWT concurrently — the pattern of
    MODWTThreadSafetyTest.java:24-148 — and every result stays bit-exact."""
    import threading
    d4, s8 = jw.by_class("Daubechies4"), jw.by_class("Symlet8")
    x = rnd(1 << 14, seed=21)
    refs = {"fwt": oracle.fwt_forward(d4, x, 14), "wpt": oracle.wpt_forward(s8, x, 5),
            "modwt": oracle.modwt_forward(d4, x[:5000], 6)}
    shared = jw.Context(0, "exact")
    own = [jw.Context(0, "exact") for _ in range(2)]
    errors = []

    def worker(c, i):
        try:
            for k in range(12):
                op = ("fwt", "wpt", "modwt")[(i + k) % 3]
                if op == "fwt":
                    got = T.fwt_forward(x, d4, 14, c)
                elif op == "wpt":
                    got = T.wpt_forward(x, s8, 5, c)
                else:
                    got = T.modwt_forward(x[:5000], d4, 6, c)
                if not np.array_equal(np.asarray(got), refs[op]):
                    errors.append("%s thread %d iter %d" % (op, i, k))
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(own[0], 0)),
           threading.Thread(target=worker, args=(own[1], 1)),
           threading.Thread(target=worker, args=(shared, 2)),
           threading.Thread(target=worker, args=(shared, 3))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    for c in own + [shared]:
        c.close()
    assert not errors, errors[:5]


def test_complex_entry(ctx):
    """BasicTransform.forward/reverse(Complex[]) (BasicTransform.java:257-322):
    {re, im} interleaved into one real array of 2n at full depth."""
    import torch
    w = jw.by_class("Daubechies4")
    fwt = jw.FastWaveletTransform(w, ctx)
    n = 512
    re, im = rnd(n, seed=3), rnd(n, seed=4)
    z = re + 1j * im
    bulk = np.empty(2 * n)
    bulk[0::2], bulk[1::2] = re, im
    ref = oracle.fwt_forward(w, bulk, 10)
    y = fwt.forward(z)
    assert_exact(np.asarray(y.real), ref[0::2], "complex fwd re")
    assert_exact(np.asarray(y.imag), ref[1::2], "complex fwd im")
    back = oracle.fwt_reverse(w, ref, 10)
    zr = fwt.reverse(y)
    assert_exact(np.asarray(zr.real), back[0::2], "complex rev re")
    yd = fwt.forward(torch.from_numpy(z).cuda())
    assert_exact(torch.view_as_real(yd).reshape(-1).cpu().numpy(), ref, "complex fwd device")


@pytest.mark.parametrize("n,thr", [(1 << 12, 1.0), (1 << 20, 2.5), (1000, 0.0), (1, 1.0)])
def test_compress_magnitude(ctx, n, thr):
    """CompressorMagnitude.compress (CompressorMagnitude.java:73-84) on the
    device vs the oracle's left-to-right restatement: magnitude within the
    summation-order tolerance, output identical (no coefficient of this data
    lies within n*eps of the cut)."""
    w = jw.by_class("Daubechies4")
    x = rnd(n, seed=5)
    pow2 = n > 1 and (n & (n - 1)) == 0  # non-pow-2 sizes compress raw samples
    c = oracle.fwt_forward(w, x, n.bit_length() - 1) if pow2 else x
    ref, mag_ref = oracle.compress_magnitude(c, thr)
    y, mag = jw.compress_magnitude(c, thr, ctx)
    assert abs(mag - mag_ref) <= 1e-13 * max(1.0, abs(mag_ref)) * max(1.0, np.log2(n))
    assert_exact(y, ref, "compress")
    comp = jw.CompressorMagnitude(thr, ctx)
    assert_exact(comp.compress(c), ref, "CompressorMagnitude")
    assert comp.calcCompressionRate(ref) == pytest.approx(
        100.0 * np.count_nonzero(ref == 0) / n if np.count_nonzero(ref == 0) else 0.0)


def _thr_at(c, k):
    """A threshold for which Java's cut (magnitude * threshold, magnitude summed
    left to right, CompressorMagnitude.java:78-82) equals |c[k]| exactly."""
    _, mag = oracle.compress_magnitude(c, 1.0)
    a = abs(float(c[k]))
    thr = a / mag
    for _ in range(256):
        cut = mag * thr
        if cut == a:
            return thr
        thr = float(np.nextafter(thr, np.inf if cut < a else -np.inf))
    pytest.skip("no threshold hits |c[k]| exactly")


@pytest.mark.parametrize("n", [4096, 1 << 20, 1000003])
def test_compress_magnitude_at_cut(ctx, n):
    """A coefficient exactly on Java's cut: the tree sum alone cannot decide it
    (it lies within the n*eps band), so the device forms the left-to-right sum
    and must keep exactly what Java keeps, with Java's magnitude."""
    x = rnd(n, seed=11) - 0.5
    k = n // 3
    thr = _thr_at(x, k)
    ref, mag_ref = oracle.compress_magnitude(x, thr)
    assert ref[k] == x[k]
    y, mag = jw.compress_magnitude(x, thr, ctx)
    assert_exact(y, ref, "compress at cut")
    assert mag == mag_ref  # the serial pass ran: Java's magnitude bit for bit


@pytest.mark.parametrize("special", ["nan", "inf", "overflow", "zeros"])
def test_compress_magnitude_special_values(ctx, special):
    """Non-finite and degenerate magnitudes decide as Java's doubles do: a NaN
    magnitude zeroes everything, an infinite one keeps only infinities, a sum
    that overflows goes through the left-to-right pass, all-zero input stays
    zero."""
    x = rnd(5000, seed=17) - 0.5
    if special == "nan":
        x[123] = np.nan
    elif special == "inf":
        x[77] = -np.inf
    elif special == "overflow":
        x[:] = 1.7e308 * np.sign(x)
    else:
        x[:] = 0.0
    ref, mag_ref = oracle.compress_magnitude(x, 1.0)
    y, mag = jw.compress_magnitude(x, 1.0, ctx)
    assert np.array_equal(np.isnan(y), np.isnan(ref))
    assert_exact(np.nan_to_num(y), np.nan_to_num(ref), "compress " + special)


@pytest.mark.parametrize("wname,n,lev", [("Daubechies4", 1 << 16, 16), ("Haar1", 1 << 12, 12)])
def test_fwt_denoise_at_cut(ctx, wname, n, lev):
    """In-place compress inside the fused denoise with a coefficient exactly on
    Java's cut (classify pass, serial magnitude, apply)."""
    w = jw.by_class(wname)
    x = rnd(n, seed=13)
    c = oracle.fwt_forward(w, x, lev)
    thr = _thr_at(c, n // 2 + 7)
    cc, _ = oracle.compress_magnitude(c, thr)
    ref = oracle.fwt_reverse(w, cc, lev)
    assert_exact(jw.fwt_denoise(x, w, lev, thr, ctx), ref, "denoise at cut")


@pytest.mark.parametrize("wname,n,lev", [("Daubechies4", 1 << 16, 16), ("Symlet8", 1 << 20, 12),
                                         ("Haar1", 1 << 10, 10)])
def test_fwt_denoise(ctx, wname, n, lev):
    """forward -> CompressorMagnitude -> reverse fused on the device, vs the
    same sequence on the oracle."""
    import torch
    w = jw.by_class(wname)
    x = rnd(n, seed=9)
    c = oracle.fwt_forward(w, x, lev)
    cc, _ = oracle.compress_magnitude(c, 1.5)
    ref = oracle.fwt_reverse(w, cc, lev)
    assert_exact(jw.fwt_denoise(x, w, lev, 1.5, ctx), ref, "denoise")
    yd = jw.fwt_denoise(torch.from_numpy(x).cuda(), w, lev, 1.5, ctx)
    assert_exact(yd.cpu().numpy(), ref, "denoise device")


def test_host_entry_staging_paths(ctx):
    """The host-pointer entries (Transform.forward(double[]) semantics) move
    pageable arrays through the pinned staging ring (4 slots of 32 MiB,
    capi.cpp PinRing) and DMA page-locked arrays (jwv_host_alloc) directly: every
    combination gives the device entry's bits, for sizes that end mid-chunk
    or wrap the ring, and the caller's current device is left as it was."""
    import ctypes
    import torch
    from jwave_amd import _lib as L
    from jwave_amd.transforms import _TapsHolder
    lib = L.lib()
    w = jw.by_class("Daubechies4")
    t = _TapsHolder.of(w)
    for n, lev in ((1 << 22, 22), ((1 << 20) * 3, 0), (1 << 10, 10), (1 << 24, 24)):
        if lev == 0:  # 3 Mi doubles (not a power of two): AED path of one call
            x = rnd(n, 5)
            ref = T.aed_transform(torch.from_numpy(x).cuda(), w, "fwt", True, ctx).cpu().numpy()
            got = T.aed_transform(x, w, "fwt", True, ctx)
            assert_exact(got, ref, "aed host entry n=%d" % n)
            continue
        x = rnd(n, 3)
        ref = T.fwt_forward(torch.from_numpy(x).cuda(), w, lev, ctx).cpu().numpy()
        assert_exact(T.fwt_forward(x, w, lev, ctx), ref, "pageable n=%d" % n)
        pin = [ctypes.c_void_p(), ctypes.c_void_p()]
        for p in pin:
            assert lib.jwv_host_alloc(ctx.handle, n * 8, ctypes.byref(p)) == 0
        try:
            px = np.ctypeslib.as_array((ctypes.c_double * n).from_address(pin[0].value))
            py = np.ctypeslib.as_array((ctypes.c_double * n).from_address(pin[1].value))
            px[:] = x
            dp = ctypes.POINTER(ctypes.c_double)
            # pageable arrays 8 B off a 64-B line (the staging copies stream
            # 64-B aligned stores after a memcpy head)
            xo = np.empty(n + 3)[3:]
            xo[:] = x
            for src, dst in ((px, py), (px, np.empty(n)), (x, py), (xo, np.empty(n + 1)[1:]),
                             (xo, py)):
                dst[:] = np.nan
                rc = lib.jwv_fwt_fwd_f64(src.ctypes.data_as(dp), dst.ctypes.data_as(dp), n, lev,
                                         t, ctx.handle)
                assert rc == 0, lib.jwv_last_error(ctx.handle)
                assert_exact(dst, ref, "pinned/pageable mix n=%d" % n)
        finally:
            for p in pin:
                assert lib.jwv_host_free(ctx.handle, p) == 0
    assert torch.cuda.current_device() == 0
