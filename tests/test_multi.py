"""Multi-device batches (include/jwave_hip.h jwv_mctx_*, jwv_m_*_batch_f64):
the split arithmetic on CPU, and on the GPU box the multi-context over one
device (n = 1) and over the same device listed several times (the split,
the per-device threads and staging run for real), bit-exact against the
oracle's batch and with the single-device messages for bad arguments.
Reference batch: src/test/java/jwave/ParallelizationOpportunityTest.java:80-98
(independent signals on an executor)."""
import numpy as np
import pytest

import jwave_amd as jw


def _ref_split(batch, n, i):
    a, b = batch * i // n, batch * (i + 1) // n
    return a, b - a


@pytest.mark.parametrize("n", [1, 2, 3, 7, 8])
def test_batch_split_arithmetic(n):
    for batch in list(range(0, 40)) + [4096, 4097, 65535, 10 ** 9 + 7, (1 << 62) + 3]:
        blocks = [jw.batch_split(batch, n, i) for i in range(n)]
        assert blocks == [_ref_split(batch, n, i) for i in range(n)]
        # contiguous, covering, balanced within one signal
        assert blocks[0][0] == 0
        for (s0, c0), (s1, _) in zip(blocks, blocks[1:]):
            assert s0 + c0 == s1
        assert blocks[-1][0] + blocks[-1][1] == batch
        counts = [c for _, c in blocks]
        assert max(counts) - min(counts) <= 1


def test_batch_split_rejects_bad_arguments():
    for args in ((-1, 2, 0), (5, 0, 0), (5, 2, 2), (5, 2, -1)):
        with pytest.raises(jw.JWaveError, match="jwv_batch_split"):
            jw.batch_split(*args)


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_context_batches(devices):
    import oracle
    w = jw.by_class("Symlet8")
    m = jw.MultiContext(devices)
    try:
        for kind in ("fwt", "wpt"):
            for b, n, lev in ((13, 4096, 6), (2, 1024, 10), (64, 65536, 6)):
                x = np.stack([oracle.java_random_doubles(b * 7 + i, n) for i in range(b)])
                yr = oracle.batch(kind, True, w, x, lev)
                y = m.batch(x, w, lev, True, kind)
                assert np.array_equal(y, yr), "%s fwd %s %dx%d" % (devices, kind, b, n)
                xr = m.batch(yr, w, lev, False, kind)
                assert np.array_equal(xr, oracle.batch(kind, False, w, yr, lev))
        # the transform classes take the multi-context for host batches
        t = jw.WaveletPacketTransform(w)
        x = np.stack([oracle.java_random_doubles(3 + i, 8192) for i in range(5)])
        assert np.array_equal(t.forward_batch(x, 6, mctx=m), oracle.batch("wpt", True, w, x, 6))
        # validation once, with the single-device messages, before any device runs
        with pytest.raises(jw.JWaveFailure, match="^FastWaveletTransform#forward - given level"):
            m.batch(np.ones((4, 64)), w, 7, True, "fwt")
        with pytest.raises(jw.JWaveFailure, match="given array length is not 2"):
            m.batch(np.ones((4, 48)), w, 2, True, "wpt")
    finally:
        m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0], [0, 0, 0, 0]])
def test_multi_context_2d(devices):
    """ParallelTransform.forward / reverse(double[][]) over the listed devices
    (jwv_m_fwt2d_* / jwv_m_wpt2d_*, ParallelTransform.java:70-126): row
    blocks, one device-to-device exchange (hipMemcpyPeerAsync), column slabs,
    row-strided staging of the host matrix.  Bit-exact against the oracle at
    2048^2 and 8192^2 (config 3), forward and reverse; [0, 0, 0] runs on 2
    (the largest power of two <= 3), and the 4-column matrix on 4 devices
    runs on 2 (chunks of at least 2 columns).  One physical GPU
    listed several times: the exchange, threads and staging run for real;
    distinct physical devices are not available on this pool."""
    import oracle
    m = jw.MultiContext(devices)
    try:
        for kind, wname, rows, cols, lm, ln in (
                ("fwt", "Daubechies8", 2048, 2048, 11, 11), ("fwt", "Daubechies8", 8192, 8192, 13, 13),
                ("fwt", "Haar1", 64, 4, 6, 2), ("fwt", "Daubechies4", 16, 4096, 4, 12),
                ("wpt", "Symlet8", 1024, 512, 5, 4), ("fwt", "Coiflet1", 256, 128, 0, 3)):
            w = jw.by_class(wname)
            x = oracle.java_random_doubles(123456789, rows * cols).reshape(rows, cols)
            ref = oracle.transform_2d_par(kind, True, w, x, lm, ln, 8)
            y = m.transform_2d(x, w, lm, ln, True, kind)
            assert np.array_equal(y, ref), "%s %s fwd %dx%d" % (devices, kind, rows, cols)
            xr = m.transform_2d(ref, w, lm, ln, False, kind)
            assert np.array_equal(xr, oracle.transform_2d_par(kind, False, w, ref, lm, ln, 8)), \
                "%s %s rev %dx%d" % (devices, kind, rows, cols)
        w = jw.by_class("Daubechies4")
        with pytest.raises(jw.JWaveFailure, match="given level"):
            m.transform_2d(np.ones((64, 64)), w, 7, 3)
    finally:
        m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_multi_context_modwt_batches(devices):
    """forwardMODWT / inverseMODWT of a batch of signals, contiguous blocks
    per device (jwv_m_modwt_*_batch_f64): each signal's coefficients equal
    the oracle's (MODWTTransform.java:256-375), non-power-of-two lengths and
    the deep levels included."""
    import oracle
    w = jw.by_class("Daubechies4")
    m = jw.MultiContext(devices)
    try:
        for b, n, J in ((5, 10000, 8), (3, 1000003, 8), (2, 20000, 13), (4, 37, 5)):
            x = np.stack([oracle.java_random_doubles(b + i, n) for i in range(b)])
            c = m.modwt_forward(x, w, J)
            for i in range(b):
                assert np.array_equal(c[i], oracle.modwt_forward(w, x[i], J)), \
                    "%s fwd b=%d n=%d J=%d #%d" % (devices, b, n, J, i)
            xr = m.modwt_inverse(c, w)
            for i in range(b):
                assert np.array_equal(xr[i], oracle.modwt_inverse(w, c[i])), \
                    "%s inv n=%d J=%d #%d" % (devices, n, J, i)
        with pytest.raises(ValueError, match="exceeds theoretical limit"):
            m.modwt_forward(np.ones((2, 100)), w, 7)
    finally:
        m.close()
