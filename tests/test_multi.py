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
