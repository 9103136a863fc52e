"""Independent numpy restatement of the reference loops (test infrastructure).

Written separately from oracle/jwave_oracle.c to cross-check it bit for bit:
  forward level  Wavelet.java:236-260  (vectorised over i, j ascending, no FMA)
  reverse level  Wavelet.java:277-303  (np.add.at applies the scatter-adds in
                                        (i, j) order, exactly like the Java loop)
  MODWT          MODWTTransform.java:256-375 with circularConvolve(:677-716)
"""
import numpy as np


def level_forward(x, lo, hi, h):
    i = np.arange(h // 2)
    a = np.zeros(h // 2)
    d = np.zeros(h // 2)
    for j in range(len(lo)):
        v = x[(2 * i + j) % h]
        a = a + v * lo[j]
        d = d + v * hi[j]
    return np.concatenate([a, d])


def level_reverse(y, lo_r, hi_r, h, scale=1.0):
    half = h // 2
    L = len(lo_r)
    i = np.repeat(np.arange(half), L)
    j = np.tile(np.arange(L), half)
    t = (y[i] * np.asarray(lo_r)[j]) + (y[i + half] * np.asarray(hi_r)[j])
    if scale != 1.0:
        t = scale * t
    out = np.zeros(h)
    np.add.at(out, (2 * i + j) % h, t)
    return out


def fwt_forward(w, x, level):
    y = np.array(x, dtype=np.float64)
    h, l = len(y), 0
    while h >= w.transform_wavelength and l < level:
        y[:h] = level_forward(y, w.lo, w.hi, h)
        h >>= 1
        l += 1
    return y


def fwt_reverse(w, y, level):
    x = np.array(y, dtype=np.float64)
    n = len(x)
    steps = n.bit_length() - 1
    h = w.transform_wavelength << (steps - level) if level <= steps else 0
    while h <= n and h >= w.transform_wavelength:
        x[:h] = level_reverse(x, w.lo_r, w.hi_r, h, w.reverse_scale)
        h <<= 1
    return x


def wpt_forward(w, x, level):
    y = np.array(x, dtype=np.float64)
    n = len(y)
    h, l = n, 0
    while h >= w.transform_wavelength and l < level:
        for p in range(n // h):
            y[p * h:(p + 1) * h] = level_forward(y[p * h:(p + 1) * h], w.lo, w.hi, h)
        h >>= 1
        l += 1
    return y


def wpt_reverse(w, y, level):
    x = np.array(y, dtype=np.float64)
    n = len(x)
    steps = n.bit_length() - 1
    h = w.transform_wavelength << (steps - level)
    while h <= n and h >= w.transform_wavelength:
        for p in range(n // h):
            x[p * h:(p + 1) * h] = level_reverse(x[p * h:(p + 1) * h], w.lo_r, w.hi_r, h,
                                                 w.reverse_scale)
        h <<= 1
    return x


def modwt_filters(w):
    g = np.array(w.lo, dtype=np.float64)
    h = np.array(w.hi, dtype=np.float64)
    for f in (g, h):
        e = 0.0
        for c in f:
            e += c * c
        nrm = np.sqrt(e)
        if nrm > 1e-12:
            f /= nrm
    s = np.sqrt(2.0)
    return g / s, h / s


def modwt_forward(w, x, J):
    g, h = modwt_filters(w)
    N = len(x)
    v = np.array(x, dtype=np.float64)
    n = np.arange(N)
    out = []
    for j in range(1, J + 1):
        s = 1 << (j - 1)
        W = np.zeros(N)
        V = np.zeros(N)
        for l in range(len(g)):
            src = v[(n - l * s) % N]
            W = W + src * h[l]
            V = V + src * g[l]
        out.append(W)
        v = V
    out.append(v)
    return np.stack(out)


def modwt_inverse(w, c):
    g, h = modwt_filters(w)
    J = c.shape[0] - 1
    N = c.shape[1]
    n = np.arange(N)
    v = np.array(c[J])
    for j in range(J, 0, -1):
        s = 1 << (j - 1)
        a = np.zeros(N)
        d = np.zeros(N)
        for l in range(len(g)):
            a = a + v[(n + l * s) % N] * g[l]
            d = d + c[j - 1][(n + l * s) % N] * h[l]
        v = a + d
    return v


def _upsample(f, s):
    """MODWTTransform.upsample (MODWTTransform.java:618-630): s - 1 zeros between taps."""
    u = np.zeros((len(f) - 1) * s + 1)
    u[::s] = f
    return u


def modwt_forward_dense(w, x, J):
    """forwardMODWT with circularConvolve as written (MODWTTransform.java:677-690):
    every tap of the upsampled filter, zeros included, m ascending.  Differs from
    modwt_forward only on non-finite input (x * 0.0 is NaN for x = +-inf / NaN)."""
    g, h = modwt_filters(w)
    N = len(x)
    v = np.array(x, dtype=np.float64)
    n = np.arange(N)
    out = []
    for j in range(1, J + 1):
        gu, hu = _upsample(g, 1 << (j - 1)), _upsample(h, 1 << (j - 1))
        W = np.zeros(N)
        V = np.zeros(N)
        with np.errstate(invalid="ignore", over="ignore"):
            for m in range(len(gu)):
                src = v[(n - m) % N]
                W = W + src * hu[m]
                V = V + src * gu[m]
        out.append(W)
        v = V
    out.append(v)
    return np.stack(out)


def modwt_inverse_dense(w, c):
    """inverseMODWT with circularConvolveAdjoint as written (MODWTTransform.java:703-716)."""
    g, h = modwt_filters(w)
    J = c.shape[0] - 1
    N = c.shape[1]
    n = np.arange(N)
    v = np.array(c[J])
    for j in range(J, 0, -1):
        gu, hu = _upsample(g, 1 << (j - 1)), _upsample(h, 1 << (j - 1))
        a = np.zeros(N)
        d = np.zeros(N)
        with np.errstate(invalid="ignore", over="ignore"):
            for m in range(len(gu)):
                a = a + v[(n + m) % N] * gu[m]
                d = d + c[j - 1][(n + m) % N] * hu[m]
            v = a + d
    return v
