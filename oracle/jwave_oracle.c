/*
 * jwave_oracle.c — CPU restatement of JWave's FWT / WPT / MODWT hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libjwave_hip.so, the
 * jwave_amd package's transform path) links, loads or calls this file.  It is
 * used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as
 * the checker / CPU baseline, never as the thing measured or shipped.
 *
 * Every function restates the reference loop it cites (paths relative to
 * /root/reference/src/main/java/jwave/).  It is compiled with
 * -ffp-contract=off so that `a += x*c` rounds twice like the JVM (no FMA), and
 * it accumulates in the reference's order, so its doubles are those the Java
 * code produces.  Parity pinning: see DESIGN.md §Oracle (KATs and fixtures of
 * the reference's own tests; the Java reference cannot run in this image).
 *
 * Status codes mirror include/jwave_hip.h: 0 ok, 1 JWaveFailure-class input
 * error, 2 MODWT level limit (IllegalArgumentException).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct orc_taps {
  int L;            /* _motherWavelength */
  int tw;           /* _transformWavelength */
  const double* lo; /* _scalingDeCom */
  const double* hi; /* _waveletDeCom */
  const double* lo_r; /* _scalingReCon */
  const double* hi_r; /* _waveletReCon */
  double reverse_scale; /* 0.5 for Haar1Orthogonal (haar/Haar1Orthogonal.java:39), else 1 */
} orc_taps;

/* MathToolKit.isBinary — tools/MathToolKit.java:185-188 */
int orc_is_binary(int64_t n) { return n > 0 && ((n & (n - 1)) == 0); }

/* MathToolKit.getExponent — tools/MathToolKit.java:202-206: (int)(log f / log 2) */
int orc_get_exponent(double f) { return (int)(log(f) / log(2.)); }

/* Wavelet.forward(double[], int) — transforms/wavelets/Wavelet.java:236-260 */
void orc_wavelet_forward(const orc_taps* t, const double* arr_time, double* arr_hilb, int len) {
  int h = len >> 1;
  for (int i = 0; i < h; i++) {
    arr_hilb[i] = arr_hilb[i + h] = 0.;
    for (int j = 0; j < t->L; j++) {
      int k = (i << 1) + j;
      while (k >= len) k -= len;
      arr_hilb[i] += arr_time[k] * t->lo[j];
      arr_hilb[i + h] += arr_time[k] * t->hi[j];
    }
  }
}

/* Wavelet.reverse(double[], int) — Wavelet.java:277-303; Haar1Orthogonal's
 * override (haar/Haar1Orthogonal.java:175-207) multiplies the bracketed term by
 * its energy correction factor, expressed here as reverse_scale. */
void orc_wavelet_reverse(const orc_taps* t, const double* arr_hilb, double* arr_time, int len) {
  for (int i = 0; i < len; i++) arr_time[i] = 0.;
  int h = len >> 1;
  for (int i = 0; i < h; i++) {
    for (int j = 0; j < t->L; j++) {
      int k = (i << 1) + j;
      while (k >= len) k -= len;
      double term = (arr_hilb[i] * t->lo_r[j]) + (arr_hilb[i + h] * t->hi_r[j]);
      if (t->reverse_scale != 1.0) term = t->reverse_scale * term;
      arr_time[k] += term;
    }
  }
}

/* FastWaveletTransform.forward(double[], int) — FastWaveletTransform.java:71-101 */
int orc_fwt_forward(const orc_taps* t, const double* x, double* y, int n, int level) {
  if (!orc_is_binary(n)) return 1;
  int levels = orc_get_exponent((double)n);
  if (level < 0 || level > levels) return 1;
  double* tmp = (double*)malloc(sizeof(double) * (size_t)n);
  memcpy(y, x, sizeof(double) * (size_t)n);
  int l = 0, h = n;
  while (h >= t->tw && l < level) {
    orc_wavelet_forward(t, y, tmp, h);
    memcpy(y, tmp, sizeof(double) * (size_t)h);
    h >>= 1;
    l++;
  }
  free(tmp);
  return 0;
}

/* FastWaveletTransform.reverse(double[], int) — FastWaveletTransform.java:119-153 */
int orc_fwt_reverse(const orc_taps* t, const double* y, double* x, int n, int level) {
  if (!orc_is_binary(n)) return 1;
  int levels = orc_get_exponent((double)n);
  if (level < 0 || level > levels) return 1;
  double* tmp = (double*)malloc(sizeof(double) * (size_t)n);
  memcpy(x, y, sizeof(double) * (size_t)n);
  int h = t->tw;
  for (int l = level; l < levels; l++) h <<= 1;
  while (h <= n && h >= t->tw) {
    orc_wavelet_reverse(t, x, tmp, h);
    memcpy(x, tmp, sizeof(double) * (size_t)h);
    h <<= 1;
  }
  free(tmp);
  return 0;
}

/* WaveletPacketTransform.forward(double[], int) — WaveletPacketTransform.java:73-124 */
int orc_wpt_forward(const orc_taps* t, const double* x, double* y, int n, int level) {
  if (!orc_is_binary(n)) return 1;
  int levels = orc_get_exponent((double)n);
  if (level < 0 || level > levels) return 1;
  double* obuf = (double*)malloc(sizeof(double) * (size_t)n);
  memcpy(y, x, sizeof(double) * (size_t)n);
  int h = n, l = 0;
  while (h >= t->tw && l < level) {
    int g = n / h;
    for (int p = 0; p < g; p++) {
      orc_wavelet_forward(t, y + (size_t)p * h, obuf, h);
      memcpy(y + (size_t)p * h, obuf, sizeof(double) * (size_t)h);
    }
    h >>= 1;
    l++;
  }
  free(obuf);
  return 0;
}

/* WaveletPacketTransform.reverse(double[], int) — WaveletPacketTransform.java:141-191 */
int orc_wpt_reverse(const orc_taps* t, const double* y, double* x, int n, int level) {
  if (!orc_is_binary(n)) return 1;
  int levels = orc_get_exponent((double)n);
  if (level < 0 || level > levels) return 1;
  double* obuf = (double*)malloc(sizeof(double) * (size_t)n);
  memcpy(x, y, sizeof(double) * (size_t)n);
  int h = t->tw;
  for (int l = level; l < levels; l++) h <<= 1;
  while (h <= n && h >= t->tw) {
    int g = n / h;
    for (int p = 0; p < g; p++) {
      orc_wavelet_reverse(t, x + (size_t)p * h, obuf, h);
      memcpy(x + (size_t)p * h, obuf, sizeof(double) * (size_t)h);
    }
    h <<= 1;
  }
  free(obuf);
  return 0;
}

typedef int (*orc_1d_fn)(const orc_taps*, const double*, double*, int, int);

static orc_1d_fn pick(int kind, int forward) {
  if (kind == 0) return forward ? orc_fwt_forward : orc_fwt_reverse;
  return forward ? orc_wpt_forward : orc_wpt_reverse;
}

/* Batched 1D: an outer loop over independent signals (the batch pattern of
 * ParallelizationOpportunityTest.java:80-98); each signal as in the 1D calls. */
int orc_batch(int kind, int forward, const orc_taps* t, const double* x, double* y, int batch,
              int n, int64_t ld, int level) {
  orc_1d_fn fn = pick(kind, forward);
  for (int b = 0; b < batch; b++) {
    int rc = fn(t, x + (size_t)b * ld, y + (size_t)b * ld, n, level);
    if (rc) return rc;
  }
  return 0;
}

/* BasicTransform.forward(double[][], lvlM, lvlN) — BasicTransform.java:361-399:
 * every row with lvlN, then every column with lvlM.  Row-major contiguous. */
int orc_2d_forward(int kind, const orc_taps* t, const double* x, double* y, int rows, int cols,
                   int lvl_m, int lvl_n) {
  orc_1d_fn fn = pick(kind, 1);
  double* a = (double*)malloc(sizeof(double) * (size_t)(rows > cols ? rows : cols));
  double* b = (double*)malloc(sizeof(double) * (size_t)(rows > cols ? rows : cols));
  int rc = 0;
  for (int i = 0; i < rows && !rc; i++) {
    rc = fn(t, x + (size_t)i * cols, b, cols, lvl_n);
    memcpy(y + (size_t)i * cols, b, sizeof(double) * (size_t)cols);
  }
  for (int j = 0; j < cols && !rc; j++) {
    for (int i = 0; i < rows; i++) a[i] = y[(size_t)i * cols + j];
    rc = fn(t, a, b, rows, lvl_m);
    for (int i = 0; i < rows; i++) y[(size_t)i * cols + j] = b[i];
  }
  free(a);
  free(b);
  return rc;
}

/* BasicTransform.reverse(double[][], lvlM, lvlN) — BasicTransform.java:436-474:
 * every column with lvlM, then every row with lvlN. */
int orc_2d_reverse(int kind, const orc_taps* t, const double* y, double* x, int rows, int cols,
                   int lvl_m, int lvl_n) {
  orc_1d_fn fn = pick(kind, 0);
  double* a = (double*)malloc(sizeof(double) * (size_t)(rows > cols ? rows : cols));
  double* b = (double*)malloc(sizeof(double) * (size_t)(rows > cols ? rows : cols));
  int rc = 0;
  for (int j = 0; j < cols && !rc; j++) {
    for (int i = 0; i < rows; i++) a[i] = y[(size_t)i * cols + j];
    rc = fn(t, a, b, rows, lvl_m);
    for (int i = 0; i < rows; i++) x[(size_t)i * cols + j] = b[i];
  }
  for (int i = 0; i < rows && !rc; i++) {
    rc = fn(t, x + (size_t)i * cols, b, cols, lvl_n);
    memcpy(x + (size_t)i * cols, b, sizeof(double) * (size_t)cols);
  }
  free(a);
  free(b);
  return rc;
}

/* BasicTransform.forward(double[][][], lvlP, lvlQ, lvlR) — BasicTransform.java:509-560:
 * each [i][.][.] slice gets the 2-D forward with (lvlP, lvlQ) — i.e. its rows
 * (length R) with lvlQ and its columns (length Q) with lvlP — then every
 * (j,k) line along i gets the 1-D forward with lvlR. */
int orc_3d_forward(int kind, const orc_taps* t, const double* x, double* y, int P, int Q, int R,
                   int lvl_p, int lvl_q, int lvl_r) {
  orc_1d_fn fn = pick(kind, 1);
  size_t slice = (size_t)Q * R;
  int rc = 0;
  for (int i = 0; i < P && !rc; i++)
    rc = orc_2d_forward(kind, t, x + i * slice, y + i * slice, Q, R, lvl_p, lvl_q);
  double* a = (double*)malloc(sizeof(double) * (size_t)P);
  double* b = (double*)malloc(sizeof(double) * (size_t)P);
  for (size_t jk = 0; jk < slice && !rc; jk++) {
    for (int i = 0; i < P; i++) a[i] = y[i * slice + jk];
    rc = fn(t, a, b, P, lvl_r);
    for (int i = 0; i < P; i++) y[i * slice + jk] = b[i];
  }
  free(a);
  free(b);
  return rc;
}

/* BasicTransform.reverse(double[][][], lvlP, lvlQ, lvlR) — BasicTransform.java:602-659:
 * 2-D reverse on each slice first, then the 1-D reverse along i. */
int orc_3d_reverse(int kind, const orc_taps* t, const double* y, double* x, int P, int Q, int R,
                   int lvl_p, int lvl_q, int lvl_r) {
  orc_1d_fn fn = pick(kind, 0);
  size_t slice = (size_t)Q * R;
  int rc = 0;
  for (int i = 0; i < P && !rc; i++)
    rc = orc_2d_reverse(kind, t, y + i * slice, x + i * slice, Q, R, lvl_p, lvl_q);
  double* a = (double*)malloc(sizeof(double) * (size_t)P);
  double* b = (double*)malloc(sizeof(double) * (size_t)P);
  for (size_t jk = 0; jk < slice && !rc; jk++) {
    for (int i = 0; i < P; i++) a[i] = x[i * slice + jk];
    rc = fn(t, a, b, P, lvl_r);
    for (int i = 0; i < P; i++) x[i * slice + jk] = b[i];
  }
  free(a);
  free(b);
  return rc;
}

/* ------------------------------------------------------------------ MODWT */

/* MODWTTransform.normalize — MODWTTransform.java:599-606 */
static void modwt_normalize(double* f, int n) {
  double energy = 0.0;
  for (int i = 0; i < n; i++) energy += f[i] * f[i];
  double norm = sqrt(energy);
  if (norm > 1e-12)
    for (int i = 0; i < n; i++) f[i] /= norm;
}

/* MODWTTransform.initializeFilterCache — MODWTTransform.java:452-484:
 * g = lo/||lo||/sqrt(2), h = hi/||hi||/sqrt(2) (decomposition taps). */
void orc_modwt_filters(const orc_taps* t, double* g, double* h) {
  memcpy(g, t->lo, sizeof(double) * (size_t)t->L);
  memcpy(h, t->hi, sizeof(double) * (size_t)t->L);
  modwt_normalize(g, t->L);
  modwt_normalize(h, t->L);
  double s = sqrt(2.0);
  for (int i = 0; i < t->L; i++) {
    g[i] = g[i] / s;
    h[i] = h[i] / s;
  }
}

/* MODWTTransform.upsample — MODWTTransform.java:618-630 */
static double* modwt_upsample(const double* f, int L, int level, int* out_len) {
  if (level <= 1) {
    double* c = (double*)malloc(sizeof(double) * (size_t)L);
    memcpy(c, f, sizeof(double) * (size_t)L);
    *out_len = L;
    return c;
  }
  int gap = (1 << (level - 1)) - 1;
  int len = L + (L - 1) * gap;
  double* u = (double*)calloc((size_t)len, sizeof(double));
  for (int i = 0; i < L; i++) u[i * (gap + 1)] = f[i];
  *out_len = len;
  return u;
}

static int64_t floor_mod(int64_t a, int64_t n) {
  int64_t r = a % n;
  return r < 0 ? r + n : r;
}

/* MODWTTransform.circularConvolve — MODWTTransform.java:677-690 (DIRECT,
 * zero taps of the upsampled filter included, as written). */
static void circular_convolve(const double* s, int N, const double* f, int M, double* out) {
  for (int n = 0; n < N; n++) {
    double sum = 0.0;
    for (int m = 0; m < M; m++) sum += s[floor_mod((int64_t)n - m, N)] * f[m];
    out[n] = sum;
  }
}

/* MODWTTransform.circularConvolveAdjoint — MODWTTransform.java:703-716 */
static void circular_convolve_adjoint(const double* s, int N, const double* f, int M, double* out) {
  for (int n = 0; n < N; n++) {
    double sum = 0.0;
    for (int m = 0; m < M; m++) sum += s[floor_mod((int64_t)n + m, N)] * f[m];
    out[n] = sum;
  }
}

/* Count of non-finite samples at the circular positions a, a+1, .., a+len-1
 * (0 <= a < N, len <= N) from the prefix counts P[0..N]. */
static int64_t circ_count(const int64_t* P, int N, int64_t a, int64_t len) {
  if (a + len <= N) return P[a + len] - P[a];
  return (P[N] - P[a]) + P[a + len - N];
}

/* Same sums with the zero taps of the upsampled filter skipped: for finite
 * inputs adding x*0.0 (= +-0.0) to a sum that started at +0.0 never changes it,
 * so the sum is bit-identical to the loops above and ~2^(j-1) times faster.
 * A non-finite sample at a zero tap makes the loops above give NaN (x*0.0 is
 * NaN for x = +-inf or NaN), so the outputs whose window (m = 0 .. M-1,
 * M = (L-1)*stride + 1, wrapping mod N as often as it does) holds one at a
 * zero tap are set to NaN: the window's non-finite count (prefix sums) minus
 * the count at its L real taps.  Tests check the two forms agree bit for bit,
 * NaN positions included. */
static void circular_convolve_sparse(const double* s, int N, const double* f, int L, int stride,
                                     int adjoint, double* out) {
  for (int n = 0; n < N; n++) {
    double sum = 0.0;
    for (int l = 0; l < L; l++) {
      int64_t m = (int64_t)l * stride;
      sum += s[floor_mod(adjoint ? (int64_t)n + m : (int64_t)n - m, N)] * f[l];
    }
    out[n] = sum;
  }
  if (stride == 1 || N == 0) return;
  int64_t* P = (int64_t*)malloc(sizeof(int64_t) * ((size_t)N + 1));
  P[0] = 0;
  for (int i = 0; i < N; i++) P[i + 1] = P[i] + !isfinite(s[i]);
  const int64_t bad = P[N];
  if (bad > 0) {
    const int64_t M = (int64_t)(L - 1) * stride + 1, full = M / N, rem = M % N;
    for (int n = 0; n < N; n++) {
      /* forward: positions n, n-1, .., n-M+1; adjoint: n, n+1, .., n+M-1 */
      const int64_t a = adjoint ? n : floor_mod((int64_t)n - rem + 1, N);
      const int64_t cnt = full * bad + (rem ? circ_count(P, N, a, rem) : 0);
      int64_t real = 0;
      for (int l = 0; l < L; l++) {
        int64_t m = (int64_t)l * stride;
        real += !isfinite(s[floor_mod(adjoint ? (int64_t)n + m : (int64_t)n - m, N)]);
      }
      if (cnt > real) out[n] = NAN;
    }
  }
  free(P);
}

/* MODWTTransform.forwardMODWT — MODWTTransform.java:256-306.  out is
 * row-major [(J+1)][N] = [W_1 .. W_J, V_J].  sparse=0 runs the zero-padded
 * DIRECT loops as written; sparse=1 skips zero taps (bit-identical). */
int orc_modwt_forward(const orc_taps* t, const double* x, double* out, int N, int J, int sparse) {
  if (J < 1) return 2;
  if (J > 13) return 2;
  if (N == 0) return 0;
  int theo = 31 - __builtin_clz((unsigned)N);
  if (J > theo) return 2;
  double g[64], h[64];
  orc_modwt_filters(t, g, h);
  double* v = (double*)malloc(sizeof(double) * (size_t)N);
  double* vn = (double*)malloc(sizeof(double) * (size_t)N);
  memcpy(v, x, sizeof(double) * (size_t)N);
  for (int j = 1; j <= J; j++) {
    double* w = out + (size_t)(j - 1) * N;
    if (sparse) {
      circular_convolve_sparse(v, N, h, t->L, 1 << (j - 1), 0, w);
      circular_convolve_sparse(v, N, g, t->L, 1 << (j - 1), 0, vn);
    } else {
      int lg, lh;
      double* gu = modwt_upsample(g, t->L, j, &lg);
      double* hu = modwt_upsample(h, t->L, j, &lh);
      circular_convolve(v, N, hu, lh, w);
      circular_convolve(v, N, gu, lg, vn);
      free(gu);
      free(hu);
    }
    memcpy(v, vn, sizeof(double) * (size_t)N);
  }
  memcpy(out + (size_t)J * N, v, sizeof(double) * (size_t)N);
  free(v);
  free(vn);
  return 0;
}

/* MODWTTransform.inverseMODWT — MODWTTransform.java:337-375 */
int orc_modwt_inverse(const orc_taps* t, const double* in, double* x, int N, int J, int sparse) {
  if (J < 1 || N == 0) return 0;
  double g[64], h[64];
  orc_modwt_filters(t, g, h);
  double* v = (double*)malloc(sizeof(double) * (size_t)N);
  double* va = (double*)malloc(sizeof(double) * (size_t)N);
  double* vd = (double*)malloc(sizeof(double) * (size_t)N);
  memcpy(v, in + (size_t)J * N, sizeof(double) * (size_t)N);
  for (int j = J; j >= 1; j--) {
    const double* w = in + (size_t)(j - 1) * N;
    if (sparse) {
      circular_convolve_sparse(v, N, g, t->L, 1 << (j - 1), 1, va);
      circular_convolve_sparse(w, N, h, t->L, 1 << (j - 1), 1, vd);
    } else {
      int lg, lh;
      double* gu = modwt_upsample(g, t->L, j, &lg);
      double* hu = modwt_upsample(h, t->L, j, &lh);
      circular_convolve_adjoint(v, N, gu, lg, va);
      circular_convolve_adjoint(w, N, hu, lh, vd);
      free(gu);
      free(hu);
    }
    for (int i = 0; i < N; i++) v[i] = va[i] + vd[i];
  }
  memcpy(x, v, sizeof(double) * (size_t)N);
  free(v);
  free(va);
  free(vd);
  return 0;
}

/* java.util.Random-compatible generator (the seeded inputs of the reference's
 * tests, e.g. PropertyBasedTest.java:47 new Random(42); nextDouble()). */
void orc_java_random_doubles(int64_t seed, double* out, int64_t n) {
  const uint64_t mult = 0x5DEECE66DULL, add = 0xBULL, mask = (1ULL << 48) - 1;
  uint64_t s = ((uint64_t)seed ^ mult) & mask;
  for (int64_t i = 0; i < n; i++) {
    s = (s * mult + add) & mask;
    uint64_t a = s >> (48 - 26);
    s = (s * mult + add) & mask;
    uint64_t b = s >> (48 - 27);
    out[i] = (double)((a << 27) + b) * (1.0 / (double)(1ULL << 53));
  }
}

/* CompressorMagnitude.compress(double[]) (compressions/CompressorMagnitude.java:73-84)
 * with Compressor.compress(arr, magnitude) (Compressor.java:96-110): the
 * magnitude is the left-to-right sum of |x| divided by n; an entry survives
 * iff |x| >= magnitude * threshold.  threshold <= 0 -> 1.0 (Compressor.java:66-80).
 * Returns the magnitude. */
double orc_compress_magnitude(const double* x, double* y, int64_t n, double threshold) {
  if (threshold <= 0.0) threshold = 1.0;
  double mag = 0.0;
  for (int64_t i = 0; i < n; i++) mag += fabs(x[i]);
  mag /= (double)n;
  for (int64_t i = 0; i < n; i++) y[i] = fabs(x[i]) >= mag * threshold ? x[i] : 0.0;
  return mag;
}
