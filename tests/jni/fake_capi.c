/*
 * fake_capi.c — TEST DOUBLE of libjwave_hip.so for the JNI shim's CPU tests:
 * the C-ABI entry points the shim calls, recording their arguments and
 * writing a recognisable function of the input (out[i] = 2*in[i % n_in] + k)
 * so the tests can check the shim's marshaling (array lengths, taps, staging)
 * without a GPU.  Host allocations are counted per thread and overall.  The
 * GPU test links the same shim against the real library instead.
 */
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "jwave_hip.h"

struct jwv_ctx { int dev; };
static struct jwv_ctx g_ctx = {0};

typedef struct {
  char name[48];
  int64_t a[6];
  int L, tw;
  double scale, lo0, hi0, lor0, hirL;
  int64_t nin, nout;
  const void* xin;
} fc_call;

static fc_call g_last;
static int g_rc = JWV_OK;
static atomic_long g_allocs, g_frees, g_live_bytes;
static __thread long t_allocs, t_frees;

int fc_set_rc(int rc) { int o = g_rc; g_rc = rc; return o; }
const fc_call* fc_last(void) { return &g_last; }
long fc_allocs(void) { return atomic_load(&g_allocs); }
long fc_frees(void) { return atomic_load(&g_frees); }
long fc_live_bytes(void) { return atomic_load(&g_live_bytes); }
long fc_thread_allocs(void) { return t_allocs; }
long fc_thread_frees(void) { return t_frees; }

int jwv_ctx_create(int device, jwv_ctx** out) {
  *out = &g_ctx;
  return JWV_OK;
}
const char* jwv_last_error(const jwv_ctx* c) { return "fake error text"; }
int jwv_host_alloc(jwv_ctx* c, int64_t bytes, void** p) {
  int64_t* h = (int64_t*)malloc((size_t)bytes + 16);
  if (!h) return JWV_ERR_DEVICE;
  h[0] = bytes;
  *p = h + 2;
  atomic_fetch_add(&g_allocs, 1);
  atomic_fetch_add(&g_live_bytes, bytes);
  ++t_allocs;
  return JWV_OK;
}
int jwv_host_free(jwv_ctx* c, void* p) {
  if (!p) return JWV_OK;
  int64_t* h = (int64_t*)p - 2;
  atomic_fetch_sub(&g_live_bytes, h[0]);
  free(h);
  atomic_fetch_add(&g_frees, 1);
  ++t_frees;
  return JWV_OK;
}

static int rec(const char* name, const double* x, int64_t nin, double* y, int64_t nout, int k,
               const jwv_taps* t, int64_t a0, int64_t a1, int64_t a2, int64_t a3, int64_t a4,
               int64_t a5) {
  memset(&g_last, 0, sizeof g_last);
  strncpy(g_last.name, name, sizeof g_last.name - 1);
  int64_t a[6] = {a0, a1, a2, a3, a4, a5};
  memcpy(g_last.a, a, sizeof a);
  g_last.L = t->mother_wavelength;
  g_last.tw = t->transform_wavelength;
  g_last.scale = t->reverse_scale;
  g_last.lo0 = t->lo[0];
  g_last.hi0 = t->hi[0];
  g_last.lor0 = t->lo_r[0];
  g_last.hirL = t->hi_r[t->mother_wavelength - 1];
  g_last.nin = nin;
  g_last.nout = nout;
  g_last.xin = x;
  if (g_rc != JWV_OK) return g_rc;
  for (int64_t i = 0; i < nout; ++i) y[i] = 2.0 * x[nin ? i % nin : 0] + k;
  return JWV_OK;
}

#define T1(NAME, K)                                                                  \
  int NAME(const double* x, double* y, int64_t n, int lv, const jwv_taps* t, jwv_ctx* c) { \
    return rec(#NAME, x, n, y, n, K, t, n, lv, 0, 0, 0, 0);                          \
  }
T1(jwv_fwt_fwd_f64, 1)
T1(jwv_fwt_rev_f64, 2)
T1(jwv_wpt_fwd_f64, 3)
T1(jwv_wpt_rev_f64, 4)

#define TB(NAME, K)                                                                   \
  int NAME(const double* x, double* y, int64_t b, int64_t n, int64_t ld, int lv,     \
           const jwv_taps* t, jwv_ctx* c) {                                          \
    return rec(#NAME, x, b * ld, y, b * ld, K, t, b, n, ld, lv, 0, 0);               \
  }
TB(jwv_fwt_fwd_batch_f64, 5)
TB(jwv_fwt_rev_batch_f64, 6)
TB(jwv_wpt_fwd_batch_f64, 7)
TB(jwv_wpt_rev_batch_f64, 8)

#define T2(NAME, K)                                                                   \
  int NAME(const double* x, double* y, int64_t r, int64_t cl, int lm, int ln,         \
           const jwv_taps* t, jwv_ctx* c) {                                          \
    return rec(#NAME, x, r * cl, y, r * cl, K, t, r, cl, lm, ln, 0, 0);              \
  }
T2(jwv_fwt2d_fwd_f64, 9)
T2(jwv_fwt2d_rev_f64, 10)
T2(jwv_wpt2d_fwd_f64, 11)
T2(jwv_wpt2d_rev_f64, 12)

#define T3(NAME, K)                                                                   \
  int NAME(const double* x, double* y, int64_t p, int64_t q, int64_t r, int lp, int lq, \
           int lr, const jwv_taps* t, jwv_ctx* c) {                                  \
    return rec(#NAME, x, p * q * r, y, p * q * r, K, t, p, q, r, lp, lq, lr);        \
  }
T3(jwv_fwt3d_fwd_f64, 13)
T3(jwv_fwt3d_rev_f64, 14)
T3(jwv_wpt3d_fwd_f64, 15)
T3(jwv_wpt3d_rev_f64, 16)
T3(jwv_fwt3d_rev_pt_f64, 22)
T3(jwv_wpt3d_rev_pt_f64, 23)

int jwv_modwt_fwd_f64(const double* x, double* wv, int64_t n, int J, const jwv_taps* t,
                      jwv_ctx* c) {
  return rec("jwv_modwt_fwd_f64", x, n, wv, (J + 1) * n, 17, t, n, J, 0, 0, 0, 0);
}
int jwv_modwt_inv_f64(const double* wv, double* x, int64_t n, int J, const jwv_taps* t,
                      jwv_ctx* c) {
  return rec("jwv_modwt_inv_f64", wv, (J + 1) * n, x, n, 18, t, n, J, 0, 0, 0, 0);
}
int jwv_aed_fwd_f64(const double* x, double* y, int64_t n, int tr, const jwv_taps* t,
                    jwv_ctx* c) {
  return rec("jwv_aed_fwd_f64", x, n, y, n, 19, t, n, tr, 0, 0, 0, 0);
}
int jwv_aed_rev_f64(const double* x, double* y, int64_t n, int tr, const jwv_taps* t,
                    jwv_ctx* c) {
  return rec("jwv_aed_rev_f64", x, n, y, n, 20, t, n, tr, 0, 0, 0, 0);
}
int jwv_decompose_f64(const double* x, double* mat, int64_t n, int tr, const jwv_taps* t,
                      jwv_ctx* c) {
  int lg = 0;
  while (((int64_t)1 << lg) < n) ++lg;
  return rec("jwv_decompose_f64", x, n, mat, (lg + 1) * n, 21, t, n, tr, 0, 0, 0, 0);
}

/* multi-device context: records the device list; batches go through rec()
 * with k = 30..33 and the device count in a[4] */
struct jwv_mctx { int n; int dev[16]; };
static struct jwv_mctx g_mctx;
int fc_mctx_devices(int* out) {
  for (int i = 0; i < g_mctx.n; ++i) out[i] = g_mctx.dev[i];
  return g_mctx.n;
}
int jwv_mctx_create(const int* devices, int n, jwv_mctx** out) {
  g_mctx.n = n < 16 ? n : 16;
  for (int i = 0; i < g_mctx.n; ++i) g_mctx.dev[i] = devices[i];
  *out = &g_mctx;
  return JWV_OK;
}
const char* jwv_mctx_last_error(const jwv_mctx* m) { return "fake multi error text"; }
jwv_ctx* jwv_mctx_ctx(jwv_mctx* m, int i) { return (m && i >= 0 && i < m->n) ? &g_ctx : NULL; }
#define TM(NAME, K)                                                                   \
  int NAME(const double* x, double* y, int64_t b, int64_t n, int64_t ld, int lv,     \
           const jwv_taps* t, jwv_mctx* m) {                                         \
    return rec(#NAME, x, b * ld, y, b * ld, K, t, b, n, ld, lv, m->n, 0);            \
  }
TM(jwv_m_fwt_fwd_batch_f64, 30)
TM(jwv_m_fwt_rev_batch_f64, 31)
TM(jwv_m_wpt_fwd_batch_f64, 32)
TM(jwv_m_wpt_rev_batch_f64, 33)
#define TM2(NAME, K)                                                                  \
  int NAME(const double* x, double* y, int64_t r, int64_t cl, int lm, int ln,         \
           const jwv_taps* t, jwv_mctx* m) {                                         \
    return rec(#NAME, x, r * cl, y, r * cl, K, t, r, cl, lm, ln, m->n, 0);           \
  }
TM2(jwv_m_fwt2d_fwd_f64, 34)
TM2(jwv_m_fwt2d_rev_f64, 35)
TM2(jwv_m_wpt2d_fwd_f64, 36)
TM2(jwv_m_wpt2d_rev_f64, 37)
int jwv_m_modwt_fwd_batch_f64(const double* x, double* wv, int64_t b, int64_t n, int J,
                              const jwv_taps* t, jwv_mctx* m) {
  return rec("jwv_m_modwt_fwd_batch_f64", x, b * n, wv, b * (J + 1) * n, 38, t, b, n, J, m->n, 0,
             0);
}
int jwv_m_modwt_inv_batch_f64(const double* wv, double* x, int64_t b, int64_t n, int J,
                              const jwv_taps* t, jwv_mctx* m) {
  return rec("jwv_m_modwt_inv_batch_f64", wv, b * (J + 1) * n, x, b * n, 39, t, b, n, J, m->n, 0,
             0);
}
int jwv_modwt_fwd_batch_f64(const double* x, double* wv, int64_t b, int64_t n, int J,
                            const jwv_taps* t, jwv_ctx* c) {
  return rec("jwv_modwt_fwd_batch_f64", x, b * n, wv, b * (J + 1) * n, 40, t, b, n, J, 0, 0, 0);
}
int jwv_modwt_inv_batch_f64(const double* wv, double* x, int64_t b, int64_t n, int J,
                            const jwv_taps* t, jwv_ctx* c) {
  return rec("jwv_modwt_inv_batch_f64", wv, b * (J + 1) * n, x, b * n, 41, t, b, n, J, 0, 0, 0);
}
