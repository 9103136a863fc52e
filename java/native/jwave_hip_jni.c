/*
 * jwave_hip_jni.c — JNI shim between jwave.amd.HipNative and libjwave_hip.so.
 *
 * Arrays cross the boundary by copy, never by pinning the Java heap: inputs
 * are copied with GetDoubleArrayRegion into page-locked staging memory of the
 * calling thread (jwv_host_alloc), the host-pointer C ABI entry DMAs that
 * buffer straight to the GPU, computes, DMAs the result into a second
 * page-locked buffer, and SetDoubleArrayRegion copies it into the Java
 * output.  No JNI critical region is held while the GPU works, so the
 * collector is never blocked by a transform (a ForkJoin pool of callers,
 * ParallelTransform.java:240-270, keeps running).  Taps are copied into
 * small local arrays.
 *
 * Build (needs a JDK; the development image has none — source only here):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *       -I../../include jwave_hip_jni.c -L../../jwave_amd/lib -ljwave_hip \
 *       -lpthread -Wl,-rpath,'$ORIGIN' -o libjwave_hip_jni.so
 */
#include <jni.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

#include "jwave_hip.h"

#define CTX(h) ((jwv_ctx*)(intptr_t)(h))
#define STAGE_FAIL (-100) /* a Java exception is pending (bad array length) or no staging */

/* Per-thread page-locked staging: two buffers (in, out), grown on demand,
 * freed when the thread exits. */
typedef struct {
  jwv_ctx* ctx;
  void* p[2];
  int64_t bytes[2];
} staging;

static pthread_key_t g_stage_key;
static pthread_once_t g_stage_once = PTHREAD_ONCE_INIT;

static void stage_free(void* v) {
  staging* s = (staging*)v;
  for (int i = 0; i < 2; ++i)
    if (s->p[i]) jwv_host_free(s->ctx, s->p[i]);
  free(s);
}
static void stage_key_init(void) { pthread_key_create(&g_stage_key, stage_free); }

static double* stage_buf(jwv_ctx* ctx, int which, int64_t n) {
  pthread_once(&g_stage_once, stage_key_init);
  staging* s = (staging*)pthread_getspecific(g_stage_key);
  if (!s) {
    s = (staging*)calloc(1, sizeof(staging));
    if (!s) return NULL;
    s->ctx = ctx;
    pthread_setspecific(g_stage_key, s);
  }
  const int64_t bytes = (n > 0 ? n : 1) * (int64_t)sizeof(double);
  if (s->bytes[which] < bytes) {
    if (s->p[which]) jwv_host_free(s->ctx, s->p[which]);
    s->p[which] = NULL;
    s->bytes[which] = 0;
    s->ctx = ctx;
    if (jwv_host_alloc(ctx, bytes, &s->p[which]) != JWV_OK) return NULL;
    s->bytes[which] = bytes;
  }
  return (double*)s->p[which];
}

/* Java array -> staging buffer `which` (n doubles) */
static double* stage_in(JNIEnv* env, jwv_ctx* ctx, int which, jdoubleArray a, int64_t n) {
  double* d = stage_buf(ctx, which, n);
  if (!d) return NULL;
  if (n > 0) (*env)->GetDoubleArrayRegion(env, a, 0, (jsize)n, d);
  return (*env)->ExceptionCheck(env) ? NULL : d;
}
/* staging buffer -> Java array, only after a successful call */
static int stage_out(JNIEnv* env, jdoubleArray a, const double* d, int64_t n, int rc) {
  if (rc == JWV_OK && n > 0) {
    (*env)->SetDoubleArrayRegion(env, a, 0, (jsize)n, d);
    if ((*env)->ExceptionCheck(env)) return STAGE_FAIL;
  }
  return rc;
}

typedef struct {
  double lo[JWV_MAX_TAPS], hi[JWV_MAX_TAPS], lor[JWV_MAX_TAPS], hir[JWV_MAX_TAPS];
  jwv_taps t;
} taps_buf;

/* taps: copied (L <= JWV_MAX_TAPS, checked again by the library) */
static int taps_of(JNIEnv* env, taps_buf* b, jint L, jint tw, jdouble scale, jdoubleArray jlo,
                   jdoubleArray jhi, jdoubleArray jlor, jdoubleArray jhir) {
  if (L < 1 || L > JWV_MAX_TAPS) return JWV_ERR_BAD_CALL;
  (*env)->GetDoubleArrayRegion(env, jlo, 0, L, b->lo);
  (*env)->GetDoubleArrayRegion(env, jhi, 0, L, b->hi);
  (*env)->GetDoubleArrayRegion(env, jlor, 0, L, b->lor);
  (*env)->GetDoubleArrayRegion(env, jhir, 0, L, b->hir);
  if ((*env)->ExceptionCheck(env)) return STAGE_FAIL;
  b->t.mother_wavelength = L;
  b->t.transform_wavelength = tw;
  b->t.lo = b->lo;
  b->t.hi = b->hi;
  b->t.lo_r = b->lor;
  b->t.hi_r = b->hir;
  b->t.reverse_scale = scale;
  return JWV_OK;
}

JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_ctxCreate(JNIEnv* env, jclass cls, jint dev,
                                                          jlongArray out) {
  jwv_ctx* c = NULL;
  int rc = jwv_ctx_create(dev, &c);
  jlong h = (jlong)(intptr_t)c;
  (*env)->SetLongArrayRegion(env, out, 0, 1, &h);
  return rc;
}

JNIEXPORT jstring JNICALL Java_jwave_amd_HipNative_lastError(JNIEnv* env, jclass cls, jlong ctx) {
  return (*env)->NewStringUTF(env, jwv_last_error(CTX(ctx)));
}

#define TAPS(B)                                                      \
  taps_buf B;                                                        \
  {                                                                  \
    const int trc = taps_of(env, &B, L, tw, scale, jlo, jhi, jlor, jhir); \
    if (trc != JWV_OK) return trc;                                   \
  }                                                                  \
  const jwv_taps* t = &B.t

/* x (nx doubles) and y (ny doubles) staged; body sets rc from x, y */
#define STAGED(NX, NY, BODY)                                         \
  do {                                                               \
    const double* x = stage_in(env, CTX(ctx), 0, jx, (NX));          \
    double* y = stage_buf(CTX(ctx), 1, (NY));                        \
    if (!x || !y) return STAGE_FAIL;                                 \
    int rc;                                                          \
    BODY;                                                            \
    return stage_out(env, jy, y, (NY), rc);                          \
  } while (0)

/* FastWaveletTransform / WaveletPacketTransform forward|reverse(double[], int) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transform1d(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint level, jint L, jint tw, jdouble scale, jdoubleArray jlo, jdoubleArray jhi,
    jdoubleArray jlor, jdoubleArray jhir) {
  const int64_t n = (*env)->GetArrayLength(env, jx);
  TAPS(B);
  STAGED(n, n, {
    if (kind == 0)
      rc = fwd ? jwv_fwt_fwd_f64(x, y, n, level, t, CTX(ctx))
               : jwv_fwt_rev_f64(x, y, n, level, t, CTX(ctx));
    else
      rc = fwd ? jwv_wpt_fwd_f64(x, y, n, level, t, CTX(ctx))
               : jwv_wpt_rev_f64(x, y, n, level, t, CTX(ctx));
  });
}

/* batched signals (one native call for many rows) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transformBatch(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint batch, jint n, jint level, jint L, jint tw, jdouble scale, jdoubleArray jlo,
    jdoubleArray jhi, jdoubleArray jlor, jdoubleArray jhir) {
  const int64_t tot = (int64_t)batch * n;
  TAPS(B);
  STAGED(tot, tot, {
    if (kind == 0)
      rc = fwd ? jwv_fwt_fwd_batch_f64(x, y, batch, n, n, level, t, CTX(ctx))
               : jwv_fwt_rev_batch_f64(x, y, batch, n, n, level, t, CTX(ctx));
    else
      rc = fwd ? jwv_wpt_fwd_batch_f64(x, y, batch, n, n, level, t, CTX(ctx))
               : jwv_wpt_rev_batch_f64(x, y, batch, n, n, level, t, CTX(ctx));
  });
}

/* BasicTransform.forward|reverse(double[][], lvlM, lvlN), rows packed by Java */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transform2d(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint rows, jint cols, jint lm, jint ln, jint L, jint tw, jdouble scale, jdoubleArray jlo,
    jdoubleArray jhi, jdoubleArray jlor, jdoubleArray jhir) {
  const int64_t tot = (int64_t)rows * cols;
  TAPS(B);
  STAGED(tot, tot, {
    if (kind == 0)
      rc = fwd ? jwv_fwt2d_fwd_f64(x, y, rows, cols, lm, ln, t, CTX(ctx))
               : jwv_fwt2d_rev_f64(x, y, rows, cols, lm, ln, t, CTX(ctx));
    else
      rc = fwd ? jwv_wpt2d_fwd_f64(x, y, rows, cols, lm, ln, t, CTX(ctx))
               : jwv_wpt2d_rev_f64(x, y, rows, cols, lm, ln, t, CTX(ctx));
  });
}

/* BasicTransform.forward|reverse(double[][][], lvlP, lvlQ, lvlR) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transform3d(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint p, jint q, jint r, jint lp, jint lq, jint lr, jint L, jint tw, jdouble scale,
    jdoubleArray jlo, jdoubleArray jhi, jdoubleArray jlor, jdoubleArray jhir) {
  const int64_t tot = (int64_t)p * q * r;
  TAPS(B);
  STAGED(tot, tot, {
    if (kind == 0)
      rc = fwd ? jwv_fwt3d_fwd_f64(x, y, p, q, r, lp, lq, lr, t, CTX(ctx))
               : jwv_fwt3d_rev_f64(x, y, p, q, r, lp, lq, lr, t, CTX(ctx));
    else
      rc = fwd ? jwv_wpt3d_fwd_f64(x, y, p, q, r, lp, lq, lr, t, CTX(ctx))
               : jwv_wpt3d_rev_f64(x, y, p, q, r, lp, lq, lr, t, CTX(ctx));
  });
}

/* MODWTTransform.forwardMODWT(x, J) -> wv ; inverseMODWT(wv) -> x */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_modwt(
    JNIEnv* env, jclass cls, jlong ctx, jboolean fwd, jdoubleArray jx, jdoubleArray jwv, jint n,
    jint J, jint L, jint tw, jdoubleArray jlo, jdoubleArray jhi, jdoubleArray jlor,
    jdoubleArray jhir) {
  const jdouble scale = 1.0;
  const int64_t nw = (int64_t)(J + 1) * n;
  TAPS(B);
  if (fwd) {
    const double* x = stage_in(env, CTX(ctx), 0, jx, n);
    double* wv = stage_buf(CTX(ctx), 1, nw);
    if (!x || !wv) return STAGE_FAIL;
    return stage_out(env, jwv, wv, nw, jwv_modwt_fwd_f64(x, wv, n, J, t, CTX(ctx)));
  }
  const double* wv = stage_in(env, CTX(ctx), 0, jwv, nw);
  double* x = stage_buf(CTX(ctx), 1, n);
  if (!wv || !x) return STAGE_FAIL;
  return stage_out(env, jx, x, n, jwv_modwt_inv_f64(wv, x, n, J, t, CTX(ctx)));
}

/* AncientEgyptianDecomposition(FWT | WPT).forward|reverse(double[]) of any
 * length: one call, the small pieces in one varlen launch (jwv_aed_*) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_aed(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint L, jint tw, jdouble scale, jdoubleArray jlo, jdoubleArray jhi, jdoubleArray jlor,
    jdoubleArray jhir) {
  const int64_t n = (*env)->GetArrayLength(env, jx);
  TAPS(B);
  STAGED(n, n, {
    rc = fwd ? jwv_aed_fwd_f64(x, y, n, kind, t, CTX(ctx))
             : jwv_aed_rev_f64(x, y, n, kind, t, CTX(ctx));
  });
}

/* WaveletTransform.decompose(double[]): mat = (log2 n + 1) * n, row p =
 * forward(x, p) (jwv_decompose_f64) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_decompose(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jdoubleArray jx, jdoubleArray jmat, jint L,
    jint tw, jdouble scale, jdoubleArray jlo, jdoubleArray jhi, jdoubleArray jlor,
    jdoubleArray jhir) {
  const int64_t n = (*env)->GetArrayLength(env, jx);
  const int64_t nm = (*env)->GetArrayLength(env, jmat);
  jdoubleArray jy = jmat;
  TAPS(B);
  STAGED(n, nm, { rc = jwv_decompose_f64(x, y, n, kind, t, CTX(ctx)); });
}
