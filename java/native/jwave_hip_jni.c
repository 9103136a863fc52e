/*
 * jwave_hip_jni.c — JNI shim between jwave.amd.HipNative and libjwave_hip.so.
 *
 * Arrays cross the boundary by copy, never by pinning the Java heap: inputs
 * are copied with GetDoubleArrayRegion into page-locked staging memory of the
 * calling thread (jwv_host_alloc; arrays above 64 MiB into pageable memory
 * of the call), the host-pointer C ABI entry DMAs that buffer to the GPU,
 * computes, DMAs the result into a second staging buffer, and
 * SetDoubleArrayRegion copies it into the Java output.  Bad arrays (too
 * short), bad taps and allocation failures leave a Java exception pending
 * (ArrayIndexOutOfBounds / IllegalArgument / OutOfMemoryError) and return
 * STAGE_FAIL before any GPU work; other statuses go to HipNative.check.  No JNI critical region is held while the GPU works, so the
 * collector is never blocked by a transform (a ForkJoin pool of callers,
 * ParallelTransform.java:240-270, keeps running).  Taps are copied into
 * small local arrays.
 *
 * Build (needs a JDK; the development image has none: tests/jni compiles and
 * runs this file against a JNI test double, tests/test_jni_shim.py):
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
#define STAGE_FAIL (-100) /* a Java exception is pending: bad array, bad taps, no memory */

/* Per-thread page-locked staging: two buffers (in, out) of at most
 * STAGE_PIN_MAX bytes each, grown on demand and kept for the thread's next
 * call, freed when the thread exits.  Larger arrays are staged in pageable
 * memory allocated for the one call (the library's host entries then move
 * them through their own pinned chunk ring), so a pool thread that once
 * transformed a big matrix does not keep gigabytes pinned. */
#define STAGE_PIN_MAX ((int64_t)64 << 20)

typedef struct {
  jwv_ctx* ctx;
  void* p[2];
  int64_t bytes[2];
} staging;

typedef struct {
  double* p;
  int owned; /* 1: pageable, freed by buf_put */
} buf_t;

static pthread_key_t g_stage_key;
static pthread_once_t g_stage_once = PTHREAD_ONCE_INIT;

static void stage_free(void* v) {
  staging* s = (staging*)v;
  for (int i = 0; i < 2; ++i)
    if (s->p[i]) jwv_host_free(s->ctx, s->p[i]);
  free(s);
}
static void stage_key_init(void) { pthread_key_create(&g_stage_key, stage_free); }

static void throw_java(JNIEnv* env, const char* cls, const char* msg) {
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, msg);
}

/* staging buffer `which` for n doubles; 0, or STAGE_FAIL with an
 * OutOfMemoryError pending */
static int buf_get(JNIEnv* env, jwv_ctx* ctx, int which, int64_t n, buf_t* b) {
  const int64_t bytes = (n > 0 ? n : 1) * (int64_t)sizeof(double);
  b->p = NULL;
  b->owned = 0;
  if (bytes > STAGE_PIN_MAX) {
    b->p = (double*)malloc((size_t)bytes);
    b->owned = 1;
  } else {
    pthread_once(&g_stage_once, stage_key_init);
    staging* s = (staging*)pthread_getspecific(g_stage_key);
    if (!s && (s = (staging*)calloc(1, sizeof(staging))) != NULL) {
      s->ctx = ctx;
      pthread_setspecific(g_stage_key, s);
    }
    if (s && s->bytes[which] < bytes) {
      if (s->p[which]) jwv_host_free(s->ctx, s->p[which]);
      s->p[which] = NULL;
      s->bytes[which] = 0;
      s->ctx = ctx;
      if (jwv_host_alloc(ctx, bytes, &s->p[which]) == JWV_OK) s->bytes[which] = bytes;
    }
    if (s && s->bytes[which] >= bytes) b->p = (double*)s->p[which];
  }
  if (!b->p) {
    throw_java(env, "java/lang/OutOfMemoryError", "jwave_hip_jni: no staging memory");
    return STAGE_FAIL;
  }
  return 0;
}
static void buf_put(buf_t* b) {
  if (b->owned) free(b->p);
  b->p = NULL;
}

/* Java array a (n doubles read) -> staging buffer `which` */
static int stage_in(JNIEnv* env, jwv_ctx* ctx, int which, jdoubleArray a, int64_t n, buf_t* b) {
  if (buf_get(env, ctx, which, n, b)) return STAGE_FAIL;
  if (n > 0) (*env)->GetDoubleArrayRegion(env, a, 0, (jsize)n, b->p);
  if ((*env)->ExceptionCheck(env)) {
    buf_put(b);
    return STAGE_FAIL;
  }
  return 0;
}
/* the output array must hold n doubles: checked before any GPU work */
static int out_fits(JNIEnv* env, jdoubleArray a, int64_t n) {
  if ((int64_t)(*env)->GetArrayLength(env, a) >= n) return 1;
  throw_java(env, "java/lang/ArrayIndexOutOfBoundsException",
             "jwave_hip_jni: output array shorter than the transform");
  return 0;
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

/* taps: copied (1 <= L <= JWV_MAX_TAPS, else IllegalArgumentException) */
static int taps_of(JNIEnv* env, taps_buf* b, jint L, jint tw, jdouble scale, jdoubleArray jlo,
                   jdoubleArray jhi, jdoubleArray jlor, jdoubleArray jhir) {
  if (L < 1 || L > JWV_MAX_TAPS) {
    throw_java(env, "java/lang/IllegalArgumentException",
               "jwave_hip_jni: filter length outside 1..64");
    return STAGE_FAIL;
  }
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

/* jx (NX doubles) and jy (NY doubles) staged; BODY sets rc from x, y */
#define STAGED(JX, NX, JY, NY, BODY)                                 \
  do {                                                               \
    if (!out_fits(env, (JY), (NY))) return STAGE_FAIL;               \
    buf_t bx_, by_;                                                  \
    if (stage_in(env, CTX(ctx), 0, (JX), (NX), &bx_)) return STAGE_FAIL; \
    if (buf_get(env, CTX(ctx), 1, (NY), &by_)) {                     \
      buf_put(&bx_);                                                 \
      return STAGE_FAIL;                                             \
    }                                                                \
    const double* x = bx_.p;                                         \
    double* y = by_.p;                                               \
    int rc;                                                          \
    BODY;                                                            \
    rc = stage_out(env, (JY), y, (NY), rc);                          \
    buf_put(&bx_);                                                   \
    buf_put(&by_);                                                   \
    return rc;                                                       \
  } while (0)

/* FastWaveletTransform / WaveletPacketTransform forward|reverse(double[], int) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transform1d(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint level, jint L, jint tw, jdouble scale, jdoubleArray jlo, jdoubleArray jhi,
    jdoubleArray jlor, jdoubleArray jhir) {
  const int64_t n = (*env)->GetArrayLength(env, jx);
  TAPS(B);
  STAGED(jx, n, jy, n, {
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
  STAGED(jx, tot, jy, tot, {
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
  STAGED(jx, tot, jy, tot, {
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
  STAGED(jx, tot, jy, tot, {
    if (kind == 0)
      rc = fwd ? jwv_fwt3d_fwd_f64(x, y, p, q, r, lp, lq, lr, t, CTX(ctx))
               : jwv_fwt3d_rev_f64(x, y, p, q, r, lp, lq, lr, t, CTX(ctx));
    else
      rc = fwd ? jwv_wpt3d_fwd_f64(x, y, p, q, r, lp, lq, lr, t, CTX(ctx))
               : jwv_wpt3d_rev_f64(x, y, p, q, r, lp, lq, lr, t, CTX(ctx));
  });
}

/* ParallelTransform.reverse(double[][][], lvlP, lvlQ, lvlR) order: the P axis
 * first, then the slices (ParallelTransform.java:183-216; jwv_*3d_rev_pt_f64) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transform3dPt(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jdoubleArray jx, jdoubleArray jy, jint p,
    jint q, jint r, jint lp, jint lq, jint lr, jint L, jint tw, jdouble scale, jdoubleArray jlo,
    jdoubleArray jhi, jdoubleArray jlor, jdoubleArray jhir) {
  const int64_t tot = (int64_t)p * q * r;
  TAPS(B);
  STAGED(jx, tot, jy, tot, {
    rc = kind == 0 ? jwv_fwt3d_rev_pt_f64(x, y, p, q, r, lp, lq, lr, t, CTX(ctx))
                   : jwv_wpt3d_rev_pt_f64(x, y, p, q, r, lp, lq, lr, t, CTX(ctx));
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
  if (fwd) STAGED(jx, n, jwv, nw, { rc = jwv_modwt_fwd_f64(x, y, n, J, t, CTX(ctx)); });
  STAGED(jwv, nw, jx, n, { rc = jwv_modwt_inv_f64(x, y, n, J, t, CTX(ctx)); });
}

/* AncientEgyptianDecomposition(FWT | WPT).forward|reverse(double[]) of any
 * length: one call, the small pieces in one varlen launch (jwv_aed_*) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_aed(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint L, jint tw, jdouble scale, jdoubleArray jlo, jdoubleArray jhi, jdoubleArray jlor,
    jdoubleArray jhir) {
  const int64_t n = (*env)->GetArrayLength(env, jx);
  TAPS(B);
  STAGED(jx, n, jy, n, {
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
  TAPS(B);
  STAGED(jx, n, jmat, nm, { rc = jwv_decompose_f64(x, y, n, kind, t, CTX(ctx)); });
}

/* ---- multi-device batches (jwv_mctx; HipNative.mctx, jwave.hip.devices) ---- */
#define MCTX(h) ((jwv_mctx*)(intptr_t)(h))

JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_mctxCreate(JNIEnv* env, jclass cls,
                                                           jintArray jdev, jlongArray out) {
  const jsize n = (*env)->GetArrayLength(env, jdev);
  if (n < 1 || n > 1024) {
    throw_java(env, "java/lang/IllegalArgumentException", "jwave_hip_jni: 1..1024 devices");
    return STAGE_FAIL;
  }
  jint dev[1024];
  (*env)->GetIntArrayRegion(env, jdev, 0, n, dev);
  if ((*env)->ExceptionCheck(env)) return STAGE_FAIL;
  int d[1024];
  for (jsize i = 0; i < n; ++i) d[i] = (int)dev[i];
  jwv_mctx* m = NULL;
  const int rc = jwv_mctx_create(d, (int)n, &m);
  jlong h = (jlong)(intptr_t)m;
  (*env)->SetLongArrayRegion(env, out, 0, 1, &h);
  return rc;
}

JNIEXPORT jstring JNICALL Java_jwave_amd_HipNative_mctxLastError(JNIEnv* env, jclass cls,
                                                                 jlong mctx) {
  return (*env)->NewStringUTF(env, jwv_mctx_last_error(MCTX(mctx)));
}

/* batched signals split over the devices of a multi-context: staged once
 * through the calling thread's pinned staging (device 0's context allocates
 * it; page-locked memory is DMA-able by every device), then one call that
 * runs every device's block concurrently */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transformBatchMulti(
    JNIEnv* env, jclass cls, jlong mctx, jint kind, jboolean fwd, jdoubleArray jx,
    jdoubleArray jy, jint batch, jint n, jint level, jint L, jint tw, jdouble scale,
    jdoubleArray jlo, jdoubleArray jhi, jdoubleArray jlor, jdoubleArray jhir) {
  const int64_t tot = (int64_t)batch * n;
  const jlong ctx = (jlong)(intptr_t)jwv_mctx_ctx(MCTX(mctx), 0);
  if (!ctx) {
    throw_java(env, "java/lang/IllegalArgumentException", "jwave_hip_jni: no multi-context");
    return STAGE_FAIL;
  }
  TAPS(B);
  STAGED(jx, tot, jy, tot, {
    if (kind == 0)
      rc = fwd ? jwv_m_fwt_fwd_batch_f64(x, y, batch, n, n, level, t, MCTX(mctx))
               : jwv_m_fwt_rev_batch_f64(x, y, batch, n, n, level, t, MCTX(mctx));
    else
      rc = fwd ? jwv_m_wpt_fwd_batch_f64(x, y, batch, n, n, level, t, MCTX(mctx))
               : jwv_m_wpt_rev_batch_f64(x, y, batch, n, n, level, t, MCTX(mctx));
  });
}

/* BasicTransform / ParallelTransform forward|reverse(double[][]) over the
 * devices of a multi-context: row blocks, one device-to-device exchange,
 * column slabs (jwv_m_{fwt,wpt}2d_*); staged once like transformBatchMulti */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transform2dMulti(
    JNIEnv* env, jclass cls, jlong mctx, jint kind, jboolean fwd, jdoubleArray jx,
    jdoubleArray jy, jint rows, jint cols, jint lvlM, jint lvlN, jint L, jint tw, jdouble scale,
    jdoubleArray jlo, jdoubleArray jhi, jdoubleArray jlor, jdoubleArray jhir) {
  const int64_t tot = (int64_t)rows * cols;
  const jlong ctx = (jlong)(intptr_t)jwv_mctx_ctx(MCTX(mctx), 0);
  if (!ctx) {
    throw_java(env, "java/lang/IllegalArgumentException", "jwave_hip_jni: no multi-context");
    return STAGE_FAIL;
  }
  TAPS(B);
  STAGED(jx, tot, jy, tot, {
    if (kind == 0)
      rc = fwd ? jwv_m_fwt2d_fwd_f64(x, y, rows, cols, lvlM, lvlN, t, MCTX(mctx))
               : jwv_m_fwt2d_rev_f64(x, y, rows, cols, lvlM, lvlN, t, MCTX(mctx));
    else
      rc = fwd ? jwv_m_wpt2d_fwd_f64(x, y, rows, cols, lvlM, lvlN, t, MCTX(mctx))
               : jwv_m_wpt2d_rev_f64(x, y, rows, cols, lvlM, lvlN, t, MCTX(mctx));
  });
}

/* MODWTTransform.forwardMODWT / inverseMODWT of `batch` signals of length n:
 * x [batch][n], wv [batch][J+1][n] (jwv_m_modwt_*_batch_f64: contiguous
 * blocks of signals per device) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_modwtBatchMulti(
    JNIEnv* env, jclass cls, jlong mctx, jboolean fwd, jdoubleArray jx, jdoubleArray jwv,
    jint batch, jint n, jint J, jint L, jint tw, jdoubleArray jlo, jdoubleArray jhi,
    jdoubleArray jlor, jdoubleArray jhir) {
  const jdouble scale = 1.0;
  const int64_t nx = (int64_t)batch * n, nw = (int64_t)batch * (J + 1) * n;
  const jlong ctx = (jlong)(intptr_t)jwv_mctx_ctx(MCTX(mctx), 0);
  if (!ctx) {
    throw_java(env, "java/lang/IllegalArgumentException", "jwave_hip_jni: no multi-context");
    return STAGE_FAIL;
  }
  TAPS(B);
  if (fwd) STAGED(jx, nx, jwv, nw, {
    rc = jwv_m_modwt_fwd_batch_f64(x, y, batch, n, J, t, MCTX(mctx));
  });
  STAGED(jwv, nw, jx, nx, { rc = jwv_m_modwt_inv_batch_f64(x, y, batch, n, J, t, MCTX(mctx)); });
}

/* the same batch on this thread's device (jwv_modwt_*_batch_f64) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_modwtBatch(
    JNIEnv* env, jclass cls, jlong ctx, jboolean fwd, jdoubleArray jx, jdoubleArray jwv,
    jint batch, jint n, jint J, jint L, jint tw, jdoubleArray jlo, jdoubleArray jhi,
    jdoubleArray jlor, jdoubleArray jhir) {
  const jdouble scale = 1.0;
  const int64_t nx = (int64_t)batch * n, nw = (int64_t)batch * (J + 1) * n;
  TAPS(B);
  if (fwd) STAGED(jx, nx, jwv, nw, {
    rc = jwv_modwt_fwd_batch_f64(x, y, batch, n, J, t, CTX(ctx));
  });
  STAGED(jwv, nw, jx, nx, { rc = jwv_modwt_inv_batch_f64(x, y, batch, n, J, t, CTX(ctx)); });
}
