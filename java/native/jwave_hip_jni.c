/*
 * jwave_hip_jni.c — JNI shim between jwave.amd.HipNative and libjwave_hip.so.
 *
 * Every native pins the Java arrays (GetPrimitiveArrayCritical: no JNI calls
 * inside the window), calls the host-pointer C ABI entry (which copies to the
 * GPU, computes and copies back before returning) and unpins.  Inputs are
 * released with JNI_ABORT (never written back), outputs with 0.
 *
 * Build (needs a JDK; the development image has none — source only here):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *       -I../../include jwave_hip_jni.c -L../../jwave_amd/lib -ljwave_hip \
 *       -Wl,-rpath,'$ORIGIN' -o libjwave_hip_jni.so
 */
#include <jni.h>
#include <stdint.h>

#include "jwave_hip.h"

#define CTX(h) ((jwv_ctx*)(intptr_t)(h))

typedef struct {
  JNIEnv* env;
  jdoubleArray arr[6];
  double* ptr[6];
  jint mode[6];
  int n;
} pins;

static double* pin(pins* p, jdoubleArray a, jint mode) {
  double* d = (double*)(*p->env)->GetPrimitiveArrayCritical(p->env, a, NULL);
  p->arr[p->n] = a;
  p->ptr[p->n] = d;
  p->mode[p->n] = mode;
  p->n++;
  return d;
}

static void unpin_all(pins* p) {
  for (int i = p->n - 1; i >= 0; --i)
    if (p->ptr[i]) (*p->env)->ReleasePrimitiveArrayCritical(p->env, p->arr[i], p->ptr[i], p->mode[i]);
}

static jwv_taps taps_of(jint L, jint tw, jdouble scale, const double* lo, const double* hi,
                        const double* lor, const double* hir) {
  jwv_taps t;
  t.mother_wavelength = L;
  t.transform_wavelength = tw;
  t.lo = lo;
  t.hi = hi;
  t.lo_r = lor;
  t.hi_r = hir;
  t.reverse_scale = scale;
  return t;
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

#define PIN_TAPS(P)                                          \
  const double* lo = pin(&P, jlo, JNI_ABORT);                \
  const double* hi = pin(&P, jhi, JNI_ABORT);                \
  const double* lor = pin(&P, jlor, JNI_ABORT);              \
  const double* hir = pin(&P, jhir, JNI_ABORT);              \
  jwv_taps t = taps_of(L, tw, scale, lo, hi, lor, hir)

/* FastWaveletTransform / WaveletPacketTransform forward|reverse(double[], int) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transform1d(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint level, jint L, jint tw, jdouble scale, jdoubleArray jlo, jdoubleArray jhi,
    jdoubleArray jlor, jdoubleArray jhir) {
  const jsize n = (*env)->GetArrayLength(env, jx);
  pins P = {env, {0}, {0}, {0}, 0};
  PIN_TAPS(P);
  const double* x = pin(&P, jx, JNI_ABORT);
  double* y = pin(&P, jy, 0);
  int rc;
  if (kind == 0)
    rc = fwd ? jwv_fwt_fwd_f64(x, y, n, level, &t, CTX(ctx)) : jwv_fwt_rev_f64(x, y, n, level, &t, CTX(ctx));
  else
    rc = fwd ? jwv_wpt_fwd_f64(x, y, n, level, &t, CTX(ctx)) : jwv_wpt_rev_f64(x, y, n, level, &t, CTX(ctx));
  unpin_all(&P);
  return rc;
}

/* batched signals (one native call for many rows) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transformBatch(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint batch, jint n, jint level, jint L, jint tw, jdouble scale, jdoubleArray jlo,
    jdoubleArray jhi, jdoubleArray jlor, jdoubleArray jhir) {
  pins P = {env, {0}, {0}, {0}, 0};
  PIN_TAPS(P);
  const double* x = pin(&P, jx, JNI_ABORT);
  double* y = pin(&P, jy, 0);
  int rc;
  if (kind == 0)
    rc = fwd ? jwv_fwt_fwd_batch_f64(x, y, batch, n, n, level, &t, CTX(ctx))
             : jwv_fwt_rev_batch_f64(x, y, batch, n, n, level, &t, CTX(ctx));
  else
    rc = fwd ? jwv_wpt_fwd_batch_f64(x, y, batch, n, n, level, &t, CTX(ctx))
             : jwv_wpt_rev_batch_f64(x, y, batch, n, n, level, &t, CTX(ctx));
  unpin_all(&P);
  return rc;
}

/* BasicTransform.forward|reverse(double[][], lvlM, lvlN), rows packed by Java */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transform2d(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint rows, jint cols, jint lm, jint ln, jint L, jint tw, jdouble scale, jdoubleArray jlo,
    jdoubleArray jhi, jdoubleArray jlor, jdoubleArray jhir) {
  pins P = {env, {0}, {0}, {0}, 0};
  PIN_TAPS(P);
  const double* x = pin(&P, jx, JNI_ABORT);
  double* y = pin(&P, jy, 0);
  int rc;
  if (kind == 0)
    rc = fwd ? jwv_fwt2d_fwd_f64(x, y, rows, cols, lm, ln, &t, CTX(ctx))
             : jwv_fwt2d_rev_f64(x, y, rows, cols, lm, ln, &t, CTX(ctx));
  else
    rc = fwd ? jwv_wpt2d_fwd_f64(x, y, rows, cols, lm, ln, &t, CTX(ctx))
             : jwv_wpt2d_rev_f64(x, y, rows, cols, lm, ln, &t, CTX(ctx));
  unpin_all(&P);
  return rc;
}

/* BasicTransform.forward|reverse(double[][][], lvlP, lvlQ, lvlR) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_transform3d(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint p, jint q, jint r, jint lp, jint lq, jint lr, jint L, jint tw, jdouble scale,
    jdoubleArray jlo, jdoubleArray jhi, jdoubleArray jlor, jdoubleArray jhir) {
  pins P = {env, {0}, {0}, {0}, 0};
  PIN_TAPS(P);
  const double* x = pin(&P, jx, JNI_ABORT);
  double* y = pin(&P, jy, 0);
  int rc;
  if (kind == 0)
    rc = fwd ? jwv_fwt3d_fwd_f64(x, y, p, q, r, lp, lq, lr, &t, CTX(ctx))
             : jwv_fwt3d_rev_f64(x, y, p, q, r, lp, lq, lr, &t, CTX(ctx));
  else
    rc = fwd ? jwv_wpt3d_fwd_f64(x, y, p, q, r, lp, lq, lr, &t, CTX(ctx))
             : jwv_wpt3d_rev_f64(x, y, p, q, r, lp, lq, lr, &t, CTX(ctx));
  unpin_all(&P);
  return rc;
}

/* MODWTTransform.forwardMODWT(x, J) -> wv ; inverseMODWT(wv) -> x */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_modwt(
    JNIEnv* env, jclass cls, jlong ctx, jboolean fwd, jdoubleArray jx, jdoubleArray jwv, jint n,
    jint J, jint L, jint tw, jdoubleArray jlo, jdoubleArray jhi, jdoubleArray jlor,
    jdoubleArray jhir) {
  const jdouble scale = 1.0;
  pins P = {env, {0}, {0}, {0}, 0};
  PIN_TAPS(P);
  int rc;
  if (fwd) {
    const double* x = pin(&P, jx, JNI_ABORT);
    double* wv = pin(&P, jwv, 0);
    rc = jwv_modwt_fwd_f64(x, wv, n, J, &t, CTX(ctx));
  } else {
    const double* wv = pin(&P, jwv, JNI_ABORT);
    double* x = pin(&P, jx, 0);
    rc = jwv_modwt_inv_f64(wv, x, n, J, &t, CTX(ctx));
  }
  unpin_all(&P);
  return rc;
}

/* AncientEgyptianDecomposition(FWT | WPT).forward|reverse(double[]) of any
 * length: one call, the small pieces in one varlen launch (jwv_aed_*) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_aed(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jboolean fwd, jdoubleArray jx, jdoubleArray jy,
    jint L, jint tw, jdouble scale, jdoubleArray jlo, jdoubleArray jhi, jdoubleArray jlor,
    jdoubleArray jhir) {
  const jsize n = (*env)->GetArrayLength(env, jx);
  pins P = {env, {0}, {0}, {0}, 0};
  PIN_TAPS(P);
  const double* x = pin(&P, jx, JNI_ABORT);
  double* y = pin(&P, jy, 0);
  const int rc = fwd ? jwv_aed_fwd_f64(x, y, n, kind, &t, CTX(ctx))
                     : jwv_aed_rev_f64(x, y, n, kind, &t, CTX(ctx));
  unpin_all(&P);
  return rc;
}

/* WaveletTransform.decompose(double[]): mat = (log2 n + 1) * n, row p =
 * forward(x, p) (jwv_decompose_f64) */
JNIEXPORT jint JNICALL Java_jwave_amd_HipNative_decompose(
    JNIEnv* env, jclass cls, jlong ctx, jint kind, jdoubleArray jx, jdoubleArray jmat, jint L,
    jint tw, jdouble scale, jdoubleArray jlo, jdoubleArray jhi, jdoubleArray jlor,
    jdoubleArray jhir) {
  const jsize n = (*env)->GetArrayLength(env, jx);
  pins P = {env, {0}, {0}, {0}, 0};
  PIN_TAPS(P);
  const double* x = pin(&P, jx, JNI_ABORT);
  double* mat = pin(&P, jmat, 0);
  const int rc = jwv_decompose_f64(x, mat, n, kind, &t, CTX(ctx));
  unpin_all(&P);
  return rc;
}
