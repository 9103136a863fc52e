/*
 * fake_jvm.c — TEST DOUBLE of the JVM side of JNI for the shim's CPU tests
 * (see tests/jni/jni.h).  Java arrays are {kind, length, data}; a region
 * access outside [0, length) leaves a pending java/lang/ArrayIndexOutOfBounds-
 * Exception and touches nothing, as the JVM does.  One pending exception per
 * thread (a JNIEnv is per thread).  Helpers fj_* are for the Python tests
 * (ctypes).
 */
#include "jni.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct fake_jobject {
  int kind; /* 1 double[], 2 long[], 3 String, 4 Class, 5 int[] */
  jsize len;
  void* data;
  char name[128];
};

static __thread char t_exc[128];
static __thread char t_msg[256];

static void throw_(const char* cls, const char* msg) {
  if (t_exc[0]) return; /* the first exception stays pending */
  snprintf(t_exc, sizeof t_exc, "%s", cls);
  snprintf(t_msg, sizeof t_msg, "%s", msg ? msg : "");
}

static int region_ok(jarray a, int kind, jsize start, jsize len) {
  if (!a || a->kind != kind) {
    throw_("java/lang/NullPointerException", "array");
    return 0;
  }
  if (start < 0 || len < 0 || (int64_t)start + len > a->len) {
    char m[96];
    snprintf(m, sizeof m, "Array region %d..%d out of bounds for length %d", start,
             start + len, a->len);
    throw_("java/lang/ArrayIndexOutOfBoundsException", m);
    return 0;
  }
  return 1;
}

static jsize GetArrayLength(JNIEnv* env, jarray a) { return a ? a->len : 0; }
static void GetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize s, jsize n, jdouble* b) {
  if (region_ok(a, 1, s, n)) memcpy(b, (double*)a->data + s, (size_t)n * sizeof(double));
}
static void SetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize s, jsize n, const jdouble* b) {
  if (region_ok(a, 1, s, n)) memcpy((double*)a->data + s, b, (size_t)n * sizeof(double));
}
static void SetLongArrayRegion(JNIEnv* env, jlongArray a, jsize s, jsize n, const jlong* b) {
  if (region_ok(a, 2, s, n)) memcpy((jlong*)a->data + s, b, (size_t)n * sizeof(jlong));
}
static void GetIntArrayRegion(JNIEnv* env, jintArray a, jsize s, jsize n, jint* b) {
  if (region_ok(a, 5, s, n)) memcpy(b, (jint*)a->data + s, (size_t)n * sizeof(jint));
}
static jboolean ExceptionCheck(JNIEnv* env) { return t_exc[0] != 0; }
static jstring NewStringUTF(JNIEnv* env, const char* s) {
  struct fake_jobject* o = calloc(1, sizeof *o);
  o->kind = 3;
  snprintf(o->name, sizeof o->name, "%s", s ? s : "");
  return o;
}
static jclass FindClass(JNIEnv* env, const char* name) {
  struct fake_jobject* o = calloc(1, sizeof *o);
  o->kind = 4;
  snprintf(o->name, sizeof o->name, "%s", name);
  return o;
}
static jint ThrowNew(JNIEnv* env, jclass cls, const char* msg) {
  throw_(cls ? cls->name : "?", msg);
  return 0;
}

static const struct JNINativeInterface_ g_table = {
    GetArrayLength, GetDoubleArrayRegion, SetDoubleArrayRegion, SetLongArrayRegion,
    GetIntArrayRegion, ExceptionCheck,    NewStringUTF,         FindClass,
    ThrowNew};
static const struct JNINativeInterface_* g_env = &g_table;

/* ---- helpers for the Python tests */
JNIEnv* fj_env(void) { return (JNIEnv*)&g_env; }
jdoubleArray fj_darray(jsize n, const double* init) {
  struct fake_jobject* o = calloc(1, sizeof *o);
  o->kind = 1;
  o->len = n;
  o->data = calloc(n > 0 ? (size_t)n : 1, sizeof(double));
  if (init) memcpy(o->data, init, (size_t)n * sizeof(double));
  return o;
}
jlongArray fj_larray(jsize n) {
  struct fake_jobject* o = calloc(1, sizeof *o);
  o->kind = 2;
  o->len = n;
  o->data = calloc(n > 0 ? (size_t)n : 1, sizeof(jlong));
  return o;
}
jintArray fj_iarray(jsize n, const jint* init) {
  struct fake_jobject* o = calloc(1, sizeof *o);
  o->kind = 5;
  o->len = n;
  o->data = calloc(n > 0 ? (size_t)n : 1, sizeof(jint));
  if (init) memcpy(o->data, init, (size_t)n * sizeof(jint));
  return o;
}
void* fj_data(jarray a) { return a->data; }
const char* fj_string(jstring s) { return s ? s->name : NULL; }
void fj_free(jobject o) {
  if (o) free(o->data);
  free(o);
}
const char* fj_exception(void) { return t_exc; }
const char* fj_exception_msg(void) { return t_msg; }
void fj_clear(void) { t_exc[0] = 0; t_msg[0] = 0; }
