/*
 * jni.h — TEST DOUBLE, not a JDK header.  The development image has no JDK,
 * so the JNI shim (java/native/jwave_hip_jni.c) is compiled for its CPU tests
 * against this minimal stand-in: the JNI types and the nine JNIEnv functions
 * the shim calls, with the real JNI calling shape ((*env)->Fn(env, ...)).
 * The function table is filled by tests/jni/fake_jvm.c, which models Java
 * arrays and the pending-exception state (ArrayIndexOutOfBounds on a bad
 * region, ThrowNew).  A real build uses $JAVA_HOME/include/jni.h instead
 * (INTEGRATION.md); nothing here is shipped.
 */
#ifndef JWV_TEST_FAKE_JNI_H
#define JWV_TEST_FAKE_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_TRUE 1
#define JNI_FALSE 0

typedef int32_t jint;
typedef int64_t jlong;
typedef double jdouble;
typedef uint8_t jboolean;
typedef jint jsize;

typedef struct fake_jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jdoubleArray;
typedef jarray jlongArray;
typedef jarray jintArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jsize (*GetArrayLength)(JNIEnv* env, jarray a);
  void (*GetDoubleArrayRegion)(JNIEnv* env, jdoubleArray a, jsize start, jsize len, jdouble* buf);
  void (*SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray a, jsize start, jsize len,
                               const jdouble* buf);
  void (*SetLongArrayRegion)(JNIEnv* env, jlongArray a, jsize start, jsize len, const jlong* buf);
  void (*GetIntArrayRegion)(JNIEnv* env, jintArray a, jsize start, jsize len, jint* buf);
  jboolean (*ExceptionCheck)(JNIEnv* env);
  jstring (*NewStringUTF)(JNIEnv* env, const char* s);
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass cls, const char* msg);
};

#endif
