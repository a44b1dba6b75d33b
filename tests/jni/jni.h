/*
 * TEST-ONLY stand-in for <jni.h>: just the types and the JNIEnv functions that
 * zarr-java_amd/java/jni/zarrhip_jni.c calls, with the JNI specification's signatures, so that
 * the shim compiles and runs against tests/jni/fake_jvm.c without a JDK (none exists in this
 * container or on the GPU box).  It is not ABI-compatible with a real JVM (the function table
 * holds only these members); the product shim is built against $JAVA_HOME/include/jni.h
 * (INTEGRATION.md).
 */
#ifndef ZH_TEST_JNI_H
#define ZH_TEST_JNI_H

#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_OK 0
#define JNI_ABORT 2
#define JNI_COMMIT 1
#define JNI_FALSE 0
#define JNI_TRUE 1

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jobjectArray;
typedef jobject jstring;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  void* fake_state; /* the harness's JVM state (tests/jni/fake_jvm.c) */
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
  jobject (*NewLocalRef)(JNIEnv* env, jobject ref);
  void (*DeleteLocalRef)(JNIEnv* env, jobject obj);
  jint (*EnsureLocalCapacity)(JNIEnv* env, jint capacity);
  jsize (*GetArrayLength)(JNIEnv* env, jarray array);
  jobjectArray (*NewObjectArray)(JNIEnv* env, jsize len, jclass clazz, jobject init);
  jobject (*GetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index);
  void (*SetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index, jobject val);
  jbyteArray (*NewByteArray)(JNIEnv* env, jsize len);
  jlongArray (*NewLongArray)(JNIEnv* env, jsize len);
  void (*GetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf);
  void (*GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf);
  void (*GetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, jlong* buf);
  void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len,
                             const jbyte* buf);
  void (*SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len,
                             const jlong* buf);
  void* (*GetPrimitiveArrayCritical)(JNIEnv* env, jarray array, jboolean* isCopy);
  void (*ReleasePrimitiveArrayCritical)(JNIEnv* env, jarray array, void* carray, jint mode);
  const char* (*GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* isCopy);
  void (*ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* chars);
};

#endif
