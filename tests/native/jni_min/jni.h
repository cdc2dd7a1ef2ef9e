/* Minimal JNI declarations for a syntax/type check of native/ndfl_jni.c in an image without a JDK
 * (tests/test_jni_glue.py).  Only the types and the JNIEnv functions the glue uses, with the
 * signatures of the JNI specification (member order does not matter for a compile-only check).
 * Test infrastructure: never used to build the shipped glue, which compiles against a real JDK. */
#ifndef NDFL_TEST_JNI_MIN_H
#define NDFL_TEST_JNI_MIN_H
#include <stdint.h>
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;
struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_ABORT 2
struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv*, const char*);
    jint (*ThrowNew)(JNIEnv*, jclass, const char*);
    jboolean (*ExceptionCheck)(JNIEnv*);
    jsize (*GetArrayLength)(JNIEnv*, jarray);
    jbyte* (*GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*);
    void (*ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint);
    void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);
    void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*);
    void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);
    void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
    void* (*GetDirectBufferAddress)(JNIEnv*, jobject);
    jlong (*GetDirectBufferCapacity)(JNIEnv*, jobject);
    jstring (*NewStringUTF)(JNIEnv*, const char*);
};
#endif
