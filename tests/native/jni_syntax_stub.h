/*
 * jni_syntax_stub.h -- NOT a JDK header.  This container has no JDK, so
 * tests/test_jni.py checks the generated JNI forwarders (jni/ecx_jni.c) with
 * `gcc -fsyntax-only` against this file: the JNI types and the function-table entries
 * ecx_jni.c uses, declared with the shapes of the JNI specification (jni.h of any JDK).
 * The table here holds only those entries (not the JDK's slot layout), which is all the
 * forwarders reference by name; tests/native/jni_fake_env.c fills it with fakes so that
 * tests/test_jni_runtime.py can execute the forwarders.  The real build (jni/Makefile)
 * uses $JAVA_HOME's jni.h.
 */
#ifndef JNI_SYNTAX_STUB_H
#define JNI_SYNTAX_STUB_H
#include <stdint.h>
typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef int16_t jshort;
typedef uint8_t jboolean;
typedef jint jsize;
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jobjectArray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jshortArray;
#define JNIEXPORT
#define JNICALL
#define JNI_ABORT 2
struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
    jsize (*GetArrayLength)(JNIEnv *env, jarray array);
    jobject (*GetObjectArrayElement)(JNIEnv *env, jobjectArray array, jsize index);
    void (*GetIntArrayRegion)(JNIEnv *env, jintArray array, jsize start, jsize len, jint *buf);
    void (*GetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, jbyte *buf);
    void (*SetLongArrayRegion)(JNIEnv *env, jlongArray array, jsize start, jsize len, const jlong *buf);
    void *(*GetPrimitiveArrayCritical)(JNIEnv *env, jarray array, jboolean *isCopy);
    void (*ReleasePrimitiveArrayCritical)(JNIEnv *env, jarray array, void *carray, jint mode);
    void (*DeleteLocalRef)(JNIEnv *env, jobject obj);
    jstring (*NewStringUTF)(JNIEnv *env, const char *utf);
    void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);
    jobject (*NewDirectByteBuffer)(JNIEnv *env, void *address, jlong capacity);
    jlong (*GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
};
#endif
