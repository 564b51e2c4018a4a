/*
 * jni_fake_env.c -- test harness, NOT a JVM.  A JNIEnv whose function table (the entries
 * jni/ecx_jni.c uses, declared in jni_syntax_stub.h) is backed by fakes over C memory,
 * so the generated JNI forwarders can be EXECUTED without a JDK: a
 * "primitive array" wraps caller memory (no copy, so GetPrimitiveArrayCritical hands the
 * export the caller's bytes, as HotSpot does for non-moving pins), an "object array"
 * holds element references.  The fakes also check the JNI rules the forwarders promise:
 * no non-critical JNI call while a critical pin is held, every pin released, indexes in
 * range, and critical pins only on primitive arrays.  tests/test_jni_runtime.py drives
 * it through ctypes (tests/native/Makefile builds libjnitest.so = this file + ecx_jni.c,
 * linked against libecx.so).
 */
#define _POSIX_C_SOURCE 200809L
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

struct _jobject {
    int kind;       /* 1 = primitive array, 2 = object array, 3 = string, 4 = direct ByteBuffer */
    jsize len;      /* elements */
    int elem_size;  /* bytes per element (primitive arrays) */
    void *data;     /* primitive / direct buffer: caller memory; object: jobject[len]; string: char[] */
    jlong capacity; /* direct buffer: bytes */
};

static int64_t g_pins_now, g_pins_total, g_unpins_total, g_violations, g_deleted, g_jni_calls_pinned;
static int64_t g_last_release_mode = -1;

static void jni_call(void) {
    if (g_pins_now > 0) {
        ++g_jni_calls_pinned;
        ++g_violations;
    }
}

static jsize f_GetArrayLength(JNIEnv *env, jarray a) {
    (void)env;
    jni_call();
    if (!a || (a->kind != 1 && a->kind != 2)) {
        ++g_violations;
        return 0;
    }
    return a->len;
}

static jobject f_GetObjectArrayElement(JNIEnv *env, jobjectArray a, jsize i) {
    (void)env;
    jni_call();
    if (!a || a->kind != 2 || i < 0 || i >= a->len) {
        ++g_violations;
        return NULL;
    }
    return ((jobject *)a->data)[i];
}

static void f_GetIntArrayRegion(JNIEnv *env, jintArray a, jsize start, jsize len, jint *buf) {
    (void)env;
    jni_call();
    if (!a || a->kind != 1 || a->elem_size != 4 || start < 0 || len < 0 || start + len > a->len) {
        ++g_violations;
        return;
    }
    memcpy(buf, (jint *)a->data + start, (size_t)len * 4);
}

static void f_GetByteArrayRegion(JNIEnv *env, jbyteArray a, jsize start, jsize len, jbyte *buf) {
    (void)env;
    jni_call();
    if (!a || a->kind != 1 || a->elem_size != 1 || start < 0 || len < 0 || start + len > a->len) {
        ++g_violations;
        return;
    }
    memcpy(buf, (jbyte *)a->data + start, (size_t)len);
}

static void f_SetLongArrayRegion(JNIEnv *env, jlongArray a, jsize start, jsize len, const jlong *buf) {
    (void)env;
    jni_call();
    if (!a || a->kind != 1 || a->elem_size != 8 || start < 0 || len < 0 || start + len > a->len) {
        ++g_violations;
        return;
    }
    memcpy((jlong *)a->data + start, buf, (size_t)len * 8);
}

static void *f_GetPrimitiveArrayCritical(JNIEnv *env, jarray a, jboolean *is_copy) {
    (void)env;
    if (!a || a->kind != 1) {
        ++g_violations;
        return NULL;
    }
    if (is_copy) *is_copy = 0;
    ++g_pins_now;
    ++g_pins_total;
    return a->data;
}

static void f_ReleasePrimitiveArrayCritical(JNIEnv *env, jarray a, void *p, jint mode) {
    (void)env;
    if (!a || a->kind != 1 || p != a->data || g_pins_now <= 0) ++g_violations;
    --g_pins_now;
    ++g_unpins_total;
    g_last_release_mode = mode;
}

static void f_DeleteLocalRef(JNIEnv *env, jobject o) {
    (void)env;
    (void)o;
    jni_call();
    ++g_deleted;
}

static jstring f_NewStringUTF(JNIEnv *env, const char *s) {
    (void)env;
    jni_call();
    struct _jobject *o = (struct _jobject *)calloc(1, sizeof(*o));
    o->kind = 3;
    o->len = (jsize)strlen(s);
    o->data = strdup(s);
    return o;
}

/* As the JNI specification: NULL / -1 for a buffer that is not direct (a heap ByteBuffer,
 * modelled here by any non-direct object). */
static void *f_GetDirectBufferAddress(JNIEnv *env, jobject b) {
    (void)env;
    jni_call();
    return b && b->kind == 4 ? b->data : NULL;
}

static jlong f_GetDirectBufferCapacity(JNIEnv *env, jobject b) {
    (void)env;
    jni_call();
    return b && b->kind == 4 ? b->capacity : -1;
}

static jobject f_NewDirectByteBuffer(JNIEnv *env, void *address, jlong capacity) {
    (void)env;
    jni_call();
    struct _jobject *o = (struct _jobject *)calloc(1, sizeof(*o));
    o->kind = 4;
    o->elem_size = 1;
    o->capacity = capacity;
    o->data = address;
    return o;
}

static const struct JNINativeInterface_ g_table = {
    f_GetArrayLength,          f_GetObjectArrayElement, f_GetIntArrayRegion,    f_GetByteArrayRegion,
    f_SetLongArrayRegion,
    f_GetPrimitiveArrayCritical, f_ReleasePrimitiveArrayCritical, f_DeleteLocalRef, f_NewStringUTF,
    f_GetDirectBufferAddress,  f_NewDirectByteBuffer,    f_GetDirectBufferCapacity,
};
static JNIEnv g_env = &g_table;

/* ---------------------------------------------------------------- harness API (ctypes) */
JNIEnv *fake_env(void) { return &g_env; }

jobject fake_array(void *data, int32_t len, int32_t elem_size) {
    struct _jobject *o = (struct _jobject *)calloc(1, sizeof(*o));
    o->kind = 1;
    o->len = len;
    o->elem_size = elem_size;
    o->data = data;
    return o;
}

/* A direct ByteBuffer over caller memory (ByteBuffer.allocateDirect / wrapAddress). */
jobject fake_direct_buffer(void *data, int64_t capacity) {
    struct _jobject *o = (struct _jobject *)calloc(1, sizeof(*o));
    o->kind = 4;
    o->elem_size = 1;
    o->capacity = capacity;
    o->data = data;
    return o;
}

jobject fake_object_array(int32_t len) {
    struct _jobject *o = (struct _jobject *)calloc(1, sizeof(*o));
    o->kind = 2;
    o->len = len;
    o->data = calloc((size_t)len + 1, sizeof(jobject));
    return o;
}

void fake_set_element(jobject a, int32_t i, jobject e) { ((jobject *)a->data)[i] = e; }

const char *fake_string(jobject s) { return s && s->kind == 3 ? (const char *)s->data : NULL; }

void fake_free(jobject o) {
    if (!o) return;
    if (o->kind == 2 || o->kind == 3) free(o->data);
    free(o);
}

/* pins held now, pins taken, pins released, rule violations, local refs deleted,
 * non-critical JNI calls made while a pin was held, mode of the last release */
void fake_counters(int64_t *out) {
    out[0] = g_pins_now;
    out[1] = g_pins_total;
    out[2] = g_unpins_total;
    out[3] = g_violations;
    out[4] = g_deleted;
    out[5] = g_jni_calls_pinned;
    out[6] = g_last_release_mode;
}

void fake_reset(void) {
    g_pins_now = g_pins_total = g_unpins_total = g_violations = g_deleted = g_jni_calls_pinned = 0;
    g_last_release_mode = -1;
}
