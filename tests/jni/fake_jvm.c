/*
 * fake_jvm.c — TEST-ONLY JNIEnv for zarrhip_jni.c (compiled with tests/jni/jni.h; no JDK).
 *
 * Java arrays are plain heap buffers; every reference the shim receives or creates is a handle
 * whose liveness is tracked.  The fake enforces and records the JNI rules the shim relies on:
 *   - between GetPrimitiveArrayCritical and its Release no other JNI call is made;
 *   - every Get has a Release (per array: the output written back with mode 0, sources left
 *     with JNI_ABORT and never modified);
 *   - no use of a deleted local reference, no JNI call (other than Release) with an exception
 *     pending, no array region access out of bounds (recorded as the JVM's exception);
 *   - the critical windows (first Get to last Release at depth 0) are timed.
 * In copy mode GetPrimitiveArrayCritical hands out a copy (as a JVM may), so a shim that wrote
 * into a source, or released its output with JNI_ABORT, would be caught by the content checks.
 * Python drives it through ctypes (tests/jni_harness.py).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "jni.h"

typedef struct FObj {
  char kind;          /* 'B' 'Z' 'S' 'I' 'J' 'F' 'D' primitive arrays, 'L' object array, 'C' class,
                         'T' java.lang.String (data: its UTF-8 bytes, NUL-terminated) */
  int esize;          /* element bytes (primitive arrays) */
  int64_t len;        /* elements */
  void* data;         /* elements (object arrays: struct FObj*[]) */
  char name[64];      /* class name ('C'), element class ('L') */
  int crit_depth;     /* critical sections held on this array */
  void* crit_copy;    /* copy handed out in copy mode */
  int64_t releases_commit, releases_abort, gets;
  int modified_under_abort;
  struct FObj* next;
} FObj;

typedef struct FRef {
  FObj* obj;
  int live;
  int local;          /* created by a JNI call (DeleteLocalRef applies) */
  struct FRef* next;
} FRef;

typedef struct {
  int64_t gets, releases, releases_commit, releases_abort, max_depth;
  int64_t calls_in_critical, dead_ref_uses, calls_with_pending, oob, modified_sources;
  int64_t windows, max_window_ns, total_window_ns, live_local_refs, peak_local_refs;
  int64_t capacity_requested, bad_release;
  int64_t string_gets, string_releases;
} FStats;

static FObj* g_objs;
static FRef* g_refs;
static FStats g_st;
static int g_depth, g_copy_mode;
static struct timespec g_win_start;
static char g_exc_cls[128], g_exc_msg[4096];
static int g_exc_pending;
static char g_last_violation[256];

static void violation(const char* what) {
  snprintf(g_last_violation, sizeof g_last_violation, "%s", what);
}

static int64_t now_ns(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (int64_t)t.tv_sec * 1000000000ll + t.tv_nsec;
}

static FObj* new_obj(char kind, int esize, int64_t len, const char* name) {
  FObj* o = (FObj*)calloc(1, sizeof(FObj));
  o->kind = kind;
  o->esize = esize;
  o->len = len;
  size_t bytes = kind == 'L' ? (size_t)len * sizeof(FObj*) : (size_t)len * (size_t)esize;
  o->data = calloc(bytes > 0 ? bytes : 1, 1);
  if (name) snprintf(o->name, sizeof o->name, "%s", name);
  o->next = g_objs;
  g_objs = o;
  return o;
}

static jobject new_ref(FObj* o, int local) {
  if (!o) return NULL;
  FRef* r = (FRef*)calloc(1, sizeof(FRef));
  r->obj = o;
  r->live = 1;
  r->local = local;
  r->next = g_refs;
  g_refs = r;
  if (local && ++g_st.live_local_refs > g_st.peak_local_refs) g_st.peak_local_refs = g_st.live_local_refs;
  return (jobject)r;
}

static FObj* deref(jobject ref) {
  if (!ref) return NULL;
  FRef* r = (FRef*)ref;
  if (!r->live) {
    g_st.dead_ref_uses++;
    violation("use of a deleted local reference");
    return NULL;
  }
  return r->obj;
}

/* every JNI call but the critical pair: not inside a critical section, no pending exception */
static void enter_call(const char* fn) {
  if (g_depth > 0) {
    g_st.calls_in_critical++;
    char b[160];
    snprintf(b, sizeof b, "%s called inside a critical section", fn);
    violation(b);
  }
  if (g_exc_pending) {
    g_st.calls_with_pending++;
    char b[160];
    snprintf(b, sizeof b, "%s called with an exception pending", fn);
    violation(b);
  }
}

static void throw_jvm(const char* cls, const char* msg) {
  if (g_exc_pending) return;
  g_exc_pending = 1;
  snprintf(g_exc_cls, sizeof g_exc_cls, "%s", cls);
  snprintf(g_exc_msg, sizeof g_exc_msg, "%s", msg ? msg : "");
}

static int region_ok(FObj* o, jsize start, jsize len) {
  if (!o || start < 0 || len < 0 || (int64_t)start + len > o->len) {
    g_st.oob++;
    throw_jvm("java/lang/ArrayIndexOutOfBoundsException", "array region out of bounds");
    return 0;
  }
  return 1;
}

/* ---- the JNIEnv functions ---------------------------------------------------------------- */
static jclass f_FindClass(JNIEnv* env, const char* name) {
  (void)env;
  enter_call("FindClass");
  for (FObj* o = g_objs; o; o = o->next)
    if (o->kind == 'C' && strcmp(o->name, name) == 0) return new_ref(o, 1);
  return new_ref(new_obj('C', 0, 0, name), 1);
}

static jint f_ThrowNew(JNIEnv* env, jclass clazz, const char* msg) {
  (void)env;
  enter_call("ThrowNew");
  FObj* c = deref(clazz);
  throw_jvm(c ? c->name : "?", msg);
  return 0;
}

static jobject f_NewLocalRef(JNIEnv* env, jobject ref) {
  (void)env;
  enter_call("NewLocalRef");
  return new_ref(deref(ref), 1);
}

static void f_DeleteLocalRef(JNIEnv* env, jobject obj) {
  (void)env;
  enter_call("DeleteLocalRef");
  if (!obj) return;
  FRef* r = (FRef*)obj;
  if (!r->live) {
    g_st.dead_ref_uses++;
    violation("DeleteLocalRef of a deleted reference");
    return;
  }
  if (!r->local) {
    violation("DeleteLocalRef of an argument reference");
    g_st.dead_ref_uses++;
    return;
  }
  r->live = 0;
  g_st.live_local_refs--;
}

static jint f_EnsureLocalCapacity(JNIEnv* env, jint capacity) {
  (void)env;
  enter_call("EnsureLocalCapacity");
  if (capacity > g_st.capacity_requested) g_st.capacity_requested = capacity;
  return 0;
}

static jsize f_GetArrayLength(JNIEnv* env, jarray array) {
  (void)env;
  enter_call("GetArrayLength");
  FObj* o = deref(array);
  return o ? (jsize)o->len : 0;
}

static jobjectArray f_NewObjectArray(JNIEnv* env, jsize len, jclass clazz, jobject init) {
  (void)env;
  enter_call("NewObjectArray");
  FObj* c = deref(clazz);
  FObj* o = new_obj('L', 0, len, c ? c->name : "?");
  FObj* iv = deref(init);
  for (jsize i = 0; i < len; i++) ((FObj**)o->data)[i] = iv;
  return new_ref(o, 1);
}

static jobject f_GetObjectArrayElement(JNIEnv* env, jobjectArray array, jsize index) {
  (void)env;
  enter_call("GetObjectArrayElement");
  FObj* o = deref(array);
  if (!o || !region_ok(o, index, 1)) return NULL;
  return new_ref(((FObj**)o->data)[index], 1);
}

static void f_SetObjectArrayElement(JNIEnv* env, jobjectArray array, jsize index, jobject val) {
  (void)env;
  enter_call("SetObjectArrayElement");
  FObj* o = deref(array);
  if (!o || !region_ok(o, index, 1)) return;
  ((FObj**)o->data)[index] = deref(val);
}

static jbyteArray f_NewByteArray(JNIEnv* env, jsize len) {
  (void)env;
  enter_call("NewByteArray");
  return new_ref(new_obj('B', 1, len, NULL), 1);
}

static jlongArray f_NewLongArray(JNIEnv* env, jsize len) {
  (void)env;
  enter_call("NewLongArray");
  return new_ref(new_obj('J', 8, len, NULL), 1);
}

#define REGION_GET(NAME, T)                                                         \
  static void NAME(JNIEnv* env, jarray array, jsize start, jsize len, T* buf) {     \
    (void)env;                                                                      \
    enter_call(#NAME);                                                              \
    FObj* o = deref(array);                                                         \
    if (!o || !region_ok(o, start, len)) return;                                    \
    memcpy(buf, (const char*)o->data + (size_t)start * o->esize, (size_t)len * o->esize); \
  }
REGION_GET(f_GetByteArrayRegion, jbyte)
REGION_GET(f_GetIntArrayRegion, jint)
REGION_GET(f_GetLongArrayRegion, jlong)

#define REGION_SET(NAME, T)                                                           \
  static void NAME(JNIEnv* env, jarray array, jsize start, jsize len, const T* buf) { \
    (void)env;                                                                        \
    enter_call(#NAME);                                                                \
    FObj* o = deref(array);                                                           \
    if (!o || !region_ok(o, start, len)) return;                                      \
    memcpy((char*)o->data + (size_t)start * o->esize, buf, (size_t)len * o->esize);   \
  }
REGION_SET(f_SetByteArrayRegion, jbyte)
REGION_SET(f_SetLongArrayRegion, jlong)

static void* f_GetPrimitiveArrayCritical(JNIEnv* env, jarray array, jboolean* isCopy) {
  (void)env;
  if (g_exc_pending) {
    g_st.calls_with_pending++;
    violation("GetPrimitiveArrayCritical called with an exception pending");
  }
  FObj* o = deref(array);
  if (!o || o->kind == 'L' || o->kind == 'C') {
    violation("GetPrimitiveArrayCritical of a non-primitive array");
    return NULL;
  }
  if (g_depth == 0) clock_gettime(CLOCK_MONOTONIC, &g_win_start);
  g_depth++;
  if (g_depth > g_st.max_depth) g_st.max_depth = g_depth;
  g_st.gets++;
  o->gets++;
  o->crit_depth++;
  if (isCopy) *isCopy = g_copy_mode ? 1 : 0;
  if (!g_copy_mode) return o->data;
  if (o->crit_depth > 1) {
    violation("one array held twice at once in copy mode");
    return NULL;
  }
  size_t bytes = (size_t)o->len * (size_t)o->esize;
  o->crit_copy = malloc(bytes > 0 ? bytes : 1);
  memcpy(o->crit_copy, o->data, bytes);
  return o->crit_copy;
}

static void f_ReleasePrimitiveArrayCritical(JNIEnv* env, jarray array, void* carray, jint mode) {
  (void)env;
  FObj* o = deref(array);
  if (!o || o->crit_depth <= 0 || g_depth <= 0) {
    g_st.bad_release++;
    violation("ReleasePrimitiveArrayCritical without a matching Get");
    return;
  }
  if (carray != (g_copy_mode ? o->crit_copy : o->data)) {
    g_st.bad_release++;
    violation("ReleasePrimitiveArrayCritical with another address than Get returned");
  }
  g_st.releases++;
  size_t bytes = (size_t)o->len * (size_t)o->esize;
  if (mode == 0 || mode == JNI_COMMIT) {
    g_st.releases_commit++;
    o->releases_commit++;
    if (g_copy_mode) memcpy(o->data, o->crit_copy, bytes);
  } else if (mode == JNI_ABORT) {
    g_st.releases_abort++;
    o->releases_abort++;
    if (g_copy_mode && memcmp(o->data, o->crit_copy, bytes) != 0) {
      o->modified_under_abort = 1;
      g_st.modified_sources++;
      violation("a source array was written inside its critical section");
    }
  } else {
    g_st.bad_release++;
    violation("ReleasePrimitiveArrayCritical with an unknown mode");
  }
  if (g_copy_mode && mode != JNI_COMMIT) {
    free(o->crit_copy);
    o->crit_copy = NULL;
  }
  o->crit_depth--;
  if (--g_depth == 0) {
    const int64_t w = now_ns() - ((int64_t)g_win_start.tv_sec * 1000000000ll + g_win_start.tv_nsec);
    g_st.windows++;
    g_st.total_window_ns += w;
    if (w > g_st.max_window_ns) g_st.max_window_ns = w;
  }
}

/* GetStringUTFChars hands out a copy (as a JVM may), freed by the matching Release */
static const char* f_GetStringUTFChars(JNIEnv* env, jstring str, jboolean* isCopy) {
  (void)env;
  enter_call("GetStringUTFChars");
  FObj* o = deref(str);
  if (!o || o->kind != 'T') {
    violation("GetStringUTFChars of a non-string");
    return NULL;
  }
  if (isCopy) *isCopy = 1;
  g_st.string_gets++;
  char* c = (char*)malloc((size_t)o->len + 1);
  memcpy(c, o->data, (size_t)o->len + 1);
  return c;
}

static void f_ReleaseStringUTFChars(JNIEnv* env, jstring str, const char* chars) {
  (void)env;
  enter_call("ReleaseStringUTFChars");
  FObj* o = deref(str);
  if (!o || o->kind != 'T' || !chars) {
    g_st.bad_release++;
    violation("ReleaseStringUTFChars without a matching Get");
    return;
  }
  g_st.string_releases++;
  free((void*)chars);
}

static struct JNINativeInterface_ g_table = {
    NULL,
    f_FindClass,
    f_ThrowNew,
    f_NewLocalRef,
    f_DeleteLocalRef,
    f_EnsureLocalCapacity,
    f_GetArrayLength,
    f_NewObjectArray,
    f_GetObjectArrayElement,
    f_SetObjectArrayElement,
    f_NewByteArray,
    f_NewLongArray,
    (void (*)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*))f_GetByteArrayRegion,
    (void (*)(JNIEnv*, jintArray, jsize, jsize, jint*))f_GetIntArrayRegion,
    (void (*)(JNIEnv*, jlongArray, jsize, jsize, jlong*))f_GetLongArrayRegion,
    (void (*)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*))f_SetByteArrayRegion,
    (void (*)(JNIEnv*, jlongArray, jsize, jsize, const jlong*))f_SetLongArrayRegion,
    f_GetPrimitiveArrayCritical,
    f_ReleasePrimitiveArrayCritical,
    f_GetStringUTFChars,
    f_ReleaseStringUTFChars,
};
static JNIEnv g_env = &g_table;

/* ---- the harness side (ctypes) ----------------------------------------------------------- */
JNIEXPORT JNIEnv* fj_env(void) { return &g_env; }

JNIEXPORT void fj_reset(int copy_mode) {
  while (g_refs) {
    FRef* r = g_refs->next;
    free(g_refs);
    g_refs = r;
  }
  while (g_objs) {
    FObj* o = g_objs->next;
    free(g_objs->data);
    free(g_objs->crit_copy);
    free(g_objs);
    g_objs = o;
  }
  memset(&g_st, 0, sizeof g_st);
  g_depth = 0;
  g_copy_mode = copy_mode;
  g_exc_pending = 0;
  g_exc_cls[0] = g_exc_msg[0] = g_last_violation[0] = 0;
}

static int esize_of(char kind) {
  switch (kind) {
    case 'B': case 'Z': return 1;
    case 'S': return 2;
    case 'I': case 'F': return 4;
    case 'J': case 'D': return 8;
    default: return 0;
  }
}

/* a primitive array ('B' 'Z' 'S' 'I' 'J' 'F' 'D') of len elements, copied from data (or zeroed) */
JNIEXPORT jobject fj_new_array(char kind, int64_t len, const void* data) {
  const int es = esize_of(kind);
  if (!es) return NULL;
  FObj* o = new_obj(kind, es, len, NULL);
  if (data) memcpy(o->data, data, (size_t)len * (size_t)es);
  return new_ref(o, 0);
}

/* a java.lang.String holding the UTF-8 text s */
JNIEXPORT jobject fj_new_string(const char* s) {
  const size_t n = strlen(s);
  FObj* o = new_obj('T', 1, (int64_t)n + 1, "java/lang/String");
  memcpy(o->data, s, n + 1);
  o->len = (int64_t)n;
  return new_ref(o, 0);
}

JNIEXPORT jobject fj_new_object_array(int64_t len, const char* elem_class) {
  return new_ref(new_obj('L', 0, len, elem_class), 0);
}

JNIEXPORT void fj_set(jobject arr, int64_t i, jobject val) {
  FObj* o = ((FRef*)arr)->obj;
  ((FObj**)o->data)[i] = val ? ((FRef*)val)->obj : NULL;
}

/* element i of an object array as a new argument reference (NULL for a null element) */
JNIEXPORT jobject fj_get(jobject arr, int64_t i) {
  FObj* o = ((FRef*)arr)->obj;
  FObj* e = ((FObj**)o->data)[i];
  return e ? new_ref(e, 0) : NULL;
}

JNIEXPORT void* fj_data(jobject ref) { return ref ? ((FRef*)ref)->obj->data : NULL; }
JNIEXPORT int64_t fj_len(jobject ref) { return ref ? ((FRef*)ref)->obj->len : -1; }
JNIEXPORT char fj_kind(jobject ref) { return ref ? ((FRef*)ref)->obj->kind : 0; }

/* per array: Gets, Releases with 0 / JNI_COMMIT, Releases with JNI_ABORT, written under abort */
JNIEXPORT void fj_obj_stats(jobject ref, int64_t* out4) {
  FObj* o = ((FRef*)ref)->obj;
  out4[0] = o->gets;
  out4[1] = o->releases_commit;
  out4[2] = o->releases_abort;
  out4[3] = o->modified_under_abort + 2 * o->crit_depth;  /* 2·k: k critical sections left open */
}

JNIEXPORT void fj_stats(FStats* out) {
  *out = g_st;
}

/* the counters only (the arrays stay): between timed calls of a lab */
JNIEXPORT void fj_reset_stats(void) {
  const int64_t live = g_st.live_local_refs;
  memset(&g_st, 0, sizeof g_st);
  g_st.live_local_refs = live;
}

JNIEXPORT int fj_depth(void) { return g_depth; }

JNIEXPORT int fj_exception(char* cls, int64_t clen, char* msg, int64_t mlen) {
  if (!g_exc_pending) return 0;
  snprintf(cls, (size_t)clen, "%s", g_exc_cls);
  snprintf(msg, (size_t)mlen, "%s", g_exc_msg);
  return 1;
}

JNIEXPORT void fj_clear_exception(void) { g_exc_pending = 0; }

JNIEXPORT const char* fj_last_violation(void) { return g_last_violation; }
