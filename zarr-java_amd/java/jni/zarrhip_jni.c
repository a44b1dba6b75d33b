/*
 * zarrhip_jni.c — thin JNI shim from zarr-java to the zarrhip C-ABI (include/zarrhip.h).
 * Built only where a JDK exists (needs $JAVA_HOME/include/jni.h); see INTEGRATION.md.  The
 * test harness (tests/jni/) compiles it against a test-only stand-in header and drives every
 * entry point through a fake JNIEnv.
 *
 * Every native method assembles a zh_array_meta from Java primitives and maps zh_status to the
 * reference's exceptions:
 *   ZH_EDATA → dev.zarr.zarrjava.ZarrException, ZH_EINVAL → IllegalArgumentException,
 *   ZH_EARITH → ArithmeticException, ZH_EIO → dev.zarr.zarrjava.store.StoreException (a
 *   RuntimeException, as FilesystemStore's readFailed), ZH_EUNSUPPORTED → returned as 3 (Java
 *   falls back to the reference codec), anything else → RuntimeException.
 *
 * Critical sections, one policy for every entry point: a Java array is held with
 * GetPrimitiveArrayCritical only for one slab of the work, and no JNI call is made while one
 * is held.  A read is cut into C-order slabs of at most ZH_JNI_SLAB_MB (default 1024) MiB of
 * output along the region's first axis of extent >= 2 (so each slab is one contiguous part of
 * the result), at stored-chunk boundaries along that axis where a slab spans several; per slab
 * the shim enters the critical sections of the sources that slab needs and of the result,
 * makes one library call on the slab's sub-region straight into the result (no copy on this
 * side: the library's pipelined read copies each source once into its page-locked ring), and
 * leaves them: sources with JNI_ABORT (never written), the result with 0.  arrayWrite copies
 * its region out of the heap in windows of the same size.  On collectors with a GC locker
 * (JDK 8-21) a held critical section defers every GC; this bounds the deferral by one slab's
 * read time instead of the whole read's (INTEGRATION.md "GC and critical sections").
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zarrhip.h"

static int throw_status(JNIEnv* env, int st, const char* msg) {
  const char* cls = "java/lang/RuntimeException";
  if (st == ZH_EDATA) cls = "dev/zarr/zarrjava/ZarrException";
  else if (st == ZH_EINVAL) cls = "java/lang/IllegalArgumentException";
  else if (st == ZH_EARITH) cls = "java/lang/ArithmeticException";
  else if (st == ZH_EIO) cls = "dev/zarr/zarrjava/store/StoreException";
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, msg && *msg ? msg : "zarrhip error");
  return st;
}

JNIEXPORT jlong JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_ctxCreate(JNIEnv* env, jclass cls,
                                                                    jint device) {
  (void)cls;
  zh_ctx* ctx = NULL;
  int st = zh_ctx_create(device, &ctx);
  if (st != ZH_OK) {
    throw_status(env, ZH_EHIP, "zh_ctx_create failed: no usable MI355X device");
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_ctxDestroy(JNIEnv* env, jclass cls,
                                                                    jlong ctx) {
  (void)env;
  (void)cls;
  zh_ctx_destroy((zh_ctx*)(intptr_t)ctx);
}

/* meta: int[] {ndim, dtypeSize, isBool, sharded, hasTranspose, endian, indexEndian,
 *              indexCrc32c, indexLocation[, nested, nestedIndexEndian, nestedIndexCrc32c,
 *              nestedIndexLocation, innerCrc32c[, isFloat]]}; shape long[ndim]; chunkShape/order int[ndim];
 *              innerShape int[ndim] (nested: int[2*ndim], inner then leaf shape);
 *              fill byte[dtypeSize] (little-endian element bytes). */
static int build_meta(JNIEnv* env, jintArray jm, jlongArray jshape, jintArray jchunk,
                      jintArray jinner, jintArray jorder, jbyteArray jfill, zh_array_meta* m) {
  memset(m, 0, sizeof(*m));
  jint mi[15] = {0};
  jsize nm = (*env)->GetArrayLength(env, jm);
  (*env)->GetIntArrayRegion(env, jm, 0, nm < 15 ? nm : 15, mi);
  m->ndim = mi[0];
  if (m->ndim <= 0 || m->ndim > ZH_MAX_DIMS) return ZH_EUNSUPPORTED;
  m->dtype_size = mi[1];
  m->dtype_is_bool = mi[2];
  m->chain.sharded = mi[3];
  m->chain.has_transpose = mi[4];
  m->chain.endian = mi[5];
  m->chain.index_endian = mi[6];
  m->chain.index_has_crc32c = mi[7];
  m->chain.index_location = mi[8];
  m->chain.nested = mi[9];
  m->chain.nested_index_endian = mi[10];
  m->chain.nested_index_has_crc32c = mi[11];
  m->chain.nested_index_location = mi[12];
  m->chain.inner_crc32c = mi[13];
  m->dtype_is_float = mi[14];
  jlong sh[ZH_MAX_DIMS];
  jint ch[ZH_MAX_DIMS];
  (*env)->GetLongArrayRegion(env, jshape, 0, m->ndim, sh);
  (*env)->GetIntArrayRegion(env, jchunk, 0, m->ndim, ch);
  for (int d = 0; d < m->ndim; d++) {
    m->shape[d] = sh[d];
    m->chunk_shape[d] = ch[d];
  }
  if (m->chain.sharded) (*env)->GetIntArrayRegion(env, jinner, 0, m->ndim, m->chain.inner_chunk_shape);
  if (m->chain.sharded && m->chain.nested)
    (*env)->GetIntArrayRegion(env, jinner, m->ndim, m->ndim, m->chain.nested_chunk_shape);
  if (m->chain.has_transpose) (*env)->GetIntArrayRegion(env, jorder, 0, m->ndim, m->chain.transpose_order);
  if (jfill) {
    jsize n = (*env)->GetArrayLength(env, jfill);
    (*env)->GetByteArrayRegion(env, jfill, 0, n < 8 ? n : 8, (jbyte*)m->fill_value);
  }
  return ZH_OK;
}

/* ---- slabs ------------------------------------------------------------------------------ */
static int64_t slab_cap_bytes(void) {
  const char* e = getenv("ZH_JNI_SLAB_MB");
  long v = e ? strtol(e, NULL, 10) : 1024;
  return (int64_t)(v < 1 ? 1 : v) << 20;
}

/* A region (or a shard part) cut into slabs along `axis`, the first axis of extent >= 2
 * (axis 0 when there is none: one slab).  row = output bytes of one index along the axis. */
typedef struct {
  int axis;
  int64_t row;   /* bytes per step along the axis                       */
  int64_t unit;  /* stored-chunk extent along the axis (slab boundaries) */
  int64_t cap;   /* output bytes per slab                               */
} SlabPlan;

static SlabPlan slab_plan(const zh_array_meta* m, const int64_t* shp, int64_t unit_of_axis[],
                          int64_t cap) {
  SlabPlan P;
  P.axis = 0;
  for (int d = 0; d < m->ndim; d++)
    if (shp[d] >= 2) {
      P.axis = d;
      break;
    }
  P.row = m->dtype_size;
  for (int d = P.axis + 1; d < m->ndim; d++) P.row *= shp[d];
  P.unit = unit_of_axis[P.axis] > 0 ? unit_of_axis[P.axis] : 1;
  P.cap = cap;
  return P;
}

/* End (exclusive, absolute coordinate) of the slab that starts at s; `end` = region end. */
static int64_t slab_end(const SlabPlan* P, int64_t s, int64_t end) {
  int64_t t = P->row > 0 ? P->cap / P->row : 1;
  if (t < 1) t = 1;
  if (t >= end - s) return end;
  int64_t e = s + t;
  const int64_t al = e / P->unit * P->unit;  /* the last unit boundary inside the slab */
  return al > s ? al : e;
}

/* The stored unit along each axis: the inner chunk (sharded: a piece names inner chunks) or
 * the chunk. */
static void units_of(const zh_array_meta* m, int sharded_part, int64_t* u) {
  for (int d = 0; d < m->ndim; d++)
    u[d] = m->chain.sharded && sharded_part ? m->chain.inner_chunk_shape[d] : m->chunk_shape[d];
}

/* computeChunkCoords order of the region's chunks: the slab [s, e) along P->axis is the
 * contiguous index range [*first, *first + *count) of that list (every earlier axis has
 * extent 1). */
static void slab_chunks(const zh_array_meta* m, const int64_t* off, const int64_t* shp, int a,
                        int64_t s, int64_t e, jsize* first, jsize* count) {
  int64_t stride = 1;
  for (int d = m->ndim - 1; d > a; d--) {
    const int64_t c0 = off[d] / m->chunk_shape[d], c1 = (off[d] + shp[d] - 1) / m->chunk_shape[d];
    stride *= c1 - c0 + 1;
  }
  const int64_t lo = off[a] / m->chunk_shape[a];
  const int64_t b0 = s / m->chunk_shape[a], b1 = (e - 1) / m->chunk_shape[a];
  *first = (jsize)((b0 - lo) * stride);
  *count = (jsize)((b1 - b0 + 1) * stride);
}

/* ---- critical sections ------------------------------------------------------------------ */
/* The arrays one call holds: sources first, the output last.  pin_enter collects nothing and
 * makes no JNI call but the Get; pin_release leaves every one (sources JNI_ABORT, the output
 * 0) in reverse order and frees the bookkeeping. */
typedef struct {
  jsize n;                 /* arrays held */
  jarray* arr;             /* sources (byte[]s), then the output */
  void** ptr;              /* their critical addresses */
  int has_out;             /* the last entry is the output */
  zh_shard_piece* pieces;  /* piece table of a pieces call */
} Pinned;

static int pin_alloc(Pinned* P, jsize narr, jsize npieces) {
  memset(P, 0, sizeof(*P));
  P->arr = (jarray*)calloc((size_t)(narr > 0 ? narr : 1), sizeof(jarray));
  P->ptr = (void**)calloc((size_t)(narr > 0 ? narr : 1), sizeof(void*));
  P->pieces = (zh_shard_piece*)calloc((size_t)(npieces > 0 ? npieces : 1), sizeof(zh_shard_piece));
  return P->arr && P->ptr && P->pieces ? ZH_OK : ZH_ENOMEM;
}

static int pin_enter(JNIEnv* env, Pinned* P) {
  for (jsize k = 0; k < P->n; k++) {
    if (!P->arr[k]) continue;
    P->ptr[k] = (*env)->GetPrimitiveArrayCritical(env, P->arr[k], NULL);
    if (!P->ptr[k]) return ZH_ENOMEM;
  }
  return ZH_OK;
}

static void pin_release(JNIEnv* env, Pinned* P) {
  for (jsize k = P->n - 1; k >= 0; k--)
    if (P->ptr && P->ptr[k])
      (*env)->ReleasePrimitiveArrayCritical(env, P->arr[k], P->ptr[k],
                                            P->has_out && k == P->n - 1 ? 0 : JNI_ABORT);
  /* local references of the sources (the output is the caller's) */
  for (jsize k = 0; P->arr && k < P->n - (P->has_out ? 1 : 0); k++)
    if (P->arr[k]) (*env)->DeleteLocalRef(env, P->arr[k]);
  free(P->arr);
  free(P->ptr);
  free(P->pieces);
  memset(P, 0, sizeof(*P));
}

static void region_of(JNIEnv* env, int n, jlongArray joffset, jlongArray jregion, int64_t* o64,
                      int64_t* r64) {
  jlong off[ZH_MAX_DIMS], reg[ZH_MAX_DIMS];
  (*env)->GetLongArrayRegion(env, joffset, 0, n, off);
  (*env)->GetLongArrayRegion(env, jregion, 0, n, reg);
  for (int d = 0; d < n; d++) {
    o64[d] = off[d];
    r64[d] = reg[d];
  }
}

/* core.Array.read replacement: chunks[i] = bytes of the i-th chunk of
 * computeChunkCoords(shape, chunkShape, offset, regionShape) or null (missing key);
 * out = the primitive array behind the result ucar.ma2.Array (C order).
 * Returns 0 on success, 3 (ZH_EUNSUPPORTED) to request the Java fallback. */
static jint array_read_common(JNIEnv* env, zh_ctx* const* ctxs, int nctx, jintArray jm,
                              jlongArray jshape, jintArray jchunk, jintArray jinner,
                              jintArray jorder, jbyteArray jfill, jobjectArray jchunks,
                              jlongArray joffset, jlongArray jregion, jobject out) {
  zh_array_meta m;
  int st = build_meta(env, jm, jshape, jchunk, jinner, jorder, jfill, &m);
  if (st != ZH_OK) return st;
  char err[1024] = {0};
  st = zh_validate_meta(&m, err, sizeof err);
  if (st == ZH_EUNSUPPORTED) return st;
  if (st != ZH_OK) return throw_status(env, st, err);
  int64_t o64[ZH_MAX_DIMS], r64[ZH_MAX_DIMS], u[ZH_MAX_DIMS];
  region_of(env, m.ndim, joffset, jregion, o64, r64);
  int64_t nel = 1;
  for (int d = 0; d < m.ndim; d++) nel *= r64[d];
  if ((int64_t)(*env)->GetArrayLength(env, (jarray)out) != nel)
    return throw_status(env, ZH_EINVAL, "output array size does not match the region");
  const jsize nchunks = (*env)->GetArrayLength(env, jchunks);
  units_of(&m, 0, u);
  const SlabPlan SP = slab_plan(&m, r64, u, slab_cap_bytes());
  const int a = SP.axis;
  for (int64_t s = o64[a]; st == ZH_OK && s < o64[a] + r64[a];) {
    const int64_t e = slab_end(&SP, s, o64[a] + r64[a]);
    jsize first = 0, cnt = 0;
    slab_chunks(&m, o64, r64, a, s, e, &first, &cnt);
    if (first < 0 || first + cnt > nchunks) {
      st = ZH_EINVAL;
      snprintf(err, sizeof err, "%d chunk arrays for a region of more chunks", (int)nchunks);
      break;
    }
    Pinned P;
    /* the slab's chunk arrays stay referenced until pin_release: room for all of them (the
     * JNI spec guarantees 16 local references) */
    if ((*env)->EnsureLocalCapacity(env, cnt + 16) != 0) {
      st = ZH_ENOMEM;
      snprintf(err, sizeof err, "out of local references for %d chunk arrays", (int)cnt);
      break;
    }
    zh_chunk_src* srcs = (zh_chunk_src*)calloc((size_t)(cnt > 0 ? cnt : 1), sizeof(zh_chunk_src));
    if (!srcs || pin_alloc(&P, cnt + 1, 0) != ZH_OK) {
      free(srcs);
      free(P.arr);
      free(P.ptr);
      free(P.pieces);
      st = ZH_ENOMEM;
      snprintf(err, sizeof err, "out of host memory");
      break;
    }
    for (jsize i = 0; i < cnt; i++) {  /* references and lengths first: JNI calls */
      P.arr[i] = (jarray)(*env)->GetObjectArrayElement(env, jchunks, first + i);
      srcs[i].nbytes = P.arr[i] ? (*env)->GetArrayLength(env, P.arr[i]) : 0;
    }
    P.arr[cnt] = (jarray)out;
    P.n = cnt + 1;
    P.has_out = 1;
    int64_t so[ZH_MAX_DIMS], ss[ZH_MAX_DIMS];
    for (int d = 0; d < m.ndim; d++) {
      so[d] = o64[d];
      ss[d] = r64[d];
    }
    so[a] = s;
    ss[a] = e - s;
    st = pin_enter(env, &P);
    if (st == ZH_OK) {
      for (jsize i = 0; i < cnt; i++) srcs[i].data = P.ptr[i];
      uint8_t* dst = (uint8_t*)P.ptr[cnt] + (size_t)((s - o64[a]) * SP.row);
      st = nctx == 1 ? zh_array_read(ctxs[0], &m, srcs, cnt, so, ss, dst, 0, NULL, err, sizeof err)
                     : zh_array_read_multi(ctxs, nctx, 0, &m, srcs, cnt, so, ss, dst, 0, err,
                                           sizeof err);
    } else {
      snprintf(err, sizeof err, "could not access the chunk or output arrays");
    }
    pin_release(env, &P);
    free(srcs);
    s = e;
  }
  if (st == ZH_EUNSUPPORTED) return st;
  if (st != ZH_OK) return throw_status(env, st, err);
  return 0;
}

JNIEXPORT jint JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_arrayRead(
    JNIEnv* env, jclass cls, jlong ctx, jintArray jm, jlongArray jshape, jintArray jchunk,
    jintArray jinner, jintArray jorder, jbyteArray jfill, jobjectArray jchunks,
    jlongArray joffset, jlongArray jregion, jobject out) {
  (void)cls;
  zh_ctx* c = (zh_ctx*)(intptr_t)ctx;
  return array_read_common(env, &c, 1, jm, jshape, jchunk, jinner, jorder, jfill, jchunks,
                           joffset, jregion, out);
}

/* The same read spread over several devices (zh_array_read_multi, host-terminated). */
JNIEXPORT jint JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_arrayReadMulti(
    JNIEnv* env, jclass cls, jlongArray jctxs, jintArray jm, jlongArray jshape,
    jintArray jchunk, jintArray jinner, jintArray jorder, jbyteArray jfill,
    jobjectArray jchunks, jlongArray joffset, jlongArray jregion, jobject out) {
  (void)cls;
  jsize k = (*env)->GetArrayLength(env, jctxs);
  if (k <= 0 || k > 64) return throw_status(env, ZH_EINVAL, "bad device context list");
  jlong raw[64];
  zh_ctx* ctxs[64];
  (*env)->GetLongArrayRegion(env, jctxs, 0, k, raw);
  for (jsize i = 0; i < k; i++) ctxs[i] = (zh_ctx*)(intptr_t)raw[i];
  return array_read_common(env, ctxs, (int)k, jm, jshape, jchunk, jinner, jorder, jfill,
                           jchunks, joffset, jregion, out);
}

/* Copies a Java string into malloc'd UTF-8 (NULL for a null string); *st = ZH_ENOMEM when the
 * copy fails.  (GetStringUTFChars' modified UTF-8 equals UTF-8 for every path without NUL or
 * supplementary characters.) */
static char* dup_string(JNIEnv* env, jstring js, int* st) {
  if (!js) return NULL;
  const char* c = (*env)->GetStringUTFChars(env, js, NULL);
  char* r = c ? strdup(c) : NULL;
  if (c) (*env)->ReleaseStringUTFChars(env, js, c);
  if (!r) *st = ZH_ENOMEM;
  return r;
}

/* The chunk paths of a files call, each copied (null stays NULL). */
static char** dup_paths(JNIEnv* env, jobjectArray jpaths, jsize n, int* st) {
  char** paths = (char**)calloc((size_t)(n > 0 ? n : 1), sizeof(char*));
  if (!paths) {
    *st = ZH_ENOMEM;
    return NULL;
  }
  for (jsize i = 0; *st == ZH_OK && i < n; i++) {
    jstring js = (jstring)(*env)->GetObjectArrayElement(env, jpaths, i);
    paths[i] = dup_string(env, js, st);
    if (js) (*env)->DeleteLocalRef(env, js);
  }
  return paths;
}

static void free_paths(char** paths, jsize n, zh_file_store* store) {
  for (jsize i = 0; paths && i < n; i++) free(paths[i]);
  free(paths);
  free((char*)store->root);
  free((char*)store->name);
}

/* core.Array.read over a FilesystemStore (HipArray.read): paths[i] = StoreHandle.toPath() of the
 * i-th chunk of computeChunkCoords(shape, chunkShape, offset, regionShape), or null; storeRoot =
 * the store's directory and storeName = FilesystemStore.toString(), which StoreException's
 * messages name (zh_file_store).  The library
 * reads the files itself (zh_array_read_files; with several contexts zh_array_read_files_multi,
 * one slab per device): no source array crosses the boundary, so per slab only the result is
 * held critical.  The paths are converted before any critical section
 * (GetStringUTFChars is a JNI call; its modified UTF-8 equals UTF-8 for every path without
 * NUL or supplementary characters). */
JNIEXPORT jint JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_arrayReadFiles(
    JNIEnv* env, jclass cls, jlongArray jctxs, jintArray jm, jlongArray jshape, jintArray jchunk,
    jintArray jinner, jintArray jorder, jbyteArray jfill, jstring jroot, jstring jname,
    jobjectArray jpaths, jlongArray joffset, jlongArray jregion, jobject out) {
  (void)cls;
  zh_array_meta m;
  int st = build_meta(env, jm, jshape, jchunk, jinner, jorder, jfill, &m);
  if (st != ZH_OK) return st;
  char err[1024] = {0};
  st = zh_validate_meta(&m, err, sizeof err);
  if (st == ZH_EUNSUPPORTED) return st;
  if (st != ZH_OK) return throw_status(env, st, err);
  const jsize k = (*env)->GetArrayLength(env, jctxs);
  if (k <= 0 || k > 64) return throw_status(env, ZH_EINVAL, "bad device context list");
  jlong raw[64];
  zh_ctx* ctxs[64];
  (*env)->GetLongArrayRegion(env, jctxs, 0, k, raw);
  for (jsize i = 0; i < k; i++) ctxs[i] = (zh_ctx*)(intptr_t)raw[i];
  int64_t o64[ZH_MAX_DIMS], r64[ZH_MAX_DIMS], u[ZH_MAX_DIMS], nel = 1;
  region_of(env, m.ndim, joffset, jregion, o64, r64);
  for (int d = 0; d < m.ndim; d++) nel *= r64[d];
  if ((int64_t)(*env)->GetArrayLength(env, (jarray)out) != nel)
    return throw_status(env, ZH_EINVAL, "output array size does not match the region");
  const jsize n = (*env)->GetArrayLength(env, jpaths);
  zh_file_store store = {dup_string(env, jroot, &st), dup_string(env, jname, &st)};
  char** paths = dup_paths(env, jpaths, n, &st);
  if (st != ZH_OK) snprintf(err, sizeof err, "out of host memory");
  units_of(&m, 0, u);
  const SlabPlan SP = slab_plan(&m, r64, u, slab_cap_bytes());
  const int a = SP.axis;
  for (int64_t s = o64[a]; st == ZH_OK && s < o64[a] + r64[a];) {
    const int64_t e = slab_end(&SP, s, o64[a] + r64[a]);
    jsize first = 0, cnt = 0;
    slab_chunks(&m, o64, r64, a, s, e, &first, &cnt);
    if (first < 0 || first + cnt > n) {
      st = ZH_EINVAL;
      snprintf(err, sizeof err, "%d chunk paths for a region of more chunks", (int)n);
      break;
    }
    int64_t so[ZH_MAX_DIMS], ss[ZH_MAX_DIMS];
    for (int d = 0; d < m.ndim; d++) {
      so[d] = o64[d];
      ss[d] = r64[d];
    }
    so[a] = s;
    ss[a] = e - s;
    void* pin = (*env)->GetPrimitiveArrayCritical(env, (jarray)out, NULL);
    if (pin) {
      uint8_t* dst = (uint8_t*)pin + (size_t)((s - o64[a]) * SP.row);
      st = k == 1 ? zh_array_read_files(ctxs[0], &m, &store, (const char* const*)(paths + first),
                                        cnt, so, ss, dst, 0, err, sizeof err)
                  : zh_array_read_files_multi(ctxs, (int)k, 0, &m, &store,
                                              (const char* const*)(paths + first), cnt, so, ss,
                                              dst, 0, NULL, err, sizeof err);
      (*env)->ReleasePrimitiveArrayCritical(env, (jarray)out, pin, 0);
    } else {
      st = ZH_ENOMEM;
      snprintf(err, sizeof err, "could not access the output array");
    }
    s = e;
  }
  free_paths(paths, n, &store);
  if (st == ZH_EUNSUPPORTED) return st;
  if (st != ZH_OK) return throw_status(env, st, err);
  return 0;
}

/* ShardingIndexedCodec.decode / decodePartial replacement for one shard's bytes: the part
 * [offset, offset + partShape) of the shard, in slabs (the shard array and the result held per
 * slab). */
JNIEXPORT jint JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_shardDecodePartial(
    JNIEnv* env, jclass cls, jlong ctx, jintArray jm, jlongArray jshape, jintArray jchunk,
    jintArray jinner, jintArray jorder, jbyteArray jfill, jbyteArray shard, jlongArray joffset,
    jintArray jpart, jobject out) {
  (void)cls;
  zh_array_meta m;
  int st = build_meta(env, jm, jshape, jchunk, jinner, jorder, jfill, &m);
  if (st != ZH_OK) return st;
  char err[1024] = {0};
  jlong off[ZH_MAX_DIMS];
  jint part[ZH_MAX_DIMS];
  (*env)->GetLongArrayRegion(env, joffset, 0, m.ndim, off);
  (*env)->GetIntArrayRegion(env, jpart, 0, m.ndim, part);
  int64_t o64[ZH_MAX_DIMS], p64[ZH_MAX_DIMS], u[ZH_MAX_DIMS], nel = 1;
  for (int d = 0; d < m.ndim; d++) {
    o64[d] = off[d];
    p64[d] = part[d];
    nel *= part[d];
  }
  if ((int64_t)(*env)->GetArrayLength(env, (jarray)out) != nel)
    return throw_status(env, ZH_EINVAL, "output array size does not match the part shape");
  const jsize len = (*env)->GetArrayLength(env, shard);
  units_of(&m, 1, u);
  const SlabPlan SP = slab_plan(&m, p64, u, slab_cap_bytes());
  const int a = SP.axis;
  for (int64_t s = o64[a]; st == ZH_OK && s < o64[a] + p64[a];) {
    const int64_t e = slab_end(&SP, s, o64[a] + p64[a]);
    int64_t so[ZH_MAX_DIMS];
    int32_t sp[ZH_MAX_DIMS];
    for (int d = 0; d < m.ndim; d++) {
      so[d] = o64[d];
      sp[d] = (int32_t)p64[d];
    }
    so[a] = s;
    sp[a] = (int32_t)(e - s);
    Pinned P;
    if (pin_alloc(&P, 2, 0) != ZH_OK) {
      pin_release(env, &P);
      return throw_status(env, ZH_ENOMEM, "out of host memory");
    }
    P.arr[0] = (jarray)(*env)->NewLocalRef(env, shard);
    P.arr[1] = (jarray)out;
    P.n = 2;
    P.has_out = 1;
    st = pin_enter(env, &P);
    if (st == ZH_OK)
      st = zh_sharding_decode_partial((zh_ctx*)(intptr_t)ctx, &m, P.ptr[0], len, so, sp,
                                      (uint8_t*)P.ptr[1] + (size_t)((s - o64[a]) * SP.row), 0,
                                      NULL, err, sizeof err);
    else
      snprintf(err, sizeof err, "could not access the shard or output arrays");
    pin_release(env, &P);
    s = e;
  }
  if (st == ZH_EUNSUPPORTED) return st;
  if (st != ZH_OK) return throw_status(env, st, err);
  return 0;
}

/* ---- sub-shard reads: stored index + pieces (zh_array_read_pieces) ---------------------
 * Pure argument marshalling, no copy on this side: per slab the index and piece byte[]s of
 * the shards the slab touches and the result's primitive array are held with
 * GetPrimitiveArrayCritical and handed to the library as host memory (the policy at the top).
 * The library's pipelined read copies each referenced source range once, on several threads,
 * into its page-locked ring and DMAs it, and the region back out into the result the same way;
 * a single-threaded copy here (GetByteArrayRegion into a staging buffer, then a memcpy into the
 * result) would cost more than the whole read for GiB-sized regions.  The shim never reads the
 * index unless asked to check it (shardRanges' checkIndex; otherwise the device checks it). */

JNIEXPORT jlongArray JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_shardRanges(
    JNIEnv* env, jclass cls, jintArray jm, jlongArray jshape, jintArray jchunk, jintArray jinner,
    jintArray jorder, jbyteArray jfill, jbyteArray jindex, jlong size, jlongArray jlo,
    jlongArray jhi, jlong max_run, jboolean check_index) {
  (void)cls;
  zh_array_meta m;
  if (build_meta(env, jm, jshape, jchunk, jinner, jorder, jfill, &m) != ZH_OK) {
    throw_status(env, ZH_EINVAL, "bad array metadata");
    return NULL;
  }
  jsize ilen = (*env)->GetArrayLength(env, jindex);
  void* idx = malloc((size_t)(ilen > 0 ? ilen : 1));
  jlong lo[ZH_MAX_DIMS], hi[ZH_MAX_DIMS];
  int64_t lo64[ZH_MAX_DIMS], hi64[ZH_MAX_DIMS];
  if (!idx) {
    throw_status(env, ZH_ENOMEM, "out of host memory for the shard index");
    return NULL;
  }
  (*env)->GetByteArrayRegion(env, jindex, 0, ilen, (jbyte*)idx);
  if (check_index) {  /* Crc32cCodec.decode of the index before any range read (:205) */
    char err[1024] = {0};
    const int st = zh_shard_index_check(&m, idx, ilen, err, sizeof err);
    if (st != ZH_OK) {
      free(idx);
      throw_status(env, st, err);
      return NULL;
    }
  }
  (*env)->GetLongArrayRegion(env, jlo, 0, m.ndim, lo);
  (*env)->GetLongArrayRegion(env, jhi, 0, m.ndim, hi);
  for (int d = 0; d < m.ndim; d++) {
    lo64[d] = lo[d];
    hi64[d] = hi[d];
  }
  const int64_t n = zh_shard_ranges(&m, idx, ilen, size, lo64, hi64, max_run, NULL, 0);
  jlongArray res = NULL;
  if (n < 0) {
    throw_status(env, (int)-n, "zh_shard_ranges: invalid shard index or part");
  } else {
    int64_t* r = (int64_t*)malloc((size_t)(2 * n > 0 ? 2 * n : 1) * sizeof(int64_t));
    if (r && zh_shard_ranges(&m, idx, ilen, size, lo64, hi64, max_run, r, n) == n) {
      res = (*env)->NewLongArray(env, (jsize)(2 * n));
      if (res) (*env)->SetLongArrayRegion(env, res, 0, (jsize)(2 * n), (const jlong*)r);
    } else {
      throw_status(env, ZH_ENOMEM, "out of host memory for the shard ranges");
    }
    free(r);
  }
  free(idx);
  return res;
}

/* Shards [first, first + count) of a pieces call as zh_shard_src: every index / piece array of
 * those shards is collected (local references, lengths, offsets: JNI calls) into P, followed by
 * the output, before any critical section is entered.  pin_enter / pin_release then hold and
 * leave them; pieces_bind points srcs at the held addresses. */
static int pieces_collect(JNIEnv* env, jobjectArray jidx, jlongArray jsizes, jobjectArray joffs,
                          jobjectArray jlens, jobjectArray jdata, jsize first, jsize count,
                          jobject out_arr, zh_shard_src* srcs, Pinned* P, jsize* slot) {
  jsize total = 0;
  for (jsize i = 0; i < count; i++) {
    jobjectArray ps = (jobjectArray)(*env)->GetObjectArrayElement(env, jdata, first + i);
    if (ps) {
      total += (*env)->GetArrayLength(env, ps);
      (*env)->DeleteLocalRef(env, ps);
    }
  }
  /* one local reference per held array (+ the per-shard arrays, released as we go) */
  if ((*env)->EnsureLocalCapacity(env, count + total + 16) != 0) return ZH_ENOMEM;
  if (pin_alloc(P, count + total + 1, total) != ZH_OK) return ZH_ENOMEM;
  jsize na = 0, used = 0;
  for (jsize i = 0; i < count; i++) {
    memset(&srcs[i], 0, sizeof(srcs[i]));
    jlong size = -1;
    (*env)->GetLongArrayRegion(env, jsizes, first + i, 1, &size);
    srcs[i].shard_nbytes = size;
    slot[2 * i] = -1;  /* index array slot */
    jbyteArray ib = (jbyteArray)(*env)->GetObjectArrayElement(env, jidx, first + i);
    if (ib) {
      srcs[i].index_nbytes = (*env)->GetArrayLength(env, ib);
      slot[2 * i] = na;
      P->arr[na++] = ib;
    }
    jobjectArray ps = (jobjectArray)(*env)->GetObjectArrayElement(env, jdata, first + i);
    jlongArray po = (jlongArray)(*env)->GetObjectArrayElement(env, joffs, first + i);
    jlongArray pl = (jlongArray)(*env)->GetObjectArrayElement(env, jlens, first + i);
    jsize np = ps ? (*env)->GetArrayLength(env, ps) : 0;
    slot[2 * i + 1] = na;  /* first piece slot */
    srcs[i].pieces = P->pieces + used;
    srcs[i].npieces = np;
    for (jsize k = 0; k < np; k++) {
      jbyteArray b = (jbyteArray)(*env)->GetObjectArrayElement(env, ps, k);
      jlong off = 0, nb = 0;
      (*env)->GetLongArrayRegion(env, po, k, 1, &off);
      (*env)->GetLongArrayRegion(env, pl, k, 1, &nb);
      P->pieces[used + k].offset = off;
      P->pieces[used + k].nbytes = nb;
      P->pieces[used + k].data_nbytes = b ? (*env)->GetArrayLength(env, b) : 0;
      P->arr[na++] = b; /* may be NULL: an empty piece */
    }
    used += np;
    if (ps) (*env)->DeleteLocalRef(env, ps);
    if (po) (*env)->DeleteLocalRef(env, po);
    if (pl) (*env)->DeleteLocalRef(env, pl);
  }
  P->arr[na++] = (jarray)out_arr;
  P->n = na;
  P->has_out = 1;
  return ZH_OK;
}

static void pieces_bind(Pinned* P, zh_shard_src* srcs, jsize count, const jsize* slot) {
  for (jsize i = 0; i < count; i++) {
    srcs[i].index = slot[2 * i] >= 0 ? P->ptr[slot[2 * i]] : NULL;
    zh_shard_piece* q = (zh_shard_piece*)srcs[i].pieces;
    for (jsize k = 0; k < (jsize)srcs[i].npieces; k++) q[k].data = P->ptr[slot[2 * i + 1] + k];
  }
}

JNIEXPORT jint JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_arrayReadPieces(
    JNIEnv* env, jclass cls, jlongArray jctxs, jintArray jm, jlongArray jshape,
    jintArray jchunk, jintArray jinner, jintArray jorder, jbyteArray jfill, jobjectArray jidx,
    jlongArray jsizes, jobjectArray joffs, jobjectArray jlens, jobjectArray jdata,
    jlongArray joffset, jlongArray jregion, jobject out) {
  (void)cls;
  zh_array_meta m;
  int st = build_meta(env, jm, jshape, jchunk, jinner, jorder, jfill, &m);
  if (st != ZH_OK) return st;
  char err[1024] = {0};
  st = zh_validate_meta(&m, err, sizeof err);
  if (st == ZH_EUNSUPPORTED) return st;
  if (st != ZH_OK) return throw_status(env, st, err);
  jsize k = (*env)->GetArrayLength(env, jctxs);
  if (k <= 0 || k > 64) return throw_status(env, ZH_EINVAL, "bad device context list");
  jlong raw[64];
  zh_ctx* ctxs[64];
  (*env)->GetLongArrayRegion(env, jctxs, 0, k, raw);
  for (jsize i = 0; i < k; i++) ctxs[i] = (zh_ctx*)(intptr_t)raw[i];
  int64_t o64[ZH_MAX_DIMS], r64[ZH_MAX_DIMS], u[ZH_MAX_DIMS], nel = 1;
  region_of(env, m.ndim, joffset, jregion, o64, r64);
  for (int d = 0; d < m.ndim; d++) nel *= r64[d];
  if ((int64_t)(*env)->GetArrayLength(env, (jarray)out) != nel)
    return throw_status(env, ZH_EINVAL, "output array size does not match the region");
  const jsize n = (*env)->GetArrayLength(env, jidx);
  units_of(&m, 1, u);
  const SlabPlan SP = slab_plan(&m, r64, u, slab_cap_bytes());
  const int a = SP.axis;
  for (int64_t s = o64[a]; st == ZH_OK && s < o64[a] + r64[a];) {
    const int64_t e = slab_end(&SP, s, o64[a] + r64[a]);
    jsize first = 0, cnt = 0;
    slab_chunks(&m, o64, r64, a, s, e, &first, &cnt);
    if (first < 0 || first + cnt > n) {
      st = ZH_EINVAL;
      snprintf(err, sizeof err, "%d shard sources for a region of more shards", (int)n);
      break;
    }
    zh_shard_src* srcs = (zh_shard_src*)calloc((size_t)(cnt > 0 ? cnt : 1), sizeof(zh_shard_src));
    jsize* slot = (jsize*)malloc((size_t)(cnt > 0 ? 2 * cnt : 2) * sizeof(jsize));
    Pinned P;
    memset(&P, 0, sizeof P);
    st = srcs && slot ? pieces_collect(env, jidx, jsizes, joffs, jlens, jdata, first, cnt, out,
                                       srcs, &P, slot)
                      : ZH_ENOMEM;
    if (st == ZH_OK) st = pin_enter(env, &P);
    if (st == ZH_OK) {
      int64_t so[ZH_MAX_DIMS], ss[ZH_MAX_DIMS];
      for (int d = 0; d < m.ndim; d++) {
        so[d] = o64[d];
        ss[d] = r64[d];
      }
      so[a] = s;
      ss[a] = e - s;
      pieces_bind(&P, srcs, cnt, slot);
      uint8_t* dst = (uint8_t*)P.ptr[P.n - 1] + (size_t)((s - o64[a]) * SP.row);
      st = k == 1 ? zh_array_read_pieces(ctxs[0], &m, srcs, cnt, so, ss, dst, 0, NULL, err,
                                         sizeof err)
                  : zh_array_read_pieces_multi(ctxs, (int)k, 0, &m, srcs, cnt, so, ss, dst, 0,
                                               NULL, err, sizeof err);
    } else {
      snprintf(err, sizeof err, "could not access the source or output arrays");
    }
    pin_release(env, &P);
    free(slot);
    free(srcs);
    s = e;
  }
  if (st == ZH_EUNSUPPORTED) return st;
  if (st != ZH_OK) return throw_status(env, st, err);
  return 0;
}

JNIEXPORT jint JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_shardDecodePieces(
    JNIEnv* env, jclass cls, jlong ctx, jintArray jm, jlongArray jshape, jintArray jchunk,
    jintArray jinner, jintArray jorder, jbyteArray jfill, jbyteArray jindex, jlong size,
    jlongArray joffs, jlongArray jlens, jobjectArray jdata, jlongArray joffset, jintArray jpart,
    jobject out) {
  (void)cls;
  zh_array_meta m;
  int st = build_meta(env, jm, jshape, jchunk, jinner, jorder, jfill, &m);
  if (st != ZH_OK) return st;
  char err[1024] = {0};
  jlong off[ZH_MAX_DIMS];
  jint part[ZH_MAX_DIMS];
  (*env)->GetLongArrayRegion(env, joffset, 0, m.ndim, off);
  (*env)->GetIntArrayRegion(env, jpart, 0, m.ndim, part);
  int64_t o64[ZH_MAX_DIMS], p64[ZH_MAX_DIMS], u[ZH_MAX_DIMS], nel = 1;
  for (int d = 0; d < m.ndim; d++) {
    o64[d] = off[d];
    p64[d] = part[d];
    nel *= part[d];
  }
  if ((int64_t)(*env)->GetArrayLength(env, (jarray)out) != nel)
    return throw_status(env, ZH_EINVAL, "output array size does not match the part shape");
  /* one shard: wrap its arrays as the one-element arrays of the read form */
  jclass bcls = (*env)->FindClass(env, "[B"), lcls = (*env)->FindClass(env, "[J"),
         bbcls = (*env)->FindClass(env, "[[B");
  jobjectArray jidx = (*env)->NewObjectArray(env, 1, bcls, jindex);
  jobjectArray jo = (*env)->NewObjectArray(env, 1, lcls, joffs);
  jobjectArray jl = (*env)->NewObjectArray(env, 1, lcls, jlens);
  jobjectArray jd = (*env)->NewObjectArray(env, 1, bbcls, jdata);
  jlongArray js = (*env)->NewLongArray(env, 1);
  if (!jidx || !jo || !jl || !jd || !js) return throw_status(env, ZH_ENOMEM, "out of memory");
  (*env)->SetLongArrayRegion(env, js, 0, 1, &size);
  zh_ctx* c = (zh_ctx*)(intptr_t)ctx;
  units_of(&m, 1, u);
  const SlabPlan SP = slab_plan(&m, p64, u, slab_cap_bytes());
  const int a = SP.axis;
  for (int64_t s = o64[a]; st == ZH_OK && s < o64[a] + p64[a];) {
    const int64_t e = slab_end(&SP, s, o64[a] + p64[a]);
    int64_t so[ZH_MAX_DIMS];
    int32_t sp[ZH_MAX_DIMS];
    for (int d = 0; d < m.ndim; d++) {
      so[d] = o64[d];
      sp[d] = (int32_t)p64[d];
    }
    so[a] = s;
    sp[a] = (int32_t)(e - s);
    zh_shard_src src;
    jsize slot[2];
    Pinned P;
    memset(&P, 0, sizeof P);
    st = pieces_collect(env, jidx, js, jo, jl, jd, 0, 1, out, &src, &P, slot);
    if (st == ZH_OK) st = pin_enter(env, &P);
    if (st == ZH_OK) {
      pieces_bind(&P, &src, 1, slot);
      st = zh_sharding_decode_pieces(c, &m, &src, so, sp,
                                     (uint8_t*)P.ptr[P.n - 1] + (size_t)((s - o64[a]) * SP.row),
                                     0, NULL, err, sizeof err);
    } else {
      snprintf(err, sizeof err, "could not access the source or output arrays");
    }
    pin_release(env, &P);
    s = e;
  }
  (*env)->DeleteLocalRef(env, jidx);
  (*env)->DeleteLocalRef(env, jo);
  (*env)->DeleteLocalRef(env, jl);
  (*env)->DeleteLocalRef(env, jd);
  (*env)->DeleteLocalRef(env, js);
  if (st == ZH_EUNSUPPORTED) return st;
  if (st != ZH_OK) return throw_status(env, st, err);
  return 0;
}

/* The region of a Java array copied out of the heap in windows of one slab, each under its own
 * critical section (released with JNI_ABORT): the write paths' one use of a critical section.
 * Returns a malloc'd copy (the caller frees it) or NULL. */
static uint8_t* copy_region_out(JNIEnv* env, jobject data, size_t rbytes) {
  const size_t win = (size_t)slab_cap_bytes();
  uint8_t* src = (uint8_t*)malloc(rbytes > 0 ? rbytes : 1);
  for (size_t o = 0; src && o < rbytes; o += win) {
    void* pin = (*env)->GetPrimitiveArrayCritical(env, (jarray)data, NULL);
    if (!pin) {
      free(src);
      return NULL;
    }
    memcpy(src + o, (const uint8_t*)pin + o, rbytes - o < win ? rbytes - o : win);
    (*env)->ReleasePrimitiveArrayCritical(env, (jarray)data, pin, JNI_ABORT);
  }
  return src;
}

/* core.Array.write of a region of whole chunks into a FilesystemStore (HipArray.write):
 * paths[i] = StoreHandle.toPath() of the i-th chunk of computeChunkCoords; the library encodes
 * on the device and writes (or, all fill_value, deletes) the chunk files itself
 * (zh_array_write_files).  Returns 0, or 3 (ZH_EUNSUPPORTED: the caller keeps its own write) for
 * a chain, region or Java array the device path does not take. */
JNIEXPORT jint JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_arrayWriteFiles(
    JNIEnv* env, jclass cls, jlong ctx, jintArray jm, jlongArray jshape, jintArray jchunk,
    jintArray jinner, jintArray jorder, jbyteArray jfill, jlongArray joffset,
    jlongArray jregion, jobject data, jstring jroot, jstring jname, jobjectArray jpaths) {
  (void)cls;
  zh_array_meta m;
  int st = build_meta(env, jm, jshape, jchunk, jinner, jorder, jfill, &m);
  if (st != ZH_OK) return st;
  char err[1024] = {0};
  st = zh_validate_meta(&m, err, sizeof err);
  if (st == ZH_EUNSUPPORTED) return st;
  if (st != ZH_OK) return throw_status(env, st, err);
  int64_t o64[ZH_MAX_DIMS], r64[ZH_MAX_DIMS], want = 1;
  region_of(env, m.ndim, joffset, jregion, o64, r64);
  for (int d = 0; d < m.ndim; d++) want *= r64[d];
  /* a Java array of another length than the region: never read past its end */
  if ((int64_t)(*env)->GetArrayLength(env, (jarray)data) != want) return ZH_EUNSUPPORTED;
  const jsize n = (*env)->GetArrayLength(env, jpaths);
  zh_file_store store = {dup_string(env, jroot, &st), dup_string(env, jname, &st)};
  char** paths = dup_paths(env, jpaths, n, &st);
  if (st != ZH_OK) snprintf(err, sizeof err, "out of host memory");
  uint8_t* src = NULL;
  if (st == ZH_OK) {
    src = copy_region_out(env, data, (size_t)want * (size_t)m.dtype_size);
    if (!src) {
      st = ZH_ENOMEM;
      snprintf(err, sizeof err, "could not copy the region out of the Java heap");
    }
  }
  if (st == ZH_OK)
    st = zh_array_write_files((zh_ctx*)(intptr_t)ctx, &m, src, o64, r64, &store,
                              (const char* const*)paths, n, 0, NULL, err, sizeof err);
  free(src);
  free_paths(paths, n, &store);
  if (st == ZH_EUNSUPPORTED) return st;
  if (st != ZH_OK) return throw_status(env, st, err);
  return 0;
}

/* core.Array.write replacement for a region of whole chunks (clipped only by the array
 * boundary): data = the primitive array of the region in C order (ucar storage copied to
 * 1-D); returns byte[][] in computeChunkCoords order, null = chunk all fill_value (the
 * caller deletes the key, Array.java:150-151), or null when the chain or region is not
 * device-supported (the caller keeps core.Array.write). */
JNIEXPORT jobjectArray JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_arrayWrite(
    JNIEnv* env, jclass cls, jlong ctx, jintArray jm, jlongArray jshape, jintArray jchunk,
    jintArray jinner, jintArray jorder, jbyteArray jfill, jlongArray joffset,
    jlongArray jregion, jobject data) {
  (void)cls;
  zh_array_meta m;
  int st = build_meta(env, jm, jshape, jchunk, jinner, jorder, jfill, &m);
  if (st != ZH_OK) return NULL;
  char err[1024] = {0};
  st = zh_validate_meta(&m, err, sizeof err);
  if (st == ZH_EUNSUPPORTED) return NULL;
  if (st != ZH_OK) {
    throw_status(env, st, err);
    return NULL;
  }
  jlong off[ZH_MAX_DIMS], reg[ZH_MAX_DIMS];
  (*env)->GetLongArrayRegion(env, joffset, 0, m.ndim, off);
  (*env)->GetLongArrayRegion(env, jregion, 0, m.ndim, reg);
  int64_t o64[ZH_MAX_DIMS], r64[ZH_MAX_DIMS], sh64[ZH_MAX_DIMS];
  int32_t cs32[ZH_MAX_DIMS];
  for (int d = 0; d < m.ndim; d++) {
    o64[d] = off[d];
    r64[d] = reg[d];
    sh64[d] = m.shape[d];
    cs32[d] = m.chunk_shape[d];
  }
  const int64_t n = zh_compute_chunk_coords(m.ndim, sh64, cs32, o64, r64, NULL, 0);
  if (n < 0) {
    throw_status(env, ZH_EINVAL, "chunk coordinates out of range");
    return NULL;
  }
  const int64_t bound = zh_array_encoded_bound(&m);
  void** outs = (void**)calloc((size_t)(n > 0 ? n : 1), sizeof(void*));
  int64_t* caps = (int64_t*)calloc((size_t)(n > 0 ? n : 1), sizeof(int64_t));
  int64_t* sizes = (int64_t*)calloc((size_t)(n > 0 ? n : 1), sizeof(int64_t));
  int ok = outs && caps && sizes;
  for (int64_t i = 0; ok && i < n; i++) {
    outs[i] = malloc((size_t)(bound > 0 ? bound : 1));
    caps[i] = bound;
    ok = outs[i] != NULL;
  }
  jobjectArray res = NULL;
  if (!ok) {
    throw_status(env, ZH_ENOMEM, "out of host memory for the encoded chunks");
  } else {
    jsize nel = (*env)->GetArrayLength(env, (jarray)data);
    int64_t want = 1;
    for (int d = 0; d < m.ndim; d++) want *= r64[d];
    if ((int64_t)nel != want) {
      /* a Java array of another length (or element type) than the region: never read past
       * its end; the caller keeps core.Array.write */
      for (int64_t i = 0; i < n; i++) free(outs[i]);
      free(outs);
      free(caps);
      free(sizes);
      return NULL;
    }
    /* copy the region out of the heap in windows of one slab (the critical-section policy):
     * the call stages it to the device */
    uint8_t* src = copy_region_out(env, data, (size_t)nel * (size_t)m.dtype_size);
    const int pinned = src != NULL;
    st = pinned ? zh_array_write_host((zh_ctx*)(intptr_t)ctx, &m, src, o64, r64, outs, caps,
                                      sizes, n, err, sizeof err)
                : ZH_ENOMEM;
    free(src);
    if (st == ZH_OK) {
      jclass bcls = (*env)->FindClass(env, "[B");
      res = bcls ? (*env)->NewObjectArray(env, (jsize)n, bcls, NULL) : NULL;
      for (int64_t i = 0; res && i < n; i++) {
        if (sizes[i] == 0) continue;  /* all fill: null → delete the key */
        jbyteArray b = (*env)->NewByteArray(env, (jsize)sizes[i]);
        if (!b) {
          res = NULL;
          break;
        }
        (*env)->SetByteArrayRegion(env, b, 0, (jsize)sizes[i], (const jbyte*)outs[i]);
        (*env)->SetObjectArrayElement(env, res, (jsize)i, b);
        (*env)->DeleteLocalRef(env, b);
      }
    } else if (st != ZH_EUNSUPPORTED) {
      throw_status(env, st, err);
    }
  }
  for (int64_t i = 0; outs && i < n; i++) free(outs[i]);
  free(outs);
  free(caps);
  free(sizes);
  return res;
}
