/*
 * zarrhip_jni.c — thin JNI shim from zarr-java to the zarrhip C-ABI (include/zarrhip.h).
 * Built only where a JDK exists (needs $JAVA_HOME/include/jni.h); see INTEGRATION.md.
 *
 * Every native method assembles a zh_array_meta from Java primitives, pins the Java
 * arrays for the duration of the call (GetPrimitiveArrayCritical: no JNI calls while
 * pinned), and maps zh_status to the reference's exceptions:
 *   ZH_EDATA → dev.zarr.zarrjava.ZarrException, ZH_EINVAL → IllegalArgumentException,
 *   ZH_EARITH → ArithmeticException, ZH_EUNSUPPORTED → returned as 3 (Java falls back to
 *   the reference codec), anything else → RuntimeException.
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
 *              nestedIndexLocation, innerCrc32c]}; shape long[ndim]; chunkShape/order int[ndim];
 *              innerShape int[ndim] (nested: int[2*ndim], inner then leaf shape);
 *              fill byte[dtypeSize] (little-endian element bytes). */
static int build_meta(JNIEnv* env, jintArray jm, jlongArray jshape, jintArray jchunk,
                      jintArray jinner, jintArray jorder, jbyteArray jfill, zh_array_meta* m) {
  memset(m, 0, sizeof(*m));
  jint mi[14] = {0};
  jsize nm = (*env)->GetArrayLength(env, jm);
  (*env)->GetIntArrayRegion(env, jm, 0, nm < 14 ? nm : 14, mi);
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
  jsize n = (*env)->GetArrayLength(env, jchunks);
  zh_chunk_src* srcs = (zh_chunk_src*)calloc((size_t)(n > 0 ? n : 1), sizeof(zh_chunk_src));
  jbyteArray* arrs = (jbyteArray*)calloc((size_t)(n > 0 ? n : 1), sizeof(jbyteArray));
  /* copy chunk bytes out of the heap (several may be large: no long critical sections) */
  void** copies = (void**)calloc((size_t)(n > 0 ? n : 1), sizeof(void*));
  for (jsize i = 0; i < n; i++) {
    arrs[i] = (jbyteArray)(*env)->GetObjectArrayElement(env, jchunks, i);
    if (!arrs[i]) continue;
    jsize len = (*env)->GetArrayLength(env, arrs[i]);
    copies[i] = malloc((size_t)(len > 0 ? len : 1));
    (*env)->GetByteArrayRegion(env, arrs[i], 0, len, (jbyte*)copies[i]);
    srcs[i].data = copies[i];
    srcs[i].nbytes = len;
    (*env)->DeleteLocalRef(env, arrs[i]);
  }
  jlong off[ZH_MAX_DIMS], reg[ZH_MAX_DIMS];
  (*env)->GetLongArrayRegion(env, joffset, 0, m.ndim, off);
  (*env)->GetLongArrayRegion(env, jregion, 0, m.ndim, reg);
  int64_t o64[ZH_MAX_DIMS], r64[ZH_MAX_DIMS];
  for (int d = 0; d < m.ndim; d++) {
    o64[d] = off[d];
    r64[d] = reg[d];
  }
  /* decode into native memory, then hold the critical section only for the final copy
   * (a critical section around device work would stall every other Java thread's GC) */
  int64_t nel = 1;
  for (int d = 0; d < m.ndim; d++) nel *= r64[d];
  const size_t obytes = (size_t)nel * (size_t)m.dtype_size;
  void* tmp = NULL;
  if ((int64_t)(*env)->GetArrayLength(env, (jarray)out) != nel) {
    st = ZH_EINVAL;
    snprintf(err, sizeof err, "output array holds %lld elements, the region %lld",
             (long long)(*env)->GetArrayLength(env, (jarray)out), (long long)nel);
  } else if (!(tmp = malloc(obytes > 0 ? obytes : 1))) {
    st = ZH_ENOMEM;
    snprintf(err, sizeof err, "out of host memory for the decoded region");
  } else if (nctx == 1) {
    st = zh_array_read(ctxs[0], &m, srcs, n, o64, r64, tmp, 0, NULL, err, sizeof err);
  } else { /* one slab per device, each D2H'd into its slice of the region */
    st = zh_array_read_multi(ctxs, nctx, 0, &m, srcs, n, o64, r64, tmp, 0, err, sizeof err);
  }
  if (st == ZH_OK) {
    void* dst = (*env)->GetPrimitiveArrayCritical(env, (jarray)out, NULL);
    if (dst) {
      memcpy(dst, tmp, obytes);
      (*env)->ReleasePrimitiveArrayCritical(env, (jarray)out, dst, 0);
    } else {
      st = ZH_ENOMEM;
      snprintf(err, sizeof err, "could not access the output array");
    }
  }
  free(tmp);
  for (jsize i = 0; i < n; i++) free(copies[i]);
  free(copies);
  free(arrs);
  free(srcs);
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

/* ShardingIndexedCodec.decode / decodePartial replacement for one shard's bytes. */
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
  int64_t o64[ZH_MAX_DIMS];
  for (int d = 0; d < m.ndim; d++) o64[d] = off[d];
  jsize len = (*env)->GetArrayLength(env, shard);
  int64_t nel = 1;
  for (int d = 0; d < m.ndim; d++) nel *= part[d];
  const size_t obytes = (size_t)nel * (size_t)m.dtype_size;
  if ((int64_t)(*env)->GetArrayLength(env, (jarray)out) != nel)
    return throw_status(env, ZH_EINVAL, "output array size does not match the part shape");
  void* src = malloc((size_t)(len > 0 ? len : 1));
  void* tmp = malloc(obytes > 0 ? obytes : 1);
  if (!src || !tmp) {
    free(src);
    free(tmp);
    return throw_status(env, ZH_ENOMEM, "out of host memory for the shard");
  }
  (*env)->GetByteArrayRegion(env, shard, 0, len, (jbyte*)src);
  /* decode into native memory; the critical section covers only the final copy */
  st = zh_sharding_decode_partial((zh_ctx*)(intptr_t)ctx, &m, src, len, o64, part, tmp, 0, NULL,
                                  err, sizeof err);
  if (st == ZH_OK) {
    void* dst = (*env)->GetPrimitiveArrayCritical(env, (jarray)out, NULL);
    if (dst) {
      memcpy(dst, tmp, obytes);
      (*env)->ReleasePrimitiveArrayCritical(env, (jarray)out, dst, 0);
    } else {
      st = ZH_ENOMEM;
      snprintf(err, sizeof err, "could not access the output array");
    }
  }
  free(tmp);
  free(src);
  if (st == ZH_EUNSUPPORTED) return st;
  if (st != ZH_OK) return throw_status(env, st, err);
  return 0;
}

/* ---- sub-shard reads: stored index + pieces (zh_array_read_pieces) ---------------------
 * Pure argument marshalling, no copy on this side: the index and piece byte[]s and the
 * result's primitive array are held with GetPrimitiveArrayCritical for the duration of the
 * call and handed to the library as host memory.  The library's pipelined read copies each
 * source once, on several threads, into its page-locked ring and DMAs it (and back out into
 * the result the same way); a single-threaded copy here (GetByteArrayRegion into a staging
 * buffer, then a memcpy into the result) would cost more than the whole read for GiB-sized
 * regions.  While the critical sections are held the call makes no JNI call; the GC waits for
 * at most the read itself.  The shim never reads the index (the device checks it).
 * tests/helpers.py jni_fetch / jni_read restate this call sequence in ctypes, and the GPU
 * tests run it (tests/test_gpu_pieces.py). */

JNIEXPORT jlongArray JNICALL Java_dev_zarr_zarrjava_hip_ZarrHip_shardRanges(
    JNIEnv* env, jclass cls, jintArray jm, jlongArray jshape, jintArray jchunk, jintArray jinner,
    jintArray jorder, jbyteArray jfill, jbyteArray jindex, jlong size, jlongArray jlo,
    jlongArray jhi, jlong max_run) {
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

/* The shards of a read as zh_shard_src: every index / piece array is collected (local
 * references, lengths, offsets: JNI calls) first, then all of them and the output enter their
 * critical sections together (no JNI call in between).  pin_release() leaves them. */
typedef struct {
  jsize n;                 /* arrays held */
  jarray* arr;             /* index / piece byte[]s, then the output */
  void** ptr;              /* their critical addresses */
  zh_shard_piece* pieces;
} Pinned;

static void pin_release(JNIEnv* env, Pinned* P, jsize n_out) {
  /* the output (the last `n_out` entries) is written back; the sources are not */
  for (jsize k = P->n - 1; k >= 0; k--)
    if (P->ptr[k])
      (*env)->ReleasePrimitiveArrayCritical(env, P->arr[k], P->ptr[k],
                                            k >= P->n - n_out ? 0 : JNI_ABORT);
  free(P->arr);
  free(P->ptr);
  free(P->pieces);
  memset(P, 0, sizeof(*P));
}

/* srcs[i] for each shard i; out_arr (may be NULL) is pinned last, its address in *out_ptr. */
static int pin_pieces(JNIEnv* env, jobjectArray jidx, jlongArray jsizes, jobjectArray joffs,
                      jobjectArray jlens, jobjectArray jdata, jobject out_arr, zh_shard_src* srcs,
                      Pinned* P, void** out_ptr) {
  memset(P, 0, sizeof(*P));
  jsize n = (*env)->GetArrayLength(env, jidx), total = 0;
  for (jsize i = 0; i < n; i++) {
    jobjectArray ps = (jobjectArray)(*env)->GetObjectArrayElement(env, jdata, i);
    if (ps) total += (*env)->GetArrayLength(env, ps);
    if (ps) (*env)->DeleteLocalRef(env, ps);
  }
  /* one local reference per held array (+ the per-shard arrays, released as we go) */
  if ((*env)->EnsureLocalCapacity(env, n + total + 16) != 0) return ZH_ENOMEM;
  P->arr = (jarray*)calloc((size_t)(n + total + 1), sizeof(jarray));
  P->ptr = (void**)calloc((size_t)(n + total + 1), sizeof(void*));
  P->pieces = (zh_shard_piece*)calloc((size_t)(total > 0 ? total : 1), sizeof(zh_shard_piece));
  if (!P->arr || !P->ptr || !P->pieces) return ZH_ENOMEM;
  jsize na = 0, used = 0;
  /* per shard: the index array, then its pieces (references and lengths only) */
  jsize* idx_slot = (jsize*)malloc((size_t)(n > 0 ? n : 1) * sizeof(jsize));
  jsize* piece_first = (jsize*)malloc((size_t)(n > 0 ? n : 1) * sizeof(jsize));
  if (!idx_slot || !piece_first) {
    free(idx_slot);
    free(piece_first);
    return ZH_ENOMEM;
  }
  for (jsize i = 0; i < n; i++) {
    memset(&srcs[i], 0, sizeof(srcs[i]));
    jlong size = -1;
    (*env)->GetLongArrayRegion(env, jsizes, i, 1, &size);
    srcs[i].shard_nbytes = size;
    idx_slot[i] = -1;
    jbyteArray ib = (jbyteArray)(*env)->GetObjectArrayElement(env, jidx, i);
    if (ib) {
      srcs[i].index_nbytes = (*env)->GetArrayLength(env, ib);
      idx_slot[i] = na;
      P->arr[na++] = ib;
    }
    jobjectArray ps = (jobjectArray)(*env)->GetObjectArrayElement(env, jdata, i);
    jlongArray po = (jlongArray)(*env)->GetObjectArrayElement(env, joffs, i);
    jlongArray pl = (jlongArray)(*env)->GetObjectArrayElement(env, jlens, i);
    jsize np = ps ? (*env)->GetArrayLength(env, ps) : 0;
    piece_first[i] = na;
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
  if (out_arr) P->arr[na++] = (jarray)out_arr;
  P->n = na;
  /* enter every critical section; from here on no JNI call until pin_release */
  int st = ZH_OK;
  for (jsize k = 0; k < na && st == ZH_OK; k++) {
    if (!P->arr[k]) continue;
    P->ptr[k] = (*env)->GetPrimitiveArrayCritical(env, P->arr[k], NULL);
    if (!P->ptr[k]) st = ZH_ENOMEM;
  }
  if (st == ZH_OK) {
    used = 0;
    for (jsize i = 0; i < n; i++) {
      if (idx_slot[i] >= 0) srcs[i].index = P->ptr[idx_slot[i]];
      for (jsize k = 0; k < srcs[i].npieces; k++)
        P->pieces[used + k].data = P->ptr[piece_first[i] + k];
      used += (jsize)srcs[i].npieces;
    }
    if (out_arr && out_ptr) *out_ptr = P->ptr[na - 1];
  }
  free(idx_slot);
  free(piece_first);
  return st;
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
  jlong off[ZH_MAX_DIMS], reg[ZH_MAX_DIMS];
  int64_t o64[ZH_MAX_DIMS], r64[ZH_MAX_DIMS];
  (*env)->GetLongArrayRegion(env, joffset, 0, m.ndim, off);
  (*env)->GetLongArrayRegion(env, jregion, 0, m.ndim, reg);
  int64_t nel = 1;
  for (int d = 0; d < m.ndim; d++) {
    o64[d] = off[d];
    r64[d] = reg[d];
    nel *= r64[d];
  }
  if ((int64_t)(*env)->GetArrayLength(env, (jarray)out) != nel)
    return throw_status(env, ZH_EINVAL, "output array size does not match the region");
  jsize n = (*env)->GetArrayLength(env, jidx);
  zh_shard_src* srcs = (zh_shard_src*)calloc((size_t)(n > 0 ? n : 1), sizeof(zh_shard_src));
  if (!srcs) return throw_status(env, ZH_ENOMEM, "out of host memory");
  Pinned P;
  void* dst = NULL;
  st = pin_pieces(env, jidx, jsizes, joffs, jlens, jdata, out, srcs, &P, &dst);
  if (st == ZH_OK)
    st = k == 1 ? zh_array_read_pieces(ctxs[0], &m, srcs, n, o64, r64, dst, 0, NULL, err, sizeof err)
                : zh_array_read_pieces_multi(ctxs, (int)k, 0, &m, srcs, n, o64, r64, dst, 0, NULL,
                                             err, sizeof err);
  else
    snprintf(err, sizeof err, "could not access the source or output arrays");
  pin_release(env, &P, 1);
  free(srcs);
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
  int64_t o64[ZH_MAX_DIMS], nel = 1;
  for (int d = 0; d < m.ndim; d++) {
    o64[d] = off[d];
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
  zh_shard_src src;
  Pinned P;
  void* dst = NULL;
  st = pin_pieces(env, jidx, js, jo, jl, jd, out, &src, &P, &dst);
  if (st == ZH_OK)
    st = zh_sharding_decode_pieces(c, &m, &src, o64, (const int32_t*)part, dst, 0, NULL, err,
                                   sizeof err);
  else
    snprintf(err, sizeof err, "could not access the source or output arrays");
  pin_release(env, &P, 1);
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
    /* copy the region out of the heap: the call stages it to the device (no long critical
     * section around device work) */
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
    const size_t rbytes = (size_t)nel * (size_t)m.dtype_size;
    void* src = malloc(rbytes > 0 ? rbytes : 1);
    void* pin = (*env)->GetPrimitiveArrayCritical(env, (jarray)data, NULL);
    if (src && pin) memcpy(src, pin, rbytes);
    if (pin) (*env)->ReleasePrimitiveArrayCritical(env, (jarray)data, pin, JNI_ABORT);
    st = src && pin ? zh_array_write_host((zh_ctx*)(intptr_t)ctx, &m, src, o64, r64, outs, caps,
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
