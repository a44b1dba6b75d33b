/*
 * zh_oracle.c — TEST INFRASTRUCTURE ONLY (see zh_oracle.h).
 *
 * Plain-C restatement of the zarr-java read/write chain for the device-supported codec
 * chains.  Each function names the reference lines it follows
 * (M/ = /root/reference/src/main/java/dev/zarr/zarrjava/).  It deliberately keeps the
 * reference's structure — zero-initialised per-shard part array, two region copies,
 * byte-at-a-time CRC — because it is the checker, not the thing measured for speed.
 *
 * Knowing divergences (also in DESIGN.md):
 *  - Q12: an inner chunk whose stored length differs from the decoded chunk size is an
 *    error here ("unexpected inner chunk byte length"); ucar.ma2.Array.factory would
 *    read a prefix or underflow.
 *  - Q7: encode lays inner chunks out in C order (the reference appends in parallel,
 *    non-deterministic order); decode is index-driven, so both read identically.
 */
#include "zh_oracle.h"

#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define INT_MAX_J 2147483647LL

static void set_err(char* err, size_t errlen, const char* fmt, ...) {
  if (!err || errlen == 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err, errlen, fmt, ap);
  va_end(ap);
}

/* ---------------------------------------------------------------------------------
 * CRC-32C: M/utils/CRC32C.java.  Table :14-80 is the reflected Castagnoli table
 * (poly 0x82F63B78); update(ByteBuffer) :119-125 runs updateByte :160-164 per byte
 * between the ^0xFFFFFFFF pre/post conditioning.
 * ------------------------------------------------------------------------------- */
static uint32_t g_crc_table[256];
static int g_crc_init = 0;

static void crc_table_init(void) {
  if (g_crc_init) return;
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
    g_crc_table[i] = c;
  }
  g_crc_init = 1;
}

uint32_t zo_crc32c(uint32_t crc, const void* data, size_t n) {
  crc_table_init();
  const uint8_t* p = (const uint8_t*)data;
  uint32_t c = crc ^ 0xFFFFFFFFu;                       /* CRC32C.java:120 */
  for (size_t i = 0; i < n; i++)                        /* :121-123 */
    c = g_crc_table[(c ^ p[i]) & 0xFFu] ^ (c >> 8);      /* updateByte :160-164 */
  return c ^ 0xFFFFFFFFu;                               /* :124 */
}

/* ---------------------------------------------------------------------------------
 * IndexingUtils.computeChunkCoords — M/utils/IndexingUtils.java:16-51
 * ------------------------------------------------------------------------------- */
int64_t zo_compute_chunk_coords(int ndim, const int64_t* array_shape, const int32_t* chunk_shape,
                                const int64_t* sel_offset, const int64_t* sel_shape,
                                int64_t* coords_out, int64_t max_coords) {
  (void)array_shape;
  int64_t start[ZH_MAX_DIMS], end[ZH_MAX_DIMS];
  int64_t num = 1;
  for (int d = 0; d < ndim; d++) {                      /* :22-28 */
    int64_t s = (int64_t)(int32_t)(sel_offset[d] / chunk_shape[d]);
    int64_t e = (int64_t)(int32_t)((sel_offset[d] + sel_shape[d] - 1) / chunk_shape[d]);
    num *= (e - s + 1);
    start[d] = s;
    end[d] = e;
  }
  if (num > INT_MAX_J) return -1;                       /* :30-32 ArithmeticException */
  if (!coords_out) return num;
  int64_t cur[ZH_MAX_DIMS];
  memcpy(cur, start, sizeof(int64_t) * ndim);
  for (int64_t i = 0; i < num && i < max_coords; i++) { /* :36-49 */
    memcpy(coords_out + i * ndim, cur, sizeof(int64_t) * ndim);
    int d = ndim - 1;
    while (d >= 0) {
      if (cur[d] >= end[d]) {
        cur[d] = start[d];
        d--;
      } else {
        cur[d]++;
        d = -1;
      }
    }
  }
  return num;
}

/* IndexingUtils.computeProjection (5-arg) — M/utils/IndexingUtils.java:65-117 */
int zo_compute_projection(int ndim, const int64_t* chunk_coords, const int64_t* array_shape,
                          const int32_t* chunk_shape, const int64_t* sel_offset,
                          const int64_t* sel_shape, int32_t* chunk_offset, int32_t* out_offset,
                          int32_t* shape) {
  for (int d = 0; d < ndim; d++) {
    int64_t dim_off = (int64_t)chunk_shape[d] * chunk_coords[d];                  /* :77 */
    int64_t lim_a = array_shape[d], lim_b = (chunk_coords[d] + 1) * (int64_t)chunk_shape[d];
    int64_t dim_limit = lim_a < lim_b ? lim_a : lim_b;                            /* :78-79 */
    if (sel_offset[d] < dim_off) {                                                /* :81-90 */
      chunk_offset[d] = 0;
      int64_t v = dim_off - sel_offset[d];
      if (v > INT_MAX_J) return ZH_EARITH;
      out_offset[d] = (int32_t)v;
    } else {                                                                      /* :91-100 */
      int64_t v = sel_offset[d] - dim_off;
      if (v > INT_MAX_J) return ZH_EARITH;
      chunk_offset[d] = (int32_t)v;
      out_offset[d] = 0;
    }
    if (sel_offset[d] + sel_shape[d] > dim_limit) {                               /* :102-105 */
      shape[d] = chunk_shape[d] - chunk_offset[d];
    } else {                                                                      /* :106-113 */
      int64_t v = sel_offset[d] + sel_shape[d] - dim_off - chunk_offset[d];
      if (v > INT_MAX_J || v < 0) return ZH_EARITH;
      shape[d] = (int32_t)v;
    }
  }
  return ZH_OK;
}

/* Utils.isPermutation / inversePermutation — M/utils/Utils.java:91-109 */
int zo_is_permutation(int n, const int32_t* order) {
  if (n <= 0) return 0;
  int seen[64] = {0};
  if (n > 64) return 0;
  for (int i = 0; i < n; i++) {
    if (order[i] < 0 || order[i] >= n || seen[order[i]]) return 0;
    seen[order[i]] = 1;
  }
  return 1;
}

int zo_inverse_permutation(int n, const int32_t* order, int32_t* inverse) {
  if (!zo_is_permutation(n, order)) return ZH_EINVAL;
  for (int i = 0; i < n; i++) inverse[order[i]] = i;
  return ZH_OK;
}

/* ---------------------------------------------------------------------------------
 * A minimal strided N-d array standing in for ucar.ma2.Array (views by strides).
 * ------------------------------------------------------------------------------- */
typedef struct {
  uint8_t* data;
  int ndim;
  int dsize;
  int64_t shape[ZH_MAX_DIMS];
  int64_t stride[ZH_MAX_DIMS]; /* in elements */
} nd_t;

static void nd_c_order(nd_t* a) {
  int64_t s = 1;
  for (int d = a->ndim - 1; d >= 0; d--) {
    a->stride[d] = s;
    s *= a->shape[d];
  }
}

static int64_t prod64(const int64_t* v, int n) {
  int64_t p = 1;
  for (int i = 0; i < n; i++) p *= v[i];
  return p;
}

/* MultiArrayUtils.copyRegion — M/utils/MultiArrayUtils.java:14-57: element-wise copy
 * between two range iterators walking the logical index space in C order. */
static void copy_region(const nd_t* src, const int64_t* soff, nd_t* dst, const int64_t* doff,
                        const int64_t* shape) {
  int n = src->ndim, ds = src->dsize;
  int64_t total = prod64(shape, n);
  if (total <= 0) return;
  int64_t idx[ZH_MAX_DIMS] = {0};
  for (int64_t t = 0; t < total; t++) {
    int64_t so = 0, dof = 0;
    for (int d = 0; d < n; d++) {
      so += (soff[d] + idx[d]) * src->stride[d];
      dof += (doff[d] + idx[d]) * dst->stride[d];
    }
    memcpy(dst->data + dof * ds, src->data + so * ds, ds);
    for (int d = n - 1; d >= 0; d--) {
      if (++idx[d] < shape[d]) break;
      idx[d] = 0;
    }
  }
}

/* MultiArrayUtils.fill — M/utils/MultiArrayUtils.java:59-67 (C-order contiguous array) */
static void fill_elems(uint8_t* p, int64_t n, int dsize, const uint8_t* fill) {
  for (int64_t i = 0; i < n; i++) memcpy(p + i * dsize, fill, dsize);
}

static void swap_elem(uint8_t* e, int dsize) {
  for (int i = 0; i < dsize / 2; i++) {
    uint8_t t = e[i];
    e[i] = e[dsize - 1 - i];
    e[dsize - 1 - i] = t;
  }
}

static int elem_swaps(const zh_array_meta* m, int endian) {
  /* core BytesCodec.decode :16-19: byte order only matters for >1-byte types; the host
   * (and every ucar array) is little-endian. */
  return m->dtype_size > 1 && endian == ZH_ENDIAN_BIG;
}


static void fmt_coords(char* buf, size_t len, const int64_t* c, int n) {
  /* java.util.Arrays.toString(long[]) */
  size_t o = 0;
  o += snprintf(buf + o, len - o, "[");
  for (int i = 0; i < n && o < len; i++)
    o += snprintf(buf + o, len - o, i ? ", %lld" : "%lld", (long long)c[i]);
  if (o < len) snprintf(buf + o, len - o, "]");
}

/* Inner codec pipeline decode (CodecPipeline.decode, M/core/codec/CodecPipeline.java:104-137):
 *   BytesCodec.decode (M/core/codec/core/BytesCodec.java:15-35) turns the bytes into an
 *   array of the *encoded* shape in the configured byte order (bool: b != 0), then
 *   TransposeCodec.decode (M/v3/codec/core/TransposeCodec.java:34-44) returns the view
 *   permute(inversePermutation(order)).  `buf` receives the decoded bytes (caller frees)
 *   and `view` the logical (decoded-shape) strided view over it. */
static int inner_decode(const zh_array_meta* m, const int32_t* chunk_shape, const uint8_t* bytes,
                        int64_t nbytes, uint8_t** buf, nd_t* view, char* err, size_t errlen) {
  const zh_codec_chain* ch = &m->chain;
  int n = m->ndim, ds = m->dtype_size;
  int64_t nel = 1;
  for (int d = 0; d < n; d++) nel *= chunk_shape[d];
  if (ch->inner_crc32c) { /* Crc32cCodec.decode (Crc32cCodec.java:24-48), last BB codec */
    if (nbytes < 4) {
      set_err(err, errlen, "unexpected inner chunk byte length: %lld (expected %lld)",
              (long long)nbytes, (long long)(nel * ds + 4));
      return ZH_EDATA;
    }
    nbytes -= 4;
    int32_t computed = (int32_t)zo_crc32c(0, bytes, nbytes);
    const uint8_t* s = bytes + nbytes;
    int32_t stored = (int32_t)((uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) |
                               ((uint32_t)s[3] << 24));
    if (computed != stored) {
      set_err(err, errlen,
              "The checksum of the sharding index is invalid. Stored: %d Computed: %d", stored,
              computed);
      return ZH_EDATA;
    }
  }
  if (nbytes != nel * ds) { /* Q12, see header */
    set_err(err, errlen, "unexpected inner chunk byte length: %lld (expected %lld)",
            (long long)(nbytes + (ch->inner_crc32c ? 4 : 0)),
            (long long)(nel * ds + (ch->inner_crc32c ? 4 : 0)));
    return ZH_EDATA;
  }
  uint8_t* b = (uint8_t*)malloc(nel * ds > 0 ? nel * ds : 1);
  memcpy(b, bytes, nel * ds);
  if (elem_swaps(m, ch->endian))
    for (int64_t i = 0; i < nel; i++) swap_elem(b + i * ds, ds);
  if (m->dtype_is_bool)
    for (int64_t i = 0; i < nel; i++) b[i] = b[i] != 0;
  /* encoded array: shape[j] = chunkShape[order[j]] (TransposeCodec.resolveArrayMetadata :70-71) */
  nd_t enc;
  enc.data = b;
  enc.ndim = n;
  enc.dsize = ds;
  int32_t order[ZH_MAX_DIMS] = {0}, inv[ZH_MAX_DIMS] = {0};
  for (int d = 0; d < n; d++) order[d] = ch->has_transpose ? ch->transpose_order[d] : d;
  if (ch->has_transpose) {
    if (!zo_is_permutation(n, order)) {                       /* :36-38 */
      free(b);
      set_err(err, errlen, "Order is no permutation array");
      return ZH_EDATA;
    }
  }
  for (int j = 0; j < n; j++) enc.shape[j] = chunk_shape[order[j]];
  nd_c_order(&enc);
  zo_inverse_permutation(n, order, inv);
  /* ucar Array.permute(dims): view dim i = source dim dims[i] */
  view->data = b;
  view->ndim = n;
  view->dsize = ds;
  for (int i = 0; i < n; i++) {
    view->shape[i] = enc.shape[inv[i]];
    view->stride[i] = enc.stride[inv[i]];
  }
  *buf = b;
  return ZH_OK;
}

static int64_t shard_index_size(const zh_array_meta* m) {
  /* ShardingIndexedCodec.getShardIndexSize :176-181 — 16 * prod(chunksPerShard) through the
   * index pipeline's computeEncodedSize (+4 for crc32c, Crc32cCodec.java:157-160) */
  int64_t n = 1;
  for (int d = 0; d < m->ndim; d++) n *= m->chunk_shape[d] / m->chain.inner_chunk_shape[d];
  return 16 * n + (m->chain.index_has_crc32c ? 4 : 0);
}

/* Nested sharding: the inner codec pipeline of the outer ShardingIndexedCodec is itself
 * [sharding_indexed{...}] (ZarrPythonTests.java:177-179).  Its CoreArrayMetadata is the
 * outer codec's inner-chunk metadata (ShardingIndexedCodec.java:44-55 builds codecPipeline
 * with chunkShape = inner chunk shape), so the level-2 codec sees a "shard" whose shape is
 * the level-1 inner chunk. */
static void nested_meta(const zh_array_meta* m, zh_array_meta* m2) {
  *m2 = *m;
  for (int d = 0; d < m->ndim; d++) {
    m2->chunk_shape[d] = m->chain.inner_chunk_shape[d];
    m2->shape[d] = m->chain.inner_chunk_shape[d];
    m2->chain.inner_chunk_shape[d] = m->chain.nested_chunk_shape[d];
  }
  m2->chain.index_endian = m->chain.nested_index_endian;
  m2->chain.index_has_crc32c = m->chain.nested_index_has_crc32c;
  m2->chain.index_location = m->chain.nested_index_location;
  m2->chain.nested = 0;
}

static int sharding_decode_internal(const zh_array_meta* m, const uint8_t* shard, int64_t nbytes,
                                    const char* path, const int64_t* offset, const int32_t* shape,
                                    uint8_t* out, int nthreads, char* err, size_t errlen);

/* FilesystemStore.get(keys, start, end) and get(keys, start) — M/store/FilesystemStore.java:
 * 59-102: one Files.newByteChannel open per call; a negative start counts from the end
 * (:63-68, :87-91: the suffix read of the index); Utils.allocateNative(end - start) (a fresh,
 * zeroed heap buffer, M/utils/Utils.java:17-20), position(start), one read of what the file
 * holds, close.  So a range past the end of the file comes back zero-padded to its length.
 *   FR_OK       *out = malloc'd buffer of `len` bytes (the file's bytes, then zeros)
 *   FR_MISSING  the file does not exist (NoSuchFileException → null)
 *   FR_NEGATIVE the resolved start is below 0 (position(< 0) throws IllegalArgumentException)
 * *fsize (may be NULL) = the file's size. */
enum { FR_OK = 0, FR_MISSING = 1, FR_NEGATIVE = 2 };
static int file_range_read(const char* path, int64_t start, int64_t len, uint8_t** out,
                           int64_t* fsize) {
  *out = NULL;
  int fd = open(path, O_RDONLY);
  if (fd < 0) return FR_MISSING;
  struct stat sb;
  if (fstat(fd, &sb) != 0) {
    close(fd);
    return FR_MISSING;
  }
  if (fsize) *fsize = (int64_t)sb.st_size;
  if (start < 0) start += (int64_t)sb.st_size;
  if (start < 0) {
    close(fd);
    return FR_NEGATIVE;
  }
  uint8_t* b = (uint8_t*)calloc(len > 0 ? len : 1, 1);
  int64_t got = 0;
  while (got < len) {
    ssize_t r = pread(fd, b + got, (size_t)(len - got), (off_t)(start + got));
    if (r <= 0) break; /* end of file: the rest stays zero */
    got += r;
  }
  close(fd);
  *out = b;
  return FR_OK;
}

static uint64_t load_u64(const uint8_t* p, int big) {
  uint64_t v = 0;
  if (big)
    for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
  else
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}

static void store_u64(uint8_t* p, uint64_t v, int big) {
  for (int i = 0; i < 8; i++) {
    int sh = big ? (56 - 8 * i) : (8 * i);
    p[i] = (uint8_t)(v >> sh);
  }
}

typedef struct {
  const zh_array_meta* m;
  const uint8_t* shard;       /* ByteBufferDataProvider (:301-331), or NULL with ... */
  const char* path;           /* ... StoreHandleDataProvider over a file (:333-357) */
  int64_t nbytes;
  const uint8_t* index;       /* index entries (CRC stripped) */
  const int64_t* inner_coords;
  const int64_t* offset;
  const int32_t* shape;
  nd_t* part;
  int status;
  char* err;
  size_t errlen;
} inner_job_t;

/* Body of the parallel inner-chunk loop, ShardingIndexedCodec.java:213-239 */
static int decode_one_inner(inner_job_t* J, int64_t k, char* err, size_t errlen) {
  const zh_array_meta* m = J->m;
  int n = m->ndim;
  const int32_t* inner = m->chain.inner_chunk_shape;
  const int64_t* c = J->inner_coords + k * n;
  int64_t lin = 0;
  for (int d = 0; d < n; d++) lin = lin * (m->chunk_shape[d] / inner[d]) + c[d];
  int big = m->chain.index_endian == ZH_ENDIAN_BIG;
  int64_t off = (int64_t)load_u64(J->index + 16 * lin, big);        /* :215-218 */
  int64_t len = (int64_t)load_u64(J->index + 16 * lin + 8, big);
  if (off == -1 || len == -1) return ZH_OK;                          /* :219-221 (Q1, Q2) */
  int64_t shard_shape[ZH_MAX_DIMS], sel_off[ZH_MAX_DIMS], sel_shape[ZH_MAX_DIMS];
  for (int d = 0; d < n; d++) {
    shard_shape[d] = m->chunk_shape[d];
    sel_off[d] = J->offset[d];
    sel_shape[d] = J->shape[d];
  }
  int32_t co[ZH_MAX_DIMS], oo[ZH_MAX_DIMS], ps[ZH_MAX_DIMS];
  if (zo_compute_projection(n, c, shard_shape, inner, sel_off, sel_shape, co, oo, ps) != ZH_OK) {
    set_err(err, errlen, "projection overflow");
    return ZH_EARITH;                                                /* :222-225 */
  }
  /* :226-230.  An entry the provider cannot serve: in memory (ByteBufferDataProvider.read,
   * :323-330) a slice beyond the buffer; from a store a negative position or length, or a
   * length beyond a Java buffer (the (int) allocation).  The reference throws
   * IllegalArgumentException there; the oracle (like the device) reports "Could not load
   * byte data" (DESIGN.md quirk Q14).  A store range past the end of the file is no error: it
   * reads zero-padded (file_range_read). */
  if (off < 0 || len < 0 ||
      (J->path ? (len > 2147483647LL || off > INT64_MAX - len) : off + len > J->nbytes)) {
    char cs[256];
    fmt_coords(cs, sizeof cs, c, n);
    set_err(err, errlen, "Could not load byte data for chunk %s", cs);
    return ZH_EDATA;
  }
  const uint8_t* bytes = J->shard ? J->shard + off : NULL;
  uint8_t* fbuf = NULL;
  if (J->path) { /* dataProvider.read(off, len) → storeHandle.read(off, off + len) :354-356 */
    if (file_range_read(J->path, off, len, &fbuf, NULL) != FR_OK) { /* null → :227-229 */
      char cs[256];
      fmt_coords(cs, sizeof cs, c, n);
      set_err(err, errlen, "Could not load byte data for chunk %s", cs);
      return ZH_EDATA;
    }
    bytes = fbuf;
  }
  uint8_t* buf = NULL;
  nd_t arr;
  int st;
  if (m->chain.nested) {  /* codecPipeline.decode → the level-2 ShardingIndexedCodec.decode
                           * (:97-103): decodeInternal over the whole sub-shard buffer */
    zh_array_meta m2;
    nested_meta(m, &m2);
    int64_t nel1 = 1, zoff[ZH_MAX_DIMS] = {0};
    for (int d = 0; d < n; d++) nel1 *= inner[d];
    buf = (uint8_t*)malloc(nel1 * m->dtype_size > 0 ? nel1 * m->dtype_size : 1);
    st = sharding_decode_internal(&m2, bytes, len, NULL, zoff, inner, buf, 1, err, errlen);
    if (st != ZH_OK) {
      free(buf);
      free(fbuf);
      return st;
    }
    arr.data = buf;
    arr.ndim = n;
    arr.dsize = m->dtype_size;
    for (int d = 0; d < n; d++) arr.shape[d] = inner[d];
    nd_c_order(&arr);
  } else {
    st = inner_decode(m, inner, bytes, len, &buf, &arr, err, errlen); /* :231 */
    if (st != ZH_OK) {
      free(fbuf);
      return st;
    }
  }
  free(fbuf);
  int64_t so[ZH_MAX_DIMS], dof[ZH_MAX_DIMS], sh[ZH_MAX_DIMS];
  for (int d = 0; d < n; d++) {
    so[d] = co[d];
    dof[d] = oo[d];
    sh[d] = ps[d];
  }
  copy_region(&arr, so, J->part, dof, sh);                           /* :232-236 */
  free(buf);
  return ZH_OK;
}

/* ShardingIndexedCodec.decodeInternal — ShardingIndexedCodec.java:183-243, with the shard
 * bytes in memory (ByteBufferDataProvider :301-331). */
static int sharding_decode_internal(const zh_array_meta* m, const uint8_t* shard, int64_t nbytes,
                                    const char* path, const int64_t* offset, const int32_t* shape,
                                    uint8_t* out, int nthreads, char* err, size_t errlen) {
  int n = m->ndim, ds = m->dtype_size;
  nd_t part;                                                          /* :189 zero-filled */
  part.data = out;
  part.ndim = n;
  part.dsize = ds;
  int64_t nel = 1;
  for (int d = 0; d < n; d++) {
    part.shape[d] = shape[d];
    nel *= shape[d];
  }
  nd_c_order(&part);
  memset(out, 0, nel * ds);
  int64_t isz = shard_index_size(m);                                  /* :190 */
  uint8_t* fidx = NULL;
  if (path) { /* StoreHandleDataProvider.readPrefix / readSuffix :340-352 */
    int rc = file_range_read(path, m->chain.index_location == ZH_INDEX_START ? 0 : -isz, isz,
                             &fidx, &nbytes);
    if (rc == FR_MISSING) { /* a null index buffer → fill_value (:199-204) */
      fill_elems(out, nel, ds, m->fill_value);
      return ZH_OK;
    }
    if (rc == FR_NEGATIVE) { /* a suffix longer than the file: position(< 0) throws
                              * IllegalArgumentException; reported as the device does (Q14) */
      set_err(err, errlen, "Shard of %lld bytes is smaller than its index (%lld bytes).",
              (long long)nbytes, (long long)isz);
      return ZH_EDATA;
    }
    /* a prefix read is zero-padded like any range: a file shorter than the index gives an
     * index of isz bytes (whose crc32c, if any, then fails) */
  } else if (nbytes < isz) {
    set_err(err, errlen, "Shard of %lld bytes is smaller than its index (%lld bytes).",
            (long long)nbytes, (long long)isz);
    free(fidx);
    return ZH_EDATA;
  }
  const uint8_t* ib = fidx ? fidx
                           : m->chain.index_location == ZH_INDEX_START ? shard  /* :192-193 */
                                                                       : shard + nbytes - isz; /* :194-195 */
  int64_t ilen = isz;
  if (m->chain.index_has_crc32c) {                /* Crc32cCodec.decode, Crc32cCodec.java:24-48 */
    ilen -= 4;
    int32_t computed = (int32_t)zo_crc32c(0, ib, ilen);
    int32_t stored = (int32_t)((uint32_t)ib[ilen] | ((uint32_t)ib[ilen + 1] << 8) |
                               ((uint32_t)ib[ilen + 2] << 16) | ((uint32_t)ib[ilen + 3] << 24));
    if (computed != stored) {
      set_err(err, errlen,
              "The checksum of the sharding index is invalid. Stored: %d Computed: %d", stored,
              computed);
      free(fidx);
      return ZH_EDATA;
    }
  }
  int64_t shard_shape[ZH_MAX_DIMS], sel_shape[ZH_MAX_DIMS];
  for (int d = 0; d < n; d++) {
    shard_shape[d] = m->chunk_shape[d];
    sel_shape[d] = shape[d];
  }
  int64_t ninner = zo_compute_chunk_coords(n, shard_shape, m->chain.inner_chunk_shape, offset,
                                           sel_shape, NULL, 0);       /* :206-208 */
  if (ninner < 0) {
    set_err(err, errlen, "Number of chunks exceeds Integer.MAX_VALUE");
    free(fidx);
    return ZH_EARITH;
  }
  int64_t* coords = (int64_t*)malloc(sizeof(int64_t) * n * (ninner > 0 ? ninner : 1));
  zo_compute_chunk_coords(n, shard_shape, m->chain.inner_chunk_shape, offset, sel_shape, coords,
                          ninner);
  inner_job_t J = {m, shard, path, nbytes, ib, coords, offset, shape, &part, ZH_OK, err, errlen};
  int status = ZH_OK;
  /* :210-212 parallel stream over inner chunks; each copy targets a disjoint region. */
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
#endif
  for (int64_t k = 0; k < ninner; k++) {
    if (status != ZH_OK) continue;
    char lerr[512];
    int st = decode_one_inner(&J, k, lerr, sizeof lerr);
    if (st != ZH_OK) {
#ifdef _OPENMP
#pragma omp critical
#endif
      {
        if (status == ZH_OK) {
          status = st;
          set_err(err, errlen, "%s", lerr);
        }
      }
    }
  }
  (void)nthreads;
  free(coords);
  free(fidx);
  return status;
}

int zo_sharding_decode_partial(const zh_array_meta* m, const void* shard, int64_t nbytes,
                               const int64_t* offset, const int32_t* shape, void* out,
                               int nthreads, char* err, size_t errlen) {
  return sharding_decode_internal(m, (const uint8_t*)shard, nbytes, NULL, offset, shape,
                                  (uint8_t*)out, nthreads, err, errlen);
}

/* core.Array.read — M/core/Array.java:378-441 */
static int array_read_impl(const zh_array_meta* m, const zh_chunk_src* chunks,
                           const char* const* paths, int64_t nchunks, const int64_t* offset,
                           const int64_t* shape, void* out_v, int nthreads, char* err,
                           size_t errlen) {
  int n = m->ndim, ds = m->dtype_size;
  uint8_t* out = (uint8_t*)out_v;
  for (int d = 0; d < n; d++)                                          /* :386-390 */
    if (offset[d] < 0 || offset[d] + shape[d] > m->shape[d]) {
      set_err(err, errlen, "Requested data is outside of the array's domain.");
      return ZH_EDATA;
    }
  int64_t ncoords = zo_compute_chunk_coords(n, m->shape, m->chunk_shape, offset, shape, NULL, 0);
  if (ncoords < 0) {
    set_err(err, errlen, "Number of chunks exceeds Integer.MAX_VALUE");
    return ZH_EARITH;
  }
  if (ncoords != nchunks) {
    set_err(err, errlen, "expected %lld chunk sources, got %lld", (long long)ncoords,
            (long long)nchunks);
    return ZH_EINVAL;
  }
  int64_t* coords = (int64_t*)malloc(sizeof(int64_t) * n * (ncoords > 0 ? ncoords : 1));
  zo_compute_chunk_coords(n, m->shape, m->chunk_shape, offset, shape, coords, ncoords);
  nd_t outa;
  outa.data = out;
  outa.ndim = n;
  outa.dsize = ds;
  int64_t nel = 1;
  for (int d = 0; d < n; d++) {
    outa.shape[d] = shape[d];
    nel *= shape[d];
  }
  nd_c_order(&outa);
  /* :392-395 isSingleFullChunk → readChunk: same values as the general path below (Q4),
   * which the oracle therefore uses for every region. */
  fill_elems(out, nel, ds, m->fill_value);                             /* :397-402 */
  int status = ZH_OK;
  for (int64_t i = 0; i < ncoords && status == ZH_OK; i++) {          /* :403-439 */
    const int64_t* c = coords + i * n;
    int32_t co[ZH_MAX_DIMS], oo[ZH_MAX_DIMS], ps[ZH_MAX_DIMS];
    if (zo_compute_projection(n, c, m->shape, m->chunk_shape, offset, shape, co, oo, ps) !=
        ZH_OK) {
      set_err(err, errlen, "projection overflow");
      status = ZH_EARITH;
      break;
    }
    zh_chunk_src fsrc = {NULL, 0};
    uint8_t* whole = NULL; /* StoreHandle.read() = FilesystemStore.get(keys) (:49-59) */
    const char* spath = NULL;
    if (paths) {
      int full = 1;
      for (int d = 0; d < n; d++) full &= ps[d] == m->chunk_shape[d];
      if (paths[i] && (!m->chain.sharded || full)) { /* decodePartial :246-252 / readChunk */
        int64_t fsz = 0;
        struct stat sb;
        if (stat(paths[i], &sb) == 0) {
          fsz = (int64_t)sb.st_size;
          (void)file_range_read(paths[i], 0, fsz, &whole, NULL);
        }
        fsrc.data = whole;
        fsrc.nbytes = fsz;
      } else if (paths[i]) {
        spath = paths[i]; /* StoreHandleDataProvider (:253) */
        fsrc.data = (const void*)1; /* exists (:419) */
      }
    }
    const zh_chunk_src* s = paths ? &fsrc : &chunks[i];
    int64_t pdoff[ZH_MAX_DIMS], psh[ZH_MAX_DIMS], zero[ZH_MAX_DIMS] = {0}, so[ZH_MAX_DIMS];
    int64_t pnel = 1;
    for (int d = 0; d < n; d++) {
      pdoff[d] = oo[d];
      psh[d] = ps[d];
      so[d] = co[d];
      pnel *= ps[d];
    }
    if (m->chain.sharded) {                                           /* :418 partial decode */
      if (!s->data) continue;                                         /* :419-421 */
      uint8_t* pbuf = (uint8_t*)malloc(pnel * ds > 0 ? pnel * ds : 1);
      int64_t coff[ZH_MAX_DIMS];
      for (int d = 0; d < n; d++) coff[d] = co[d];
      status = sharding_decode_internal(m, spath ? NULL : (const uint8_t*)s->data, s->nbytes,
                                        spath, coff, ps, pbuf, nthreads, err,
                                        errlen); /* :422-423 */
      if (status == ZH_OK) {
        nd_t part;
        part.data = pbuf;
        part.ndim = n;
        part.dsize = ds;
        for (int d = 0; d < n; d++) part.shape[d] = ps[d];
        nd_c_order(&part);
        copy_region(&part, zero, &outa, pdoff, psh);                  /* :424-426 */
      }
      free(pbuf);
    } else {
      if (!s->data) continue;                                         /* :429 null → keep fill */
      uint8_t* buf = NULL;
      nd_t arr;
      status = inner_decode(m, m->chunk_shape, (const uint8_t*)s->data, s->nbytes, &buf, &arr,
                            err, errlen);                             /* :430 */
      if (status == ZH_OK) copy_region(&arr, so, &outa, pdoff, psh);  /* :430-432 */
      free(buf);
    }
    free(whole);
  }
  free(coords);
  return status;
}

int zo_array_read(const zh_array_meta* m, const zh_chunk_src* chunks, int64_t nchunks,
                  const int64_t* offset, const int64_t* shape, void* out_v, int nthreads,
                  char* err, size_t errlen) {
  return array_read_impl(m, chunks, NULL, nchunks, offset, shape, out_v, nthreads, err, errlen);
}

/* core.Array.read against a FilesystemStore: one file path per chunk key (NULL = the key
 * does not exist).  Sub-shard regions take StoreHandleDataProvider's range reads (suffix
 * read of the index, then one open + read + close per referenced inner chunk,
 * ShardingIndexedCodec.java:253,333-357); whole chunks and unsharded chunks are read whole
 * (FilesystemStore.get(keys), M/store/FilesystemStore.java:49-59). */
int zo_array_read_store(const zh_array_meta* m, const char* const* paths, int64_t nchunks,
                        const int64_t* offset, const int64_t* shape, void* out_v, int nthreads,
                        char* err, size_t errlen) {
  return array_read_impl(m, NULL, paths, nchunks, offset, shape, out_v, nthreads, err, errlen);
}

/* ---------------------------------------------------------------------------------
 * Write path
 * ------------------------------------------------------------------------------- */
/* One element against the fill value as ValueAccessor.isEqual compares them
 * (M/utils/MultiArrayUtils.java:104-280): Java's == on float / double (NaN equals nothing,
 * +0.0 == -0.0), the integer value otherwise (= the bits). */
static int elem_equal(const uint8_t* e, const uint8_t* fill, int ds, int is_float) {
  if (is_float && ds == 4) {
    float x, y;
    memcpy(&x, e, 4);
    memcpy(&y, fill, 4);
    return x == y;
  }
  if (is_float && ds == 8) {
    double x, y;
    memcpy(&x, e, 8);
    memcpy(&y, fill, 8);
    return x == y;
  }
  return memcmp(e, fill, ds) == 0;
}

/* MultiArrayUtils.allValuesEqual — M/utils/MultiArrayUtils.java:69-80 */
static int all_equal(const nd_t* a, const int64_t* off, const int64_t* shape, const uint8_t* fill,
                     int is_float) {
  int n = a->ndim, ds = a->dsize;
  int64_t total = prod64(shape, n);
  int64_t idx[ZH_MAX_DIMS] = {0};
  for (int64_t t = 0; t < total; t++) {
    int64_t o = 0;
    for (int d = 0; d < n; d++) o += (off[d] + idx[d]) * a->stride[d];
    if (!elem_equal(a->data + o * ds, fill, ds, is_float)) return 0;
    for (int d = n - 1; d >= 0; d--) {
      if (++idx[d] < shape[d]) break;
      idx[d] = 0;
    }
  }
  return 1;
}

/* Inner pipeline encode (CodecPipeline.encode :140-153): TransposeCodec.encode
 * (TransposeCodec.java:47-57, permute(order)) then BytesCodec.encode
 * (M/core/codec/core/BytesCodec.java:38-78) in the configured byte order.  Writes
 * prod(shape)*dsize bytes to dst. */
static void inner_encode(const zh_array_meta* m, const nd_t* src, const int64_t* off,
                         const int32_t* chunk_shape, uint8_t* dst) {
  int n = m->ndim, ds = m->dtype_size;
  int32_t order[ZH_MAX_DIMS];
  for (int d = 0; d < n; d++) order[d] = m->chain.has_transpose ? m->chain.transpose_order[d] : d;
  int64_t eshape[ZH_MAX_DIMS];
  for (int j = 0; j < n; j++) eshape[j] = chunk_shape[order[j]];
  int64_t total = prod64(eshape, n);
  int64_t idx[ZH_MAX_DIMS] = {0};
  int sw = elem_swaps(m, m->chain.endian);
  for (int64_t t = 0; t < total; t++) {
    /* encoded coord idx[j] = decoded coord x[order[j]] */
    int64_t o = 0;
    for (int j = 0; j < n; j++) o += (off[order[j]] + idx[j]) * src->stride[order[j]];
    uint8_t* e = dst + t * ds;
    memcpy(e, src->data + o * ds, ds);
    if (m->dtype_is_bool) e[0] = e[0] != 0;
    if (sw) swap_elem(e, ds);
    for (int d = n - 1; d >= 0; d--) {
      if (++idx[d] < eshape[d]) break;
      idx[d] = 0;
    }
  }
  if (m->chain.inner_crc32c) { /* Crc32cCodec.encode (Crc32cCodec.java:50-60) */
    uint32_t c = zo_crc32c(0, dst, (size_t)(total * ds));
    for (int i = 0; i < 4; i++) dst[total * ds + i] = (uint8_t)(c >> (8 * i));
  }
}

/* ShardingIndexedCodec.encode — ShardingIndexedCodec.java:105-168, C-order layout (Q7) */
static int sharding_encode(const zh_array_meta* m, const nd_t* chunk, uint8_t** out,
                           int64_t* out_n) {
  int n = m->ndim, ds = m->dtype_size;
  const int32_t* inner = m->chain.inner_chunk_shape;
  int64_t cps[ZH_MAX_DIMS] = {0}, shard_shape[ZH_MAX_DIMS] = {0}, zero[ZH_MAX_DIMS] = {0};
  int64_t ninner = 1, inner_nel = 1;
  for (int d = 0; d < n; d++) {
    cps[d] = m->chunk_shape[d] / inner[d];
    shard_shape[d] = m->chunk_shape[d];
    ninner *= cps[d];
    inner_nel *= inner[d];
  }
  int64_t isz = shard_index_size(m);
  int64_t* coords = (int64_t*)malloc(sizeof(int64_t) * n * ninner);
  zo_compute_chunk_coords(n, shard_shape, inner, zero, shard_shape, coords, ninner);
  int64_t* offs = (int64_t*)malloc(sizeof(int64_t) * ninner);
  int64_t* lens = (int64_t*)malloc(sizeof(int64_t) * ninner);
  uint8_t** subs = (uint8_t**)calloc((size_t)ninner, sizeof(uint8_t*)); /* nested payloads */
  int64_t payload = 0;
  for (int64_t k = 0; k < ninner; k++) {                              /* :116-152 */
    int64_t o[ZH_MAX_DIMS], sh[ZH_MAX_DIMS];
    for (int d = 0; d < n; d++) {
      o[d] = coords[k * n + d] * inner[d];
      sh[d] = inner[d];
    }
    if (all_equal(chunk, o, sh, m->fill_value, m->dtype_is_float)) { /* :129-133 */
      offs[k] = -1;
      lens[k] = 0;
    } else {
      offs[k] = payload;                                              /* :137-143 */
      lens[k] = inner_nel * ds + (m->chain.inner_crc32c ? 4 : 0);
      if (m->chain.nested) {  /* codecPipeline.encode(chunkArray) = level-2 sharding encode */
        zh_array_meta m2;
        nested_meta(m, &m2);
        nd_t view = *chunk;
        int64_t eo = 0;
        for (int d = 0; d < n; d++) {
          eo += o[d] * chunk->stride[d];
          view.shape[d] = inner[d];
        }
        view.data = chunk->data + eo * ds;
        sharding_encode(&m2, &view, &subs[k], &lens[k]);
      }
      payload += lens[k];
    }
  }
  int64_t total = payload + isz;                                      /* :153-156 */
  uint8_t* buf = (uint8_t*)malloc(total);
  int start = m->chain.index_location == ZH_INDEX_START;
  uint8_t* pay = buf + (start ? isz : 0);
  uint8_t* idx = buf + (start ? 0 : payload);
  int big = m->chain.index_endian == ZH_ENDIAN_BIG;
  for (int64_t k = 0; k < ninner; k++) {
    int64_t o[ZH_MAX_DIMS];
    for (int d = 0; d < n; d++) o[d] = coords[k * n + d] * inner[d];
    if (offs[k] < 0) {
      store_u64(idx + 16 * k, (uint64_t)-1, big);
      store_u64(idx + 16 * k + 8, (uint64_t)-1, big);
    } else {
      if (subs[k]) {
        memcpy(pay + offs[k], subs[k], (size_t)lens[k]);
        free(subs[k]);
      } else {
        inner_encode(m, chunk, o, inner, pay + offs[k]);
      }
      store_u64(idx + 16 * k, (uint64_t)(offs[k] + (start ? isz : 0)), big); /* :140-143 */
      store_u64(idx + 16 * k + 8, (uint64_t)lens[k], big);
    }
  }
  if (m->chain.index_has_crc32c) {                                    /* Crc32cCodec.encode :50-60 */
    uint32_t c = zo_crc32c(0, idx, 16 * ninner);
    for (int i = 0; i < 4; i++) idx[16 * ninner + i] = (uint8_t)(c >> (8 * i));
  }
  free(coords);
  free(offs);
  free(lens);
  free(subs);
  *out = buf;
  *out_n = total;
  return ZH_OK;
}

/* core.Array.write over whole chunks (M/core/Array.java:83-133) + writeChunk (:144-156). */
int zo_array_write(const zh_array_meta* m, const void* src_v, const int64_t* offset,
                   const int64_t* shape, void** out_bufs, int64_t* out_sizes, int64_t nchunks,
                   char* err, size_t errlen) {
  int n = m->ndim, ds = m->dtype_size;
  for (int d = 0; d < n; d++) {
    if (offset[d] < 0 || offset[d] + shape[d] > m->shape[d]) {
      set_err(err, errlen, "Requested data is outside of the array's domain.");
      return ZH_EDATA;
    }
    int64_t e = offset[d] + shape[d];
    if (offset[d] % m->chunk_shape[d] != 0 || (e % m->chunk_shape[d] != 0 && e != m->shape[d])) {
      set_err(err, errlen, "region does not cover whole chunks");
      return ZH_EUNSUPPORTED;
    }
  }
  int64_t ncoords = zo_compute_chunk_coords(n, m->shape, m->chunk_shape, offset, shape, NULL, 0);
  if (ncoords != nchunks) {
    set_err(err, errlen, "expected %lld chunk destinations", (long long)ncoords);
    return ZH_EINVAL;
  }
  int64_t* coords = (int64_t*)malloc(sizeof(int64_t) * n * ncoords);
  zo_compute_chunk_coords(n, m->shape, m->chunk_shape, offset, shape, coords, ncoords);
  nd_t src;
  src.data = (uint8_t*)src_v;
  src.ndim = n;
  src.dsize = ds;
  for (int d = 0; d < n; d++) src.shape[d] = shape[d];
  nd_c_order(&src);
  int64_t cnel = 1;
  for (int d = 0; d < n; d++) cnel *= m->chunk_shape[d];
  uint8_t* cbuf = (uint8_t*)malloc(cnel * ds);
  for (int64_t i = 0; i < ncoords; i++) {
    int32_t co[ZH_MAX_DIMS], oo[ZH_MAX_DIMS], ps[ZH_MAX_DIMS];
    zo_compute_projection(n, coords + i * n, m->shape, m->chunk_shape, offset, shape, co, oo, ps);
    /* chunk array = fill (allocateFillValueChunk, ArrayMetadata.java:182-186; a fresh
     * store is assumed for the boundary read-modify-write) + copied region */
    fill_elems(cbuf, cnel, ds, m->fill_value);
    nd_t ch;
    ch.data = cbuf;
    ch.ndim = n;
    ch.dsize = ds;
    for (int d = 0; d < n; d++) ch.shape[d] = m->chunk_shape[d];
    nd_c_order(&ch);
    int64_t so[ZH_MAX_DIMS], dof[ZH_MAX_DIMS], sh[ZH_MAX_DIMS], zero[ZH_MAX_DIMS] = {0};
    for (int d = 0; d < n; d++) {
      so[d] = oo[d];
      dof[d] = co[d];
      sh[d] = ps[d];
    }
    copy_region(&src, so, &ch, dof, sh);
    int64_t full[ZH_MAX_DIMS];
    for (int d = 0; d < n; d++) full[d] = m->chunk_shape[d];
    if (all_equal(&ch, zero, full, m->fill_value, m->dtype_is_float)) { /* writeChunk :150-151 */
      out_bufs[i] = NULL;
      out_sizes[i] = 0;
      continue;
    }
    if (m->chain.sharded) {
      uint8_t* b;
      int64_t nb;
      sharding_encode(m, &ch, &b, &nb);
      out_bufs[i] = b;
      out_sizes[i] = nb;
    } else {
      const int64_t extra = m->chain.inner_crc32c ? 4 : 0;
      uint8_t* b = (uint8_t*)malloc(cnel * ds + extra);
      inner_encode(m, &ch, zero, m->chunk_shape, b);
      out_bufs[i] = b;
      out_sizes[i] = cnel * ds + extra;
    }
  }
  free(cbuf);
  free(coords);
  return ZH_OK;
}

void zo_free(void* p) { free(p); }
