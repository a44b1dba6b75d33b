/*
 * zarrhip.h — C-ABI of the MI355X-native Zarr v3 chunk codec path.
 *
 * This is the drop-in boundary that zarr-java's JNI shim binds.
 * Every entry point is `extern "C"`, takes plain pointers and sizes, and returns an
 * `int` status (ZH_OK = 0).  No torch / HIP types appear in any signature: streams
 * and device buffers travel as `void*`.
 *
 * Reference interfaces replaced (zarr-java snapshot 2026-08-07,
 * M/ = src/main/java/dev/zarr/zarrjava/):
 *   zh_array_read               core.Array.read(long[],long[],boolean)       M/core/Array.java:378-441
 *   zh_plan_* (prepared read)   same, split into plan (host) + execute (device)
 *   zh_sharding_decode          ShardingIndexedCodec.decode(ByteBuffer)      M/v3/codec/core/ShardingIndexedCodec.java:98-103
 *   zh_sharding_decode_partial  ShardingIndexedCodec.decodePartial(...)      M/v3/codec/core/ShardingIndexedCodec.java:245-255
 *   zh_shard_ranges             StoreHandleDataProvider reads of decodeInternal ShardingIndexedCodec.java:190-230, 333-357
 *   zh_array_read_pieces        core.Array.read with sub-shard parts         M/core/Array.java:378-441 + the above
 *   zh_sharding_decode_pieces   ShardingIndexedCodec.decodePartial(StoreHandle, ...) ShardingIndexedCodec.java:245-255
 *   zh_shard_index_check        Crc32cCodec.decode of a shard index (host)    M/v3/codec/core/Crc32cCodec.java:24-48
 *   zh_array_read_files(_multi) core.Array.read over a FilesystemStore        M/core/Array.java:378-441 +
 *                               (exists / get(keys,start,end) per chunk)     M/store/FilesystemStore.java:43-102
 *   zh_array_write(_files)      core.Array.write + writeChunk + ShardingIndexedCodec.encode
 *                                                                            M/core/Array.java:83-156, ShardingIndexedCodec.java:105-168
 *   zh_shard_index_size         ShardingIndexedCodec.getShardIndexSize       ShardingIndexedCodec.java:176-181
 *   zh_crc32c                   utils.CRC32C.update/getValue                 M/utils/CRC32C.java:119-125,137-139
 *   zh_compute_chunk_coords     IndexingUtils.computeChunkCoords             M/utils/IndexingUtils.java:16-51
 *   zh_compute_projection       IndexingUtils.computeProjection (5-arg)      M/utils/IndexingUtils.java:65-117
 *   zh_is_permutation           Utils.isPermutation                          M/utils/Utils.java:91-100
 *   zh_inverse_permutation      Utils.inversePermutation                     M/utils/Utils.java:102-109
 *
 * Status → Java exception mapping used by the JNI shim:
 *   ZH_EINVAL  → IllegalArgumentException      (rank mismatches, Array.java:380-385)
 *   ZH_EDATA   → dev.zarr.zarrjava.ZarrException (message text reproduces the reference's)
 *   ZH_EUNSUPPORTED → caller falls back to the Java codec (chain not device-supported)
 *   ZH_EARITH  → ArithmeticException            (IndexingUtils overflow checks)
 *   ZH_EIO     → dev.zarr.zarrjava.store.StoreException (a RuntimeException; zh_array_read_files)
 *   ZH_EHIP / ZH_ENOMEM → RuntimeException
 */
#ifndef ZARRHIP_H
#define ZARRHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZH_MAX_DIMS 8

enum zh_status {
  ZH_OK = 0,
  ZH_EINVAL = 1,
  ZH_EDATA = 2,
  ZH_EUNSUPPORTED = 3,
  ZH_EHIP = 4,
  ZH_ENOMEM = 5,
  ZH_EARITH = 6,
  ZH_EIO = 7 /* a store file could not be read (StoreException.readFailed) */
};

enum zh_endian { ZH_ENDIAN_LITTLE = 0, ZH_ENDIAN_BIG = 1 };
enum zh_index_location { ZH_INDEX_END = 0, ZH_INDEX_START = 1 };

/* call flags */
#define ZH_SRC_DEVICE 0x1u /* chunk/shard byte sources are device pointers            */
#define ZH_OUT_DEVICE 0x2u /* output buffer is a device pointer                      */

/*
 * Codec chain the device path executes.  Mirrors the JSON `codecs` list of a v3 array
 * (v3/ArrayMetadata.java) restricted to the device-supported chains:
 *   sharded = 0 :  [transpose?, bytes]                          (BASELINE config 2)
 *   sharded = 1 :  [sharding_indexed{ codecs=[transpose?, bytes, crc32c?],
 *                                     index_codecs=[bytes, crc32c?],
 *                                     index_location }]          (configs 3, 4, 5)
 *   plus one nested sharding_indexed level as the sole inner codec (nested* fields) and a
 *   trailing chunk crc32c (inner_crc32c).  Anything else (blosc/gzip/zstd inside the chain,
 *   array-level codecs next to sharding) is rejected with ZH_EUNSUPPORTED so the caller
 *   keeps the Java path (host byte-to-byte stages: INTEGRATION.md §3).
 */
typedef struct zh_codec_chain {
  int32_t sharded;                          /* 1: outer codec is sharding_indexed              */
  int32_t inner_chunk_shape[ZH_MAX_DIMS];   /* sharding configuration.chunk_shape              */
  int32_t has_transpose;                    /* transpose codec present in the (inner) chain    */
  int32_t transpose_order[ZH_MAX_DIMS];     /* TransposeCodec.Configuration.order              */
  int32_t endian;                           /* bytes codec endian (ignored for 1-byte types)   */
  int32_t index_endian;                     /* index_codecs bytes endian                       */
  int32_t index_has_crc32c;                 /* index_codecs contains crc32c                    */
  int32_t index_location;                   /* ZH_INDEX_END (default) / ZH_INDEX_START          */
  /* Nested sharding (ZarrPythonTests.java:177-179, ZarrV3Test.java:197-200): the sharding
   * codec's inner codecs are [sharding_indexed{nested_chunk_shape, codecs [transpose?,
   * bytes], index_codecs [bytes(nested_index_endian), crc32c?], nested_index_location}].
   * Each inner chunk is then itself a shard; transpose/endian above apply to its leaves. */
  int32_t nested;
  int32_t nested_chunk_shape[ZH_MAX_DIMS];
  int32_t nested_index_endian;
  int32_t nested_index_has_crc32c;
  int32_t nested_index_location;
  /* The chunk codecs end with crc32c ([transpose?, bytes, crc32c]; ZarrPythonTests "crc32c",
   * ZarrPythonTests.java:180-182): each stored (inner/leaf) chunk is its payload followed by
   * the payload's CRC-32C, little-endian (Crc32cCodec.java:24-60), verified on the device. */
  int32_t inner_crc32c;
} zh_codec_chain;

/* CoreArrayMetadata (M/core/ArrayMetadata.java:154-187) + the codec chain. */
typedef struct zh_array_meta {
  int32_t ndim;
  int32_t dtype_size;                 /* DataType.getByteCount(): 1, 2, 4 or 8             */
  int32_t dtype_is_bool;              /* bool decodes as b != 0 (core BytesCodec.java:24-33) */
  int32_t dtype_is_float;             /* float32 / float64: the write path's all-fill test
                                       * compares as Java's == (MultiArrayUtils.allValuesEqual,
                                       * MultiArrayUtils.java:69-80), so a ±0 fill matches
                                       * both zeros; other types compare bits */
  int64_t shape[ZH_MAX_DIMS];         /* array shape                                       */
  int32_t chunk_shape[ZH_MAX_DIMS];   /* regular chunk grid shape (= shard shape)          */
  uint8_t fill_value[8];              /* parsed fill value, element bytes little-endian     */
  zh_codec_chain chain;
} zh_array_meta;

/* One stored chunk (or shard) object.  data == NULL means the key does not exist in the
 * store (StoreHandle.exists() == false, M/core/Array.java:419-421). */
typedef struct zh_chunk_src {
  const void* data;
  int64_t nbytes;
} zh_chunk_src;

/* Destination of one encoded chunk object for zh_array_write. */
typedef struct zh_chunk_dst {
  void* data;          /* device buffer for the encoded bytes                         */
  int64_t capacity;    /* bytes available                                            */
  int64_t nbytes;      /* out: encoded size; 0 = chunk is all fill → delete key      */
} zh_chunk_dst;

typedef struct zh_ctx zh_ctx;
typedef struct zh_plan zh_plan;

/* ---- context -------------------------------------------------------------------- */
int zh_ctx_create(int device, zh_ctx** out);
void zh_ctx_destroy(zh_ctx* ctx);
int zh_ctx_device(const zh_ctx* ctx);
/* The context's default stream (a hipStream_t).  Calls with stream == NULL use it. */
void* zh_ctx_stream(zh_ctx* ctx);
/* Device blocks of finished plans are kept by the context (at most 8 GiB, blocks up to
 * 4 GiB) and reused by later plans: fresh device memory pays for its first touch.  Returns
 * them to the runtime; returns the bytes released.  No reference counterpart. */
int64_t zh_ctx_release_cache(zh_ctx* ctx);
const char* zh_version(void);

/* ---- host-side metadata helpers (no device needed) ------------------------------- */
/* Validates the chain against the reference rules (CodecPipeline ctor, sharding
 * divisibility ArrayMetadata.java:285-306, TransposeCodec.decode :35-41,
 * v3 BytesCodec.getByteOrder :43-48).  Returns ZH_EUNSUPPORTED for valid-but-not-
 * device-supported chains. */
int zh_validate_meta(const zh_array_meta* meta, char* err, size_t errlen);
/* 16 * prod(chunks per shard) (+4 with crc32c).  -1 for unsharded metas. */
int64_t zh_shard_index_size(const zh_array_meta* meta);
/* CRC32C.update over n bytes starting from a previous getValue() (0 for a fresh CRC32C). */
uint32_t zh_crc32c(uint32_t crc, const void* data, size_t n);
/* IndexingUtils.computeChunkCoords: writes up to max_coords rows of ndim int64 into
 * coords_out (may be NULL) in C order; returns the number of chunks, or -1 (ZH_EARITH
 * condition: more than Integer.MAX_VALUE chunks). */
int64_t zh_compute_chunk_coords(int ndim, const int64_t* array_shape, const int32_t* chunk_shape,
                                const int64_t* sel_offset, const int64_t* sel_shape,
                                int64_t* coords_out, int64_t max_coords);
/* IndexingUtils.computeProjection (5-arg).  Returns ZH_OK or ZH_EARITH. */
int zh_compute_projection(int ndim, const int64_t* chunk_coords, const int64_t* array_shape,
                          const int32_t* chunk_shape, const int64_t* sel_offset,
                          const int64_t* sel_shape, int32_t* chunk_offset_out,
                          int32_t* out_offset_out, int32_t* shape_out);
int zh_is_permutation(int n, const int32_t* order);
int zh_inverse_permutation(int n, const int32_t* order, int32_t* inverse_out);

/* ---- decode (the hot path) ------------------------------------------------------ */
/*
 * Prepared region read: the host half of core.Array.read (domain check, chunk
 * enumeration, projection, per-shard inner-chunk boxes) runs once in zh_plan_create;
 * zh_plan_execute only enqueues device work on `stream` (no allocation, no sync:
 * hipGraph-capturable); zh_plan_wait synchronises and reports deferred device errors
 * (CRC mismatch, corrupt index) with the reference's messages.
 *   chunks[i] belongs to the i-th chunk coordinate of
 *   computeChunkCoords(meta->shape, meta->chunk_shape, offset, shape) (C order).
 *   out = C-order buffer of prod(shape) elements.
 */
int zh_plan_create(zh_ctx* ctx, const zh_array_meta* meta, const zh_chunk_src* chunks,
                   int64_t nchunks, const int64_t* offset, const int64_t* shape, uint32_t flags,
                   zh_plan** out, char* err, size_t errlen);
int zh_plan_execute(zh_plan* plan, void* out, void* stream);
int zh_plan_wait(zh_plan* plan, char* err, size_t errlen);
/* Where the data error (ZH_EDATA) that the last read call on this thread reported sits in the
 * reference's sequential order: the failing chunk's grid coordinates (ndim
 * values into coords[0..cap)) and *key, its place inside that chunk (larger = earlier: the
 * index crc32c is ~0, else the failing inner chunk's C-order rank, complemented).  Returns
 * ndim, or 0 when that call placed no data error; the position is cleared once reported.
 * Multi-rank callers order the ranks' errors
 * by (coords, -key) so every rank reports the one a sequential read would have
 * (zarrhip.parallel.pick_error; the reference throws from its parallel chunk loop,
 * M/core/Array.java:403-407, 436-438). */
int zh_last_data_error(int64_t* coords, int cap, uint64_t* key);
void zh_plan_destroy(zh_plan* plan);
/* Plan statistics: bytes of encoded input read, output bytes written, number of
 * inner-chunk work items, shards touched. */
int zh_plan_stats(const zh_plan* plan, int64_t* in_bytes, int64_t* out_bytes,
                  int64_t* items, int64_t* nshards);
/* Diagnostic: the fast-path selection of the last decode scatter launch in this process
 * (encode = 0: aligned windows * 10^9 + fast_mode * 1000000 + kernel variant * 1000 +
 *  row group * 4 + (pieces ? 1 : 0))
 * or of the last write's encode view (encode = 1: fast_mode * 1000000 + chunk group * 1000 +
 * kernel form), or -1.  Tests use it to check that a switch reached the kernel it names. */
int64_t zh_debug_last_fast_path(int encode);
/* Per-kernel timing (HIP events around the scatter kernel on the launch stream).
 * enable=1 starts recording; zh_plan_kernel_time synchronises and returns the summed
 * scatter-kernel milliseconds and launch count since the last call. */
/* Bytes the plan copies host→device per execute (0 for device sources).  With host sources a
 * sub-shard part stages only its index + referenced inner chunks (StoreHandleDataProvider
 * semantics, ShardingIndexedCodec.java:333-357). */
int64_t zh_plan_staged_bytes(const zh_plan* plan);
int zh_plan_set_timing(zh_plan* plan, int enable);
/* enable=1: zh_plan_execute replays the plan as one hipGraph (captured on the first execute
 * for a given (out, stream); device sources and device output only, timing off).  For small
 * repeated reads this replaces ~8 enqueues with one graph launch. */
int zh_plan_set_graph(zh_plan* plan, int enable);
int zh_plan_kernel_time(zh_plan* plan, double* scatter_ms, int64_t* launches,
                        double* index_ms);

/* One-shot synchronous region read: plan + execute + wait. */
int zh_array_read(zh_ctx* ctx, const zh_array_meta* meta, const zh_chunk_src* chunks,
                  int64_t nchunks, const int64_t* offset, const int64_t* shape, void* out,
                  uint32_t flags, void* stream, char* err, size_t errlen);
/*
 * Multi-GPU region read in ONE process: the single-JVM form of SURVEY §8(b)'s
 * zh_decode_region_multi (one zarr-java Array.read spread over the GPUs of a node).
 *   The region splits into `ndev` contiguous C-order slabs along its first axis of extent
 *   >= ndev (all earlier axes must have extent 1; otherwise ctxs[root] decodes it whole),
 *   with boundaries on inner-chunk multiples (zh_slab_partition).  Slab r is planned on
 *   ctxs[r] over the chunks it touches and decoded there; all devices work concurrently,
 *   one host thread each.  chunks[] follows computeChunkCoords of the WHOLE region, as in
 *   zh_array_read; flags as there:
 *     no ZH_OUT_DEVICE : host-terminated — slab r is copied D2H straight into its slice of
 *                        the host buffer `out`, each device over its own PCIe link (pin
 *                        `out` with zh_host_register for the full rate);
 *     ZH_OUT_DEVICE    : `out` is a buffer on ctxs[root]'s device; the other devices decode
 *                        into their own HBM and copy their slab to the root's slice over
 *                        xGMI (hipMemcpyPeerAsync), or through pinned host memory when the
 *                        pair has no peer access (see zh_array_read_multi_routed).
 *   Errors: zh_array_read's messages; when the slabs' failures are all data errors the
 *   device placed (checksums, index entries), the first of them in zh_array_read's order (the
 *   chunk first in C order, then the error within it; slabs may cut a shard), else the first
 *   failing slab in C order.
 * zh_slab_partition writes nslabs rows of ndim int64 offsets / shapes (ZH_EINVAL when the
 * region cannot be split into nslabs contiguous slabs).
 */
int zh_array_read_multi(zh_ctx* const* ctxs, int ndev, int root, const zh_array_meta* meta,
                        const zh_chunk_src* chunks, int64_t nchunks, const int64_t* offset,
                        const int64_t* shape, void* out, uint32_t flags, char* err,
                        size_t errlen);
/*
 * zh_array_read_multi with a per-slab route report (slab_route: ndev int32, may be NULL):
 *   output  ZH_ROUTE_DIRECT  decoded straight into its destination (root slab / host slice)
 *           ZH_ROUTE_PEER    device-to-device copy to the root over xGMI (peer access on)
 *           ZH_ROUTE_STAGED  no peer access: D2H into pinned host memory, then H2D on a fresh
 *                            stream of the root device
 *           ZH_ROUTE_SAME    two contexts on one device: a device-local copy
 *   sources (ZH_SRC_DEVICE chunks on another device than the slab's), OR-ed in:
 *           ZH_ROUTE_SRC_PEER    the kernels read them over xGMI (peer access on)
 *           ZH_ROUTE_SRC_STAGED  copied to the slab's device first (no peer access)
 *   ZH_MULTI_FORCE_STAGED=1 stages every non-root slab even on one device (tests).
 */
#define ZH_ROUTE_DIRECT 0
#define ZH_ROUTE_PEER 1
#define ZH_ROUTE_STAGED 2
#define ZH_ROUTE_SAME 3
#define ZH_ROUTE_SRC_PEER 4
#define ZH_ROUTE_SRC_STAGED 8
int zh_array_read_multi_routed(zh_ctx* const* ctxs, int ndev, int root,
                               const zh_array_meta* meta, const zh_chunk_src* chunks,
                               int64_t nchunks, const int64_t* offset, const int64_t* shape,
                               void* out, uint32_t flags, int32_t* slab_route, char* err,
                               size_t errlen);
int zh_slab_partition(int ndim, const int64_t* offset, const int64_t* shape, int nslabs,
                      int64_t align, int64_t* slab_off, int64_t* slab_shape);
/* Number of visible HIP devices (0 when none). */
int zh_device_count(void);

/* ---- sub-shard reads from the index and the referenced pieces ------------------------
 * core.Array.read of a region that covers part of a shard goes through
 * ShardingIndexedCodec.decodePartial → StoreHandleDataProvider (ShardingIndexedCodec.java:
 * 245-255, 333-357): one prefix/suffix read of the shard's index, then one range read per
 * referenced inner chunk.  The Java side does exactly that I/O and nothing else; the stored
 * index goes to the device unchanged, where its crc32c is verified (Crc32cCodec.decode,
 * Crc32cCodec.java:24-48) and its entries are parsed and mapped onto the pieces.  A shard is
 * never assembled on the host, so a part whose referenced payload exceeds 2^31 bytes (a Java
 * array) reads like any other.
 *
 * zh_shard_ranges: the byte ranges of one stored shard a part needs.  index = the
 * index_nbytes bytes the prefix/suffix read returned (16 per inner chunk [+ 4 crc32c]);
 * shard_nbytes = StoreHandle.getSize() or -1 when the store cannot tell; [part_lo, part_hi) =
 * shard-local element box.  Entries of the part's inner-chunk box (nested sharding: its
 * level-1 cells, read whole), missing ones (-1) dropped, are sorted by offset.  max_run > 0:
 * overlapping entries are united and adjacent ranges merged while a run stays <= max_run
 * bytes; no range ever exceeds 2^31 - 1 bytes (a union that would continues as a new range).
 * max_run == 0 (chains whose host stages decode each inner chunk on its own): one range per
 * entry, overlapping or not, exact duplicates once.  Entries that cannot be read (negative,
 * beyond a known shard_nbytes, longer than 2^31 - 1) are left out: the device then reports
 * them with the reference's "Could not load byte data for chunk [...]" unless the index
 * crc32c fails first.  The index crc32c is NOT checked here (zh_shard_index_check).  Writes up to `cap` (offset, nbytes) pairs to
 * `ranges` (may be NULL) and returns the number of ranges; a negative return is -zh_status
 * (EINVAL: not a sharded meta, index_nbytes below the index size, bad part box). */
int64_t zh_shard_ranges(const zh_array_meta* meta, const void* index, int64_t index_nbytes,
                        int64_t shard_nbytes, const int64_t* part_lo, const int64_t* part_hi,
                        int64_t max_run, int64_t* ranges, int64_t cap);

/* Crc32cCodec.decode of a stored shard index on the host (Crc32cCodec.java:24-48): ZH_OK when
 * the chain's index has no crc32c or it matches, ZH_EDATA with the reference's message
 * ("The checksum of the sharding index is invalid. Stored: <int> Computed: <int>") when it does
 * not.  A sub-shard read normally leaves the check to the device; a binding calls this first
 * when the index decides host work before the device sees it: inner chains with host stages
 * (each referenced range is decoded on the host) or a store that cannot tell the shard size
 * (a corrupt entry could ask for a 2^31-byte range read).  The reference checks the index
 * before any range read (ShardingIndexedCodec.java:205). */
int zh_shard_index_check(const zh_array_meta* meta, const void* index, int64_t index_nbytes,
                         char* err, size_t errlen);

/* One byte range of a stored shard as the store returned it.  Pieces are sorted by offset and
 * disjoint, except host-decoded pieces (data_nbytes != nbytes), which may overlap one another
 * at distinct offsets: each serves exactly the entry (offset, nbytes) it was read for. */
typedef struct zh_shard_piece {
  int64_t offset;      /* shard byte offset of the range                                       */
  int64_t nbytes;      /* stored bytes in the range (one inner chunk or a run of adjacent ones) */
  const void* data;    /* the bytes: host memory, or device memory with ZH_SRC_DEVICE          */
  int64_t data_nbytes; /* == nbytes: the stored bytes.  Otherwise the range is exactly one
                          inner chunk whose host byte-to-byte stages (zstd, gzip, blosc) were
                          undone: data holds its raw `bytes` payload (+ crc32c)               */
} zh_shard_piece;

/* One stored shard of a region read (computeChunkCoords order).
 *   missing key (StoreHandle.exists() false): index = NULL, npieces = 0 → fill_value;
 *   whole shard as one object: index = NULL, one piece at offset 0 holding all its bytes;
 *   sub-shard part: index = the stored index bytes, pieces = the ranges zh_shard_ranges
 *     named (in any grouping: a piece must cover each entry it serves; sorted by offset,
 *     not overlapping).  An entry no piece covers reads as "Could not load byte data". */
typedef struct zh_shard_src {
  const void* index;
  int64_t index_nbytes;
  int64_t shard_nbytes;           /* StoreHandle.getSize(), -1 when unknown                   */
  const zh_shard_piece* pieces;
  int64_t npieces;
} zh_shard_src;

/* zh_array_read over shards given as index + pieces (HipArray.read's sub-shard form).
 * Sharded chains only (ZH_EINVAL otherwise).  Host pieces are staged into the device (page-
 * locked sources by direct DMA, pageable ones through the context's pinned ring); the device
 * checks each stored index's crc32c and resolves every entry against the pieces.  Large host
 * reads run pipelined (H2D | decode | D2H) as zh_array_read does. */
int zh_array_read_pieces(zh_ctx* ctx, const zh_array_meta* meta, const zh_shard_src* shards,
                         int64_t nshards, const int64_t* offset, const int64_t* shape, void* out,
                         uint32_t flags, void* stream, char* err, size_t errlen);
/* zh_array_read_multi_routed over shards given as index + pieces (one JVM, several GPUs). */
int zh_array_read_pieces_multi(zh_ctx* const* ctxs, int ndev, int root,
                               const zh_array_meta* meta, const zh_shard_src* shards,
                               int64_t nshards, const int64_t* offset, const int64_t* shape,
                               void* out, uint32_t flags, int32_t* slab_route, char* err,
                               size_t errlen);
/* ShardingIndexedCodec.decodePartial(StoreHandle, offset, shape) over one shard given as
 * index + pieces (HipShardingIndexedCodec's form): shard-local offset/shape → shape elements. */
int zh_sharding_decode_pieces(zh_ctx* ctx, const zh_array_meta* meta, const zh_shard_src* shard,
                              const int64_t* offset, const int32_t* shape, void* out,
                              uint32_t flags, void* stream, char* err, size_t errlen);
/* Page-locked host staging owned by the context, for bindings that copy their sources out of
 * a managed heap before a read (the JNI shim does not: it hands the library its arrays in
 * bounded critical sections): at least `bytes`, valid until the next call on
 * this context or zh_ctx_destroy; grown on demand, kept across calls up to ZH_STAGING_MAX_MB
 * (default 8192; larger requests get a one-off buffer that the next call frees).  Takes the
 * context's lock, so it never replaces the staging under a read in flight on another thread;
 * the caller must not use the previous pointer once it calls again. */
int zh_host_staging(zh_ctx* ctx, size_t bytes, void** out);

/* ---- region reads straight from a FilesystemStore ---------------------------------------
 * core.Array.read when every chunk key resolves to a file (StoreHandle.toPath(),
 * M/store/StoreHandle.java:96-101): the library does the store I/O itself.
 *
 * The store: root = FilesystemStore's directory, name = FilesystemStore.toString() (its file:
 * URI without the trailing '/', FilesystemStore.java:194-197; NULL → "file://" + root).  A
 * NULL store means the filesystem root ("/", named "file://").  Errors name the store and the
 * key as StoreException does (StoreException.java:17-35): "Failed to read from store '<name>'
 * at key '<key>': <reason>", the key being the path below root ('/'-joined keys).
 *
 * paths[i] is the file of the i-th chunk of computeChunkCoords(meta->shape, meta->chunk_shape,
 * offset, shape); NULL, or a path that is not a regular file, is a missing key
 * (FilesystemStore.exists, FilesystemStore.java:42-45) → fill_value.  Per file the reads are
 * the reference's:
 *   unsharded:           the whole object (get(keys), :47-57);
 *   sharded, whole shard (the part is the full chunk: decodePartial → chunkHandle.read(),
 *                        ShardingIndexedCodec.java:246-251): the index and the referenced
 *                        ranges of the file as it is; an index or entry beyond the file is an
 *                        error (ZH_EDATA; the reference's ByteBuffer slicing throws);
 *   sharded, part        (StoreHandleDataProvider, ShardingIndexedCodec.java:333-357): the
 *                        index by a prefix (index_location start, get(keys, 0, n)) or suffix
 *                        (get(keys, -n)) read, then the referenced inner-chunk ranges
 *                        (get(keys, off, off + n), adjacent ranges merged).  As in
 *                        get(keys, start, end) (:84-102), bytes past the end of the file read as
 *                        zeros: a truncated file decodes with zeros where its bytes are missing,
 *                        and a prefix index read of a file shorter than the index is zero-padded
 *                        (its crc32c then fails).  A suffix read of a file shorter than the
 *                        index is an error (ZH_EDATA; the reference's position(< 0) throws).
 * The index crc32c and every entry are checked on the device, as with zh_array_read_pieces.
 * The range reads (pread) write straight into the page-locked ring of the pipelined read, so
 * the file bytes are copied once on the host and the reads overlap the H2D copies, the decode
 * and the D2H of earlier slabs.  At most 64 files are open at once whatever the region's
 * chunk count (a closed one is reopened by path for its next range).  `out`: host memory
 * (flags 0) or device memory (ZH_OUT_DEVICE); ZH_SRC_DEVICE is not allowed.  A file that cannot
 * be opened or read (other than missing) → ZH_EIO with the readFailed text.  The chain must be
 * device-supported (zh_validate_meta); chains with host byte-to-byte stages keep their store
 * reads on the binding side (zh_array_read_pieces). */
typedef struct zh_file_store {
  const char* root; /* FilesystemStore's directory                                          */
  const char* name; /* FilesystemStore.toString(); NULL: "file://" + root                     */
} zh_file_store;
int zh_array_read_files(zh_ctx* ctx, const zh_array_meta* meta, const zh_file_store* store,
                        const char* const* paths, int64_t npaths, const int64_t* offset,
                        const int64_t* shape, void* out, uint32_t flags, char* err,
                        size_t errlen);
/* zh_array_read_files spread over several GPUs in one process (zh_array_read_multi_routed's
 * slabs and routes; HipArray.read with ZH_DEVICES): every device reads the files of its slab
 * and decodes it, a host-terminated read copying each slab straight into its slice of `out`
 * (each device over its own PCIe link). */
int zh_array_read_files_multi(zh_ctx* const* ctxs, int ndev, int root, const zh_array_meta* meta,
                              const zh_file_store* store, const char* const* paths,
                              int64_t npaths, const int64_t* offset, const int64_t* shape,
                              void* out, uint32_t flags, int32_t* slab_route, char* err,
                              size_t errlen);
/* core.Array.write of a region of whole chunks (clipped only by the array boundary) into a
 * FilesystemStore: the device encode of zh_array_write, then per chunk writeChunk's store call
 * (M/core/Array.java:143-156) done here — all fill_value → the file deleted (FilesystemStore.delete,
 * a missing file is fine), otherwise the parent directories created and the chunk's bytes
 * stored at its path (FilesystemStore.set, M/store/FilesystemStore.java:105-128).  The encoded
 * bytes go D2H through the page-locked ring in windows that several lanes pwrite into a
 * temporary file beside the chunk's, renamed over it once complete: a failure leaves every
 * chunk it did not complete as it was (the reference truncates a file before writing it), and
 * at most 3 files per lane are open at once.  paths[i]: the i-th chunk of computeChunkCoords;
 * src: the region in C order on the host, or on the device with ZH_SRC_DEVICE; nbytes (may be
 * NULL): per chunk the bytes written (0: deleted).  A region that cuts chunks → ZH_EUNSUPPORTED
 * (the binding's read-modify-write); a store failure → ZH_EIO with StoreException's text
 * (writeFailed: "... Failed to write <n> bytes to file: <path>" or "... Failed to create parent
 * directories for path: <dir>"; deleteFailed: "... Failed to delete file: <path>"). */
int zh_array_write_files(zh_ctx* ctx, const zh_array_meta* meta, const void* src,
                         const int64_t* offset, const int64_t* shape, const zh_file_store* store,
                         const char* const* paths, int64_t npaths, uint32_t flags,
                         int64_t* nbytes, char* err, size_t errlen);
/* Diagnostic (no device needed): the store reads zh_array_read_files would make for these
 * paths, as (chunk index, file offset, bytes) triples in order — a whole object, or a shard's
 * index read followed by its merged range reads; missing keys make none.  Writes up to `cap`
 * triples to `reads` (may be NULL) and returns their number, or -zh_status with err set (the
 * same checks and messages as the read).  Tests use it to check the read plan on the host. */
int64_t zh_debug_file_reads(const zh_array_meta* meta, const zh_file_store* store,
                            const char* const* paths, int64_t npaths, const int64_t* offset,
                            const int64_t* shape, int64_t* reads, int64_t cap, char* err,
                            size_t errlen);
/* Diagnostic (no device needed): the process-wide file table of the file reads —
 * out[0] = slots in use, out[1] = descriptors open, out[2] = entries in the queue of opens
 * (bounded: stale entries are dropped as files are given back).  Returns ZH_OK. */
int zh_debug_file_table(int64_t* out);

/* ShardingIndexedCodec.decode: whole shard → chunk_shape elements. */
int zh_sharding_decode(zh_ctx* ctx, const zh_array_meta* meta, const void* shard, int64_t nbytes,
                       void* out, uint32_t flags, void* stream, char* err, size_t errlen);
/* ShardingIndexedCodec.decodePartial: shard-local offset/shape → shape elements. */
int zh_sharding_decode_partial(zh_ctx* ctx, const zh_array_meta* meta, const void* shard,
                               int64_t nbytes, const int64_t* offset, const int32_t* shape,
                               void* out, uint32_t flags, void* stream, char* err,
                               size_t errlen);

/* ---- encode (write path) ---------------------------------------------------------- */
/*
 * Device encode of every chunk intersecting [offset, offset+shape), which must cover
 * whole chunks (clipped only by the array boundary); src is that region in C order on
 * the device.  Inner chunks that are all fill_value become (-1,-1) index entries and
 * are laid out in C order (deterministic; the reference's order is not — SURVEY Q7).
 * A chunk that is entirely fill reports nbytes = 0 (writeChunk deletes it).
 * dsts[i] follows computeChunkCoords order.  zh_array_encoded_bound gives the worst-
 * case encoded size of one chunk.
 */
int64_t zh_array_encoded_bound(const zh_array_meta* meta);
int zh_array_write(zh_ctx* ctx, const zh_array_meta* meta, const void* src,
                   const int64_t* offset, const int64_t* shape, zh_chunk_dst* dsts,
                   int64_t nchunks, void* stream, char* err, size_t errlen);
/* zh_array_write for host buffers (the JNI write path: the region is a Java array, the
 * encoded chunks become byte[]s): src_host holds the region in C order; the encoded chunk i
 * is copied to outs[i] (capacities[i] bytes available) and its size stored in nbytes[i]
 * (0 = chunk is all fill → delete the key).  A capacity below the encoded size → ZH_EINVAL
 * naming the size needed; zh_array_encoded_bound always suffices.  Staging goes through the
 * context's block cache. */
int zh_array_write_host(zh_ctx* ctx, const zh_array_meta* meta, const void* src_host,
                        const int64_t* offset, const int64_t* shape, void* const* outs,
                        const int64_t* capacities, int64_t* nbytes, int64_t nchunks, char* err,
                        size_t errlen);

/* ---- device memory / stream / event plumbing for callers without their own ---------- */
/* sizeof of the public structs, for binding-side layout checks (ctypes / JNI mirrors):
 * out[0..3] = zh_codec_chain, zh_array_meta, zh_chunk_src, zh_chunk_dst.  Returns 4. */
int zh_abi_sizes(int64_t* out, int n);
/* Device memory for regions and shards, the library's default kind (zh_device_malloc_ex with
 * flags 0): a buffer of at least 1 GiB is built from 1 GiB physical chunks (ZH_MALLOC_SCATTER,
 * falling back to hipMalloc), a smaller one is hipMalloc'd.  Round 6 timed the full c4 decode
 * into 3 fresh outputs of each kind on three boxes (DESIGN.md §4 "Placement"): 1 GiB chunks had
 * the highest floor on each (2871 / 2869 / 2927 GiB/s against hipMalloc's 2841 / 2844 / 2913
 * and 16 MiB chunks' 2803 / 2830 / 2900). */
int zh_device_malloc(zh_ctx* ctx, size_t bytes, void** out);
/* Allocation flags for zh_device_malloc_ex.  The write bandwidth a large buffer gets depends
 * on where its physical memory lands (DESIGN.md §4 "Placement": writes only, any access
 * pattern, not TLB or L2-channel balance).  ZH_MALLOC_CONTIGUOUS asks for physically
 * contiguous HBM (hipDeviceMallocContiguous).  Falls back to hipMalloc unless
 * ZH_MALLOC_REQUIRE. */
#define ZH_MALLOC_CONTIGUOUS 0x1u
#define ZH_MALLOC_REQUIRE 0x2u
/* Physical chunks (hipMemCreate, ZH_SCATTER_MB MiB each, default 1024) mapped into one virtual
 * range in a coprime-stride order, so that virtually adjacent chunks are not physically
 * adjacent: the decode's output arena in bench.py (DESIGN.md §4 "Placement": mean +5.6 % over
 * hipMalloc on 18 buffers, 3 boxes).  The rest beyond the last whole chunk gets one smaller
 * chunk (rounded up to the allocation granularity), mapped last.  Freed by zh_device_free. */
#define ZH_MALLOC_SCATTER 0x4u
/* With ZH_MALLOC_SCATTER: allocate two candidate arenas (the first held while the second is
 * allocated, so each gets other physical chunks), time a contiguous
 * store probe over each (zh_device_write_rate pattern 0) and keep the fastest.  A large
 * arena's write rate is set by its physical chunks (not their order or its address) and the
 * probe predicts the decode's rate into it (DESIGN.md §4 "Placement").  Needs the memory of
 * two arenas while it runs; a candidate that does not fit ends the search.  The buffer's
 * contents are undefined.  zh_device_alloc_probes reports the probes. */
#define ZH_MALLOC_CALIBRATE 0x8u
/* hipMalloc whatever the size (the default kind's small-buffer form for every size). */
#define ZH_MALLOC_PLAIN 0x10u
int zh_device_malloc_ex(zh_ctx* ctx, size_t bytes, unsigned flags, void** out);
/* Map a ZH_MALLOC_SCATTER allocation's physical chunks a second time, at a fresh virtual
 * range, in chunk order `order` (0 = the allocation's order: slot i <- chunk (i*m) mod n;
 * k > 0: another coprime stride and a rotation).  The view aliases the allocation's memory;
 * free it with zh_device_free before the allocation.  ZH_EINVAL for a pointer that is not a
 * scatter allocation.  (Re-mapping a live range in place is not offered: on ROCm 7.2 the
 * device kept translations of the old mapping, DESIGN.md §4 "Placement".) */
/* Probe rates (GB/s) of the candidates ZH_MALLOC_CALIBRATE tried for `ptr`, in allocation
 * order; *chosen = the index of `ptr` among them.  Returns the number of candidates (0 for an
 * allocation that was not calibrated), or -ZH_EINVAL. */
int zh_device_alloc_probes(zh_ctx* ctx, void* ptr, double* gbps, int cap, int* chosen);
int zh_device_scatter_view(zh_ctx* ctx, void* ptr, uint64_t order, void** out);
/* Write bandwidth of [ptr, ptr+bytes): one untimed and `reps` timed launches of a store-only
 * probe on the context stream (pattern 0: contiguous 16-B stores; 1: the decode kernels' store
 * pattern, 128-B lines 6 KiB apart).  *gbps = bytes / median time, in 1e9 B/s.  Overwrites
 * the buffer. */
int zh_device_write_rate(zh_ctx* ctx, void* ptr, size_t bytes, int pattern, int reps,
                         double* gbps);
/* Copy ceiling of a buffer pair: one untimed and `reps` timed launches of a streaming
 * byte-swapping copy src -> dst over the first bytes rounded down to 128 KiB (non-temporal
 * 16-B loads and stores, 128 KiB per workgroup step: the fastest stream of
 * tools/copy_lab.hip).  *gbps = (bytes read + bytes written) / median time, in 1e9 B/s, the
 * decode's own traffic count.  Overwrites dst.  ZH_EINVAL below 128 KiB. */
int zh_device_copy_rate(zh_ctx* ctx, void* dst, const void* src, size_t bytes, int reps,
                        double* gbps);
int zh_device_free(zh_ctx* ctx, void* ptr);
int zh_host_malloc_pinned(zh_ctx* ctx, size_t bytes, void** out);
int zh_host_free_pinned(zh_ctx* ctx, void* ptr);
/* Page-lock caller-owned host memory (hipHostRegister), e.g. one rank's slice of a region
 * buffer shared by the processes of a multi-GPU read, so that its D2H runs at pinned rate. */
int zh_host_register(zh_ctx* ctx, void* ptr, size_t bytes);
int zh_host_unregister(zh_ctx* ctx, void* ptr);
/* kind: 0 H2D, 1 D2H, 2 D2D; asynchronous on stream */
int zh_memcpy_async(zh_ctx* ctx, void* dst, const void* src, size_t bytes, int kind, void* stream);
int zh_memset_async(zh_ctx* ctx, void* dst, int value, size_t bytes, void* stream);
int zh_stream_synchronize(zh_ctx* ctx, void* stream);
int zh_stream_create(zh_ctx* ctx, void** stream);
int zh_stream_destroy(zh_ctx* ctx, void* stream);
/* make `stream` wait for `ev` (recorded on another stream) */
int zh_stream_wait_event(zh_ctx* ctx, void* stream, void* ev);
/* pitched copy of `height` rows of `width` bytes; kind as zh_memcpy_async */
int zh_memcpy2d_async(zh_ctx* ctx, void* dst, size_t dpitch, const void* src, size_t spitch,
                      size_t width, size_t height, int kind, void* stream);
int zh_event_create(zh_ctx* ctx, void** ev);
int zh_event_destroy(zh_ctx* ctx, void* ev);
int zh_event_record(zh_ctx* ctx, void* ev, void* stream);
int zh_event_elapsed_ms(zh_ctx* ctx, void* start, void* stop, float* ms);
int zh_device_info(zh_ctx* ctx, char* name, size_t namelen, int64_t* total_mem,
                   int* cu_count, char* arch, size_t archlen);

/* ---- host byte-to-byte stage: blosc1 frames ----------------------------------------
 * Replaces the blosc-java call inside BloscCodec.decode (M/v3/codec/core/BloscCodec.java,
 * M/v2/codec/core/BloscCodec.java) for hosts without the blosc library: BloscLZ, LZ4/LZ4HC,
 * zlib and zstd payloads, byte and bit shuffle, split and unsplit blocks, memcpyed frames.
 * dst == NULL only reports the decompressed size in *nbytes_out.  Snappy payloads
 * → ZH_EUNSUPPORTED. */
int zh_blosc_decompress(const void* src, size_t srclen, void* dst, size_t dstcap,
                        size_t* nbytes_out, char* err, size_t errlen);

/* ---- host byte-to-byte stage: zstd frames (RFC 8878) ------------------------------
 * Replaces zstd-jni inside ZstdCodec.decode (M/core/codec/core/ZstdCodec.java:14-22) and the
 * zstd compressor of blosc frames (BloscCodec.java; CodecBuilder.withBlosc() defaults to
 * cname "zstd", M/v3/codec/CodecBuilder.java:58-60).  One or more frames (skippable frames
 * skipped); the XXH64 content checksum is verified when a frame carries one; frames that need
 * a dictionary → ZH_EUNSUPPORTED.  dst == NULL: *dstlen = the decoded size.
 * zh_zstd_compress_raw writes a valid frame of raw (stored) blocks with the content size and,
 * if asked, the checksum (the write path's encoder; no compression); dst == NULL: the size.
 * zh_xxh64: XXH64 of a buffer (the checksum's hash). */
int zh_zstd_decompress(const void* src, size_t srclen, void* dst, size_t dstcap, size_t* dstlen,
                       char* err, size_t errlen);
int zh_zstd_compress_raw(const void* src, size_t srclen, int checksum, void* dst, size_t dstcap,
                         size_t* dstlen);
uint64_t zh_xxh64(const void* data, size_t len, uint64_t seed);

/* dst block b ← src block src_block[b] (device buffers, blocks of block_bytes, a multiple of
 * 16; 16-byte aligned; src_block on the host), synchronous: re-lays out encoded shards, e.g.
 * the bench's shuffled inner-chunk order. */
int zh_gather_blocks(zh_ctx* ctx, void* dst, const void* src, int64_t block_bytes,
                     const int64_t* src_block, int64_t n);

/* ---- synthetic data (bench / property tests) -------------------------------------- */
/* dst[i] = low dtype_size bytes of splitmix64((first + i) ^ seed), i in [0, n). */
int zh_synth_fill(zh_ctx* ctx, void* dst, int64_t n, int dtype_size, int64_t first,
                  uint64_t seed, void* stream);
/* Counts elements of the C-order region [offset, offset+shape) of an array of
 * array_shape whose value differs from the synth value at their global index. */
int zh_synth_verify(zh_ctx* ctx, const void* region, int ndim, const int64_t* array_shape,
                    const int64_t* offset, const int64_t* shape, int dtype_size,
                    uint64_t seed, uint64_t* mismatches, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ZARRHIP_H */
