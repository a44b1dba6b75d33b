/*
 * zh_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of zarr-java's chunk codec path (reference snapshot 2026-08-07),
 * used as the parity checker for the HIP path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product (libzarrhip.so) never links
 * or calls it.
 *
 * Parity is pinned against the reference's own fixtures and known-answer tests
 * (tests/test_oracle_golden.py): testdata/sharding_index_location/{start,end},
 * TestUtils.java:15-93, ZarrV3Test.java:248-264, ZarrV3Test.java:389, and the CRC-32C
 * check value.  The reference itself (Java) cannot run in this image (no JDK).
 *
 * Structs are the public ABI types of include/zarrhip.h (types only).
 */
#ifndef ZH_ORACLE_H
#define ZH_ORACLE_H

#include "../include/zarrhip.h"

#ifdef __cplusplus
extern "C" {
#endif

uint32_t zo_crc32c(uint32_t crc, const void* data, size_t n);
int64_t zo_compute_chunk_coords(int ndim, const int64_t* array_shape, const int32_t* chunk_shape,
                                const int64_t* sel_offset, const int64_t* sel_shape,
                                int64_t* coords_out, int64_t max_coords);
int zo_compute_projection(int ndim, const int64_t* chunk_coords, const int64_t* array_shape,
                          const int32_t* chunk_shape, const int64_t* sel_offset,
                          const int64_t* sel_shape, int32_t* chunk_offset, int32_t* out_offset,
                          int32_t* shape);
int zo_is_permutation(int n, const int32_t* order);
int zo_inverse_permutation(int n, const int32_t* order, int32_t* inverse);

/* core.Array.read (M/core/Array.java:378-441).  nthreads <= 1: serial. */
int zo_array_read(const zh_array_meta* meta, const zh_chunk_src* chunks, int64_t nchunks,
                  const int64_t* offset, const int64_t* shape, void* out, int nthreads,
                  char* err, size_t errlen);
/* core.Array.read against a FilesystemStore (one path per chunk key, NULL = missing): the
 * partial path's range reads per inner chunk (StoreHandleDataProvider). */
int zo_array_read_store(const zh_array_meta* meta, const char* const* paths, int64_t nchunks,
                        const int64_t* offset, const int64_t* shape, void* out, int nthreads,
                        char* err, size_t errlen);
/* ShardingIndexedCodec.decodeInternal over a whole shard buffer (decode / decodePartial). */
int zo_sharding_decode_partial(const zh_array_meta* meta, const void* shard, int64_t nbytes,
                               const int64_t* offset, const int32_t* shape, void* out,
                               int nthreads, char* err, size_t errlen);
/* core.Array.write over whole chunks → one malloc'd buffer per chunk (NULL/0 = deleted). */
int zo_array_write(const zh_array_meta* meta, const void* src, const int64_t* offset,
                   const int64_t* shape, void** out_bufs, int64_t* out_sizes, int64_t nchunks,
                   char* err, size_t errlen);
void zo_free(void* p);

#ifdef __cplusplus
}
#endif
#endif
