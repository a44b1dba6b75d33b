// zh_internal.h — structures shared by the host planner (zh_engine.cpp) and the HIP
// kernels (zh_kernels.hip).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <stdint.h>

#include "../../include/zarrhip.h"

namespace zh {

constexpr int kMaxDims = ZH_MAX_DIMS;
constexpr int kBlock = 256;            // threads per workgroup (4 waves of 64)
constexpr int kTileTPB = 4;            // 32x32 transpose tiles per workgroup iteration
constexpr int kCrcSpan = 64 * 1024;    // chunk payload bytes per data-CRC partial
constexpr int kIdxSpan = 4096;         // index bytes per index-CRC workgroup (one 16-B vector
                                       // per lane: a 512 KiB index is 128 workgroups)
constexpr int kCrcLane = kCrcSpan / kBlock;  // 256 bytes per lane

// Per-shard status words (device, uint64 each), read back by zh_plan_wait: the flags, the
// shard index's crc32c pair (kFlagCrc: checked before any inner chunk, Crc32cCodec.java:24-48),
// and the first chunk-level error in the oracle's sequential order (chunk_error below): its
// key ((0xFFFFFFFF − rank) << 8 | kind, atomicMax) and two detail words keyed by the same rank.
enum : uint32_t { kStFlags = 0, kStCrcStored = 1, kStCrcComputed = 2, kStBadChunk = 3,
                  kStDetailA = 4, kStDetailB = 5, kStWords = 6 };
// kinds: kFlagCrc is the shard index's own checksum; the others are chunk-level (with kFlagL1
// / kFlagLeaf, below, on nested chains): an unreadable range, a wrong length, a failed chunk
// or sub-shard index crc32c (details: stored, computed), a sub-shard shorter than its index
// (detail A: its length)
enum : uint32_t { kFlagCrc = 1u, kFlagRange = 2u, kFlagLength = 4u, kFlagChunkCrc = 32u,
                  kFlagShort = 64u };

// The rank of a chunk-level error: its place in the sequential order in which the oracle
// decodes a shard (the reference decodes the inner chunks in a parallel stream,
// ShardingIndexedCodec.java:210-212, so any failing chunk's error may surface there; the
// device and the oracle both report the first in C order).  Single level: the
// inner chunk's C-order index in the shard grid.  Nested: level-1 cell lin1 ranks
// lin1·(cps2 + 1) (its entry, its sub-shard's length and index crc32c), its leaf k2
// lin1·(cps2 + 1) + 1 + k2 (the sub-shard decode visits every leaf, :97-103).
struct RankGeom {
  int64_t cps_stride[ZH_MAX_DIMS];   // single level: inner-grid C-order strides
  int64_t cps1_stride[ZH_MAX_DIMS];  // nested: level-1 cell grid strides
  int64_t k2_stride[ZH_MAX_DIMS];    // nested: leaf-in-cell C-order strides
  int64_t r2;                        // nested: cps2 + 1 (0: single level)
  int32_t r[ZH_MAX_DIMS];            // nested: leaves per cell per dim
  int32_t ndim;
  int32_t pad;
};

// Exact floor(n / d) for 0 <= n < 2^31, 1 <= d < 2^31 (Granlund–Montgomery round-up
// method with N = 31): q = (n * m) >> s.
struct FastDiv {
  uint64_t m;
  uint32_t s;
  uint32_t d;
};

__host__ __device__ inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < (uint64_t)d) l++;
  FastDiv f;
  f.d = d;
  f.s = 31 + l;
  f.m = ((1ull << (31 + l)) / d) + 1;
  return f;
}

__host__ __device__ inline uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (uint32_t)(((uint64_t)n * f.m) >> f.s);
}

// One byte range of a stored shard the device holds (sub-shard reads: the index and the
// referenced ranges only, zh_array_read_pieces / compact host staging).  Entry (off, nb) of
// the stored index is served by the piece with p.off <= off and off + nb <= p.off + p.len,
// read at p.src + (off - p.off).  A piece with dlen != len is exactly one inner chunk whose
// host byte-to-byte stages were undone: it serves only (p.off, p.len) and holds dlen bytes.
struct DevPiece {
  uint64_t off;
  uint64_t len;
  const uint8_t* src;
  uint64_t dlen;
};

// One stored chunk object (a shard when sharded) touched by a region.
struct DevShard {
  const uint8_t* data;      // decode: encoded bytes (nullptr: key missing → fill_value); with
                            // pieces: the stored index (index_off 0)
  uint8_t* wdata;           // encode: destination buffer
  int64_t nbytes;           // decode: object size (StoreHandle.getSize(); INT64_MAX unknown)
  int64_t index_off;        // decode (sharded): byte offset of the index entries
  const DevPiece* pieces;   // decode: sorted, disjoint byte ranges held (nullptr: the whole
  int64_t npieces;          //   object is at data)
  int64_t item_begin;       // prefix sum of inner-chunk items before this shard
  int64_t out_base;         // element offset of part_lo inside the region buffer
  int32_t box_start[kMaxDims];  // first inner-chunk coordinate of the box
  int32_t box_count[kMaxDims];  // inner chunks per dim in the box
  int32_t part_lo[kMaxDims];    // requested part of the shard (shard-local coords)
  int32_t part_hi[kMaxDims];
  // nested sharding: flattened leaf index (16 B LE entries over the shard's leaf grid,
  // written by nested_index_kernel; nullptr for single-level sharding) and the box of
  // level-1 cells the part references
  uint8_t* flat;
  int64_t l1_begin;             // prefix sum of referenced level-1 cells before this shard
  int32_t l1_box_start[kMaxDims];
  int32_t l1_box_count[kMaxDims];
};

// Per-inner-chunk work descriptor written by the resolve kernel (index parse) and read
// by the scatter kernel, one item ahead of use.
enum : int32_t { kFastNone = 0, kFastRowArith = 1, kFastRowTable = 2, kFastTileTable = 3 };
enum : uint32_t { kDescFullCopy = 0, kDescFullFill = 1, kDescClip = 2, kDescSkip = 3,
                  kDescModeMask = 0xFF, kDescFast = 0x100,
                  // kDescClip copy cut only along the unit-stride dim (rows keep their start,
                  // a 16-byte-multiple, power-of-two-vector prefix is in bounds): the row
                  // kernel takes it with log2(vectors per row) in ItemDesc.fill
                  kDescClipRow = 0x200 };
struct ItemDesc {
  uint64_t src;   // absolute address of the inner chunk's bytes (kDescFullCopy)
  int64_t d0;     // destination element offset of the inner chunk origin
  uint64_t fill;  // kDescFullFill value (fill_value for a missing shard, 0 for Q1)
  uint32_t kind;
  uint32_t shard;
};

// Uniform launch arguments of the decode/encode scatter kernels.
struct ScatterArgs {
  const DevShard* shards;
  int64_t nshards;
  int64_t total_items;      // (inner chunks) << piece_shift
  uint8_t* region;          // decode: output region; encode: source region (C order)
  uint64_t* status;         // decode: kStWords u64 per shard
  const int64_t* item_off;  // encode: payload byte offset per inner-chunk item (-1 = skip)
  uint8_t* flags;           // encode flag pass: 1 = item has a non-fill element
  int32_t ndim;
  int32_t swap;             // byte-swap elements (big-endian bytes codec, dtype > 1 byte)
  int32_t is_bool;          // normalise bool bytes to 0/1
  int32_t piece_shift;      // items per inner chunk = 1 << piece_shift
  int32_t fs;               // src-fast dim (decoded-dim index)
  int32_t fd;               // dst-fast dim
  int32_t index_be;         // shard index stored big-endian
  int32_t sharded;
  int32_t inner[kMaxDims];      // decoded inner chunk shape
  int64_t pstride[kMaxDims];    // payload element stride of each decoded dim
  int64_t rstride[kMaxDims];    // region element stride of each dim
  int64_t cps_stride[kMaxDims]; // index entry stride of each inner-chunk coordinate
  int64_t inner_nbytes;
  uint64_t fill;                // fill_value bytes (little-endian), replicated as needed
  uint64_t fill_mask;           // write path's all-fill test: element bits compared (a float
                                // ±0 fill drops the sign bit; else all ones), low dsize bytes
  int32_t fill_never;           // write path, a float NaN fill: no element equals it, so every
                                // chunk and inner chunk is kept, boundary padding included
  int32_t pad_fill;
  FastDiv inner_div[kMaxDims];  // divisors for unclipped extents
  // decode fast path for unclipped inner chunks
  ItemDesc* desc;               // per inner chunk (resolve kernel output)
  int32_t fast_mode;            // kFastNone / kFastRowArith / kFastRowTable / kFastTileTable
  int32_t fast_vpr_shift;       // row modes: log2(16-byte vectors per row)
  int32_t fast_rows;            // row modes: rows (tile mode: 32x32 units) per inner chunk
  const uint32_t* fast_tab;     // (src, dst) element offsets per row / tile unit
  int32_t fast_n;               // table entries (0: no table)
  int32_t rm_n;                 // kFastRowArith: row dims (innermost first)
  int32_t rm_shift[3];          //   log2 extent of each row dim
  int64_t rm_sstr[3];           //   payload element stride of each row dim
  int64_t rm_dstr[3];           //   region element stride of each row dim
  int64_t n_citems;             // inner-chunk items (without pieces)
  uint32_t* slow_list;          // inner chunks that need the generic path (resolve output)
  uint32_t* slow_count;
  int32_t dsize;
  int32_t tile;
  int32_t nt;                   // fast kernels: bit 0 non-temporal loads, bit 1 stores (the
                                // launchers require 3: every kept kernel streams)
  int32_t tile_variant;         // tile fast path: 0 row-per-tile loads, 1 row-interleaved groups,
                                // 20 + G: tiles_group_kernel over G chunks (next step's loads
                                // prefetched); 51: the row-CRC tile kernel (chunk crc32c)
  int32_t row_group;            // row fast path (decode): G > 0 = rows_group_kernel over G
                                // chunks per work item (row-clipped items then go slow)
  int32_t crc_extra;            // 4 when each stored chunk carries a trailing crc32c, else 0
  uint64_t item_mul;            // fast kernels visit items in the order (i * item_mul) mod
                                // total_items (coprime; 0 = identity): decorrelates the
                                // addresses written concurrently (DESIGN §4 placement)
  int32_t crc_fused;            // the fast kernel also computes the chunk CRC: row kernel per
                                // piece; tile kernel per chunk (shares shifted to the payload
                                // end, per-unit shifts after the (src, dst) pairs of fast_tab)
  uint32_t* crc_partials;       // raw CRC registers, XOR-accumulated: per item (rows) or per
                                // chunk (tiles)
  uint32_t crc_tile_step;       // tile CRC: x^(8Δ) when unit u + kTG ends Δ bytes after unit u
                                // for every u (a lane then folds its groups with one table
                                // shift instead of a multiply per group); 0 = irregular
  int32_t tile_align;           // row-CRC tile decode: units are consecutive 128-B payload rows
                                // and the tile rows follow each other (host-checked), so the
                                // movers load 128-B aligned lines (tiles_rowcrc_aln_kernel)
  int64_t tile_ystride;         // tile_align: unit u's region offset is u · tile_ystride
  RankGeom rank;                // chunk-level error order (decode)
};

// Chunk-payload CRC-32C pass (inner crc32c codec): one workgroup per (item, 64 KiB span) of
// every resolved chunk, then one lane per item combines the spans and verifies the stored
// value (decode) or writes it after the payload (encode, store = 1).
struct DataCrcArgs {
  const ItemDesc* desc;         // src = payload address; kinds other than copy/clip skipped
  int64_t n_items;
  int64_t len;                  // payload bytes per chunk
  int64_t span;                 // bytes per partial (kCrcSpan, or the row kernel's piece)
  int32_t nspan;                // ceil(len / span)
  int32_t store;
  int32_t skip_fast;            // partial pass skips kDescFast items (their CRC is fused)
  int32_t pad;
  uint32_t* partials;           // n_items * nspan
  uint64_t* status;             // decode: kStWords per shard
  const DevShard* shards;       // decode: the items' shards (a mismatch's rank)
  RankGeom rank;
};

// Nested sharding pre-pass (nested_index_kernel): one workgroup per referenced level-1 cell
// resolves the outer entry, CRC-checks the cell's sub-shard index and writes its leaves'
// absolute (offset, nbytes) into DevShard::flat, so that the single-level resolve/scatter
// kernels run unchanged with leaf = inner chunk.
enum : uint32_t { kFlagL1 = 8, kFlagLeaf = 16 };  // error-key level bits (status kStBadChunk)
struct NestArgs {
  const DevShard* shards;
  int64_t nshards;
  int64_t n_l1;                   // referenced level-1 cells (all shards)
  uint64_t* status;
  int32_t ndim;
  int32_t index_be;               // outer index endianness
  int32_t sub_be;                 // sub-shard index endianness
  int32_t sub_crc;                // sub-shard index has crc32c
  int32_t sub_start;              // sub-shard index at the start
  int32_t pad;
  int64_t sub_isz;                // encoded sub-shard index size (16 * cps2 [+ 4])
  int64_t cps2;                   // leaves per level-1 cell
  int64_t leaf_nbytes;            // stored leaf bytes (+ 4 with the leaf crc32c)
  int32_t leaf_crc;               // leaves carry a crc32c: the cell's leaves outside the part
  int32_t pad2;                   //   are checked here (the data-CRC pass checks the rest)
  int32_t leaf[kMaxDims];         // leaf chunk shape
  int64_t cps1_stride[kMaxDims];  // outer index entry stride per level-1 coordinate
  int64_t flat_stride[kMaxDims];  // flat index entry stride per leaf coordinate
  int32_t r[kMaxDims];            // leaves per level-1 cell along each dim
};

struct CrcJob {
  const uint8_t* base;      // first index byte (device)
  int64_t len;              // bytes under the CRC (16 * entries)
  int64_t span_begin;       // prefix sum of spans
  int32_t shard;            // status slot
  int32_t pad;
};

// one index-CRC launch: the jobs, their span count, the span registers + completion counters
// (launch_crc below), the status words (nullptr: store the CRC, the write path)
struct CrcIdxArgs {
  const CrcJob* jobs;
  int64_t njobs;
  int64_t nspans;
  uint32_t* partials;
  uint64_t* status;
  int32_t sshift;
  int32_t pad;
};
constexpr int kCrcLdsWords = 12 * 256 + kBlock + 1;  // tables, wave reduction, last flag
constexpr int64_t kSmallOneItems = 64;  // plans of at most this many inner chunks: one launch
constexpr int64_t kSmallOneBytes = 16ll << 20;  // ... of at most this many payload bytes
// one-plan reads into pageable memory up to this: staged (above it the runtime's own pageable
// copy is faster: 2 MiB 0.10 vs 0.17 ms, 4 MiB 0.15 vs 0.29 ms, profiles/r05/hout/small_hout.json)
constexpr int64_t kHoutPinBytes = 1ll << 20;

int env_int(const char* name, int def);  // zh_engine.cpp: an integer switch from the environment

// Kernel launchers (zh_kernels.hip).
// index crc32c of every job in one launch, spans of kIdxSpan << span_shift bytes (job
// span_begin set by assign_crc_spans); partials holds nspans span registers followed by njobs
// completion counters, zero before the first launch (the kernel resets them)
hipError_t launch_crc(const CrcJob* jobs, int64_t njobs, int64_t nspans, int span_shift,
                      uint32_t* partials, uint64_t* status, hipStream_t stream);
hipError_t launch_resolve(const ScatterArgs& a, hipStream_t stream);
hipError_t launch_nested_index(const NestArgs& a, int grid, hipStream_t stream);
hipError_t launch_data_crc(const DataCrcArgs& a, int grid, hipStream_t stream);
hipError_t launch_data_crc_partial(const DataCrcArgs& a, int grid, hipStream_t stream);
hipError_t launch_data_crc_finalize(const DataCrcArgs& a, hipStream_t stream);
// error path: the crc32c of a single-level chunk rejected for its length (out: 3 words)
hipError_t launch_chunk_crc_detail(const ScatterArgs& a, int64_t shard, int64_t lin,
                                   uint64_t* out, hipStream_t stream);
extern std::atomic<int64_t> g_last_fast_path;  // diagnostic, zh_debug_last_fast_path
extern std::atomic<int64_t> g_last_encode_path;
bool rowcrc_lds_at_zero();  // the row-CRC tile kernels have no static LDS
constexpr int kAlnUnitsMax = 32;  // tiles_rowcrc_aln_kernel: units per chunk (its K capacity)
hipError_t launch_scatter(const ScatterArgs& a, int dsize, int grid, hipStream_t stream);
// the slow list; with crc.nspans > 0 the index crc32c runs in the same launch (first
// crc.nspans workgroups) instead of launch_crc ahead of the resolve kernel
hipError_t launch_decode_slow(const ScatterArgs& a, int grid, const CrcIdxArgs& crc,
                              hipStream_t stream);
// small plans: resolve + decode of every item in one launch (with the index CRC as above)
hipError_t launch_decode_small(const ScatterArgs& a, int grid, const CrcIdxArgs& crc,
                               hipStream_t stream);
// write path, one pass: payload offsets + encode-view descriptors + slow list, the fast
// kernels with the all-fill test, the slow list through the generic encode, then the finish
// kernel (all-fill count, index entries, chunk-CRC descriptors); launch_crc with
// status == nullptr stores the index crc32c instead of checking it
// nested sharding on the one-pass write: per (shard, level-1 cell) {cell offset in the shard
// (-1: no in-bounds leaf, elided at level 1), sub-shard index offset}, and the cell geometry
struct EncNest {
  const int64_t* cell;          // 2 per (shard, cell); nullptr: single-level chain
  int64_t ncell;                // level-1 cells per shard
  int64_t sub_isz;              // sub-shard index bytes (16 per leaf, +4 with crc32c)
  int32_t r[kMaxDims];          // leaves per cell per dim
  int32_t g1[kMaxDims];         // cells per shard per dim
  int32_t sub_start;            // sub-shard index before the leaves
  int32_t sub_be;               // sub-shard index big-endian
};
hipError_t launch_encode_resolve(const ScatterArgs& a, const EncNest& nz, int64_t* item_off,
                                 int64_t base_off, int64_t cn, const uint8_t* vbase, int vfast,
                                 hipStream_t stream);
// group > 0: the grouped kernels over groups of `group` consecutive chunks (piece_shift 0;
// rows: group << fast_vpr_shift <= 64; view.item_mul over the groups)
hipError_t launch_encode_fast(const ScatterArgs& view, int grid, int group, hipStream_t stream);
hipError_t launch_encode_slow(const ScatterArgs& a, int grid, hipStream_t stream);
hipError_t launch_encode_finish(const ScatterArgs& a, const EncNest& nz, int64_t chunk_nbytes,
                                uint32_t* bad, ItemDesc* crc_desc, hipStream_t stream);
hipError_t launch_gather_blocks(void* dst, const void* src, const int64_t* d_idx, int64_t n,
                                int64_t bb, hipStream_t stream);
hipError_t launch_write_probe(void* dst, int64_t bytes, int pattern, hipStream_t stream);
hipError_t launch_copy_probe(void* dst, const void* src, int64_t bytes, hipStream_t stream);
hipError_t launch_synth_fill(void* dst, int64_t n, int dsize, int64_t first, uint64_t seed,
                             hipStream_t stream);
hipError_t launch_synth_verify(const void* region, int ndim, const int64_t* array_shape,
                               const int64_t* offset, const int64_t* shape, int dsize,
                               uint64_t seed, unsigned long long* d_count, hipStream_t stream);

}  // namespace zh
