// zh_pieces.cpp — sub-shard reads from the stored index and the referenced byte ranges.
//
// core.Array.read of a region that covers part of a shard reads, per shard, the index (one
// prefix or suffix read) and then each referenced inner chunk (StoreHandleDataProvider,
// M/v3/codec/core/ShardingIndexedCodec.java:190-230, 333-357).  zh_shard_ranges tells the
// binding which ranges to read; zh_array_read_pieces takes the stored index and those ranges
// as they came from the store.  The index crc32c and every entry are checked on the device
// (Crc32cCodec.java:24-48 → crc_index_kernel; ShardingIndexedCodec.java:215-230 →
// resolve_kernel), never on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "zh_ctx.h"

using namespace zh;

namespace zh {

// Entries of the part's box (level-1 cells for nested sharding, read whole), missing ones
// dropped, unreadable ones (negative, beyond a known shard size, longer than max_entry) left
// out, sorted by offset.  max_run > 0 (raw ranges): overlapping entries united and adjacent
// ones merged while a range stays within max_run bytes, and no range exceeds max_entry (an
// overlap that would continues as a new range from the previous end).  max_run == 0 (each
// range is read and decoded on its own by host stages): exact duplicates once, every other
// entry its own range, overlapping or not — the reference reads and decodes each entry
// separately (StoreHandleDataProvider.read, ShardingIndexedCodec.java:226-231, 353-356).
static int shard_ranges_impl(const zh_array_meta* m, const uint8_t* index, int64_t shard_nbytes,
                             const int64_t* part_lo, const int64_t* part_hi, int64_t max_run,
                             int64_t max_entry,
                             std::vector<std::pair<int64_t, int64_t>>& out) {
  out.clear();
  if (!m || !index || !part_lo || !part_hi || !m->chain.sharded) return ZH_EINVAL;
  const int n = m->ndim;
  if (n <= 0 || n > kMaxDims) return ZH_EINVAL;
  const int32_t* unit = m->chain.inner_chunk_shape;  // the entries the outer index holds
  int64_t cps[kMaxDims], b0[kMaxDims], cnt[kMaxDims], total = 1;
  for (int d = 0; d < n; d++) {
    if (unit[d] <= 0 || m->chunk_shape[d] % unit[d] != 0) return ZH_EINVAL;
    if (part_lo[d] < 0 || part_hi[d] <= part_lo[d] || part_hi[d] > m->chunk_shape[d])
      return ZH_EINVAL;
    cps[d] = m->chunk_shape[d] / unit[d];
    b0[d] = part_lo[d] / unit[d];  // ShardingIndexedCodec.java:206-208
    cnt[d] = (part_hi[d] - 1) / unit[d] - b0[d] + 1;
    total *= cnt[d];
  }
  const bool be = m->chain.index_endian == ZH_ENDIAN_BIG;
  std::vector<std::pair<int64_t, int64_t>> ents;
  ents.reserve((size_t)total);
  int64_t cur[kMaxDims] = {0};
  for (int64_t k = 0; k < total; k++) {
    int64_t lin = 0;
    for (int d = 0; d < n; d++) lin = lin * cps[d] + b0[d] + cur[d];
    const uint64_t off = ld_u64_host(index + 16 * lin, be);
    const uint64_t nb = ld_u64_host(index + 16 * lin + 8, be);
    for (int d = n - 1; d >= 0; d--) {
      if (++cur[d] < cnt[d]) break;
      cur[d] = 0;
    }
    if (off == ~0ull || nb == ~0ull) continue;  // missing (Q2): ShardingIndexedCodec.java:219-221
    if (off > (uint64_t)INT64_MAX || nb > (uint64_t)max_entry) continue;
    if (shard_nbytes >= 0 && (off > (uint64_t)shard_nbytes || nb > (uint64_t)shard_nbytes - off))
      continue;
    if (nb == 0) continue;
    ents.push_back({(int64_t)off, (int64_t)nb});
  }
  std::sort(ents.begin(), ents.end());
  for (const auto& e : ents) {
    if (!out.empty()) {
      auto& b = out.back();
      const int64_t bend = b.first + b.second, eend = e.first + e.second;
      if (max_run <= 0) {  // one range per entry: only exact duplicates collapse
        if (e == b) continue;
        out.push_back(e);
        continue;
      }
      if (e.first < bend) {  // overlapping entries (shared payloads): one range
        if (eend <= bend) continue;
        if (eend - b.first <= max_entry) {
          b.second = eend - b.first;
        } else {  // the union would exceed what one read may return: continue from bend
          out.push_back({bend, eend - bend});
        }
        continue;
      }
      if (e.first == bend && b.second + e.second <= max_run) {
        b.second += e.second;
        continue;
      }
    }
    out.push_back(e);
  }
  return ZH_OK;
}

int shard_ranges(const zh_array_meta* m, const uint8_t* index, int64_t shard_nbytes,
                 const int64_t* part_lo, const int64_t* part_hi, int64_t max_run,
                 std::vector<std::pair<int64_t, int64_t>>& out, int64_t max_entry) {
  return shard_ranges_impl(m, index, shard_nbytes, part_lo, part_hi, max_run, max_entry, out);
}

}  // namespace zh

namespace {

// zh_shard_src → planner source: missing, whole object (one piece at 0), or index + pieces
// (copied into `held`, which the call keeps until it returns).
int to_src(const zh_shard_src& s, int64_t i, SrcDesc& d, std::vector<Piece>& held, char* err,
           size_t errlen) {
  d = SrcDesc();
  if (s.npieces < 0 || (s.npieces > 0 && !s.pieces)) {
    set_err(err, errlen, "shard source %lld: invalid piece list", (long long)i);
    return ZH_EINVAL;
  }
  if (!s.index) {
    if (s.npieces == 0) return ZH_OK;  // missing key → fill_value
    const zh_shard_piece& q = s.pieces[0];
    if (s.npieces != 1 || q.offset != 0 || q.data_nbytes != q.nbytes || !q.data) {
      set_err(err, errlen,
              "shard source %lld: without its index a shard must be one whole piece at offset 0",
              (long long)i);
      return ZH_EINVAL;
    }
    d.data = SrcRef::memory(q.data);
    d.nbytes = q.nbytes;
    return ZH_OK;
  }
  d.index = (const uint8_t*)s.index;
  d.index_nbytes = s.index_nbytes;
  d.shard_nbytes = s.shard_nbytes;
  held.resize((size_t)s.npieces);
  for (int64_t k = 0; k < s.npieces; k++) {
    const zh_shard_piece& q = s.pieces[k];
    held[(size_t)k] = Piece{q.offset, q.nbytes, SrcRef::memory(q.data), q.data_nbytes};
  }
  d.pieces = held.data();
  d.npieces = s.npieces;
  return ZH_OK;
}

}  // namespace

extern "C" {

int64_t zh_shard_ranges(const zh_array_meta* meta, const void* index, int64_t index_nbytes,
                        int64_t shard_nbytes, const int64_t* part_lo, const int64_t* part_hi,
                        int64_t max_run, int64_t* ranges, int64_t cap) {
  if (!meta || !index || !meta->chain.sharded) return -ZH_EINVAL;
  const int64_t isz = zh_shard_index_size(meta);
  if (index_nbytes < isz) return -ZH_EINVAL;
  const uint8_t* ib = (const uint8_t*)index +
                      (meta->chain.index_location == ZH_INDEX_START ? 0 : index_nbytes - isz);
  // a Java ByteBuffer / byte[] holds at most 2^31 - 1 bytes: no entry or run beyond that
  const int64_t kJava = kIntMax;
  const int64_t run = std::min<int64_t>(std::max<int64_t>(0, max_run), kJava);
  std::vector<std::pair<int64_t, int64_t>> rs;
  const int st = shard_ranges_impl(meta, ib, shard_nbytes, part_lo, part_hi, run, kJava, rs);
  if (st != ZH_OK) return -st;
  for (size_t k = 0; ranges && k < rs.size() && (int64_t)k < cap; k++) {
    ranges[2 * k] = rs[k].first;
    ranges[2 * k + 1] = rs[k].second;
  }
  return (int64_t)rs.size();
}

int zh_array_read_pieces(zh_ctx* ctx, const zh_array_meta* meta, const zh_shard_src* shards,
                         int64_t nshards, const int64_t* offset, const int64_t* shape, void* out,
                         uint32_t flags, void* stream, char* err, size_t errlen) {
  if (!ctx || !meta) return ZH_EINVAL;
  if (!meta->chain.sharded) {
    set_err(err, errlen, "index + pieces sources need a sharding_indexed chain");
    return ZH_EINVAL;
  }
  if (nshards > 0 && !shards) return ZH_EINVAL;
  std::vector<SrcDesc> srcs((size_t)std::max<int64_t>(0, nshards));
  std::vector<std::vector<Piece>> held((size_t)std::max<int64_t>(0, nshards));
  for (int64_t i = 0; i < nshards; i++) {
    const int st = to_src(shards[i], i, srcs[(size_t)i], held[(size_t)i], err, errlen);
    if (st != ZH_OK) return st;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  return read_region(ctx, meta, srcs.data(), nshards, offset, shape, out, flags, stream, err,
                     errlen);
}

int zh_array_read_pieces_multi(zh_ctx* const* ctxs, int ndev, int root,
                               const zh_array_meta* meta, const zh_shard_src* shards,
                               int64_t nshards, const int64_t* offset, const int64_t* shape,
                               void* out, uint32_t flags, int32_t* slab_route, char* err,
                               size_t errlen) {
  if (!meta || (nshards > 0 && !shards)) return ZH_EINVAL;
  if (!meta->chain.sharded) {
    set_err(err, errlen, "index + pieces sources need a sharding_indexed chain");
    return ZH_EINVAL;
  }
  std::vector<SrcDesc> srcs((size_t)std::max<int64_t>(0, nshards));
  std::vector<std::vector<Piece>> held((size_t)std::max<int64_t>(0, nshards));
  for (int64_t i = 0; i < nshards; i++) {
    const int st = to_src(shards[i], i, srcs[(size_t)i], held[(size_t)i], err, errlen);
    if (st != ZH_OK) return st;
  }
  return read_multi_impl(ctxs, ndev, root, meta, srcs.data(), nshards, offset, shape, out, flags,
                         slab_route, err, errlen);
}

int zh_sharding_decode_pieces(zh_ctx* ctx, const zh_array_meta* meta, const zh_shard_src* shard,
                              const int64_t* offset, const int32_t* shape, void* out,
                              uint32_t flags, void* stream, char* err, size_t errlen) {
  if (!meta || !shard || !offset || !shape) return ZH_EINVAL;
  zh_array_meta sm = *meta;  // the shard viewed as a one-chunk array
  int64_t shp[kMaxDims];
  for (int d = 0; d < meta->ndim && d < kMaxDims; d++) {
    sm.shape[d] = meta->chunk_shape[d];
    shp[d] = shape[d];
  }
  return zh_array_read_pieces(ctx, &sm, shard, 1, offset, shp, out, flags, stream, err, errlen);
}

int zh_shard_index_check(const zh_array_meta* meta, const void* index, int64_t index_nbytes,
                         char* err, size_t errlen) {
  if (!meta || !index || !meta->chain.sharded) return ZH_EINVAL;
  if (!meta->chain.index_has_crc32c) return ZH_OK;
  const int64_t isz = zh_shard_index_size(meta);
  if (isz < 4 || index_nbytes < isz) return ZH_OK;  // the read reports the short index
  const uint8_t* ib = (const uint8_t*)index +
                      (meta->chain.index_location == ZH_INDEX_START ? 0 : index_nbytes - isz);
  const uint32_t computed = zh_crc32c(0, ib, (size_t)(isz - 4));
  const uint8_t* sp = ib + isz - 4;  // stored little-endian (Crc32cCodec.java:36-37)
  const uint32_t stored =
      (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) | ((uint32_t)sp[2] << 16) | ((uint32_t)sp[3] << 24);
  if (computed == stored) return ZH_OK;
  set_err(err, errlen, "The checksum of the sharding index is invalid. Stored: %d Computed: %d",
          (int32_t)stored, (int32_t)computed);  // Crc32cCodec.java:39-44 (signed ints)
  return ZH_EDATA;
}

int zh_host_staging(zh_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out) return ZH_EINVAL;
  *out = nullptr;
  // the same lock as every read on this context: a concurrent read never sees its staging
  // freed or replaced under its DMA
  std::lock_guard<std::mutex> lk(ctx->mu);
  (void)hipSetDevice(ctx->device);
  const size_t cap = (size_t)8192 << 20;  // at most 8 GiB of page-locked staging
  const size_t want = std::max<size_t>(bytes, 1);
  if (ctx->staging && (ctx->staging_oneoff || want > ctx->staging_cap)) {
    (void)hipHostFree(ctx->staging);
    ctx->staging = nullptr;
    ctx->staging_cap = 0;
    ctx->staging_oneoff = false;
  }
  if (!ctx->staging) {
    const size_t g = (size_t)64 << 20;  // grow in 64 MiB steps
    const size_t sz = want > cap ? want : std::min(cap, (want + g - 1) / g * g);
    if (hipHostMalloc(&ctx->staging, sz, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      ctx->staging = nullptr;
      return ZH_ENOMEM;
    }
    ctx->staging_cap = sz;
    ctx->staging_oneoff = want > cap;
  }
  *out = ctx->staging;
  return ZH_OK;
}

}  // extern "C"
