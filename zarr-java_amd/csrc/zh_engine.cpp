// zh_engine.cpp — host side of the MI355X Zarr v3 chunk codec path and its C-ABI
// (include/zarrhip.h).
//
// The planner restates the host half of core.Array.read (M/core/Array.java:378-441):
// domain check, chunk enumeration (IndexingUtils.computeChunkCoords :16-51), outer
// projection (computeProjection :65-117) and, per shard, the inner-chunk box that
// ShardingIndexedCodec.decodeInternal (:206-208) iterates.  Everything per element —
// index CRC, index parse, endian swap, transpose, scatter — runs on the GPU in
// zh_kernels.hip.  There is no CPU fallback: if the device is unusable every entry point
// fails with ZH_EHIP.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <array>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "zh_ctx.h"

using namespace zh;

namespace zh {



// the last message of a call made without an error buffer (zh_plan_execute), per thread
thread_local char g_quiet_err[256];

void set_err(char* err, size_t errlen, const char* fmt, ...) {
  if (!err || errlen == 0) {
    err = g_quiet_err;
    errlen = sizeof g_quiet_err;
  }
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err, errlen, fmt, ap);
  va_end(ap);
}

// A SrcRef used as the wrong kind is a planner bug: stop before a store file offset is
// dereferenced as an address (or an address read as a file).
void src_ref_misuse(const char* what) {
  fprintf(stderr, "zarrhip: internal error: %s\n", what);
  abort();
}

#define ZH_HIP(call)                                                                       \
  do {                                                                                     \
    hipError_t e_ = (call);                                                                \
    if (e_ != hipSuccess) {                                                                \
      set_err(err, errlen, "HIP error %s at %s:%d (%s)", hipGetErrorName(e_), __FILE__,     \
              __LINE__, hipGetErrorString(e_));                                            \
      return ZH_EHIP;                                                                      \
    }                                                                                      \
  } while (0)

std::string fmt_ints(const int64_t* v, int n) {  // java.util.Arrays.toString
  std::string s = "[";
  for (int i = 0; i < n; i++) {
    if (i) s += ", ";
    s += std::to_string((long long)v[i]);
  }
  return s + "]";
}
std::string fmt_ints32(const int32_t* v, int n) {
  std::vector<int64_t> t(v, v + n);
  return fmt_ints(t.data(), n);
}

// ---- CRC-32C (host; slicing-by-8 over the reference's table, CRC32C.java:14-80) ----
struct CrcTables {
  uint32_t t[8][256];
  CrcTables() {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
      t[0][i] = c;
    }
    for (int k = 1; k < 8; k++)
      for (int i = 0; i < 256; i++) t[k][i] = (t[k - 1][i] >> 8) ^ t[0][t[k - 1][i] & 0xFF];
  }
};
const CrcTables& crc_tables() {
  static CrcTables T;
  return T;
}

uint32_t crc32c_host(uint32_t crc, const uint8_t* p, size_t n) {
  const auto& T = crc_tables().t;
  uint32_t c = crc ^ 0xFFFFFFFFu;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    uint32_t lo = (uint32_t)w ^ c, hi = (uint32_t)(w >> 32);
    c = T[7][lo & 0xFF] ^ T[6][(lo >> 8) & 0xFF] ^ T[5][(lo >> 16) & 0xFF] ^ T[4][lo >> 24] ^
        T[3][hi & 0xFF] ^ T[2][(hi >> 8) & 0xFF] ^ T[1][(hi >> 16) & 0xFF] ^ T[0][hi >> 24];
  }
  for (; i < n; i++) c = T[0][(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

// GF(2) arithmetic mod the reflected CRC-32C polynomial (the device's multmodp/x2nmodp):
// a(x)·b(x) mod P, and x^(8n) mod P = the shift of a raw CRC register past n zero bytes.
uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ 0x82F63B78u : b >> 1;
  }
  return p;
}
uint32_t gf2_xpow8n(uint64_t n) {
  uint32_t p = 1u << 31, sq = 1u << 23;  // x^0, x^8 (reflected)
  while (n) {
    if (n & 1) p = gf2_mulmod(sq, p);
    sq = gf2_mulmod(sq, sq);
    n >>= 1;
  }
  return p;
}

// The tile kernels' fused chunk CRC: when every unit u + kTG (the same lane's next group)
// ends a constant Δ bytes after unit u, a lane folds its groups as r = r·x^(8Δ) ⊕ acc and
// multiplies by its last unit's K once per piece; returns x^(8Δ) (0 = irregular layout,
// the kernel then multiplies every group by its K).
uint32_t tile_crc_step(const std::vector<int64_t>& ends, size_t kGroup = 8 /* kTG */) {
  if (ends.size() <= kGroup) return 0;
  const int64_t delta = ends[kGroup] - ends[0];
  if (delta <= 0) return 0;
  for (size_t u = 0; u + kGroup < ends.size(); u++)
    if (ends[u + kGroup] - ends[u] != delta) return 0;
  return gf2_xpow8n((uint64_t)delta);
}

// ---- IndexingUtils (M/utils/IndexingUtils.java) ----
int64_t chunk_coords(int n, const int32_t* chunk, const int64_t* off, const int64_t* shp,
                     int64_t* start, int64_t* count) {
  int64_t num = 1;
  for (int d = 0; d < n; d++) {  // :22-28 (int casts reproduced)
    int64_t s = (int64_t)(int32_t)(off[d] / chunk[d]);
    int64_t e = (int64_t)(int32_t)((off[d] + shp[d] - 1) / chunk[d]);
    start[d] = s;
    count[d] = e - s + 1;
    num *= count[d];
  }
  return num;
}

int projection(int n, const int64_t* cc, const int64_t* ashape, const int32_t* chunk,
               const int64_t* soff, const int64_t* sshape, int32_t* co, int32_t* oo,
               int32_t* ps) {
  for (int d = 0; d < n; d++) {
    const int64_t dim_off = (int64_t)chunk[d] * cc[d];
    const int64_t dim_limit = std::min(ashape[d], (cc[d] + 1) * (int64_t)chunk[d]);
    if (soff[d] < dim_off) {
      co[d] = 0;
      int64_t v = dim_off - soff[d];
      if (v > kIntMax) return ZH_EARITH;
      oo[d] = (int32_t)v;
    } else {
      int64_t v = soff[d] - dim_off;
      if (v > kIntMax) return ZH_EARITH;
      co[d] = (int32_t)v;
      oo[d] = 0;
    }
    if (soff[d] + sshape[d] > dim_limit) {
      ps[d] = chunk[d] - co[d];
    } else {
      int64_t v = soff[d] + sshape[d] - dim_off - co[d];
      if (v > kIntMax || v < 0) return ZH_EARITH;
      ps[d] = (int32_t)v;
    }
  }
  return ZH_OK;
}

bool is_perm(int n, const int32_t* o) {
  if (n <= 0 || n > kMaxDims) return false;
  bool seen[kMaxDims] = {false};
  for (int i = 0; i < n; i++) {
    if (o[i] < 0 || o[i] >= n || seen[o[i]]) return false;
    seen[o[i]] = true;
  }
  return true;
}

uint32_t next_pow2_shift(uint64_t v) {
  uint32_t s = 0;
  while ((1ull << s) < v) s++;
  return s;
}

int env_int(const char* name, int def) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : def;
}

}  // namespace zh


namespace zh {
constexpr size_t kCacheMaxBlock = (size_t)4 << 30;   // larger blocks go back to the runtime
constexpr size_t kCacheMaxTotal = (size_t)8 << 30;

size_t cache_round(size_t bytes) {  // 64 KiB granules below 64 MiB, 2 MiB above
  const size_t g = bytes < ((size_t)64 << 20) ? ((size_t)64 << 10) : ((size_t)2 << 20);
  return (bytes + g - 1) / g * g;
}

// a device block of at least `bytes` (returned size in *got): a cached block of up to 1.25x
// the request, else hipMalloc
hipError_t ctx_alloc(zh_ctx* ctx, size_t bytes, void** p, size_t* got) {
  const size_t want = cache_round(bytes);
  {
    std::lock_guard<std::mutex> lk(ctx->cache_mu);
    auto it = ctx->cache.lower_bound(want);
    if (it != ctx->cache.end() && it->first <= want + want / 4) {
      *p = it->second;
      *got = it->first;
      ctx->cache_bytes -= it->first;
      ctx->cache.erase(it);
      return hipSuccess;
    }
  }
  *got = want;
  hipError_t e = hipMalloc(p, want);
  if (e == hipErrorOutOfMemory) {  // give the cached blocks back and try once more
    std::lock_guard<std::mutex> lk(ctx->cache_mu);
    for (auto& kv : ctx->cache) (void)hipFree(kv.second);
    ctx->cache.clear();
    ctx->cache_bytes = 0;
    e = hipMalloc(p, want);
  }
  return e;
}

void ctx_release(zh_ctx* ctx, void* p, size_t bytes) {
  if (!p) return;
  if (bytes <= kCacheMaxBlock) {
    std::lock_guard<std::mutex> lk(ctx->cache_mu);
    if (ctx->cache_bytes + bytes <= kCacheMaxTotal) {
      ctx->cache.emplace(bytes, p);
      ctx->cache_bytes += bytes;
      return;
    }
  }
  (void)hipFree(p);
}
}  // namespace zh


extern "C" {

const char* zh_version(void) { return "zarrhip 0.1.0 (gfx950)"; }

int zh_ctx_create(int device, zh_ctx** out) {
  char* err = nullptr;
  size_t errlen = 0;
  if (!out) return ZH_EINVAL;
  *out = nullptr;
  int ndev = 0;
  ZH_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return ZH_EINVAL;
  ZH_HIP(hipSetDevice(device));
  zh_ctx* c = new zh_ctx();
  c->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->cu_count = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return ZH_EHIP;
  }
  *out = c;
  return ZH_OK;
}

void zh_ctx_destroy(zh_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->status_pin) (void)hipHostFree(c->status_pin);
  if (c->upload_pin) (void)hipHostFree(c->upload_pin);
  if (c->file_pin) (void)hipHostFree(c->file_pin);
  if (c->hout_pin) (void)hipHostFree(c->hout_pin);
  if (c->wscratch) (void)hipFree(c->wscratch);
  for (auto& kv : c->cache) (void)hipFree(kv.second);
  pipeline_release(c);
  delete c;
}

int zh_ctx_device(const zh_ctx* c) { return c ? c->device : -1; }
void* zh_ctx_stream(zh_ctx* c) { return c ? (void*)c->stream : nullptr; }

int64_t zh_ctx_release_cache(zh_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  std::lock_guard<std::mutex> lk(c->cache_mu);
  const int64_t n = (int64_t)c->cache_bytes;
  for (auto& kv : c->cache) (void)hipFree(kv.second);
  c->cache.clear();
  c->cache_bytes = 0;
  return n;
}

// =====================================================================================
// host helpers
// =====================================================================================
uint32_t zh_crc32c(uint32_t crc, const void* data, size_t n) {
  return crc32c_host(crc, (const uint8_t*)data, n);
}

int64_t zh_compute_chunk_coords(int ndim, const int64_t* array_shape, const int32_t* chunk_shape,
                                const int64_t* sel_offset, const int64_t* sel_shape,
                                int64_t* coords_out, int64_t max_coords) {
  (void)array_shape;
  if (ndim <= 0 || ndim > kMaxDims) return -1;
  int64_t start[kMaxDims], count[kMaxDims];
  int64_t num = chunk_coords(ndim, chunk_shape, sel_offset, sel_shape, start, count);
  if (num > kIntMax) return -1;  // :30-32
  if (coords_out) {
    int64_t cur[kMaxDims] = {0};
    for (int64_t i = 0; i < num && i < max_coords; i++) {
      for (int d = 0; d < ndim; d++) coords_out[i * ndim + d] = start[d] + cur[d];
      for (int d = ndim - 1; d >= 0; d--) {
        if (++cur[d] < count[d]) break;
        cur[d] = 0;
      }
    }
  }
  return num;
}

int zh_compute_projection(int ndim, const int64_t* chunk_coords, const int64_t* array_shape,
                          const int32_t* chunk_shape, const int64_t* sel_offset,
                          const int64_t* sel_shape, int32_t* chunk_offset_out,
                          int32_t* out_offset_out, int32_t* shape_out) {
  if (ndim <= 0 || ndim > kMaxDims) return ZH_EINVAL;
  return projection(ndim, chunk_coords, array_shape, chunk_shape, sel_offset, sel_shape,
                    chunk_offset_out, out_offset_out, shape_out);
}

int zh_is_permutation(int n, const int32_t* order) { return is_perm(n, order) ? 1 : 0; }

int zh_inverse_permutation(int n, const int32_t* order, int32_t* inverse_out) {
  if (!is_perm(n, order)) return ZH_EINVAL;
  for (int i = 0; i < n; i++) inverse_out[order[i]] = i;
  return ZH_OK;
}

int64_t zh_shard_index_size(const zh_array_meta* m) {
  if (!m || !m->chain.sharded) return -1;
  int64_t n = 1;
  for (int d = 0; d < m->ndim; d++) n *= m->chunk_shape[d] / m->chain.inner_chunk_shape[d];
  return 16 * n + (m->chain.index_has_crc32c ? 4 : 0);  // ShardingIndexedCodec.java:176-181
}

int zh_validate_meta(const zh_array_meta* m, char* err, size_t errlen) {
  if (!m) return ZH_EINVAL;
  const int n = m->ndim;
  if (n <= 0 || n > kMaxDims) {
    set_err(err, errlen, "ndim %d not supported (1..%d)", n, kMaxDims);
    return ZH_EUNSUPPORTED;
  }
  if (m->dtype_size != 1 && m->dtype_size != 2 && m->dtype_size != 4 && m->dtype_size != 8) {
    set_err(err, errlen, "dtype size %d not supported", m->dtype_size);
    return ZH_EUNSUPPORTED;
  }
  for (int d = 0; d < n; d++) {
    if (m->shape[d] < 0 || m->chunk_shape[d] <= 0) {
      set_err(err, errlen, "invalid shape/chunk shape at dimension %d", d);
      return ZH_EINVAL;
    }
  }
  const zh_codec_chain& c = m->chain;
  const int32_t* inner = c.sharded ? c.inner_chunk_shape : m->chunk_shape;
  if (c.sharded) {  // v3/ArrayMetadata.java:102-116
    for (int d = 0; d < n; d++) {
      if (inner[d] <= 0 || m->chunk_shape[d] % inner[d] != 0) {
        set_err(err, errlen,
                "Sharding inner chunk shape %s does not evenly divide the outer chunk size %s",
                fmt_ints32(inner, n).c_str(), fmt_ints32(m->chunk_shape, n).c_str());
        return ZH_EDATA;
      }
    }
    if (c.index_location != ZH_INDEX_START && c.index_location != ZH_INDEX_END) {
      set_err(err, errlen, "Only index_location \"start\" or \"end\" are supported.");
      return ZH_EDATA;  // ShardingIndexedCodec.java:288-293
    }
    if (c.nested) {  // the level-2 codec validates against its own "shard" (the inner chunk)
      for (int d = 0; d < n; d++) {
        if (c.nested_chunk_shape[d] <= 0 || inner[d] % c.nested_chunk_shape[d] != 0) {
          set_err(err, errlen,
                  "Sharding inner chunk shape %s does not evenly divide the outer chunk size %s",
                  fmt_ints32(c.nested_chunk_shape, n).c_str(), fmt_ints32(inner, n).c_str());
          return ZH_EDATA;
        }
      }
      if (c.nested_index_location != ZH_INDEX_START && c.nested_index_location != ZH_INDEX_END) {
        set_err(err, errlen, "Only index_location \"start\" or \"end\" are supported.");
        return ZH_EDATA;
      }
    }
  } else if (c.nested) {
    set_err(err, errlen, "nested sharding requires an outer sharding codec");
    return ZH_EINVAL;
  }
  if (c.has_transpose && !is_perm(n, c.transpose_order)) {
    set_err(err, errlen, "Order is no permutation array");  // TransposeCodec.java:36-38
    return ZH_EDATA;
  }
  int64_t nel = 1;
  for (int d = 0; d < n; d++) nel *= inner[d];
  if (nel >= kIntMax) {  // ucar.ma2.Array / Java int limits: one inner chunk < 2^31 elements
    set_err(err, errlen, "inner chunk of %lld elements exceeds the 2^31 element limit",
            (long long)nel);
    return ZH_EUNSUPPORTED;
  }
  return ZH_OK;
}

}  // extern "C"

// =====================================================================================
// planning
// =====================================================================================
namespace zh {

// Shape of the chunks the scatter kernels move: the chunk (unsharded), the inner chunk
// (sharded) or the leaf of the level-2 shard (nested: the flattened leaf grid).
const int32_t* leaf_shape(const zh_array_meta* m) {
  const zh_codec_chain& c = m->chain;
  if (!c.sharded) return m->chunk_shape;
  return c.nested ? c.nested_chunk_shape : c.inner_chunk_shape;
}

void fill_common_args(const zh_array_meta* m, const int64_t* region_shape, bool encode,
                      ScatterArgs& a, int& tile_mode) {
  const int n = m->ndim;
  const zh_codec_chain& c = m->chain;
  const int32_t* inner = leaf_shape(m);
  int32_t order[kMaxDims];
  for (int d = 0; d < n; d++) order[d] = c.has_transpose ? c.transpose_order[d] : d;
  memset(&a, 0, sizeof(a));
  a.ndim = n;
  a.swap = (m->dtype_size > 1 && c.endian == ZH_ENDIAN_BIG) ? 1 : 0;
  a.is_bool = m->dtype_is_bool ? 1 : 0;
  a.index_be = c.index_endian == ZH_ENDIAN_BIG ? 1 : 0;
  a.sharded = c.sharded ? 1 : 0;
  // payload: C-order over P[j] = inner[order[j]] (TransposeCodec.java:70-71)
  int64_t st = 1;
  for (int j = n - 1; j >= 0; j--) {
    a.pstride[order[j]] = st;
    st *= inner[order[j]];
  }
  st = 1;
  for (int d = n - 1; d >= 0; d--) {
    a.rstride[d] = st;
    st *= region_shape[d];
  }
  st = 1;
  for (int d = n - 1; d >= 0; d--) {
    a.cps_stride[d] = st;
    a.rank.cps_stride[d] = st;
    st *= c.sharded ? (m->chunk_shape[d] / inner[d]) : 1;
  }
  a.rank.ndim = n;  // single level; plan creation adds the nested geometry
  int64_t nel = 1;
  for (int d = 0; d < n; d++) {
    a.inner[d] = inner[d];
    a.inner_div[d] = make_fastdiv((uint32_t)inner[d]);
    nel *= inner[d];
  }
  for (int d = n; d < kMaxDims; d++) {
    a.inner[d] = 1;
    a.inner_div[d] = make_fastdiv(1);
  }
  a.inner_nbytes = nel * m->dtype_size;
  a.crc_extra = c.inner_crc32c ? 4 : 0;
  a.dsize = m->dtype_size;
  uint64_t f = 0;
  for (int i = 0; i < 8; i++) f |= (uint64_t)m->fill_value[i] << (8 * i);
  a.fill = f;
  // the write path's all-fill test compares as Java's == (MultiArrayUtils.allValuesEqual,
  // M/utils/MultiArrayUtils.java:69-80, 104-150): for a float ±0 fill, +0.0 == -0.0
  // (a NaN fill equals nothing: every chunk is kept, fill_never)
  a.fill_mask = ~0ull;
  a.fill_never = 0;
  if (m->dtype_is_float && (m->dtype_size == 4 || m->dtype_size == 8)) {
    const bool d8 = m->dtype_size == 8;
    const uint64_t sign = 1ull << (8 * m->dtype_size - 1);
    const uint64_t mag = f & (d8 ? ~0ull : 0xFFFFFFFFull) & ~sign;
    const uint64_t inf = d8 ? 0x7FF0000000000000ull : 0x7F800000ull;
    if (mag == 0) a.fill_mask = ~sign;
    if (mag > inf) a.fill_never = 1;
  }
  if (encode) {
    a.fs = n - 1;
    a.fd = order[n - 1];
  } else {
    a.fs = order[n - 1];
    a.fd = n - 1;
  }
  tile_mode = a.fs != a.fd;
  a.tile = tile_mode;
  // Work-item size along a large inner chunk: 2 MiB pieces (c2's 4 GiB chunks: decode 33.5 →
  // 32.65 ms against 128 KiB, 512 KiB 32.77, 4 MiB 32.90, 8 MiB 33.05; encode view 40.66 →
  // 39.38 ms; interleaved A/B, profiles/r02/experiments/ab_c2_piece*.json).  Chunks of at most
  // 2 MiB (c3, c4: 128 KiB) are one piece either way.
  const int64_t piece_kb = std::max(1, env_int("ZH_PIECE_KB", 2048));
  const uint64_t pieces = (uint64_t)((a.inner_nbytes + piece_kb * 1024 - 1) / (piece_kb * 1024));
  a.piece_shift = (int32_t)next_pow2_shift(std::max<uint64_t>(1, pieces));
}

// Chooses the decode fast path for unclipped inner chunks and fills its launch-uniform
// parameters: rows along the unit-stride dim mapped by shift/mask arithmetic (power-of-two
// row extents, <= 3 row dims) or by a (src, dst) offset table, or 32x32 transpose tiles
// from a table.  Returns the table (empty when the mode needs none).
std::vector<uint32_t> setup_fast(const zh_array_meta* m, ScatterArgs& a, int tile_mode) {
  const int n = m->ndim, ds = m->dtype_size;
  const int64_t kMaxEntries = 4096;
  std::vector<uint32_t> tab;
  auto fits = [](int64_t v) { return v >= 0 && v < (1ll << 32); };
  a.fast_mode = kFastNone;
  a.fast_n = 0;
  a.rm_n = 0;
  if (!tile_mode) {
    const int F = a.fs;
    const int64_t rowb = (int64_t)a.inner[F] * ds;
    if (rowb % 16) return {};
    const int64_t vpr = rowb / 16;
    if (vpr > kBlock || (vpr & (vpr - 1))) return {};
    int64_t rows = 1;
    std::vector<int> rdims;  // innermost first
    for (int d = n - 1; d >= 0; d--) {
      if (d == F) continue;
      rows *= a.inner[d];
      if (a.inner[d] > 1) {
        if ((a.pstride[d] * ds) % 16 || (a.rstride[d] * ds) % 16) return {};
        rdims.push_back(d);
      }
    }
    a.fast_vpr_shift = (int32_t)next_pow2_shift((uint64_t)vpr);
    a.fast_rows = (int32_t)rows;
    bool pow2 = rdims.size() <= 3;
    for (int d : rdims) pow2 &= (a.inner[d] & (a.inner[d] - 1)) == 0;
    if (pow2 && rows < (1ll << 31)) {
      a.fast_mode = kFastRowArith;
      a.rm_n = (int32_t)rdims.size();
      for (size_t i = 0; i < rdims.size(); i++) {
        a.rm_shift[i] = (int32_t)next_pow2_shift((uint64_t)a.inner[rdims[i]]);
        a.rm_sstr[i] = a.pstride[rdims[i]];
        a.rm_dstr[i] = a.rstride[rdims[i]];
      }
      return {};
    }
    if (rows > kMaxEntries) return {};
    for (int64_t r = 0; r < rows; r++) {
      int64_t rr = r, so = 0, dof = 0;
      for (int d = n - 1; d >= 0; d--) {
        if (d == F) continue;
        const int64_t mm = rr % a.inner[d];
        rr /= a.inner[d];
        so += mm * a.pstride[d];
        dof += mm * a.rstride[d];
      }
      if (!fits(so) || !fits(dof)) return {};
      tab.push_back((uint32_t)so);
      tab.push_back((uint32_t)dof);
    }
    a.fast_mode = kFastRowTable;
    a.fast_n = (int32_t)rows;
    return tab;
  }
  const int fs = a.fs, fd = a.fd;
  if (ds != 4 || a.inner[fs] % 32 || a.inner[fd] % 32) return {};
  if (a.pstride[fd] % 4 || a.rstride[fs] % 4) return {};
  const int64_t ts = a.inner[fs] / 32, td = a.inner[fd] / 32;
  int64_t nb = 1;
  for (int d = 0; d < n; d++)
    if (d != fs && d != fd) nb *= a.inner[d];
  // the tile kernels keep the table next to 8 LDS tiles (33.8 KB): stay within 64 KiB of
  // dynamic LDS (larger inner chunks take the generic kernel)
  if (nb * ts * td > kMaxEntries - 256) return {};
  for (int64_t u = 0; u < nb * ts * td; u++) {
    const int64_t ud = u % td, us = (u / td) % ts;
    int64_t b = u / (td * ts);
    int64_t so = us * 32 * a.pstride[fs] + ud * 32 * a.pstride[fd];
    int64_t dof = us * 32 * a.rstride[fs] + ud * 32 * a.rstride[fd];
    for (int d = n - 1; d >= 0; d--) {
      if (d == fs || d == fd) continue;
      const int64_t mm = b % a.inner[d];
      b /= a.inner[d];
      so += mm * a.pstride[d];
      dof += mm * a.rstride[d];
    }
    if (!fits(so) || !fits(dof) || so % 4 || dof % 4) return {};
    tab.push_back((uint32_t)so);
    tab.push_back((uint32_t)dof);
  }
  a.fast_mode = kFastTileTable;
  a.fast_n = (int32_t)(nb * ts * td);
  a.fast_rows = a.fast_n;
  return tab;
}

// Multiplier of the golden-ratio visit order of the fast kernels (item i → i·m mod t, m odd
// and coprime to t); 0 = natural order.
uint64_t golden_item_mul(int64_t total) {
  if (total <= 1) return 0;
  const uint64_t t = (uint64_t)total;
  uint64_t m = ((uint64_t)((double)t * 0.6180339887498949)) | 1;
  auto gcd = [](uint64_t x, uint64_t y) {
    while (y) {
      const uint64_t r = x % y;
      x = y;
      y = r;
    }
    return x;
  };
  while (gcd(m, t) != 1) m += 2;
  return m % t;
}

// Index-CRC spans: 4 KiB per workgroup when the indexes are few (a small read: a 512 KiB
// index in 128 workgroups instead of 8, the span CRC no longer latency-bound), 64 KiB when
// there are enough spans to fill the chip anyway (each workgroup also loads 12 KiB of tables).
// Sets every job's span_begin; returns the span count, *shift = log2(span / kIdxSpan).
int64_t assign_crc_spans(std::vector<CrcJob>& jobs, int cu_count, int* shift) {
  int64_t small = 0;
  for (const CrcJob& J : jobs) small += (J.len + kIdxSpan - 1) / kIdxSpan;
  *shift = small >= 4 * (int64_t)cu_count ? 4 : 0;
  const int64_t span = (int64_t)kIdxSpan << *shift;
  int64_t spans = 0;
  for (CrcJob& J : jobs) {
    J.span_begin = spans;
    spans += (J.len + span - 1) / span;
  }
  return spans;
}

int grid_for(const zh_ctx* ctx, int64_t total_items) {
  int64_t g = (int64_t)ctx->cu_count * 256;  // grid-stride kernels: 256 workgroups per CU
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, total_items));
}

template <typename T>
int dev_alloc(T** p, size_t count, char* err, size_t errlen) {
  *p = nullptr;
  if (count == 0) return ZH_OK;
  hipError_t e = hipMalloc((void**)p, count * sizeof(T));
  if (e != hipSuccess) {
    set_err(err, errlen, "hipMalloc(%zu bytes) failed: %s", count * sizeof(T),
            hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? ZH_ENOMEM : ZH_EHIP;
  }
  return ZH_OK;
}

// a plan buffer from the context's block cache (released by plan_free)
template <typename T>
int plan_alloc(zh_plan* p, T** ptr, size_t count, char* err, size_t errlen) {
  *ptr = nullptr;
  if (count == 0) return ZH_OK;
  void* q = nullptr;
  size_t got = 0;
  hipError_t e = ctx_alloc(p->ctx, count * sizeof(T), &q, &got);
  if (e != hipSuccess) {
    set_err(err, errlen, "hipMalloc(%zu bytes) failed: %s", count * sizeof(T),
            hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? ZH_ENOMEM : ZH_EHIP;
  }
  p->blocks.emplace_back(q, got);
  *ptr = (T*)q;
  return ZH_OK;
}

uint64_t ld_u64_host(const uint8_t* p, bool be) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (be ? 56 - 8 * i : 8 * i);
  return v;
}

// The bytes of one stored shard the device will hold: the stored index and the byte ranges
// of the shard it needs (sub-shard reads), or the whole object.
struct HeldPieces {
  const uint8_t* index = nullptr;       // the stored index (isz bytes), host or device
  std::vector<Piece> pieces;            // sorted, disjoint
};

// Host whole-shard sources, single-level sharding: StoreHandleDataProvider semantics
// (ShardingIndexedCodec.java:333-357) inside the planner.  The stored index is read on the
// host only to know which ranges the part references (shard_ranges, adjacent ranges merged);
// the device gets the stored index unchanged plus those ranges, checks the index crc32c and
// resolves every entry against the ranges (an entry outside them reads as the reference's
// "Could not load byte data").  Returns false when the part references over 90 % of the
// shard: the whole object is copied then.
bool compact_pieces(const zh_array_meta* m, const DevShard& S, int64_t isz, HeldPieces& hp) {
  int64_t lo[kMaxDims], hi[kMaxDims];
  for (int d = 0; d < m->ndim; d++) {
    lo[d] = S.part_lo[d];
    hi[d] = S.part_hi[d];
  }
  std::vector<std::pair<int64_t, int64_t>> rs;
  if (shard_ranges(m, S.data + S.index_off, S.nbytes, lo, hi, INT64_MAX, rs) != ZH_OK)
    return false;
  int64_t ref = isz;
  for (auto& r : rs) ref += r.second;
  // H2D is bandwidth-bound: compacting pays whenever it skips a tenth of the shard
  if (10 * ref > 9 * S.nbytes) return false;
  hp.index = S.data + S.index_off;
  hp.pieces.clear();
  for (auto& r : rs)
    hp.pieces.push_back({r.first, r.second, SrcRef::memory(S.data + r.first), r.second});
  return true;
}

int caller_pieces_all(const zh_array_meta* m, const SrcDesc& src, int64_t isz, const int64_t* cc,
                      HeldPieces& hp, char* err, size_t errlen);

// Validates a caller's sub-shard form (zh_shard_src) and collects its pieces.  For host
// sources only what this part references is kept (a pipelined read plans one part per slab,
// and each slab must copy only its own ranges): the caller's raw pieces cut to the ranges
// the stored index names for the part (read on the host only to know what to copy; checked
// on the device), host-decoded pieces kept whole when referenced.
int caller_pieces(const zh_array_meta* m, const SrcDesc& src, int64_t isz, const int64_t* cc,
                  const DevShard& S, bool src_dev, HeldPieces& hp, char* err, size_t errlen) {
  int st = caller_pieces_all(m, src, isz, cc, hp, err, errlen);
  if (st != ZH_OK || src_dev) return st;
  int64_t lo[kMaxDims], hi[kMaxDims];
  for (int d = 0; d < m->ndim; d++) {
    lo[d] = S.part_lo[d];
    hi[d] = S.part_hi[d];
  }
  std::vector<std::pair<int64_t, int64_t>> need;
  if (shard_ranges(m, hp.index, src.shard_nbytes, lo, hi, INT64_MAX, need) != ZH_OK) return ZH_OK;
  std::vector<Piece> kept;
  size_t r = 0;
  for (const Piece& q : hp.pieces) {
    const int64_t qe = q.offset + q.nbytes;
    while (r < need.size() && need[r].first + need[r].second <= q.offset) r++;
    for (size_t k = r; k < need.size() && need[k].first < qe; k++) {
      const int64_t a = std::max(q.offset, need[k].first);
      const int64_t b = std::min(qe, need[k].first + need[k].second);
      if (b <= a) continue;
      if (q.data_nbytes != q.nbytes) {  // one host-decoded chunk: whole or nothing
        kept.push_back(q);
        break;
      }
      kept.push_back({a, b - a, q.data + (a - q.offset), b - a});
    }
  }
  hp.pieces.swap(kept);
  return ZH_OK;
}

int caller_pieces_all(const zh_array_meta* m, const SrcDesc& src, int64_t isz, const int64_t* cc,
                      HeldPieces& hp, char* err, size_t errlen) {
  const int n = m->ndim;
  if (src.index_nbytes < isz) {  // worded as for a whole shard when its size is known
    if (src.shard_nbytes >= 0)
      set_err(err, errlen, "Shard %s of %lld bytes is smaller than its index (%lld bytes).",
              fmt_ints(cc, n).c_str(), (long long)src.shard_nbytes, (long long)isz);
    else
      set_err(err, errlen, "Shard %s is smaller than its index (%lld bytes).",
              fmt_ints(cc, n).c_str(), (long long)isz);
    return ZH_EDATA;
  }
  hp.index = src.index + (m->chain.index_location == ZH_INDEX_START ? 0 : src.index_nbytes - isz);
  hp.pieces.assign(src.pieces, src.pieces + std::max<int64_t>(0, src.npieces));
  for (size_t k = 0; k < hp.pieces.size(); k++) {
    const Piece& q = hp.pieces[k];
    // disjoint, except host-decoded pieces among themselves at distinct offsets: each serves
    // exactly the entry it was read for (piece_src), as the reference decodes each entry
    const bool dec = q.data_nbytes != q.nbytes;
    const bool overlap =
        k > 0 && (q.offset < hp.pieces[k - 1].offset + hp.pieces[k - 1].nbytes) &&
        !(dec && hp.pieces[k - 1].data_nbytes != hp.pieces[k - 1].nbytes &&
          q.offset > hp.pieces[k - 1].offset);
    const bool bad = q.offset < 0 || q.nbytes < 0 || q.data_nbytes < 0 ||
                     (q.data_nbytes > 0 && q.data.empty()) || overlap ||
                     (k > 0 && q.offset < hp.pieces[k - 1].offset) || (dec && m->chain.nested);
    if (bad) {
      set_err(err, errlen,
              "shard %s: piece %lld (offset %lld, %lld bytes, %lld held) is invalid: pieces "
              "must be sorted by offset, disjoint (host-decoded ones: distinct offsets), and "
              "hold their bytes (host-decoded pieces only below single-level sharding)",
              fmt_ints(cc, n).c_str(), (long long)k, (long long)q.offset, (long long)q.nbytes,
              (long long)q.data_nbytes);
      return ZH_EINVAL;
    }
  }
  return ZH_OK;
}

// A page-locked status slot of the context for plans of at most 32 shards (−1: none; the plan
// then reads its status back with a blocking copy).
static int status_slot_take(zh_ctx* c, int64_t nshards) {
  if (nshards * kStWords > kStatusSlotWords) return -1;
  std::lock_guard<std::mutex> lk(c->status_mu);
  if (!c->status_pin && !c->status_failed) {
    void* h = nullptr;
    if (hipHostMalloc(&h, (size_t)kStatusSlots * kStatusSlotWords * sizeof(uint64_t)) != hipSuccess) {
      c->status_failed = true;
      return -1;
    }
    c->status_pin = (uint64_t*)h;
    for (int i = kStatusSlots - 1; i >= 0; i--) c->status_free.push_back(i);
  }
  if (c->status_free.empty()) return -1;
  const int k = c->status_free.back();
  c->status_free.pop_back();
  return k;
}

// A page-locked upload slot of the context for a plan whose table prefix fits one (−1: none).
static int upload_slot_take(zh_ctx* c, size_t bytes) {
  if (bytes > kUploadSlotBytes) return -1;
  std::lock_guard<std::mutex> lk(c->status_mu);
  if (!c->upload_pin && !c->upload_failed) {
    void* h = nullptr;
    if (hipHostMalloc(&h, (size_t)kUploadSlots * kUploadSlotBytes) != hipSuccess) {
      c->upload_failed = true;
      return -1;
    }
    c->upload_pin = (uint8_t*)h;
    for (int i = kUploadSlots - 1; i >= 0; i--) c->upload_free.push_back(i);
  }
  if (c->upload_free.empty()) return -1;
  const int k = c->upload_free.back();
  c->upload_free.pop_back();
  return k;
}

void plan_free(zh_plan* p) {
  if (!p) return;
  (void)hipSetDevice(p->ctx->device);
  // the blocks go back to the context's cache: the plan's last work on them must be done
  if (p->early_h2d) (void)hipStreamSynchronize(p->ctx->stream);  // and file_pin is free again
  if (p->done_ev) {
    (void)hipEventSynchronize(p->done_ev);
    (void)hipEventDestroy(p->done_ev);
  }
  if (p->status_slot >= 0 || p->upload_slot >= 0) {  // after done_ev: copies may be queued
    std::lock_guard<std::mutex> lk(p->ctx->status_mu);
    if (p->status_slot >= 0) p->ctx->status_free.push_back(p->status_slot);
    if (p->upload_slot >= 0) p->ctx->upload_free.push_back(p->upload_slot);
  }
  for (auto& b : p->blocks) ctx_release(p->ctx, b.first, b.second);
  for (auto& e : p->ev_pending)
    for (auto ev : e) p->ev_pool.push_back(ev);
  for (auto ev : p->ev_pool) (void)hipEventDestroy(ev);
  if (p->graph_exec) (void)hipGraphExecDestroy(p->graph_exec);
  delete p;
}

}  // namespace zh

namespace zh {

// zh_ctx::file_pin with at least n bytes (grown to a power of two from 4 MiB), or null when
// the page-locked allocation fails.  Caller holds ctx->mu.
uint8_t* ctx_file_pin(zh_ctx* ctx, size_t n) {
  if (ctx->file_pin_cap >= n) return ctx->file_pin;
  if (ctx->file_pin) (void)hipHostFree(ctx->file_pin);
  ctx->file_pin = nullptr;
  ctx->file_pin_cap = 0;
  size_t cap = (size_t)4 << 20;
  while (cap < n) cap <<= 1;
  void* q = nullptr;
  if (hipHostMalloc(&q, cap, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  ctx->file_pin = (uint8_t*)q;
  ctx->file_pin_cap = cap;
  return ctx->file_pin;
}

int plan_create(zh_ctx* ctx, const zh_array_meta* m, const SrcDesc* srcs, int64_t nchunks,
                const int64_t* offset, const int64_t* shape, uint32_t flags, bool external_h2d,
                zh_plan** out, char* err, size_t errlen) {
  if (!ctx || !m || !offset || !shape || !out) return ZH_EINVAL;
  *out = nullptr;
  int st = zh_validate_meta(m, err, errlen);
  if (st != ZH_OK) return st;
  const int n = m->ndim;
  for (int d = 0; d < n; d++) {  // M/core/Array.java:386-390
    if (offset[d] < 0 || offset[d] + shape[d] > m->shape[d]) {
      set_err(err, errlen, "Requested data is outside of the array's domain.");
      return ZH_EDATA;
    }
    if (shape[d] <= 0) {
      set_err(err, errlen, "empty selection at dimension %d", d);
      return ZH_EINVAL;
    }
  }
  int64_t cstart[kMaxDims], ccount[kMaxDims];
  const int64_t ncoords = chunk_coords(n, m->chunk_shape, offset, shape, cstart, ccount);
  if (ncoords > kIntMax) {
    set_err(err, errlen, "Number of chunks exceeds Integer.MAX_VALUE");
    return ZH_EARITH;
  }
  if (ncoords != nchunks || (nchunks > 0 && !srcs)) {
    set_err(err, errlen, "expected %lld chunk sources (computeChunkCoords order), got %lld",
            (long long)ncoords, (long long)nchunks);
    return ZH_EINVAL;
  }
  (void)hipSetDevice(ctx->device);
  zh_plan* p = new zh_plan();
  p->ctx = ctx;
  p->meta = *m;
  p->flags = flags;
  p->nshards = ncoords;
  p->external_h2d = external_h2d;
  fill_common_args(m, shape, false, p->args, p->tile_mode);
  const zh_codec_chain& c = m->chain;
  const int32_t* inner = leaf_shape(m);
  const int64_t isz = zh_shard_index_size(m);
  const bool src_dev = (flags & ZH_SRC_DEVICE) != 0;
  // nested sharding: level-1 cells and the flattened leaf index per shard
  const bool nested = c.sharded && c.nested;
  int64_t cps_leaf = 1, cps2 = 1;
  for (int d = 0; d < n; d++) {
    cps_leaf *= m->chunk_shape[d] / inner[d];
    if (nested) cps2 *= c.inner_chunk_shape[d] / c.nested_chunk_shape[d];
  }
  const int64_t sub_isz = nested ? 16 * cps2 + (c.nested_index_has_crc32c ? 4 : 0) : 0;
  int64_t l1_items = 0, flat_bytes = 0;
  std::vector<int64_t> flat_off(ncoords, -1);
  std::vector<DevShard> hs(ncoords);
  std::vector<CrcJob> jobs;
  p->coords.resize(ncoords * n);
  int64_t cur[kMaxDims] = {0};
  int64_t items = 0, staged = 0, in_bytes = 0;
  std::vector<int64_t> stage_off(ncoords, -1);
  // shards held as index + pieces (sub-shard forms): the pieces of shard i are
  // held[i].pieces, laid out after its index in its staging block at piece_dst
  std::vector<HeldPieces> held(ncoords);
  std::vector<char> is_held(ncoords, 0);
  std::vector<std::vector<int64_t>> piece_dst(ncoords);
  auto fail = [&](int code) {
    plan_free(p);
    return code;
  };
  for (int64_t i = 0; i < ncoords; i++) {
    int64_t cc[kMaxDims];
    for (int d = 0; d < n; d++) cc[d] = p->coords[i * n + d] = cstart[d] + cur[d];
    for (int d = n - 1; d >= 0; d--) {
      if (++cur[d] < ccount[d]) break;
      cur[d] = 0;
    }
    int32_t co[kMaxDims], oo[kMaxDims], ps[kMaxDims];
    if (projection(n, cc, m->shape, m->chunk_shape, offset, shape, co, oo, ps) != ZH_OK) {
      set_err(err, errlen, "projection exceeds Integer.MAX_VALUE");
      return fail(ZH_EARITH);
    }
    const SrcDesc& src = srcs[i];
    DevShard& S = hs[i];
    memset(&S, 0, sizeof(S));
    const bool pieced = src.index != nullptr;
    if (pieced && !c.sharded) {
      set_err(err, errlen, "chunk %s: index + pieces sources need a sharding_indexed chain",
              fmt_ints(cc, n).c_str());
      return fail(ZH_EINVAL);
    }
    // a whole object in a store file has no address until it is staged (its bytes are read
    // into host memory or the pipelined read's ring first)
    const bool present = pieced || !src.data.empty();
    S.data = pieced ? src.index : src.data.is_file() ? nullptr : src.data.mem();
    S.nbytes = pieced ? (src.shard_nbytes >= 0 ? src.shard_nbytes : INT64_MAX) : src.nbytes;
    S.item_begin = items;
    int64_t ob = 0, nit = 1;
    for (int d = 0; d < n; d++) {
      ob += (int64_t)oo[d] * p->args.rstride[d];
      S.part_lo[d] = co[d];
      S.part_hi[d] = co[d] + ps[d];
      // inner-chunk box of the part (ShardingIndexedCodec.java:206-208)
      const int32_t b0 = co[d] / inner[d], b1 = (co[d] + ps[d] - 1) / inner[d];
      S.box_start[d] = b0;
      S.box_count[d] = b1 - b0 + 1;
      nit *= S.box_count[d];
    }
    for (int d = n; d < kMaxDims; d++) {
      S.box_count[d] = 1;
      S.part_hi[d] = 1;
    }
    S.out_base = ob;
    S.l1_begin = l1_items;
    items += nit;
    if (!present) continue;
    if (pieced) {
      if ((st = caller_pieces(m, src, isz, cc, S, src_dev, held[i], err, errlen)) != ZH_OK) return fail(st);
      is_held[i] = 1;
      S.index_off = 0;
    } else if (c.sharded) {
      if (S.nbytes < isz) {
        set_err(err, errlen, "Shard %s of %lld bytes is smaller than its index (%lld bytes).",
                fmt_ints(cc, n).c_str(), (long long)S.nbytes, (long long)isz);
        return fail(ZH_EDATA);
      }
      S.index_off = c.index_location == ZH_INDEX_START ? 0 : S.nbytes - isz;
    } else if (S.nbytes != p->args.inner_nbytes + p->args.crc_extra &&
               !(p->args.crc_extra && S.nbytes >= 4)) {  // Q12 (knowing divergence); with a
      // crc32c the checksum decides first: the resolve kernel flags the chunk, zh_plan_wait
      // checks its crc on the device (chunk_crc_detail_kernel)
      set_err(err, errlen,
              "unexpected inner chunk byte length: %lld (expected %lld) for chunk %s",
              (long long)S.nbytes, (long long)(p->args.inner_nbytes + p->args.crc_extra),
              fmt_ints(cc, n).c_str());
      return fail(ZH_EDATA);
    }
    if (nested) {
      int64_t ncell = 1;
      S.l1_begin = l1_items;
      for (int d = 0; d < n; d++) {
        const int32_t i1 = c.inner_chunk_shape[d];
        S.l1_box_start[d] = co[d] / i1;
        S.l1_box_count[d] = (co[d] + ps[d] - 1) / i1 - S.l1_box_start[d] + 1;
        ncell *= S.l1_box_count[d];
      }
      for (int d = n; d < kMaxDims; d++) S.l1_box_count[d] = 1;
      l1_items += ncell;
      flat_off[i] = flat_bytes;
      flat_bytes += 16 * cps_leaf;
      in_bytes += ncell * sub_isz;  // the referenced sub-shard indexes
    }
    // algorithmic input bytes: referenced inner chunks + the index for a
    // shard; only the in-bounds part of an unsharded chunk
    if (c.sharded) {
      in_bytes += nit * (p->args.inner_nbytes + p->args.crc_extra) + isz;
    } else {
      int64_t pb = m->dtype_size;
      for (int d = 0; d < n; d++) pb *= ps[d];
      in_bytes += pb;
    }
    if (src_dev) continue;  // device sources are read where they are
    // host sources: a whole object is staged as it is, unless the part references little
    // of a single-level shard (then its index + the referenced ranges, as a caller's pieces)
    if (!is_held[i] && c.sharded && !nested && !src.data.is_file() &&
        compact_pieces(m, S, isz, held[i])) {
      is_held[i] = 1;
      S.index_off = 0;  // the staging block starts with the stored index
    }
    stage_off[i] = staged;
    if (!is_held[i]) {
      staged += (S.nbytes + 255) & ~(int64_t)255;
      continue;
    }
    // staging block: [index][pieces], each raw piece at its shard offset's residue mod 256
    // (the payload alignment the fast kernels see is the stored one)
    int64_t pos = isz;
    for (const Piece& q : held[i].pieces) {
      pos = ((pos + 255) & ~(int64_t)255) + (q.data_nbytes == q.nbytes ? (q.offset & 255) : 0);
      piece_dst[i].push_back(pos);
      pos += q.data_nbytes;
    }
    staged += (pos + 255) & ~(int64_t)255;
  }
  p->n_items = items;
  p->in_bytes = in_bytes;
  int64_t onel = 1;
  for (int d = 0; d < n; d++) onel *= shape[d];
  p->out_bytes = onel * m->dtype_size;
  // stage host sources
  if (staged > 0) {
    if ((st = plan_alloc(p, &p->d_input, (size_t)staged, err, errlen)) != ZH_OK) return fail(st);
    for (int64_t i = 0; i < ncoords; i++) {
      if (stage_off[i] < 0) continue;
      if (is_held[i]) {
        p->h2d.push_back({stage_off[i], SrcRef::memory(held[i].index)});
        p->h2d_len.push_back(isz);
        const auto& pv = held[i].pieces;
        for (size_t k = 0; k < pv.size(); k++) {
          if (pv[k].data_nbytes <= 0) continue;
          p->h2d.push_back({stage_off[i] + piece_dst[i][k], pv[k].data});
          p->h2d_len.push_back(pv[k].data_nbytes);
        }
      } else {
        p->h2d.push_back({stage_off[i], srcs[i].data});
        p->h2d_len.push_back(hs[i].nbytes);
      }
      hs[i].data = p->d_input + stage_off[i];
    }
    // copies adjacent on both sides become one (a run of pieces read side by side into one
    // host buffer lands side by side in the staging when their stored offsets share a residue
    // mod 256): fewer, larger DMAs
    size_t w = 0;
    for (size_t k = 0; k < p->h2d.size(); k++) {
      if (w > 0 && p->h2d[w - 1].first + p->h2d_len[w - 1] == p->h2d[k].first &&
          p->h2d[k].second.follows(p->h2d[w - 1].second, p->h2d_len[w - 1])) {
        p->h2d_len[w - 1] += p->h2d_len[k];
        continue;
      }
      p->h2d[w] = p->h2d[k];
      p->h2d_len[w] = p->h2d_len[k];
      w++;
    }
    p->h2d.resize(w);
    p->h2d_len.resize(w);
    // store-file sources (zh_array_read_files): a plan that does its own h2d copies reads
    // their bytes now (the pipelined read's in lanes read them instead).  They go into the
    // context's page-locked buffer at their staging offsets, the host entries (the stored
    // indexes) copied beside them, and the plan's H2D becomes one DMA of that extent (several
    // pageable copies cost ~30 us each in the runtime's staging); into buffers the plan keeps
    // when the extent is large or sparse, or the buffer cannot be had
    std::vector<FileRead> freads;
    bool files = false;
    int64_t lo = INT64_MAX, hi = 0, sum = 0;
    for (size_t k = 0; !external_h2d && k < p->h2d.size(); k++) {
      files = files || p->h2d[k].second.is_file();
      lo = std::min(lo, p->h2d[k].first);
      hi = std::max(hi, p->h2d[k].first + p->h2d_len[k]);
      sum += p->h2d_len[k];
    }
    uint8_t* pin = nullptr;
    if (files && env_int("ZH_FILE_PIN", 1) != 0 && hi - lo <= kFilePinMax &&
        hi - lo <= 2 * sum + ((int64_t)1 << 20))
      pin = ctx_file_pin(ctx, (size_t)(hi - lo));
    // staged in batches of about 1 MiB, each DMA'd on the context's stream (the one the plan
    // runs on: read_one_plan, read_multi_impl) as soon as it is in, so the H2D of one batch
    // runs under the reads of the next
    int64_t b_lo = INT64_MAX, b_hi = 0;
    auto flush = [&]() -> int {
      if (b_lo >= b_hi) return ZH_OK;
      const std::string m = file_fetch_all(freads);
      freads.clear();
      if (!m.empty()) {
        set_err(err, errlen, "%s", m.c_str());
        return ZH_EIO;
      }
      p->early_h2d = true;
      if (hipMemcpyAsync(p->d_input + b_lo, pin + (b_lo - lo), (size_t)(b_hi - b_lo),
                         hipMemcpyHostToDevice, ctx->stream) != hipSuccess) {
        (void)hipGetLastError();
        set_err(err, errlen, "host-to-device copy of store file bytes failed");
        return ZH_EHIP;
      }
      b_lo = INT64_MAX;
      b_hi = 0;
      return ZH_OK;
    };
    for (size_t k = 0; files && k < p->h2d.size(); k++) {
      const bool f = p->h2d[k].second.is_file();
      if (pin) {
        uint8_t* dst = pin + (p->h2d[k].first - lo);
        if (f)
          freads.push_back({dst, p->h2d[k].second, p->h2d_len[k]});
        else
          std::memcpy(dst, p->h2d[k].second.mem(), (size_t)p->h2d_len[k]);
        b_lo = std::min(b_lo, p->h2d[k].first);
        b_hi = std::max(b_hi, p->h2d[k].first + p->h2d_len[k]);
        if (b_hi - b_lo >= ((int64_t)1 << 20)) {
          const int rc = flush();
          if (rc != ZH_OK) return fail(rc);
        }
        continue;
      }
      if (!f) continue;
      // uninitialised: the read fills every byte
      p->h2d_keep.emplace_back(new uint8_t[(size_t)std::max<int64_t>(1, p->h2d_len[k])]);
      freads.push_back({p->h2d_keep.back().get(), p->h2d[k].second, p->h2d_len[k]});
      p->h2d[k].second = SrcRef::memory(p->h2d_keep.back().get());
    }
    if (pin) {
      const int rc = flush();
      if (rc != ZH_OK) return fail(rc);
      p->h2d.clear();  // queued already
      p->h2d_len.clear();
    }
    if (!freads.empty()) {  // the small reads of a plan
      const std::string m = file_fetch_all(freads);
      if (!m.empty()) {
        set_err(err, errlen, "%s", m.c_str());
        return fail(ZH_EIO);
      }
    }
  }
  // the piece tables (device addresses of every held range)
  std::vector<DevPiece> dpieces;
  std::vector<int64_t> piece_first(ncoords, -1);
  for (int64_t i = 0; i < ncoords; i++) {
    if (!is_held[i]) continue;
    piece_first[i] = (int64_t)dpieces.size();
    const auto& pv = held[i].pieces;
    for (size_t k = 0; k < pv.size(); k++) {
      const uint8_t* dsrc = src_dev ? pv[k].data.mem() : hs[i].data + piece_dst[i][k];
      dpieces.push_back({(uint64_t)pv[k].offset, (uint64_t)pv[k].nbytes, dsrc,
                         (uint64_t)pv[k].data_nbytes});
    }
    hs[i].npieces = (int64_t)pv.size();
  }
  if (nested && flat_bytes > 0) {
    if ((st = plan_alloc(p, &p->d_flat, (size_t)flat_bytes, err, errlen)) != ZH_OK) return fail(st);
    for (int64_t i = 0; i < ncoords; i++)
      if (flat_off[i] >= 0) hs[i].flat = p->d_flat + flat_off[i];
    NestArgs& N = p->nest;
    N.nshards = ncoords;
    N.n_l1 = l1_items;
    N.ndim = n;
    N.index_be = c.index_endian == ZH_ENDIAN_BIG;
    N.sub_be = c.nested_index_endian == ZH_ENDIAN_BIG;
    N.sub_crc = c.nested_index_has_crc32c ? 1 : 0;
    N.sub_start = c.nested_index_location == ZH_INDEX_START;
    N.sub_isz = sub_isz;
    N.cps2 = cps2;
    N.leaf_nbytes = p->args.inner_nbytes + p->args.crc_extra;
    N.leaf_crc = c.inner_crc32c ? 1 : 0;
    RankGeom& R = p->args.rank;
    R.r2 = cps2 + 1;
    int64_t s1 = 1, sf = 1, s2 = 1;
    for (int d = n - 1; d >= 0; d--) {
      N.cps1_stride[d] = s1;
      R.cps1_stride[d] = s1;
      s1 *= m->chunk_shape[d] / c.inner_chunk_shape[d];
      N.flat_stride[d] = sf;
      sf *= m->chunk_shape[d] / inner[d];
      N.r[d] = c.inner_chunk_shape[d] / inner[d];
      R.r[d] = N.r[d];
      R.k2_stride[d] = s2;
      s2 *= N.r[d];
      N.leaf[d] = inner[d];
    }
    p->nest_grid = (int)std::min<int64_t>(l1_items, (int64_t)ctx->cu_count * 16);
  }
  // CRC jobs over the device copies of the stored indexes (Crc32cCodec.decode, :24-48): every
  // shard's, the sub-shard forms' included — the host never checks an index
  if (c.sharded && c.index_has_crc32c) {
    for (int64_t i = 0; i < ncoords; i++) {
      if (!hs[i].data) continue;
      CrcJob J;
      J.base = hs[i].data + hs[i].index_off;
      J.len = isz - 4;
      J.span_begin = 0;
      J.shard = (int32_t)i;
      J.pad = 0;
      jobs.push_back(J);
    }
    p->n_crc_jobs = (int64_t)jobs.size();
    p->n_crc_spans = assign_crc_spans(jobs, ctx->cu_count, &p->crc_shift);
    p->idx_crc_fused = env_int("ZH_IDX_CRC_FUSE", 1) != 0;
  }
  if (!(flags & ZH_OUT_DEVICE)) {
    if ((st = plan_alloc(p, &p->d_out, (size_t)p->out_bytes, err, errlen)) != ZH_OK) {
      plan_free(p);
      return st;
    }
  }
  // Small reads: split inner chunks into more pieces until the launch covers the chip (a
  // 64^3 read touches 27 inner chunks: one workgroup each left the other CUs idle and the
  // clipped ones ran 43 us).  Pieces stay whole 4 KiB CRC rounds, at most 256 per chunk.
  if (env_int("ZH_SMALL_SPLIT", 1) != 0)
    while ((items << p->args.piece_shift) < 2 * (int64_t)ctx->cu_count &&
           p->args.piece_shift < 8 && (p->args.inner_nbytes >> (p->args.piece_shift + 1)) >= 4096 &&
           (p->args.inner_nbytes >> (p->args.piece_shift + 1)) % 4096 == 0)
      p->args.piece_shift++;
  std::vector<uint32_t> tab = setup_fast(m, p->args, p->tile_mode);
  p->args.tile_variant = 1;  // the row-interleaved per-chunk tile kernel unless grouped below
  // Chunk CRC fused into the row-interleaved tile kernel: every payload byte of a fast item
  // is loaded exactly once by some lane, and each lane's share is shifted to the payload end
  // by K[u] = x^(8(L − E_u)) (E_u = end of unit u's last row, appended to the table) and a
  // lane constant.  Dynamic LDS (table, 8 tiles, CRC tables, K) stays within 64 KiB.
  const bool tile_crc =
      c.inner_crc32c && items > 0 && p->tile_mode && p->args.fast_mode == kFastTileTable &&
      p->args.tile_variant == 1 && env_int("ZH_CRC_FUSE", 1) != 0 &&
      ((int64_t)p->args.fast_n * 8 + 15) / 16 * 16 + 8 * 1057 * 4 + 16 * 256 * 4 +
              (int64_t)p->args.fast_n * 4 <= 65536;
  p->args.crc_tile_step = 0;
  p->args.tile_align = 0;
  p->args.tile_ystride = 0;
  std::vector<int64_t> ends;  // per-unit payload ends (tile CRC; the grouped step below)
  if (tile_crc) {
    const ScatterArgs& g = p->args;
    const int64_t L = g.inner_nbytes, s_fd = g.pstride[g.fd];
    for (int32_t u = 0; u < g.fast_n; u++) {
      const int64_t end = 4 * (int64_t)tab[2 * (size_t)u] + 4 * 31 * s_fd + 128;
      ends.push_back(end);
      tab.push_back(gf2_xpow8n((uint64_t)(L - end)));
    }
    p->args.crc_tile_step = tile_crc_step(ends);
  }
  // All plan tables in one allocation, the uploaded ones (shards, CRC jobs, zeroed CRC
  // partials + completion counters, fast-path table) as one prefix in one copy: a one-shot
  // small read paid ~15-20 us per synchronous upload and per allocation.
  {
    size_t off = 0;
    auto carve = [&](size_t bytes) {
      const size_t o = off;
      off += (bytes + 255) & ~(size_t)255;
      return o;
    };
    const size_t o_shards = carve(hs.size() * sizeof(DevShard));
    const size_t o_jobs = carve(jobs.size() * sizeof(CrcJob));
    const size_t o_part = carve((size_t)(p->n_crc_spans + p->n_crc_jobs) * 4);
    const size_t o_tab = carve(tab.size() * 4);
    const size_t o_pieces = carve(dpieces.size() * sizeof(DevPiece));
    const size_t up = off;  // uploaded prefix
    const size_t o_status = carve((size_t)ncoords * kStWords * 8);
    const size_t o_slow = carve(((size_t)items + 4) * 4);  // right after the status: one memset
    const size_t o_desc = carve((size_t)items * sizeof(ItemDesc));
    if ((st = plan_alloc(p, &p->d_tables, off, err, errlen)) != ZH_OK) {
      plan_free(p);
      return st;
    }
    std::vector<uint8_t> blob(up, 0);
    for (int64_t i = 0; i < ncoords; i++)
      if (piece_first[i] >= 0)
        hs[i].pieces = (const DevPiece*)(p->d_tables + o_pieces) + piece_first[i];
    memcpy(blob.data() + o_shards, hs.data(), hs.size() * sizeof(DevShard));
    if (!dpieces.empty())
      memcpy(blob.data() + o_pieces, dpieces.data(), dpieces.size() * sizeof(DevPiece));
    if (!jobs.empty()) memcpy(blob.data() + o_jobs, jobs.data(), jobs.size() * sizeof(CrcJob));
    if (!tab.empty()) memcpy(blob.data() + o_tab, tab.data(), tab.size() * 4);
    uint8_t* T = p->d_tables;
    p->d_shards = (DevShard*)(T + o_shards);
    p->d_crc_jobs = jobs.empty() ? nullptr : (CrcJob*)(T + o_jobs);
    p->d_crc_partials = (uint32_t*)(T + o_part);
    p->d_fast_tab = tab.empty() ? nullptr : (uint32_t*)(T + o_tab);
    p->d_status = (uint64_t*)(T + o_status);
    p->d_desc = (ItemDesc*)(T + o_desc);
    p->d_slow = (uint32_t*)(T + o_slow);
    // small plans: the prefix and zeroed status words + slow-list count go to a page-locked
    // slot and ride on the first execute's stream (no blocking copy here, no memset there)
    const size_t upz = o_slow + sizeof(uint32_t);
    const int slot = upload_slot_take(ctx, upz);
    if (slot >= 0) {
      uint8_t* h = ctx->upload_pin + (size_t)slot * kUploadSlotBytes;
      memcpy(h, blob.data(), up);
      memset(h + up, 0, upz - up);
      p->upload_slot = slot;
      p->upload_bytes = upz;
      p->upload_pending = true;
    } else if (hipMemcpy(T, blob.data(), up, hipMemcpyHostToDevice) != hipSuccess) {
      set_err(err, errlen, "plan upload failed");
      plan_free(p);
      return ZH_EHIP;
    }
  }
  if (c.inner_crc32c && items > 0) {
    // Fuse the chunk CRC into the row kernel when its lanes read each piece's payload in
    // the CRC pass's order: rows sequential in the payload (pstride[F] == 1, row dims in
    // C order) and equal pieces of whole 4 KiB rounds (256 lanes x 16 B); or into the tile
    // kernel (tile_crc above: one partial per chunk).
    ScatterArgs& g = p->args;
    const int64_t pieces = 1ll << g.piece_shift;
    bool fuse = !p->tile_mode && env_int("ZH_CRC_FUSE", 1) != 0 &&
                (g.fast_mode == kFastRowArith || g.fast_mode == kFastRowTable);
    if (fuse) {
      const int F = g.fs;
      int64_t stv = g.inner[F];
      fuse = g.pstride[F] == 1;
      for (int d = n - 1; d >= 0; d--) {
        if (d == F) continue;
        if (g.inner[d] > 1 && g.pstride[d] != stv) fuse = false;
        stv *= g.inner[d];
      }
      fuse = fuse && g.inner_nbytes % pieces == 0 && (g.inner_nbytes / pieces) % 4096 == 0 &&
             g.fast_rows % pieces == 0;
    }
    const int64_t span = tile_crc ? g.inner_nbytes
                                  : (fuse ? g.inner_nbytes / pieces : (int64_t)kCrcSpan);
    fuse = fuse || tile_crc;
    const int64_t nspan = (g.inner_nbytes + span - 1) / span;
    if ((st = plan_alloc(p, &p->d_dcrc, (size_t)(items * nspan), err, errlen)) != ZH_OK) {
      plan_free(p);
      return st;
    }
    DataCrcArgs& D = p->dcrc;
    D.desc = p->d_desc;
    D.n_items = items;
    D.len = g.inner_nbytes;
    D.span = span;
    D.nspan = (int32_t)nspan;
    D.store = 0;
    D.skip_fast = fuse ? 1 : 0;
    D.partials = p->d_dcrc;
    D.status = p->d_status;
    D.shards = p->d_shards;
    D.rank = p->args.rank;
    g.crc_fused = fuse ? 1 : 0;
    g.crc_partials = p->d_dcrc;
    p->dcrc_grid = (int)std::min<int64_t>(items * nspan, (int64_t)ctx->cu_count * 32);
  }
  p->args.desc = p->d_desc;
  p->args.fast_tab = p->d_fast_tab;
  p->args.n_citems = items;
  p->args.slow_count = p->d_slow;
  p->args.slow_list = p->d_slow + 4;
  p->args.shards = p->d_shards;
  p->args.nshards = ncoords;
  p->args.total_items = items << p->args.piece_shift;
  p->args.status = p->d_status;
  p->nest.shards = p->d_shards;
  p->nest.status = p->d_status;
  p->grid = grid_for(ctx, p->args.total_items);
  // non-temporal loads + stores: +4 % on the row path, +1 % on the tile path (interleaved
  // A/B in one process, profiles/r01/experiments/tune_*.json); every decode fast kernel
  // streams (the grouped row-CRC decode loads its payloads through the cache, launcher)
  p->args.nt = 3;
  // Visit items in a golden-ratio stride order: +3.6 % on the tile path (c4) on every normal
  // allocation (profiles/placement_perm.py); on the row paths it evens out where the output
  // lands — half-array c2 into three hipMalloc outputs: 18.10 / 16.14 / 16.13 → 16.45 / 16.03 /
  // 16.03 ms, c3 19.16 / 18.42 / 17.33 → 19.62 / 16.87 / 16.52 ms (round 5,
  // profiles/r05/perm/) — so every decode fast path uses it (the switch that turned it off
  // was removed in round 6).
  p->args.item_mul = golden_item_mul(p->args.total_items);
  p->slow_grid = p->grid;
  // The tile decode over G consecutive (z-adjacent) chunks per work item, the next step's
  // loads issued before this step's stores (tiles_group_kernel; tile_variant 20 + G): c4
  // 33.4 → 32.9 ms (G = 4), interleaved A/B in profiles/r02/experiments/ab_r02abdtgpf*.txt.
  // G = 4 (round 6 removed the switch and the other group sizes of this direction).
  //
  // With the fused chunk CRC: tiles_rowcrc_kernel, one chunk per work item (tile_variant 51:
  // every lane also CRCs one payload row from the LDS tiles, 16 lookups per 16-B vector):
  // c4crc 38.27 → 36.92 ms, profiles/r02/crc/ab_rowcrc.json.  Round 4 removed the variants that
  // measured slower (the fused grouped CRC decode, CRC waves of their own, rows per lane, field
  // tables); their A/B records stay under profiles/.
  {
    const bool crc = p->args.crc_fused != 0;
    const int G = crc ? 1 : 4;
    const bool rowcrc_ok = !crc || zh::rowcrc_lds_at_zero();
    if (rowcrc_ok && p->tile_mode && p->args.fast_mode == kFastTileTable &&
        (!crc || tile_crc) && p->args.piece_shift == 0 && items > 0) {
      const int64_t groups = (items + G - 1) / G;
      p->args.tile_variant = crc ? 51 : 20 + G;
      // Aligned windows for the row-CRC kernel: every payload after a 4-byte crc32c starts at
      // 4·i mod 128, so a 1 KiB wave load of it touched 9 lines and the shared line was
      // fetched twice.  When unit u's rows start at 32u elements and row r + 1 follows row r
      // (the payload is [32 rows][units][32 words], c4's layout), the movers load 128-B aligned
      // lines and route each word to its tile in LDS; other layouts keep the unaligned loads.
      if (crc) {
        const ScatterArgs& g = p->args;
        const int64_t nu = g.fast_n;
        // [32 rows][nu units][32 words], 2-4 steps of 8 units (K fits the kernel's K area),
        // unit u's region offset u·ys, the stores' lane offsets 4·(u·ys) + 128 within 32 bits
        bool al = nu >= 16 && nu <= zh::kAlnUnitsMax && nu % 8 == 0 &&
                  g.pstride[g.fd] == 32 * nu && g.inner_nbytes == 4096 * nu &&
                  (int64_t)tab.size() >= 2 * nu;
        const uint64_t ys = al ? tab[3] : 0;
        for (int64_t u = 0; al && u < nu; u++)
          al = tab[2 * (size_t)u] == (uint32_t)(32 * u) &&
               tab[2 * (size_t)u + 1] == (uint64_t)u * ys && 4 * (uint64_t)u * ys + 128 <= 0xFFFFFFFFull;
        p->args.tile_align = al ? 1 : 0;
        p->args.tile_ystride = al ? (int64_t)ys : 0;
      }
      if (crc) p->args.crc_tile_step = tile_crc_step(ends, (size_t)(8 / G));
      p->args.item_mul = golden_item_mul(groups);
      p->grid = grid_for(ctx, groups);
    }
  }
  // The row decode over G consecutive chunks per work item (rows_group_kernel, narrow rows:
  // G·row bytes of a region row per wave store).  With the fused chunk CRC, G·row = 256 B
  // (c3crc 37.2 → 35.9 ms); without it, 128-B rows take rows_xpose_kernel (8 chunks, 1 KiB
  // contiguous on both sides through an LDS lane exchange; c3, quarter array: 8.71 → 8.49 ms,
  // profiles/r02/experiments/ab_xpose_c3.json) and other rows the per-chunk row kernel (plain
  // c3 with G = 2: 33.2 → 33.5 ms, profiles/r02/experiments/ab_r02drg_*.txt).  Row-clipped
  // items then take the generic kernel (is_fast).
  {
    const int want = p->args.crc_fused ? -1 : p->args.fast_vpr_shift == 3 ? 8 : 0;
    const ScatterArgs& g = p->args;
    if (want != 0 && !p->tile_mode && (g.fast_mode == kFastRowArith || g.fast_mode == kFastRowTable) &&
        g.piece_shift == 0 && items > 0) {
      int G = want > 0 ? want : (16 >> std::min(g.fast_vpr_shift, 5));
      // 8: rows_xpose_kernel (128-B rows, no fused CRC, rows a multiple of 8)
      const bool xpose = G == 8 && g.fast_vpr_shift == 3 && !g.crc_fused && g.fast_rows % 8 == 0;
      G = xpose ? 8 : G >= 4 ? 4 : G >= 2 ? 2 : G;
      if (G >= 1 && (xpose || (G << g.fast_vpr_shift) <= 64)) {
        const int64_t groups = (items + G - 1) / G;
        p->args.row_group = G;
        p->args.item_mul = golden_item_mul(groups);
        p->grid = grid_for(ctx, groups);
      }
    }
  }
  // small plans (at most kSmallOneItems inner chunks of at most kSmallOneBytes together, no
  // chunk crc32c, no nested index): the resolve and the decode of every item in one launch
  // beside the index CRC (decode_small_kernel): a 64³ region of a c4 shard took four dependent
  // launches.  The byte bound keeps few large chunks (c2: 24 chunks of 4 GiB) on the fast
  // kernels.
  if (env_int("ZH_SMALL_ONE", 1) != 0 && items > 0 && items <= kSmallOneItems &&
      items * p->args.inner_nbytes <= kSmallOneBytes && !p->d_flat && !p->d_dcrc &&
      !p->args.crc_fused) {
    p->small_one = true;
    p->small_grid = (int)std::min<int64_t>(p->args.total_items, std::max(p->grid, 1));
  }
  *out = p;
  return ZH_OK;
}

// Enqueues one execution of the plan on stream s (also the body a hipGraph captures).
int plan_enqueue_impl(zh_plan* p, void* out, hipStream_t s) {
  char* err = nullptr;
  size_t errlen = 0;
  if (p->early_h2d && s != p->ctx->stream) {  // the staged bytes were queued on ctx->stream
    hipEvent_t e;
    ZH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    const bool ok = hipEventRecord(e, p->ctx->stream) == hipSuccess &&
                    hipStreamWaitEvent(s, e, 0) == hipSuccess;
    (void)hipEventDestroy(e);
    if (!ok) return ZH_EHIP;
  }
  for (size_t k = 0; !p->external_h2d && k < p->h2d.size(); k++)
    ZH_HIP(hipMemcpyAsync(p->d_input + p->h2d[k].first, p->h2d[k].second.mem(), (size_t)p->h2d_len[k],
                          hipMemcpyHostToDevice, s));
  if (p->upload_slot >= 0 && (p->upload_pending || p->use_graph)) {
    // the tables with zeroed status words and slow-list count (a graph replays the copy)
    ZH_HIP(hipMemcpyAsync(p->d_tables, p->ctx->upload_pin + (size_t)p->upload_slot * kUploadSlotBytes,
                          p->upload_bytes, hipMemcpyHostToDevice, s));
    p->upload_pending = false;
  } else {
    // the status words and the slow-list count (carved adjacent in the plan's tables)
    ZH_HIP(hipMemsetAsync(p->d_status, 0,
                          (size_t)((uint8_t*)p->d_slow - (uint8_t*)p->d_status) + sizeof(uint32_t), s));
  }
  std::array<hipEvent_t, 3> ev{};
  if (p->timing) {
    for (int k = 0; k < 3; k++) {
      if (p->ev_pool.empty()) {
        hipEvent_t e;
        ZH_HIP(hipEventCreate(&e));
        p->ev_pool.push_back(e);
      }
      ev[k] = p->ev_pool.back();
      p->ev_pool.pop_back();
    }
    ZH_HIP(hipEventRecord(ev[0], s));
  }
  // the index crc32c only writes status words: by default its workgroups ride in the slow
  // kernel's launch, beside the clipped chunks' decode, instead of ahead of the resolve kernel
  const CrcIdxArgs crc{p->d_crc_jobs, p->n_crc_jobs, p->n_crc_spans, p->d_crc_partials,
                       p->d_status, p->crc_shift, 0};
  if (!p->idx_crc_fused)
    ZH_HIP(launch_crc(p->d_crc_jobs, p->n_crc_jobs, p->n_crc_spans, p->crc_shift, p->d_crc_partials,
                      p->d_status, s));
  if (p->d_flat) ZH_HIP(launch_nested_index(p->nest, p->nest_grid, s));
  ScatterArgs a = p->args;
  a.region = (p->flags & ZH_OUT_DEVICE) ? (uint8_t*)out : p->d_out;
  if (p->d_dcrc && p->args.crc_fused)  // the row kernel XOR-accumulates per-piece partials
    ZH_HIP(hipMemsetAsync(p->d_dcrc, 0, (size_t)p->dcrc.n_items * p->dcrc.nspan * 4, s));
  if (p->small_one) {
    if (p->timing) ZH_HIP(hipEventRecord(ev[1], s));
    ZH_HIP(launch_decode_small(a, p->small_grid, p->idx_crc_fused ? crc : CrcIdxArgs{}, s));
  } else {
    ZH_HIP(launch_resolve(a, s));
    if (p->d_dcrc) ZH_HIP(launch_data_crc_partial(p->dcrc, p->dcrc_grid, s));
    if (p->timing) ZH_HIP(hipEventRecord(ev[1], s));
    ZH_HIP(launch_scatter(a, p->meta.dtype_size, p->grid, s));
    ZH_HIP(launch_decode_slow(a, p->slow_grid, p->idx_crc_fused ? crc : CrcIdxArgs{}, s));
  }
  if (p->d_dcrc) ZH_HIP(launch_data_crc_finalize(p->dcrc, s));
  if (p->timing) {
    ZH_HIP(hipEventRecord(ev[2], s));
    p->ev_pending.push_back(ev);
  }
  if (!(p->flags & ZH_OUT_DEVICE))
    ZH_HIP(hipMemcpyAsync(out, p->d_out, (size_t)p->out_bytes, hipMemcpyDeviceToHost, s));
  return ZH_OK;
}

void plan_drop_graph(zh_plan* p) {
  if (p->graph_exec) (void)hipGraphExecDestroy(p->graph_exec);
  p->graph_exec = nullptr;
  p->graph_out = nullptr;
  p->graph_stream = nullptr;
}

// Records the end of the plan's latest execution: plan_free waits on this event before its
// device blocks go back to the context's cache (an event outlives a caller's stream).
int plan_mark_done_impl(zh_plan* p, hipStream_t s) {
  if (!p->done_ev && hipEventCreateWithFlags(&p->done_ev, hipEventDisableTiming) != hipSuccess) {
    p->done_ev = nullptr;
    return ZH_EHIP;
  }
  return hipEventRecord(p->done_ev, s) == hipSuccess ? ZH_OK : ZH_EHIP;
}

}  // namespace zh

extern "C" {

int zh_plan_create(zh_ctx* ctx, const zh_array_meta* m, const zh_chunk_src* chunks,
                   int64_t nchunks, const int64_t* offset, const int64_t* shape, uint32_t flags,
                   zh_plan** out, char* err, size_t errlen) {
  std::vector<SrcDesc> srcs((size_t)std::max<int64_t>(0, nchunks));
  for (int64_t i = 0; chunks && i < nchunks; i++) {
    srcs[(size_t)i].data = SrcRef::memory(chunks[i].data);
    srcs[(size_t)i].nbytes = chunks[i].nbytes;
  }
  return plan_create(ctx, m, chunks ? srcs.data() : nullptr, nchunks, offset, shape, flags,
                     false, out, err, errlen);
}

int zh_plan_execute(zh_plan* p, void* out, void* stream_v) {
  if (!p || !out) return ZH_EINVAL;
  char* err = nullptr;
  size_t errlen = 0;
  hipStream_t s = stream_v ? (hipStream_t)stream_v : p->ctx->stream;
  (void)hipSetDevice(p->ctx->device);
  // hipGraph replay (zh_plan_set_graph): device-resident plans without timing events; the
  // graph is captured on the first execute for this (out, stream) and then relaunched as
  // one unit, so a small read pays one launch instead of ~8 enqueues
  if (p->use_graph && !p->timing && p->h2d.empty() && (p->flags & ZH_OUT_DEVICE)) {
    if (!p->graph_exec || p->graph_out != out || p->graph_stream != s) {
      plan_drop_graph(p);
      ZH_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      const int st = plan_enqueue_impl(p, out, s);
      hipGraph_t g = nullptr;
      const hipError_t e = hipStreamEndCapture(s, &g);
      if (st != ZH_OK || e != hipSuccess) {
        if (g) (void)hipGraphDestroy(g);
        return st != ZH_OK ? st : ZH_EHIP;
      }
      const hipError_t ei = hipGraphInstantiate(&p->graph_exec, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      if (ei != hipSuccess) {
        p->graph_exec = nullptr;
        return ZH_EHIP;
      }
      p->graph_out = out;
      p->graph_stream = s;
    }
    ZH_HIP(hipGraphLaunch(p->graph_exec, s));
    p->last_stream = s;
    return plan_mark_done_impl(p, s);
  }
  const int st = plan_enqueue_impl(p, out, s);
  if (st == ZH_OK) p->last_stream = s;
  return st == ZH_OK ? plan_mark_done_impl(p, s) : st;
}

int zh_plan_set_graph(zh_plan* p, int enable) {
  if (!p) return ZH_EINVAL;
  p->use_graph = enable != 0;
  if (!p->use_graph) {
    (void)hipSetDevice(p->ctx->device);
    plan_drop_graph(p);
  }
  return ZH_OK;
}

int zh_plan_wait(zh_plan* p, char* err, size_t errlen) {
  if (!p) return ZH_EINVAL;
  (void)hipSetDevice(p->ctx->device);
  p->err_shard = -1;
  g_data_err.set = false;
  std::vector<uint64_t> stv((size_t)p->nshards * kStWords);
  if (p->status_slot < 0 && p->last_stream && !stv.empty())
    p->status_slot = status_slot_take(p->ctx, p->nshards);
  if (p->status_slot >= 0 && p->last_stream && !stv.empty()) {
    // the status copy rides on the plan's stream behind its kernels: one synchronise
    uint64_t* h = p->ctx->status_pin + (size_t)p->status_slot * kStatusSlotWords;
    ZH_HIP(hipMemcpyAsync(h, p->d_status, stv.size() * sizeof(uint64_t), hipMemcpyDeviceToHost,
                          p->last_stream));
    ZH_HIP(hipStreamSynchronize(p->last_stream));
    std::copy(h, h + stv.size(), stv.begin());
  } else {
    if (p->last_stream) ZH_HIP(hipStreamSynchronize(p->last_stream));
    if (!stv.empty())
      ZH_HIP(hipMemcpy(stv.data(), p->d_status, stv.size() * sizeof(uint64_t),
                       hipMemcpyDeviceToHost));
  }
  const int n = p->meta.ndim;
  for (int64_t i = 0; i < p->nshards; i++) {
    const uint64_t* w = &stv[i * kStWords];
    if (!w[kStFlags]) continue;
    p->err_shard = i;  // where the error sits in the oracle's order (the pipelined read's pick)
    p->err_key = (w[kStFlags] & kFlagCrc) ? ~0ull : w[kStBadChunk];
    g_data_err.set = true;
    g_data_err.cc.assign(p->coords.begin() + i * n, p->coords.begin() + (i + 1) * n);
    g_data_err.key = p->err_key;
    if (w[kStFlags] & kFlagCrc) {  // Crc32cCodec.java:39-44 (signed ints)
      set_err(err, errlen, "The checksum of the sharding index is invalid. Stored: %d Computed: %d",
              (int32_t)(uint32_t)w[kStCrcStored], (int32_t)(uint32_t)w[kStCrcComputed]);
      return ZH_EDATA;
    }
    // the first chunk-level error in the oracle's order (RankGeom)
    const uint64_t key = w[kStBadChunk];
    const uint32_t rank = 0xFFFFFFFFu - (uint32_t)(key >> 8);
    const uint32_t level = (uint32_t)(key & (kFlagL1 | kFlagLeaf));
    const uint32_t kind = (uint32_t)(key & (kFlagRange | kFlagLength | kFlagChunkCrc | kFlagShort));
    const zh_codec_chain& ch = p->meta.chain;
    if (kind == kFlagChunkCrc) {  // a chunk's (or sub-shard index's) Crc32cCodec.decode :39-44
      set_err(err, errlen, "The checksum of the sharding index is invalid. Stored: %d Computed: %d",
              (int32_t)(uint32_t)w[kStDetailA], (int32_t)(uint32_t)w[kStDetailB]);
      return ZH_EDATA;
    }
    if (kind == kFlagLength && level == 0 && p->args.crc_extra) {
      // The reference's pipeline runs the crc32c stage before the bytes codec: the checksum over
      // the chunk's stored bytes decides first (error path only: one workgroup on the device).
      uint64_t o[4] = {0, 0, 0, 0};
      uint64_t* dw = p->d_status + (size_t)i * kStWords;
      hipStream_t s = p->last_stream ? p->last_stream : p->ctx->stream;
      ZH_HIP(launch_chunk_crc_detail(p->args, i, (int64_t)rank, dw, s));
      ZH_HIP(hipMemcpyAsync(o, dw, sizeof o, hipMemcpyDeviceToHost, s));
      ZH_HIP(hipStreamSynchronize(s));
      if (o[0] & 2) {
        set_err(err, errlen,
                "The checksum of the sharding index is invalid. Stored: %d Computed: %d",
                (int32_t)(uint32_t)o[1], (int32_t)(uint32_t)o[2]);
        return ZH_EDATA;
      }
      if (!ch.sharded) {  // the planner's Q12 text for a whole chunk
        set_err(err, errlen, "unexpected inner chunk byte length: %lld (expected %lld) for chunk %s",
                (long long)o[3], (long long)(p->args.inner_nbytes + p->args.crc_extra),
                fmt_ints(p->coords.data() + i * n, n).c_str());
        return ZH_EDATA;
      }
    }
    if (kind == kFlagShort) {  // the level-2 decode of a sub-shard shorter than its index
      const int64_t cps2 = (int64_t)p->args.rank.r2 - 1;
      set_err(err, errlen, "Shard of %lld bytes is smaller than its index (%lld bytes).",
              (long long)(uint32_t)w[kStDetailA],
              (long long)(16 * cps2 + (ch.nested_index_has_crc32c ? 4 : 0)));
      return ZH_EDATA;
    }
    // chunk coordinates in the grid of the codec that read the entry: the shard's inner-chunk
    // grid, (nested, kFlagL1) its level-1 cell grid, or (kFlagLeaf) the sub-shard's leaf grid
    uint64_t r = rank;
    if (level & kFlagL1) r = rank / (uint64_t)p->args.rank.r2;
    if (level & kFlagLeaf) r = rank % (uint64_t)p->args.rank.r2 - 1;
    int64_t ic[kMaxDims];
    for (int d = n - 1; d >= 0; d--) {
      int32_t cps = p->meta.chunk_shape[d] / leaf_shape(&p->meta)[d];
      if (level & kFlagL1) cps = p->meta.chunk_shape[d] / ch.inner_chunk_shape[d];
      if (level & kFlagLeaf) cps = ch.inner_chunk_shape[d] / ch.nested_chunk_shape[d];
      ic[d] = (int64_t)(r % (uint64_t)cps);
      r /= (uint64_t)cps;
    }
    if (kind == kFlagRange)  // ShardingIndexedCodec.java:227-230
      set_err(err, errlen, "Could not load byte data for chunk %s", fmt_ints(ic, n).c_str());
    else
      set_err(err, errlen, "unexpected inner chunk byte length for chunk %s",
              fmt_ints(ic, n).c_str());
    return ZH_EDATA;
  }
  return ZH_OK;
}

void zh_plan_destroy(zh_plan* p) { plan_free(p); }

int zh_plan_stats(const zh_plan* p, int64_t* in_bytes, int64_t* out_bytes, int64_t* items,
                  int64_t* nshards) {
  if (!p) return ZH_EINVAL;
  if (in_bytes) *in_bytes = p->in_bytes;
  if (out_bytes) *out_bytes = p->out_bytes;
  if (items) *items = p->n_items;
  if (nshards) *nshards = p->nshards;
  return ZH_OK;
}

int64_t zh_debug_last_fast_path(int encode) {
  return encode ? zh::g_last_encode_path.load() : zh::g_last_fast_path.load();
}

int64_t zh_plan_staged_bytes(const zh_plan* p) {
  if (!p) return -1;
  int64_t t = 0;
  for (int64_t l : p->h2d_len) t += l;
  return t;
}

int zh_plan_set_timing(zh_plan* p, int enable) {
  if (!p) return ZH_EINVAL;
  p->timing = enable != 0;
  return ZH_OK;
}

int zh_plan_kernel_time(zh_plan* p, double* scatter_ms, int64_t* launches, double* index_ms) {
  if (!p) return ZH_EINVAL;
  char* err = nullptr;
  size_t errlen = 0;
  (void)hipSetDevice(p->ctx->device);
  double sc = 0, ix = 0;
  for (auto& e : p->ev_pending) {
    ZH_HIP(hipEventSynchronize(e[2]));
    float a = 0, b = 0;
    ZH_HIP(hipEventElapsedTime(&a, e[0], e[1]));
    ZH_HIP(hipEventElapsedTime(&b, e[1], e[2]));
    ix += a;
    sc += b;
  }
  if (scatter_ms) *scatter_ms = sc;
  if (index_ms) *index_ms = ix;
  if (launches) *launches = (int64_t)p->ev_pending.size();
  for (auto& e : p->ev_pending)
    for (auto ev : e) p->ev_pool.push_back(ev);
  p->ev_pending.clear();
  return ZH_OK;
}

}  // extern "C"

namespace zh {

// A small output in pageable host memory (a Java array, a fresh numpy array) lands in the
// context's page-locked buffer as one DMA and leaves it by one memcpy after the wait, instead
// of the runtime's staged pageable copy.  Null: write to `out` directly.
static uint8_t* hout_stage(zh_ctx* ctx, const void* out, int64_t nbytes, uint32_t flags) {
  if ((flags & ZH_OUT_DEVICE) || nbytes <= 0 || nbytes > kHoutPinBytes || ctx->hout_pin_failed)
    return nullptr;
  unsigned int hf = 0;
  if (hipHostGetFlags(&hf, const_cast<void*>(out)) == hipSuccess) return nullptr;  // pinned
  (void)hipGetLastError();
  if (!ctx->hout_pin) {
    void* q = nullptr;
    if (hipHostMalloc(&q, (size_t)kHoutPinBytes, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      ctx->hout_pin_failed = true;
      return nullptr;
    }
    ctx->hout_pin = (uint8_t*)q;
  }
  return ctx->hout_pin;
}

int read_one_plan(zh_ctx* ctx, const zh_array_meta* meta, const SrcDesc* srcs, int64_t nsrc,
                  const int64_t* offset, const int64_t* shape, void* out, uint32_t flags,
                  void* stream, char* err, size_t errlen) {
  zh_plan* p = nullptr;
  int st = plan_create(ctx, meta, srcs, nsrc, offset, shape, flags, false, &p, err, errlen);
  if (st != ZH_OK) return st;
  g_quiet_err[0] = 0;
  uint8_t* stage = hout_stage(ctx, out, p->out_bytes, flags);
  st = zh_plan_execute(p, stage ? (void*)stage : out, stream);
  if (st != ZH_OK) {
    set_err(err, errlen, "kernel launch failed%s%s", g_quiet_err[0] ? ": " : "", g_quiet_err);
    plan_free(p);
    return st;
  }
  st = zh_plan_wait(p, err, errlen);
  if (st == ZH_OK && stage) std::memcpy(out, stage, (size_t)p->out_bytes);
  plan_free(p);
  return st;
}

// A region read: large reads with a host side (host sources or a host output) go through the
// pipelined path (H2D | decode | D2H per slab, zh_pipeline.cpp); everything else, and regions
// that do not split, as one plan.
thread_local DataErrPos g_data_err;

int read_region(zh_ctx* ctx, const zh_array_meta* meta, const SrcDesc* srcs, int64_t nsrc,
                const int64_t* offset, const int64_t* shape, void* out, uint32_t flags,
                void* stream, char* err, size_t errlen) {
  g_data_err.set = false;
  if (meta && offset && shape && out && env_int("ZH_PIPE", 1) != 0) {
    const int st = read_pipelined(ctx, meta, srcs, nsrc, offset, shape, out, flags, stream, err,
                                  errlen);
    if (st != ZH_EUNSUPPORTED) return st;
  }
  return read_one_plan(ctx, meta, srcs, nsrc, offset, shape, out, flags, stream, err, errlen);
}

}  // namespace zh

extern "C" {

int zh_array_read(zh_ctx* ctx, const zh_array_meta* meta, const zh_chunk_src* chunks,
                  int64_t nchunks, const int64_t* offset, const int64_t* shape, void* out,
                  uint32_t flags, void* stream, char* err, size_t errlen) {
  if (!ctx) return ZH_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  std::vector<SrcDesc> srcs((size_t)std::max<int64_t>(0, nchunks));
  for (int64_t i = 0; chunks && i < nchunks; i++) {
    srcs[(size_t)i].data = SrcRef::memory(chunks[i].data);
    srcs[(size_t)i].nbytes = chunks[i].nbytes;
  }
  return read_region(ctx, meta, chunks ? srcs.data() : nullptr, nchunks, offset, shape, out,
                     flags, stream, err, errlen);
}

}  // extern "C"

namespace {
// Peer access from device `from` to device `to` (once per pair per process), so that the
// slab copies to the root device go device to device over xGMI and kernels on `from` may
// read `to`'s memory.  Returns false when the pair has no peer access: the caller then stages
// through host memory (ZH_MULTI_FORCE_STAGED=1 takes that route for every pair).
bool enable_peer(int from, int to) {
  if (from == to) return true;
  static std::mutex mu;
  static std::vector<std::pair<std::pair<int, int>, bool>> done;
  std::lock_guard<std::mutex> lk(mu);
  for (auto& p : done)
    if (p.first.first == from && p.first.second == to) return p.second;
  int can = 0;
  bool ok = hipDeviceCanAccessPeer(&can, from, to) == hipSuccess && can;
  if (ok) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(from);
    const hipError_t e = hipDeviceEnablePeerAccess(to, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
    ok = e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
    if (!ok) (void)hipGetLastError();
    (void)hipSetDevice(cur);
  }
  done.push_back({{from, to}, ok});
  return ok;
}

// Device holding a device pointer (-1: host / unknown).
int pointer_device(const void* p) {
  hipPointerAttribute_t a;
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return a.type == hipMemoryTypeDevice ? a.device : -1;
}

// Copy `bytes` from `src` on device `sdev` to `dst` on device `ddev` through pinned host
// memory in bounded pieces (no peer access between the two), on fresh streams of each
// device.  Leaves the current device as it found it.
int staged_copy(void* dst, int ddev, const void* src, int sdev, size_t bytes) {
  const size_t piece = (size_t)256 << 20;
  int cur = 0;
  (void)hipGetDevice(&cur);
  void* host = nullptr;
  hipStream_t ss = nullptr, ds = nullptr;
  int rc = ZH_OK;
  if (hipHostMalloc(&host, std::min(piece, bytes > 0 ? bytes : 1), 0) != hipSuccess) rc = ZH_ENOMEM;
  if (rc == ZH_OK && (hipSetDevice(sdev) != hipSuccess || hipStreamCreate(&ss) != hipSuccess))
    rc = ZH_EHIP;
  if (rc == ZH_OK && (hipSetDevice(ddev) != hipSuccess || hipStreamCreate(&ds) != hipSuccess))
    rc = ZH_EHIP;
  for (size_t o = 0; rc == ZH_OK && o < bytes; o += piece) {
    const size_t b = std::min(piece, bytes - o);
    if (hipSetDevice(sdev) != hipSuccess ||
        hipMemcpyAsync(host, (const uint8_t*)src + o, b, hipMemcpyDeviceToHost, ss) != hipSuccess ||
        hipStreamSynchronize(ss) != hipSuccess || hipSetDevice(ddev) != hipSuccess ||
        hipMemcpyAsync((uint8_t*)dst + o, host, b, hipMemcpyHostToDevice, ds) != hipSuccess ||
        hipStreamSynchronize(ds) != hipSuccess)
      rc = ZH_EHIP;
  }
  if (ss) {
    (void)hipSetDevice(sdev);
    (void)hipStreamDestroy(ss);
  }
  if (ds) {
    (void)hipSetDevice(ddev);
    (void)hipStreamDestroy(ds);
  }
  if (host) (void)hipHostFree(host);
  if (rc != ZH_OK) (void)hipGetLastError();
  (void)hipSetDevice(cur);
  return rc;
}
}  // namespace

extern "C" {

// Multi-GPU region read inside one process: contiguous C-order slabs, one
// per device, decoded concurrently (one host thread per device, each on its context), then
// delivered to the caller's host buffer (each device over its own PCIe link) or to the
// root device's buffer over xGMI.
int zh_slab_partition(int ndim, const int64_t* offset, const int64_t* shape, int nslabs,
                      int64_t align, int64_t* slab_off, int64_t* slab_shape) {
  if (ndim <= 0 || ndim > kMaxDims || nslabs <= 0 || !offset || !shape || !slab_off ||
      !slab_shape)
    return ZH_EINVAL;
  int ax = -1;  // first axis long enough; all earlier axes must have extent 1
  for (int d = 0; d < ndim; d++) {
    if (shape[d] >= nslabs) {
      ax = d;
      break;
    }
    if (shape[d] != 1) break;
  }
  if (ax < 0) return ZH_EINVAL;
  const int64_t lo = offset[ax], ext = shape[ax];
  const bool units_ok = align > 1 && ext % align == 0 && ext / align >= nslabs;
  for (int r = 0; r < nslabs; r++) {
    auto bound = [&](int k) {
      return units_ok ? lo + (ext / align * k / nslabs) * align : lo + ext * k / nslabs;
    };
    for (int d = 0; d < ndim; d++) {
      slab_off[r * ndim + d] = offset[d];
      slab_shape[r * ndim + d] = shape[d];
    }
    slab_off[r * ndim + ax] = bound(r);
    slab_shape[r * ndim + ax] = bound(r + 1) - bound(r);
  }
  return ZH_OK;
}

int zh_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int zh_array_read_multi(zh_ctx* const* ctxs, int ndev, int root, const zh_array_meta* meta,
                        const zh_chunk_src* chunks, int64_t nchunks, const int64_t* offset,
                        const int64_t* shape, void* out, uint32_t flags, char* err,
                        size_t errlen) {
  return zh_array_read_multi_routed(ctxs, ndev, root, meta, chunks, nchunks, offset, shape, out,
                                    flags, nullptr, err, errlen);
}

}  // extern "C"

namespace zh {

int read_multi_impl(zh_ctx* const* ctxs, int ndev, int root, const zh_array_meta* meta,
                    const SrcDesc* chunks, int64_t nchunks, const int64_t* offset,
                    const int64_t* shape, void* out, uint32_t flags, int32_t* slab_route,
                    char* err, size_t errlen) {
  if (slab_route)
    for (int k = 0; k < ndev; k++) slab_route[k] = ZH_ROUTE_DIRECT;
  if (!ctxs || ndev <= 0 || root < 0 || root >= ndev || !meta || !offset || !shape || !out)
    return ZH_EINVAL;
  for (int k = 0; k < ndev; k++)
    if (!ctxs[k]) return ZH_EINVAL;
  int st = zh_validate_meta(meta, err, errlen);
  if (st != ZH_OK) return st;
  const int n = meta->ndim;
  for (int d = 0; d < n; d++) {  // M/core/Array.java:386-390
    if (offset[d] < 0 || shape[d] <= 0 || offset[d] + shape[d] > meta->shape[d]) {
      set_err(err, errlen, "Requested data is outside of the array's domain.");
      return ZH_EDATA;
    }
  }
  int64_t cstart[kMaxDims], ccount[kMaxDims];
  const int64_t ncoords = chunk_coords(n, meta->chunk_shape, offset, shape, cstart, ccount);
  if (ncoords != nchunks || !chunks) {
    set_err(err, errlen, "expected %lld chunk sources (computeChunkCoords order), got %lld",
            (long long)ncoords, (long long)nchunks);
    return ZH_EINVAL;
  }
  // slabs aligned to inner (leaf) chunks along the split axis, so no item is cut in two
  int ax = -1;
  for (int d = 0; d < n; d++) {
    if (shape[d] >= ndev) {
      ax = d;
      break;
    }
    if (shape[d] != 1) break;
  }
  const int nslab = ax < 0 ? 1 : ndev;
  std::vector<int64_t> so((size_t)nslab * n), ss((size_t)nslab * n);
  if (ax < 0) {  // not splittable: the root decodes it all
    std::copy(offset, offset + n, so.begin());
    std::copy(shape, shape + n, ss.begin());
  } else {
    zh_slab_partition(n, offset, shape, nslab, leaf_shape(meta)[ax], so.data(), ss.data());
  }
  const bool out_dev = (flags & ZH_OUT_DEVICE) != 0;
  int64_t rstride[kMaxDims], cstride[kMaxDims], s1 = 1, s2 = 1;
  for (int d = n - 1; d >= 0; d--) {
    rstride[d] = s1;
    s1 *= shape[d];
    cstride[d] = s2;
    s2 *= ccount[d];
  }
  std::vector<int> status(nslab, ZH_OK);
  std::vector<std::string> msgs(nslab);
  std::vector<DataErrPos> where(nslab);  // a data error's place in the oracle's order
  auto work = [&](int r) {
    const int64_t* o = &so[(size_t)r * n];
    const int64_t* s = &ss[(size_t)r * n];
    int64_t nel = 1, base = 0;
    for (int d = 0; d < n; d++) {
      nel *= s[d];
      base += (o[d] - offset[d]) * rstride[d];
    }
    if (nel == 0) return;
    zh_ctx* ctx = ctxs[ax < 0 ? root : r];
    char e[1024] = {0};
    int rc = ZH_OK;
    // this slab's chunks, picked out of the caller's (full region) list
    int64_t st0[kMaxDims], cnt[kMaxDims];
    const int64_t m = chunk_coords(n, meta->chunk_shape, o, s, st0, cnt);
    std::vector<SrcDesc> sub((size_t)m);
    std::vector<std::vector<Piece>> moved;  // pieces restaged on this device
    int64_t cur[kMaxDims] = {0};
    for (int64_t i = 0; i < m; i++) {
      int64_t lin = 0;
      for (int d = 0; d < n; d++) lin += (st0[d] + cur[d] - cstart[d]) * cstride[d];
      sub[(size_t)i] = chunks[lin];
      for (int d = n - 1; d >= 0; d--) {
        if (++cur[d] < cnt[d]) break;
        cur[d] = 0;
      }
    }
    uint8_t* dst = (uint8_t*)out + base * meta->dtype_size;
    std::lock_guard<std::mutex> lk(ctx->mu);
    (void)hipSetDevice(ctx->device);
    const int rdev = ctxs[root]->device;
    const size_t sbytes = (size_t)(nel * meta->dtype_size);
    int route = ZH_ROUTE_DIRECT;
    // device sources on another device: read them over xGMI, or stage them here
    std::vector<void*> staged;
    // ZH_MULTI_FORCE_STAGED=1 (tests): every non-root slab takes the staged routes, so the
    // no-peer fallback runs even with all contexts on one device
    const char* fenv = getenv("ZH_MULTI_FORCE_STAGED");
    const bool force = fenv && fenv[0] == '1' && ctx != ctxs[root];
    if (flags & ZH_SRC_DEVICE) {
      // a device range on another device: read over xGMI when the pair has peer access,
      // else copied here first (a whole object, or a sub-shard form's index and pieces)
      auto localize = [&](const void* p, int64_t nb, const void** to) -> bool {
        if (!p || nb <= 0) return true;
        const int sdev = pointer_device(p);
        if (sdev < 0 || (sdev == ctx->device && !force)) return true;
        if (!force && enable_peer(ctx->device, sdev)) {
          route |= ZH_ROUTE_SRC_PEER;
          return true;
        }
        void* loc = nullptr;
        if (hipMalloc(&loc, (size_t)nb) != hipSuccess) {
          (void)hipGetLastError();
          rc = ZH_ENOMEM;
          snprintf(e, sizeof(e), "hipMalloc of a staged chunk on device %d failed", ctx->device);
          return false;
        }
        staged.push_back(loc);
        rc = staged_copy(loc, ctx->device, p, sdev, (size_t)nb);
        if (rc != ZH_OK) {
          snprintf(e, sizeof(e), "staging a chunk from device %d to %d failed", sdev,
                   ctx->device);
          return false;
        }
        *to = loc;
        route |= ZH_ROUTE_SRC_STAGED;
        return true;
      };
      for (auto& c : sub) {
        const void* p = c.data.mem();
        if (!localize(p, c.nbytes, &p)) break;
        c.data = SrcRef::memory(p);
        p = c.index;
        if (!localize(c.index, c.index_nbytes, &p)) break;
        c.index = (const uint8_t*)p;
        if (c.npieces > 0) {
          moved.emplace_back(c.pieces, c.pieces + c.npieces);
          bool ok = true;
          for (auto& q : moved.back()) {
            const void* qp = q.data.mem();
            if (!(ok = localize(qp, q.data_nbytes, &qp))) break;
            q.data = SrcRef::memory(qp);
          }
          if (!ok) break;
          c.pieces = moved.back().data();
        }
      }
    }
    const bool remote = out_dev && ctx != ctxs[root];  // decode locally, then deliver
    int oroute = ZH_ROUTE_DIRECT;
    if (remote)
      oroute = force                     ? ZH_ROUTE_STAGED
               : ctx->device == rdev     ? ZH_ROUTE_SAME
               : enable_peer(ctx->device, rdev) ? ZH_ROUTE_PEER
                                         : ZH_ROUTE_STAGED;
    route |= oroute;
    void* local = nullptr;
    if (rc == ZH_OK && remote && hipMalloc(&local, sbytes) != hipSuccess) {
      (void)hipGetLastError();
      rc = ZH_ENOMEM;
      snprintf(e, sizeof(e), "hipMalloc of a slab buffer failed");
    }
    zh_plan* p = nullptr;
    uint32_t pf = (flags & ZH_SRC_DEVICE) | (out_dev ? ZH_OUT_DEVICE : 0u);
    if (rc == ZH_OK && !remote) {
      // straight into its destination: the region read itself (large host slabs pipelined)
      rc = read_region(ctx, meta, sub.data(), m, o, s, dst, pf, nullptr, e, sizeof(e));
    } else {
      if (rc == ZH_OK) rc = plan_create(ctx, meta, sub.data(), m, o, s, pf, false, &p, e, sizeof(e));
      if (rc == ZH_OK) rc = zh_plan_execute(p, local, nullptr);
      if (rc == ZH_OK && (oroute == ZH_ROUTE_PEER || oroute == ZH_ROUTE_SAME) &&
          hipMemcpyPeerAsync(dst, rdev, local, ctx->device, sbytes, ctx->stream) != hipSuccess) {
        (void)hipGetLastError();
        rc = ZH_EHIP;
        snprintf(e, sizeof(e), "slab copy to device %d failed", rdev);
      }
      if (rc == ZH_OK) rc = zh_plan_wait(p, e, sizeof(e));
      if (rc == ZH_OK && oroute == ZH_ROUTE_STAGED) {
        rc = staged_copy(dst, rdev, local, ctx->device, sbytes);
        if (rc != ZH_OK) snprintf(e, sizeof(e), "staged slab copy to device %d failed", rdev);
      }
    }
    if (p) plan_free(p);
    (void)hipSetDevice(ctx->device);
    if (local) (void)hipFree(local);
    for (void* x : staged) (void)hipFree(x);
    if (slab_route) slab_route[r] = route;
    status[r] = rc;
    msgs[r] = e;
    if (rc == ZH_EDATA && g_data_err.set) where[r] = g_data_err;
  };
  std::vector<std::thread> th;
  for (int r = 0; r < nslab; r++) th.emplace_back(work, r);
  for (auto& t : th) t.join();
  // the first failing slab in C order; when every failure is a data error the device placed,
  // the first of those in the oracle's order (slabs can cut a shard)
  int first = -1, best = -1;
  bool placed = true;
  for (int r = 0; r < nslab; r++) {
    if (status[r] == ZH_OK) continue;
    if (first < 0) first = r;
    if (status[r] != ZH_EDATA || !where[r].set) {
      placed = false;
      continue;
    }
    if (best < 0 || data_err_before(where[r].cc, where[r].key, where[best].cc, where[best].key))
      best = r;
  }
  g_data_err = DataErrPos{};
  if (first < 0) return ZH_OK;
  const int r = placed && best >= 0 ? best : first;
  if (r == best) g_data_err = where[r];  // zh_last_data_error on the calling thread
  set_err(err, errlen, "%s", msgs[r].c_str());
  return status[r];
}

}  // namespace zh

extern "C" {

int zh_array_read_multi_routed(zh_ctx* const* ctxs, int ndev, int root,
                               const zh_array_meta* meta, const zh_chunk_src* chunks,
                               int64_t nchunks, const int64_t* offset, const int64_t* shape,
                               void* out, uint32_t flags, int32_t* slab_route, char* err,
                               size_t errlen) {
  std::vector<SrcDesc> srcs((size_t)std::max<int64_t>(0, nchunks));
  for (int64_t i = 0; chunks && i < nchunks; i++) {
    srcs[(size_t)i].data = SrcRef::memory(chunks[i].data);
    srcs[(size_t)i].nbytes = chunks[i].nbytes;
  }
  return read_multi_impl(ctxs, ndev, root, meta, chunks ? srcs.data() : nullptr, nchunks, offset,
                         shape, out, flags, slab_route, err, errlen);
}

// ShardingIndexedCodec.decode / decodePartial: one shard viewed as a one-chunk array.
int zh_sharding_decode_partial(zh_ctx* ctx, const zh_array_meta* meta, const void* shard,
                               int64_t nbytes, const int64_t* offset, const int32_t* shape,
                               void* out, uint32_t flags, void* stream, char* err,
                               size_t errlen) {
  if (!meta || !shard || !offset || !shape) return ZH_EINVAL;
  if (!meta->chain.sharded) {
    set_err(err, errlen, "meta does not describe a sharding_indexed chain");
    return ZH_EINVAL;
  }
  zh_array_meta sm = *meta;
  for (int d = 0; d < meta->ndim; d++) sm.shape[d] = meta->chunk_shape[d];
  int64_t shp[kMaxDims];
  for (int d = 0; d < meta->ndim; d++) shp[d] = shape[d];
  zh_chunk_src src{shard, nbytes};
  return zh_array_read(ctx, &sm, &src, 1, offset, shp, out, flags, stream, err, errlen);
}

int zh_sharding_decode(zh_ctx* ctx, const zh_array_meta* meta, const void* shard, int64_t nbytes,
                       void* out, uint32_t flags, void* stream, char* err, size_t errlen) {
  if (!meta) return ZH_EINVAL;
  int64_t off[kMaxDims] = {0};
  return zh_sharding_decode_partial(ctx, meta, shard, nbytes, off, meta->chunk_shape, out, flags,
                                    stream, err, errlen);
}

// =====================================================================================
// write path
// =====================================================================================
int64_t zh_array_encoded_bound(const zh_array_meta* m) {
  if (!m) return -1;
  int64_t nel = 1;
  for (int d = 0; d < m->ndim; d++) nel *= m->chunk_shape[d];
  int64_t bound = nel * m->dtype_size + (m->chain.sharded ? zh_shard_index_size(m) : 0);
  if (m->chain.inner_crc32c) {  // + 4 per (inner/leaf) chunk
    int64_t nch = 1;
    const int32_t* leaf = leaf_shape(m);
    for (int d = 0; d < m->ndim; d++) nch *= m->chunk_shape[d] / leaf[d];
    bound += 4 * nch;
  }
  if (m->chain.sharded && m->chain.nested) {  // + one sub-shard index per level-1 cell
    int64_t ncell = 1, cps2 = 1;
    for (int d = 0; d < m->ndim; d++) {
      ncell *= m->chunk_shape[d] / m->chain.inner_chunk_shape[d];
      cps2 *= m->chain.inner_chunk_shape[d] / m->chain.nested_chunk_shape[d];
    }
    bound += ncell * (16 * cps2 + (m->chain.nested_index_has_crc32c ? 4 : 0));
  }
  return bound;
}

constexpr int kWriteFallback = -1;

// zh_array_write in one pass over the region (single-level chains): the layout assumes every
// in-bounds inner chunk is kept, in C order, so each chunk's payload offset is
// its rank in the shard's in-bounds box — computed on the device by the resolve kernel.  The
// fast decode kernels run on an encode view (source = region, destination = payloads) and
// test each piece against fill_value on the way, the generic kernel takes the clipped or
// misaligned chunks, and one finish kernel writes the index entries, builds the chunk-CRC
// descriptors and counts kept chunks that turned out all fill_value.  Index crc32c and
// chunk crc32c are stored on the device; the call synchronises once.  A non-zero count means
// the layout was wrong (the reference elides such a chunk): returns kWriteFallback and the
// caller runs flags → layout → encode.  Scratch tables live in the context (grow-only).
//
// keep != nullptr (the second pass after a fallback): keep[item] = the chunk holds a
// non-fill element, from the first pass's flags (flags_out).  The layout is then the
// reference's: kept chunks only, in C order, a shard (or nested cell) with none elided; the
// host computes the offsets and the same kernels run once more.
static int array_write_fast(zh_ctx* ctx, const zh_array_meta* m, ScatterArgs a,
                            std::vector<DevShard>& hs, int64_t items, int tile_mode,
                            zh_chunk_dst* dsts, const uint8_t* keep,
                            std::vector<uint8_t>* flags_out, hipStream_t s, char* err,
                            size_t errlen) {
  const zh_codec_chain& c = m->chain;
  const int n = m->ndim;
  const int64_t ncoords = (int64_t)hs.size();
  const int64_t cn = a.inner_nbytes + a.crc_extra;  // stored bytes per inner chunk
  const int64_t isz = c.sharded ? zh_shard_index_size(m) : 0;
  const bool start = c.sharded && c.index_location == ZH_INDEX_START;
  const int32_t* inner = leaf_shape(m);
  // nested sharding: each level-1 cell with an in-bounds leaf is a sub-shard in C order —
  // its in-bounds leaves in C order + its own index (ShardingIndexedCodec.encode of the
  // level-2 codec, :105-168) — and a cell without one is (-1, -1) at level 1.  The cell table
  // and the outer index (+ crc32c) are built here; leaf entries and sub-index CRCs on the
  // device.
  EncNest nz{};
  std::vector<int64_t> cells;
  std::vector<std::vector<uint8_t>> outer;
  std::vector<CrcJob> jobs;
  int64_t spans = 0;
  auto add_job = [&](const uint8_t* base, int64_t len, int64_t shard) {
    CrcJob J;
    J.base = base;
    J.len = len;
    J.span_begin = 0;
    J.shard = (int32_t)shard;
    J.pad = 0;
    jobs.push_back(J);
  };
  int64_t cps2 = 1;
  std::vector<int64_t> hoff;  // keep mode: payload offset per item (-1: elided)
  if (keep) hoff.assign((size_t)items, -1);
  int64_t cps_total = 1;
  for (int d = 0; d < n; d++) cps_total *= m->chunk_shape[d] / inner[d];
  if (c.nested) {
    nz.ncell = 1;
    for (int d = 0; d < kMaxDims; d++) {
      nz.r[d] = d < n ? c.inner_chunk_shape[d] / inner[d] : 1;
      nz.g1[d] = d < n ? m->chunk_shape[d] / c.inner_chunk_shape[d] : 1;
      nz.ncell *= nz.g1[d];
      cps2 *= nz.r[d];
    }
    nz.sub_isz = 16 * cps2 + (c.nested_index_has_crc32c ? 4 : 0);
    nz.sub_start = c.nested_index_location == ZH_INDEX_START;
    nz.sub_be = c.nested_index_endian == ZH_ENDIAN_BIG;
    cells.assign((size_t)(2 * nz.ncell * ncoords), -1);
    outer.resize((size_t)ncoords);
  }
  for (int64_t i = 0; i < ncoords; i++) {
    DevShard& S = hs[i];
    int64_t payload;
    if (c.nested) {
      std::vector<uint8_t>& idx = outer[(size_t)i];
      idx.assign((size_t)isz, 0);
      const bool be = c.index_endian == ZH_ENDIAN_BIG;
      int64_t pos = start ? isz : 0;
      for (int64_t cell = 0; cell < nz.ncell; cell++) {
        int64_t q = cell, nk = 1, c1v[kMaxDims] = {0};
        for (int d = n - 1; d >= 0; d--) {
          const int64_t c1 = q % nz.g1[d];
          q /= nz.g1[d];
          c1v[d] = c1;
          const int64_t lo = c1 * c.inner_chunk_shape[d];
          nk *= a.fill_never ? nz.r[d]  // a NaN fill: every leaf kept (padding included)
                             : std::max<int64_t>(0, std::min<int64_t>(
                                   nz.r[d], (S.part_hi[d] - lo + inner[d] - 1) / inner[d]));
        }
        if (keep) {  // the cell's kept leaves, C order over its leaf grid
          nk = 0;
          const int64_t lpos = pos + (nz.sub_start ? nz.sub_isz : 0);
          for (int64_t k2 = 0; k2 < cps2; k2++) {
            int64_t f = 0, tq = k2, fs = 1;
            for (int d = n - 1; d >= 0; d--) {
              f += (c1v[d] * nz.r[d] + tq % nz.r[d]) * fs;
              tq /= nz.r[d];
              fs *= S.box_count[d];
            }
            if (keep[S.item_begin + f]) hoff[(size_t)(S.item_begin + f)] = lpos + cn * nk++;
          }
        }
        uint64_t eo = ~0ull, en = ~0ull;
        if (nk > 0) {
          const int64_t len = nk * cn + nz.sub_isz;
          const int64_t sidx = nz.sub_start ? pos : pos + nk * cn;
          cells[(size_t)(2 * (i * nz.ncell + cell))] = pos;
          cells[(size_t)(2 * (i * nz.ncell + cell) + 1)] = sidx;
          if (c.nested_index_has_crc32c)
            add_job((const uint8_t*)dsts[i].data + sidx, 16 * cps2, i);
          eo = (uint64_t)pos;
          en = (uint64_t)len;
          pos += len;
        }
        for (int b = 0; b < 8; b++) {
          const int sh = be ? 56 - 8 * b : 8 * b;
          idx[(size_t)(16 * cell + b)] = (uint8_t)(eo >> sh);
          idx[(size_t)(16 * cell + 8 + b)] = (uint8_t)(en >> sh);
        }
      }
      if (c.index_has_crc32c) {  // Crc32cCodec.encode :50-60
        const uint32_t crc = crc32c_host(0, idx.data(), (size_t)(isz - 4));
        for (int b = 0; b < 4; b++) idx[(size_t)(isz - 4 + b)] = (uint8_t)(crc >> (8 * b));
      }
      payload = pos - (start ? isz : 0);
    } else if (keep) {
      const int64_t nit = c.sharded ? cps_total : 1;
      int64_t kept = 0;
      for (int64_t k = 0; k < nit; k++)
        if (keep[S.item_begin + k]) hoff[(size_t)(S.item_begin + k)] = (start ? isz : 0) + cn * kept++;
      payload = kept * cn;
    } else {
      int64_t kept = 1;  // in-bounds inner chunks of the shard (all kept under this layout)
      for (int d = 0; d < n; d++)
        kept *= a.fill_never ? S.box_count[d] : (S.part_hi[d] + inner[d] - 1) / inner[d];
      payload = kept * cn;
    }
    if (keep && payload == 0) {  // all fill: writeChunk deletes the key (Array.java:150-151)
      dsts[i].nbytes = 0;
      S.index_off = -1;
      continue;
    }
    const int64_t total = payload + isz;
    if (total > dsts[i].capacity || !dsts[i].data) {
      set_err(err, errlen, "chunk destination %lld too small: need %lld bytes, have %lld",
              (long long)i, (long long)total, (long long)dsts[i].capacity);
      return ZH_EINVAL;
    }
    dsts[i].nbytes = total;
    S.index_off = c.sharded && !c.nested ? (start ? 0 : payload) : -1;
  }
  const int64_t pitems = items << a.piece_shift;
  // the encode view: source strides = region, destination strides = payload, destination
  // addresses relative to the lowest shard buffer
  ScatterArgs v = a;
  for (int d = 0; d < kMaxDims; d++) std::swap(v.pstride[d], v.rstride[d]);
  std::vector<uint32_t> tab = setup_fast(m, v, tile_mode);
  uint8_t* vbase = nullptr;
  for (int64_t i = 0; i < ncoords; i++)
    if (!vbase || (uint8_t*)dsts[i].data < vbase) vbase = (uint8_t*)dsts[i].data;
  if (c.sharded && !c.nested && c.index_has_crc32c)  // Crc32cCodec.encode of each index
    for (int64_t i = 0; i < ncoords; i++)
      if (hs[i].index_off >= 0) add_job((const uint8_t*)dsts[i].data + hs[i].index_off, isz - 4, i);
  int crc_shift = 0;
  spans = assign_crc_spans(jobs, ctx->cu_count, &crc_shift);
  // chunk crc32c fused into the row encode when its lanes store each piece's payload in the
  // CRC pass's order (the decode rule, plan creation above: rows sequential in the payload,
  // equal pieces of whole 4 KiB rounds); otherwise a separate pass over the written payloads
  bool crc_fuse = false;
  const int64_t pieces = 1ll << a.piece_shift;
  if (c.inner_crc32c && !tile_mode && env_int("ZH_CRC_FUSE", 1) != 0 &&
      (v.fast_mode == kFastRowArith || v.fast_mode == kFastRowTable)) {
    const int F = a.fs;
    int64_t stv = a.inner[F];
    crc_fuse = a.pstride[F] == 1;
    for (int d = n - 1; d >= 0; d--) {
      if (d == F) continue;
      if (a.inner[d] > 1 && a.pstride[d] != stv) crc_fuse = false;
      stv *= a.inner[d];
    }
    crc_fuse = crc_fuse && a.inner_nbytes % pieces == 0 &&
               (a.inner_nbytes / pieces) % 4096 == 0 && v.fast_rows % pieces == 0;
  }
  // ... or into the tile encode (its stores have the decode loads' geometry: per-unit end
  // shifts from the payload side of the table, appended to it; one partial per chunk)
  const bool tile_crc =
      c.inner_crc32c && tile_mode && v.fast_mode == kFastTileTable &&
      env_int("ZH_CRC_FUSE", 1) != 0 &&
      ((int64_t)v.fast_n * 8 + 15) / 16 * 16 + 8 * 1057 * 4 + 16 * 256 * 4 +
              (int64_t)v.fast_n * 4 <= 65536;
  v.crc_tile_step = 0;
  v.tile_align = 0;
  v.tile_ystride = 0;
  std::vector<int64_t> tile_ends;  // per-unit payload ends (tile CRC; the grouped step below)
  if (tile_crc) {
    const int64_t L = a.inner_nbytes, d_fs = v.rstride[v.fs];
    std::vector<int64_t>& ends = tile_ends;
    for (int32_t u = 0; u < v.fast_n; u++) {
      const int64_t end = 4 * (int64_t)tab[2 * (size_t)u + 1] + 4 * 31 * d_fs + 128;
      ends.push_back(end);
      tab.push_back(gf2_xpow8n((uint64_t)(L - end)));
    }
    v.crc_tile_step = tile_crc_step(ends);
  }
  const int64_t cspan = tile_crc ? a.inner_nbytes
                                 : (crc_fuse ? a.inner_nbytes / pieces : (int64_t)kCrcSpan);
  crc_fuse = crc_fuse || tile_crc;
  const int64_t nspan = c.inner_crc32c ? (a.inner_nbytes + cspan - 1) / cspan : 0;
  // scratch carve-up (256-B aligned sub-buffers)
  size_t off = 0;
  auto carve = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  const size_t o_shards = carve(hs.size() * sizeof(DevShard));
  const size_t o_flags = carve((size_t)items);  // one all-fill flag per inner chunk
  const size_t o_off = carve((size_t)items * sizeof(int64_t));
  const size_t o_desc = carve((size_t)items * sizeof(ItemDesc));
  const size_t o_slow = carve(((size_t)items + 4) * sizeof(uint32_t));
  const size_t o_tab = carve(tab.size() * sizeof(uint32_t));
  const size_t o_jobs = carve(jobs.size() * sizeof(CrcJob));
  const size_t o_part = carve((size_t)(spans + (int64_t)jobs.size()) * sizeof(uint32_t));
  const size_t o_cdesc = carve(c.inner_crc32c ? (size_t)items * sizeof(ItemDesc) : 0);
  const size_t o_cpart = carve((size_t)(items * nspan) * sizeof(uint32_t));
  const size_t o_cnt = carve(sizeof(uint32_t));
  const size_t o_cells = carve(cells.size() * sizeof(int64_t));
  if (off > ctx->wscratch_cap) {
    (void)hipFree(ctx->wscratch);
    ctx->wscratch = nullptr;
    ctx->wscratch_cap = 0;
    const size_t cap = off + off / 4;
    int st = dev_alloc(&ctx->wscratch, cap, err, errlen);
    if (st != ZH_OK) return st;
    ctx->wscratch_cap = cap;
  }
  uint8_t* W = ctx->wscratch;
  DevShard* d_shards = (DevShard*)(W + o_shards);
  uint8_t* d_flags = W + o_flags;
  int64_t* d_off = (int64_t*)(W + o_off);
  uint32_t* d_slow = (uint32_t*)(W + o_slow);
  uint32_t* d_cnt = (uint32_t*)(W + o_cnt);
  ItemDesc* d_cdesc = c.inner_crc32c ? (ItemDesc*)(W + o_cdesc) : nullptr;
#define ZH_HIPF(call)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (call);                                                                \
    if (e_ != hipSuccess) {                                                                \
      set_err(err, errlen, "HIP error %s (%s)", hipGetErrorName(e_), hipGetErrorString(e_)); \
      return ZH_EHIP;                                                                      \
    }                                                                                      \
  } while (0)
  ZH_HIPF(hipMemcpyAsync(d_shards, hs.data(), hs.size() * sizeof(DevShard), hipMemcpyHostToDevice,
                         s));
  if (!tab.empty())
    ZH_HIPF(hipMemcpyAsync(W + o_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice, s));
  if (!jobs.empty())
    ZH_HIPF(hipMemcpyAsync(W + o_jobs, jobs.data(), jobs.size() * sizeof(CrcJob),
                           hipMemcpyHostToDevice, s));
  // a NaN fill equals nothing (Java's ==): every chunk holds a non-fill element
  ZH_HIPF(hipMemsetAsync(d_flags, a.fill_never ? 1 : 0, (size_t)items, s));
  ZH_HIPF(hipMemsetAsync(d_slow, 0, sizeof(uint32_t), s));
  ZH_HIPF(hipMemsetAsync(d_cnt, 0, sizeof(uint32_t), s));
  if (c.nested) {
    ZH_HIPF(hipMemcpyAsync(W + o_cells, cells.data(), cells.size() * sizeof(int64_t),
                           hipMemcpyHostToDevice, s));
    nz.cell = (const int64_t*)(W + o_cells);
    for (int64_t i = 0; i < ncoords; i++)  // the outer index (entries + crc32c), host-built
      if (dsts[i].nbytes)
        ZH_HIPF(hipMemcpyAsync((uint8_t*)dsts[i].data + (start ? 0 : dsts[i].nbytes - isz),
                               outer[(size_t)i].data(), (size_t)isz, hipMemcpyHostToDevice, s));
  }
  a.shards = d_shards;
  a.nshards = ncoords;
  a.n_citems = items;
  a.total_items = pitems;
  a.item_off = d_off;
  a.flags = d_flags;
  a.desc = (ItemDesc*)(W + o_desc);
  a.slow_count = d_slow;
  a.slow_list = d_slow + 4;
  if (keep)
    ZH_HIPF(hipMemcpyAsync(d_off, hoff.data(), hoff.size() * sizeof(int64_t),
                           hipMemcpyHostToDevice, s));
  ZH_HIPF(launch_encode_resolve(a, nz, keep ? nullptr : d_off, start ? isz : 0, cn, vbase,
                                v.fast_mode != kFastNone ? 1 : 0, s));
  v.shards = d_shards;
  v.nshards = ncoords;
  v.n_citems = items;
  v.total_items = pitems;
  v.region = vbase;
  v.flags = d_flags;
  v.desc = a.desc;
  v.fast_tab = (uint32_t*)(W + o_tab);
  // golden-ratio visit order and (uint32 rows) 8 rows in flight per lane: +2.4 % on c3, the
  // order +4 % on c4 (interleaved A/B, profiles/tune_write.py → profiles/r01/experiments/)
  v.item_mul = golden_item_mul(pitems);
  v.crc_fused = crc_fuse ? 1 : 0;
  v.crc_partials = (uint32_t*)(W + o_cpart);
  if (crc_fuse)
    ZH_HIPF(hipMemsetAsync(W + o_cpart, 0, (size_t)(items * nspan) * sizeof(uint32_t), s));
  v.nt = 3;  // non-temporal region loads and payload stores (launch_encode_fast_ds)
  // narrow rows: G consecutive chunks per work item so a wave load covers G·row bytes of a
  // region row (G·row = 256 B; rows_group_kernel, 4 rows in flight per lane; c3 write G × U
  // grid in profiles/r02/write/ab_enc3.txt: G = 2, U = 4 best, 40.1 → 36.2 ms)
  int group = 0;
  // (not nested: c3nest measured 42 → 48 ms grouped, profiles/r02/write/ab_enc.txt)
  // (with the chunk CRC fused: rows sequential in the payload, checked above; whole chunks)
  if ((v.fast_mode == kFastRowArith || v.fast_mode == kFastRowTable) && a.piece_shift == 0 &&
      !nz.cell) {
    int G = 16 >> std::min(v.fast_vpr_shift, 5);
    G = G >= 8 ? 8 : G >= 4 ? 4 : G >= 2 ? 2 : G;
    if (crc_fuse && G > 4) G = 4;  // the CRC variants: G 1, 2, 4
    if (G && (G << v.fast_vpr_shift) <= 64) group = G;
  }
  // tiles (uint32 transposed chunks): 2 chunks per work item, 4 tiles of each per step
  // (tiles_group_kernel; 1 and 4 measured slower, profiles/r02/write/ab_tenc.txt).  With the
  // tile CRC fused, the kernel folds each lane's units (4 apart) with the step for that stride.
  if (v.fast_mode == kFastTileTable && (!crc_fuse || tile_crc) && a.piece_shift == 0 &&
      !nz.cell) {
    group = 2;
    if (tile_crc) v.crc_tile_step = tile_crc_step(tile_ends, (size_t)(8 / group));
  }
  if (group) v.item_mul = golden_item_mul((items + group - 1) / group);
  const int grid = grid_for(ctx, group ? (items + group - 1) / group : pitems);
  ZH_HIPF(launch_encode_fast(v, grid, group, s));
  ZH_HIPF(launch_encode_slow(a, grid, s));
  ZH_HIPF(launch_encode_finish(a, nz, cn, d_cnt, d_cdesc, s));
  if (!jobs.empty()) {
    ZH_HIPF(hipMemsetAsync(W + o_part + spans * 4, 0, jobs.size() * 4, s));  // job counters
  }
  if (!jobs.empty())
    ZH_HIPF(launch_crc((const CrcJob*)(W + o_jobs), (int64_t)jobs.size(), spans, crc_shift,
                       (uint32_t*)(W + o_part), nullptr, s));
  if (c.inner_crc32c) {  // Crc32cCodec.encode (:50-60) of every kept chunk payload
    DataCrcArgs D{};
    D.desc = d_cdesc;
    D.n_items = items;
    D.len = a.inner_nbytes;
    D.span = cspan;
    D.nspan = (int32_t)nspan;
    D.store = 1;
    D.skip_fast = crc_fuse ? 1 : 0;
    D.partials = (uint32_t*)(W + o_cpart);
    ZH_HIPF(launch_data_crc(D, (int)std::min<int64_t>(items * nspan, (int64_t)ctx->cu_count * 32),
                            s));
  }
  uint32_t bad = 0;
  ZH_HIPF(hipMemcpyAsync(&bad, d_cnt, sizeof(bad), hipMemcpyDeviceToHost, s));
  ZH_HIPF(hipStreamSynchronize(s));
  if (bad && !keep && flags_out) {  // the speculative layout was wrong: hand the flags back
    flags_out->resize((size_t)items);
    ZH_HIPF(hipMemcpy(flags_out->data(), d_flags, (size_t)items, hipMemcpyDeviceToHost));
  }
#undef ZH_HIPF
  if (bad && keep) {
    set_err(err, errlen, "internal error: kept chunk without data on the second write pass");
    return ZH_EHIP;
  }
  return bad ? kWriteFallback : ZH_OK;
}

int zh_array_write(zh_ctx* ctx, const zh_array_meta* m, const void* src, const int64_t* offset,
                   const int64_t* shape, zh_chunk_dst* dsts, int64_t nchunks, void* stream_v,
                   char* err, size_t errlen) {
  if (!ctx || !m || !src || !offset || !shape) return ZH_EINVAL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  int st = zh_validate_meta(m, err, errlen);
  if (st != ZH_OK) return st;
  const int n = m->ndim;
  for (int d = 0; d < n; d++) {
    if (offset[d] < 0 || offset[d] + shape[d] > m->shape[d]) {
      set_err(err, errlen, "Requested data is outside of the array's domain.");
      return ZH_EDATA;
    }
    const int64_t e = offset[d] + shape[d];
    if (shape[d] <= 0 || offset[d] % m->chunk_shape[d] != 0 ||
        (e % m->chunk_shape[d] != 0 && e != m->shape[d])) {
      set_err(err, errlen, "region does not cover whole chunks (host read-modify-write needed)");
      return ZH_EUNSUPPORTED;
    }
  }
  int64_t cstart[kMaxDims], ccount[kMaxDims];
  const int64_t ncoords = chunk_coords(n, m->chunk_shape, offset, shape, cstart, ccount);
  if (ncoords != nchunks || !dsts) {
    set_err(err, errlen, "expected %lld chunk destinations", (long long)ncoords);
    return ZH_EINVAL;
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream_v ? (hipStream_t)stream_v : ctx->stream;
  ScatterArgs a{};
  int tile_mode = 0;
  fill_common_args(m, shape, true, a, tile_mode);
  const zh_codec_chain& c = m->chain;
  const int32_t* inner = leaf_shape(m);
  std::vector<DevShard> hs(ncoords);
  int64_t cur[kMaxDims] = {0};
  int64_t items = 0;
  int64_t cps_total = 1;
  for (int d = 0; d < n; d++) cps_total *= m->chunk_shape[d] / inner[d];
  for (int64_t i = 0; i < ncoords; i++) {
    int64_t cc[kMaxDims];
    for (int d = 0; d < n; d++) cc[d] = cstart[d] + cur[d];
    for (int d = n - 1; d >= 0; d--) {
      if (++cur[d] < ccount[d]) break;
      cur[d] = 0;
    }
    int32_t co[kMaxDims], oo[kMaxDims], ps[kMaxDims];
    projection(n, cc, m->shape, m->chunk_shape, offset, shape, co, oo, ps);
    DevShard& S = hs[i];
    memset(&S, 0, sizeof(S));
    S.wdata = (uint8_t*)dsts[i].data;
    S.item_begin = items;
    int64_t ob = 0;
    for (int d = 0; d < n; d++) {
      ob += (int64_t)oo[d] * a.rstride[d];
      S.part_lo[d] = co[d];
      S.part_hi[d] = co[d] + ps[d];
      S.box_start[d] = 0;
      S.box_count[d] = m->chunk_shape[d] / inner[d];
    }
    for (int d = n; d < kMaxDims; d++) {
      S.box_count[d] = 1;
      S.part_hi[d] = 1;
    }
    S.out_base = ob;
    items += c.sharded ? cps_total : 1;
  }
  {
    a.region = (uint8_t*)src;
    std::vector<uint8_t> flags;
    st = array_write_fast(ctx, m, a, hs, items, tile_mode, dsts, nullptr, &flags, s, err, errlen);
    if (st != kWriteFallback) return st;
    // second pass with the layout the first pass's all-fill flags give (the reference's),
    // over the shards that hold an elided inner chunk only: in every other shard the
    // speculative layout was the true one and the first pass's bytes are final
    const int32_t* leaf = leaf_shape(m);
    std::vector<DevShard> hs2;
    std::vector<zh_chunk_dst> d2;
    std::vector<int64_t> which;
    std::vector<uint8_t> keep2;
    for (int64_t i = 0; i < ncoords; i++) {
      const int64_t b = hs[i].item_begin;
      const int64_t nit = c.sharded ? cps_total : 1;
      bool dirty = false;
      int64_t ic[kMaxDims] = {0};
      for (int64_t k = 0; k < nit && !dirty; k++) {  // an in-bounds chunk without data?
        bool in = true;
        for (int d = 0; d < n; d++) in &= ic[d] * leaf[d] < hs[i].part_hi[d];
        dirty = in && !flags[(size_t)(b + k)];
        for (int d = n - 1; d >= 0; d--) {
          if (++ic[d] < hs[i].box_count[d]) break;
          ic[d] = 0;
        }
      }
      if (!dirty) continue;
      DevShard S = hs[i];
      S.index_off = 0;
      S.item_begin = (int64_t)keep2.size();
      hs2.push_back(S);
      zh_chunk_dst D = dsts[i];
      D.nbytes = 0;
      d2.push_back(D);
      which.push_back(i);
      keep2.insert(keep2.end(), flags.begin() + b, flags.begin() + b + nit);
    }
    st = array_write_fast(ctx, m, a, hs2, (int64_t)keep2.size(), tile_mode, d2.data(),
                          keep2.data(), nullptr, s, err, errlen);
    for (size_t j = 0; j < which.size(); j++) dsts[which[j]].nbytes = d2[j].nbytes;
    return st;
  }
}

int zh_array_write_host(zh_ctx* ctx, const zh_array_meta* m, const void* src_host,
                        const int64_t* offset, const int64_t* shape, void* const* outs,
                        const int64_t* capacities, int64_t* nbytes, int64_t nchunks, char* err,
                        size_t errlen) {
  if (!ctx || !m || !src_host || !offset || !shape || (nchunks > 0 && (!outs || !capacities ||
                                                                         !nbytes)))
    return ZH_EINVAL;
  int st = zh_validate_meta(m, err, errlen);
  if (st != ZH_OK) return st;
  (void)hipSetDevice(ctx->device);
  int64_t rbytes = m->dtype_size;
  for (int d = 0; d < m->ndim; d++) rbytes *= shape[d];
  const int64_t bound = zh_array_encoded_bound(m);
  void* dsrc = nullptr;
  void* ddst = nullptr;
  size_t gsrc = 0, gdst = 0;
  hipError_t e = ctx_alloc(ctx, (size_t)std::max<int64_t>(1, rbytes), &dsrc, &gsrc);
  if (e == hipSuccess)
    e = ctx_alloc(ctx, (size_t)std::max<int64_t>(1, bound * nchunks), &ddst, &gdst);
  if (e == hipSuccess) e = hipMemcpy(dsrc, src_host, (size_t)rbytes, hipMemcpyHostToDevice);
  std::vector<zh_chunk_dst> dsts((size_t)std::max<int64_t>(1, nchunks));
  if (e == hipSuccess) {
    for (int64_t i = 0; i < nchunks; i++) {
      dsts[(size_t)i].data = (uint8_t*)ddst + i * bound;
      dsts[(size_t)i].capacity = bound;
      dsts[(size_t)i].nbytes = 0;
    }
    st = zh_array_write(ctx, m, dsrc, offset, shape, dsts.data(), nchunks, nullptr, err, errlen);
    for (int64_t i = 0; st == ZH_OK && i < nchunks; i++) {
      nbytes[i] = dsts[(size_t)i].nbytes;
      if (nbytes[i] == 0) continue;
      if (nbytes[i] > capacities[i] || !outs[i]) {
        set_err(err, errlen, "chunk destination %lld too small: need %lld bytes, have %lld",
                (long long)i, (long long)nbytes[i], (long long)capacities[i]);
        st = ZH_EINVAL;
        break;
      }
      e = hipMemcpy(outs[i], dsts[(size_t)i].data, (size_t)nbytes[i], hipMemcpyDeviceToHost);
      if (e != hipSuccess) break;
    }
  }
  if (dsrc) ctx_release(ctx, dsrc, gsrc);
  if (ddst) ctx_release(ctx, ddst, gdst);
  if (e != hipSuccess) {
    set_err(err, errlen, "HIP error %s (%s)", hipGetErrorName(e), hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? ZH_ENOMEM : ZH_EHIP;
  }
  return st;
}

// =====================================================================================
// plumbing
// =====================================================================================
}  // extern "C"

namespace {
// ZH_MALLOC_SCATTER allocations: VA base → (size, chunk size, physical chunk handles).  A view
// (zh_device_scatter_view) maps another allocation's handles at a fresh VA and owns none.
struct ScatterAlloc {
  size_t size = 0, chunk = 0;
  size_t tail = 0;  // bytes of the last handle when smaller than a chunk (mapped last, unpermuted)
  int device = 0;
  bool view = false;
  std::vector<hipMemGenericAllocationHandle_t> handles;
  std::vector<double> probes;  // ZH_MALLOC_CALIBRATE: write probe of every candidate, GB/s
  int chosen = -1;             // index of this allocation among them
};
std::mutex g_scatter_mu;
std::map<void*, ScatterAlloc> g_scatter;
// Every virtual range a scatter allocation or view ever used, [begin, end), and reservations
// set aside because they overlapped one.  ROCm 7.2 did not drop the device's translations of a
// freed range: a later range reserved over it and mapped to other chunks was partly written
// through the old mapping (kernel stores lost, copies reading zeros; profiles/va_reuse_lab.py,
// profiles/r02/placement/va_reuse.jsonl).  So no range is ever mapped twice: a reservation
// that overlaps a used range stays reserved, unmapped (address space only), and another is
// taken above the highest address used so far.
std::vector<std::pair<uintptr_t, uintptr_t>> g_va_used;
std::vector<std::pair<void*, size_t>> g_va_quarantine;

uint64_t gcd_u64(uint64_t x, uint64_t y) {
  while (y) {
    const uint64_t r = x % y;
    x = y;
    y = r;
  }
  return x;
}

// Map A's chunks into [base, base+size): slot i <- chunk (a + i*m) mod n.  Order 0 is the
// golden-ratio stride with a = 0; order k > 0 takes a further stride coprime with n (from a
// second irrational fraction) and a rotation.  On failure nothing stays mapped.
int scatter_map(void* base, const ScatterAlloc& A, uint64_t order) {
  const size_t n = A.handles.size() - (A.tail ? 1 : 0), chunk = A.chunk;
  uint64_t m = 1, a = 0;
  if (n > 1) {
    const double frac = order == 0 ? 0.6180339887498949
                                   : std::fmod(0.4142135623730950 * (double)(order + 1), 1.0);
    m = ((uint64_t)((double)n * frac)) | 1;
    if (m >= n) m = 1;
    while (gcd_u64(m, n) != 1) m += 2;
    a = order == 0 ? 0 : (order * ((n + 6) / 7)) % n;
  }
  for (size_t i = 0; i < n; i++) {
    const size_t src = n > 1 ? (size_t)((a + (uint64_t)i * m) % n) : 0;
    if (hipMemMap((uint8_t*)base + i * chunk, chunk, 0, A.handles[src], 0) != hipSuccess) {
      for (size_t k = 0; k < i; k++) (void)hipMemUnmap((uint8_t*)base + k * chunk, chunk);
      (void)hipGetLastError();
      return ZH_EHIP;
    }
  }
  if (A.tail && hipMemMap((uint8_t*)base + n * chunk, A.tail, 0, A.handles[n], 0) != hipSuccess) {
    for (size_t k = 0; k < n; k++) (void)hipMemUnmap((uint8_t*)base + k * chunk, chunk);
    (void)hipGetLastError();
    return ZH_EHIP;
  }
  hipMemAccessDesc acc = {};
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = A.device;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if (hipMemSetAccess(base, A.size, &acc, 1) != hipSuccess) {
    for (size_t k = 0; k < n; k++) (void)hipMemUnmap((uint8_t*)base + k * chunk, chunk);
    if (A.tail) (void)hipMemUnmap((uint8_t*)base + n * chunk, A.tail);
    (void)hipGetLastError();
    return ZH_EHIP;
  }
  return ZH_OK;
}

void scatter_unmap(void* base, const ScatterAlloc& A) {
  const size_t n = A.handles.size() - (A.tail ? 1 : 0);
  for (size_t k = 0; k < n; k++) (void)hipMemUnmap((uint8_t*)base + k * A.chunk, A.chunk);
  if (A.tail) (void)hipMemUnmap((uint8_t*)base + n * A.chunk, A.tail);
  (void)hipGetLastError();
}

// reserve a virtual range that overlaps no range used before (see g_va_used).  The driver
// hands freed address space out again, lowest first; an answer inside a used range is kept
// reserved (quarantined, never mapped), and that whole used range is reserved too when it is
// still free, so the next answer skips it instead of walking through it one request at a time
// (after many arenas a 2 MiB request met more than 16 such answers in a row).
std::vector<uintptr_t> g_va_blocked;  // starts of used ranges reserved whole

int reserve_fresh(size_t size, size_t align, void** out) {
  std::lock_guard<std::mutex> lk(g_scatter_mu);
  uintptr_t top = 0;
  for (auto& u : g_va_used) top = std::max(top, u.second);
  for (int attempt = 0; attempt < 256; attempt++) {
    void* base = nullptr;
    void* hint = attempt == 0 || top == 0 ? nullptr
                 : (void*)((top + align - 1) / align * align + (uintptr_t)attempt * align);
    if (hipMemAddressReserve(&base, size, align, hint, 0) != hipSuccess) {
      (void)hipGetLastError();
      return ZH_ENOMEM;
    }
    const uintptr_t b = (uintptr_t)base, e = b + size;
    const std::pair<uintptr_t, uintptr_t>* hit = nullptr;
    for (auto& u : g_va_used)
      if (b < u.second && u.first < e) {
        hit = &u;
        break;
      }
    if (!hit) {
      g_va_used.emplace_back(b, e);
      *out = base;
      return ZH_OK;
    }
    g_va_quarantine.emplace_back(base, size);  // never mapped; kept out of the next answer
    const uintptr_t u0 = hit->first, u1 = hit->second;
    if (std::find(g_va_blocked.begin(), g_va_blocked.end(), u0) == g_va_blocked.end()) {
      g_va_blocked.push_back(u0);  // one try per used range
      // the parts of the used range around this answer, each reserved at its exact address
      const std::pair<uintptr_t, uintptr_t> parts[2] = {{u0, b}, {e, u1}};
      for (const auto& pr : parts) {
        if (pr.second <= pr.first) continue;
        void* q = nullptr;
        if (hipMemAddressReserve(&q, pr.second - pr.first, 0, (void*)pr.first, 0) != hipSuccess) {
          (void)hipGetLastError();
          continue;
        }
        if ((uintptr_t)q == pr.first) {
          g_va_quarantine.emplace_back(q, pr.second - pr.first);
        } else {
          (void)hipMemAddressFree(q, pr.second - pr.first);
          (void)hipGetLastError();
        }
      }
    }
  }
  return ZH_ENOMEM;
}

// reserve a fresh VA range for A and map its chunks there
int scatter_place(ScatterAlloc& A, uint64_t order, void** out) {
  void* base = nullptr;
  if (reserve_fresh(A.size, A.chunk, &base) != ZH_OK) return ZH_ENOMEM;
  const int st = scatter_map(base, A, order);
  if (st != ZH_OK) {
    (void)hipMemAddressFree(base, A.size);
    (void)hipGetLastError();
    return st;
  }
  *out = base;
  return ZH_OK;
}

int scatter_malloc(int device, size_t bytes, void** out) {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  size_t gran = 0;
  if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended) !=
          hipSuccess || gran == 0)
    return ZH_EHIP;
  size_t chunk = (size_t)std::max(1, env_int("ZH_SCATTER_MB", 1024)) << 20;
  chunk = std::min(chunk, std::max(bytes, (size_t)1));  // small buffers: one chunk
  chunk = (chunk + gran - 1) / gran * gran;
  // whole chunks, then a tail chunk only as large as the rest (rounded to the granularity):
  // a request just above a chunk multiple must not take a whole extra chunk
  const size_t n = std::max<size_t>(1, bytes / chunk);
  size_t rest = bytes > n * chunk ? bytes - n * chunk : 0;
  rest = (rest + gran - 1) / gran * gran;
  ScatterAlloc A;
  A.size = n * chunk + rest;
  A.chunk = chunk;
  A.tail = rest;
  A.device = device;
  for (size_t i = 0; i < n + (rest ? 1 : 0); i++) {
    hipMemGenericAllocationHandle_t h;
    if (hipMemCreate(&h, i < n ? chunk : rest, &prop, 0) != hipSuccess) {
      for (auto hh : A.handles) (void)hipMemRelease(hh);
      (void)hipGetLastError();
      return ZH_ENOMEM;
    }
    A.handles.push_back(h);
  }
  void* base = nullptr;
  const int st = scatter_place(A, 0, &base);
  if (st != ZH_OK) {
    for (auto h : A.handles) (void)hipMemRelease(h);
    return st;
  }
  std::lock_guard<std::mutex> lk(g_scatter_mu);
  g_scatter[base] = std::move(A);
  *out = base;
  return ZH_OK;
}

int scatter_view(void* ptr, uint64_t order, void** out) {
  ScatterAlloc V;
  {
    std::lock_guard<std::mutex> lk(g_scatter_mu);
    auto it = g_scatter.find(ptr);
    if (it == g_scatter.end() || it->second.view) return ZH_EINVAL;
    V = it->second;
  }
  V.view = true;
  void* base = nullptr;
  const int st = scatter_place(V, order, &base);
  if (st != ZH_OK) return st;
  std::lock_guard<std::mutex> lk(g_scatter_mu);
  g_scatter[base] = std::move(V);
  *out = base;
  return ZH_OK;
}

bool scatter_free(void* ptr) {
  ScatterAlloc A;
  {
    std::lock_guard<std::mutex> lk(g_scatter_mu);
    auto it = g_scatter.find(ptr);
    if (it == g_scatter.end()) return false;
    A = std::move(it->second);
    g_scatter.erase(it);
  }
  (void)hipDeviceSynchronize();
  scatter_unmap(ptr, A);
  if (!A.view)
    for (auto h : A.handles) (void)hipMemRelease(h);
  (void)hipMemAddressFree(ptr, A.size);
  (void)hipGetLastError();
  return true;
}

// median rate (GB/s of `bytes`) of `reps` timed launches after one untimed one
template <typename Launch>
int stream_rate(hipStream_t s, size_t bytes, int reps, double* gbps, Launch launch) {
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess) return ZH_EHIP;
  if (hipEventCreate(&e1) != hipSuccess) {
    (void)hipEventDestroy(e0);
    return ZH_EHIP;
  }
  int rc = ZH_OK;
  std::vector<float> ms;
  if (launch() != hipSuccess) rc = ZH_EHIP;
  for (int r = 0; rc == ZH_OK && r < reps; r++) {
    float t = 0;
    if (hipEventRecord(e0, s) != hipSuccess || launch() != hipSuccess ||
        hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
        hipEventElapsedTime(&t, e0, e1) != hipSuccess)
      rc = ZH_EHIP;
    else
      ms.push_back(t);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (rc != ZH_OK) {
    (void)hipGetLastError();
    return rc;
  }
  std::sort(ms.begin(), ms.end());
  const double med = ms[ms.size() / 2];
  *gbps = med > 0 ? (double)bytes / (med * 1e-3) / 1e9 : 0.0;
  return ZH_OK;
}

int write_rate(hipStream_t s, void* ptr, size_t bytes, int pattern, int reps, double* gbps) {
  return stream_rate(s, bytes, reps, gbps, [&] {
    return launch_write_probe(ptr, (int64_t)bytes, pattern, s);
  });
}

// ZH_MALLOC_CALIBRATE: the write rate of a large scatter arena is set by which physical chunks
// it got (not their order, not its virtual address), and a contiguous store probe predicts
// the decode's rate into it (profiles/r02/placement/calib*.jsonl).  Allocate up to
// two candidates, holding the first while allocating the second, so the driver hands out
// different chunks, probe each, keep the fastest.  A candidate that does not fit ends the
// search.  On return *out is the kept allocation, with every probe recorded on it.
void scatter_calibrate(zh_ctx* ctx, size_t bytes, void** out) {
  const int tries = 2;
  std::vector<void*> cand{*out};
  std::vector<double> rate;
  for (int k = 0;; k++) {
    double g = 0;
    if (write_rate(ctx->stream, cand[(size_t)k], bytes, 0, 2, &g) != ZH_OK) g = 0;
    rate.push_back(g);
    if (k + 1 >= tries) break;
    void* next = nullptr;
    if (scatter_malloc(ctx->device, bytes, &next) != ZH_OK) break;
    cand.push_back(next);
  }
  size_t best = 0;
  for (size_t i = 1; i < rate.size(); i++)
    if (rate[i] > rate[best]) best = i;
  for (size_t i = 0; i < cand.size(); i++)
    if (i != best) scatter_free(cand[i]);
  std::lock_guard<std::mutex> lk(g_scatter_mu);
  auto it = g_scatter.find(cand[best]);
  if (it != g_scatter.end()) {
    it->second.probes = rate;
    it->second.chosen = (int)best;
  }
  *out = cand[best];
}
}  // namespace

extern "C" {

int zh_abi_sizes(int64_t* out, int n) {
  const int64_t s[4] = {(int64_t)sizeof(zh_codec_chain), (int64_t)sizeof(zh_array_meta),
                        (int64_t)sizeof(zh_chunk_src), (int64_t)sizeof(zh_chunk_dst)};
  for (int i = 0; i < n && i < 4 && out; i++) out[i] = s[i];
  return 4;
}
int zh_device_malloc(zh_ctx* ctx, size_t bytes, void** out) {
  return zh_device_malloc_ex(ctx, bytes, 0, out);
}
int zh_device_malloc_ex(zh_ctx* ctx, size_t bytes, unsigned flags, void** out) {
  if (!ctx || !out) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  // the default kind: large buffers from 1 GiB physical chunks (the highest floor of the
  // round-6 allocation A/B, DESIGN §4 "Placement"), hipMalloc below 1 GiB or when that fails
  if (flags == 0 && bytes >= ((size_t)1 << 30)) flags = ZH_MALLOC_SCATTER;
  hipError_t e = hipErrorOutOfMemory;
  if (flags & ZH_MALLOC_SCATTER) {
    const int st = scatter_malloc(ctx->device, bytes, out);
    if (st == ZH_OK && (flags & ZH_MALLOC_CALIBRATE)) scatter_calibrate(ctx, bytes, out);
    if (st == ZH_OK || (flags & ZH_MALLOC_REQUIRE)) return st;
  }
  if (flags & ZH_MALLOC_CONTIGUOUS) {
    e = hipExtMallocWithFlags(out, bytes, hipDeviceMallocContiguous);
    if (e != hipSuccess) (void)hipGetLastError();
  }
  if (e != hipSuccess && !(flags & ZH_MALLOC_REQUIRE)) e = hipMalloc(out, bytes);
  return e == hipSuccess ? ZH_OK : (e == hipErrorOutOfMemory ? ZH_ENOMEM : ZH_EHIP);
}
int zh_device_scatter_view(zh_ctx* ctx, void* ptr, uint64_t order, void** out) {
  if (!ctx || !ptr || !out) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  return scatter_view(ptr, order, out);
}
int zh_device_alloc_probes(zh_ctx* ctx, void* ptr, double* gbps, int cap, int* chosen) {
  if (!ctx || !ptr) return -ZH_EINVAL;
  std::lock_guard<std::mutex> lk(g_scatter_mu);
  auto it = g_scatter.find(ptr);
  if (it == g_scatter.end()) return 0;
  const auto& P = it->second.probes;
  for (int i = 0; i < cap && i < (int)P.size(); i++) gbps[i] = P[(size_t)i];
  if (chosen) *chosen = it->second.chosen;
  return (int)P.size();
}
int zh_device_write_rate(zh_ctx* ctx, void* ptr, size_t bytes, int pattern, int reps,
                         double* gbps) {
  if (!ctx || !ptr || !gbps || bytes == 0 || reps <= 0 || pattern < 0 || pattern > 1)
    return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  return write_rate(ctx->stream, ptr, bytes, pattern, reps, gbps);
}
int zh_last_data_error(int64_t* coords, int cap, uint64_t* key) {
  if (!g_data_err.set) return 0;
  const int n = (int)g_data_err.cc.size();
  for (int d = 0; coords && d < n && d < cap; d++) coords[d] = g_data_err.cc[(size_t)d];
  if (key) *key = g_data_err.key;
  g_data_err.set = false;  // reported once
  return n;
}
int zh_device_copy_rate(zh_ctx* ctx, void* dst, const void* src, size_t bytes, int reps,
                        double* gbps) {
  if (!ctx || !dst || !src || !gbps || bytes < ((size_t)128 << 10) || reps <= 0)
    return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  const size_t n = bytes / ((size_t)128 << 10) * ((size_t)128 << 10);
  double g = 0;
  const int rc = stream_rate(ctx->stream, n, reps, &g, [&] {
    return launch_copy_probe(dst, src, (int64_t)n, ctx->stream);
  });
  *gbps = 2.0 * g;  // bytes read + bytes written
  return rc;
}
int zh_device_free(zh_ctx* ctx, void* ptr) {
  if (!ctx) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  if (scatter_free(ptr)) return ZH_OK;
  return hipFree(ptr) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_host_malloc_pinned(zh_ctx* ctx, size_t bytes, void** out) {
  if (!ctx || !out) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  return hipHostMalloc(out, bytes, hipHostMallocDefault) == hipSuccess ? ZH_OK : ZH_ENOMEM;
}
int zh_host_free_pinned(zh_ctx* ctx, void* ptr) {
  if (!ctx) return ZH_EINVAL;
  return hipHostFree(ptr) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_host_register(zh_ctx* ctx, void* ptr, size_t bytes) {
  if (!ctx || !ptr) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  return hipHostRegister(ptr, bytes, hipHostRegisterDefault) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_host_unregister(zh_ctx* ctx, void* ptr) {
  if (!ctx || !ptr) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  return hipHostUnregister(ptr) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_memcpy_async(zh_ctx* ctx, void* dst, const void* src, size_t bytes, int kind,
                    void* stream) {
  if (!ctx) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                              : (kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return hipMemcpyAsync(dst, src, bytes, k, s) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_memset_async(zh_ctx* ctx, void* dst, int value, size_t bytes, void* stream) {
  if (!ctx) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return hipMemsetAsync(dst, value, bytes, s) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_stream_synchronize(zh_ctx* ctx, void* stream) {
  if (!ctx) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return hipStreamSynchronize(s) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_stream_create(zh_ctx* ctx, void** stream) {
  if (!ctx || !stream) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  return hipStreamCreateWithFlags((hipStream_t*)stream, hipStreamNonBlocking) == hipSuccess
             ? ZH_OK
             : ZH_EHIP;
}
int zh_stream_destroy(zh_ctx* ctx, void* stream) {
  if (!ctx || !stream) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_stream_wait_event(zh_ctx* ctx, void* stream, void* ev) {
  if (!ctx || !ev) return ZH_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return hipStreamWaitEvent(s, (hipEvent_t)ev, 0) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_memcpy2d_async(zh_ctx* ctx, void* dst, size_t dpitch, const void* src, size_t spitch,
                      size_t width, size_t height, int kind, void* stream) {
  if (!ctx) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                              : (kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, k, s) == hipSuccess ? ZH_OK
                                                                                      : ZH_EHIP;
}
int zh_event_create(zh_ctx* ctx, void** ev) {
  if (!ctx || !ev) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  return hipEventCreate((hipEvent_t*)ev) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_event_destroy(zh_ctx* ctx, void* ev) {
  if (!ctx) return ZH_EINVAL;
  return hipEventDestroy((hipEvent_t)ev) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_event_record(zh_ctx* ctx, void* ev, void* stream) {
  if (!ctx) return ZH_EINVAL;
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return hipEventRecord((hipEvent_t)ev, s) == hipSuccess ? ZH_OK : ZH_EHIP;
}
int zh_event_elapsed_ms(zh_ctx* ctx, void* start, void* stop, float* ms) {
  if (!ctx || !ms) return ZH_EINVAL;
  if (hipEventSynchronize((hipEvent_t)stop) != hipSuccess) return ZH_EHIP;
  return hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop) == hipSuccess ? ZH_OK
                                                                                    : ZH_EHIP;
}
int zh_device_info(zh_ctx* ctx, char* name, size_t namelen, int64_t* total_mem, int* cu_count,
                   char* arch, size_t archlen) {
  if (!ctx) return ZH_EINVAL;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, ctx->device) != hipSuccess) return ZH_EHIP;
  if (name && namelen) snprintf(name, namelen, "%s", p.name);
  if (arch && archlen) snprintf(arch, archlen, "%s", p.gcnArchName);
  if (total_mem) *total_mem = (int64_t)p.totalGlobalMem;
  if (cu_count) *cu_count = p.multiProcessorCount;
  return ZH_OK;
}

int zh_gather_blocks(zh_ctx* ctx, void* dst, const void* src, int64_t block_bytes,
                     const int64_t* src_block, int64_t n) {
  if (!ctx || !dst || !src || !src_block || n < 0 || block_bytes <= 0 || block_bytes % 16 ||
      ((uintptr_t)dst | (uintptr_t)src) & 15)
    return ZH_EINVAL;
  if (n == 0) return ZH_OK;
  (void)hipSetDevice(ctx->device);
  std::lock_guard<std::mutex> lk(ctx->mu);
  int64_t* d = nullptr;
  if (hipMalloc((void**)&d, (size_t)n * sizeof(int64_t)) != hipSuccess) {
    (void)hipGetLastError();
    return ZH_ENOMEM;
  }
  int rc = ZH_OK;
  if (hipMemcpyAsync(d, src_block, (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice,
                     ctx->stream) != hipSuccess ||
      launch_gather_blocks(dst, src, d, n, block_bytes, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess) {
    (void)hipGetLastError();
    rc = ZH_EHIP;
  }
  (void)hipFree(d);
  return rc;
}

int zh_synth_fill(zh_ctx* ctx, void* dst, int64_t n, int dtype_size, int64_t first,
                  uint64_t seed, void* stream) {
  if (!ctx || !dst) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return launch_synth_fill(dst, n, dtype_size, first, seed, s) == hipSuccess ? ZH_OK : ZH_EHIP;
}

int zh_synth_verify(zh_ctx* ctx, const void* region, int ndim, const int64_t* array_shape,
                    const int64_t* offset, const int64_t* shape, int dtype_size, uint64_t seed,
                    uint64_t* mismatches, void* stream) {
  if (!ctx || !region || !mismatches || ndim <= 0 || ndim > kMaxDims) return ZH_EINVAL;
  (void)hipSetDevice(ctx->device);
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  unsigned long long* d = nullptr;
  if (hipMalloc((void**)&d, sizeof(*d)) != hipSuccess) return ZH_ENOMEM;
  int rc = ZH_OK;
  if (hipMemsetAsync(d, 0, sizeof(*d), s) != hipSuccess ||
      launch_synth_verify(region, ndim, array_shape, offset, shape, dtype_size, seed, d, s) !=
          hipSuccess ||
      hipMemcpyAsync(mismatches, d, sizeof(*d), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    rc = ZH_EHIP;
  (void)hipFree(d);
  return rc;
}

}  // extern "C"
