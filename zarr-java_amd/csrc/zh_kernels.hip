// zh_kernels.hip — hand-written CDNA4 (gfx950) kernels of the Zarr v3 chunk codec path.
//
//   crc_partial / crc_finalize   sharding index CRC-32C (Crc32cCodec.decode,
//                                M/v3/codec/core/Crc32cCodec.java:24-48; CRC32C.java:119-125):
//                                per-lane slicing-by-8 segment CRCs combined in GF(2)
//   resolve                      index parse: one 32-byte descriptor per inner chunk
//                                (ShardingIndexedCodec.java:206-230)
//   decode<DS,TILE>              the per-inner-chunk codec chain + region scatter
//                                (ShardingIndexedCodec.decodeInternal :183-243, BytesCodec.decode,
//                                TransposeCodec.decode, MultiArrayUtils.copyRegion)
//   encode<DS,TILE>              the inverse (ShardingIndexedCodec.encode payload writes)
//   flags                        encode pre-pass: inner chunk all fill_value? (:129-133)
//   synth_fill / synth_verify    synthetic data for the bench and full-size property tests
//
// Everything is byte movement: HBM-bound.  The scatter kernel streams each inner chunk
// with 16-byte per-lane loads/stores (1 KiB per wave instruction); the transpose variant
// stages 32x32-element tiles through padded LDS so that both the read (payload-fast
// axis) and the write (region-fast axis) are whole 128-byte rows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "zh_internal.h"

namespace zh {

// ---------------------------------------------------------------------------------
// element helpers
// ---------------------------------------------------------------------------------
template <int DS> struct ElemT;
template <> struct ElemT<1> { using T = uint8_t; };
template <> struct ElemT<2> { using T = uint16_t; };
template <> struct ElemT<4> { using T = uint32_t; };
template <> struct ElemT<8> { using T = uint64_t; };

template <int DS>
__device__ __forceinline__ typename ElemT<DS>::T xform1(typename ElemT<DS>::T v, int swap,
                                                         int is_bool) {
  if constexpr (DS == 1) {
    (void)swap;
    return is_bool ? (uint8_t)(v != 0) : v;
  } else if constexpr (DS == 2) {
    (void)is_bool;
    return swap ? (uint16_t)((v >> 8) | (v << 8)) : v;
  } else if constexpr (DS == 4) {
    (void)is_bool;
    return swap ? __builtin_bswap32(v) : v;
  } else {
    (void)is_bool;
    return swap ? __builtin_bswap64(v) : v;
  }
}

__device__ __forceinline__ uint32_t bool_bytes(uint32_t x) {
  // per byte: 1 if non-zero, else 0
  uint32_t t = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;
  return (t >> 7) & 0x01010101u;
}

template <int DS>
__device__ __forceinline__ uint4 xform16(uint4 v, int swap, int is_bool) {
  if constexpr (DS == 1) {
    (void)swap;
    if (is_bool) {
      v.x = bool_bytes(v.x);
      v.y = bool_bytes(v.y);
      v.z = bool_bytes(v.z);
      v.w = bool_bytes(v.w);
    }
    return v;
  } else if constexpr (DS == 2) {
    (void)is_bool;
    if (swap) {
      v.x = ((v.x & 0x00FF00FFu) << 8) | ((v.x >> 8) & 0x00FF00FFu);
      v.y = ((v.y & 0x00FF00FFu) << 8) | ((v.y >> 8) & 0x00FF00FFu);
      v.z = ((v.z & 0x00FF00FFu) << 8) | ((v.z >> 8) & 0x00FF00FFu);
      v.w = ((v.w & 0x00FF00FFu) << 8) | ((v.w >> 8) & 0x00FF00FFu);
    }
    return v;
  } else if constexpr (DS == 4) {
    (void)is_bool;
    if (swap) {
      v.x = __builtin_bswap32(v.x);
      v.y = __builtin_bswap32(v.y);
      v.z = __builtin_bswap32(v.z);
      v.w = __builtin_bswap32(v.w);
    }
    return v;
  } else {
    (void)is_bool;
    if (swap) {
      uint4 r;
      r.x = __builtin_bswap32(v.y);
      r.y = __builtin_bswap32(v.x);
      r.z = __builtin_bswap32(v.w);
      r.w = __builtin_bswap32(v.z);
      return r;
    }
    return v;
  }
}

template <int DS>
__device__ __forceinline__ uint4 fill16(uint64_t f) {
  uint32_t lo = (uint32_t)f, hi = (uint32_t)(f >> 32);
  uint32_t w;
  if constexpr (DS == 1) {
    w = (lo & 0xFFu) * 0x01010101u;
  } else if constexpr (DS == 2) {
    w = (lo & 0xFFFFu) * 0x00010001u;
  } else {
    w = lo;
  }
  if constexpr (DS == 8) return make_uint4(lo, hi, lo, hi);
  return make_uint4(w, w, w, w);
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld16(const uint8_t* p) {
  return *reinterpret_cast<const uint4*>(p);
}
__device__ __forceinline__ void st16(uint8_t* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }

// streaming (non-temporal) forms: once-read source, once-written destination; measured
// +4-6 % on 96 GiB copies (zarr-java_amd/tools/copy_lab.hip)
template <bool NT>
__device__ __forceinline__ uint4 ld16s(const uint8_t* p) {
  if constexpr (NT) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return ld16(p);
  }
}
// non-temporal 16-B global load at a wave-uniform base + a 32-bit lane offset (global_load with
// a scalar base: no 64-bit address per load in VGPRs)
__device__ __forceinline__ uint4 ld16g(const uint8_t* base, uint32_t off) {
  const v4u v = __builtin_nontemporal_load(
      reinterpret_cast<const __attribute__((address_space(1))) v4u*>(
          (const __attribute__((address_space(1))) uint8_t*)base + off));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16g(uint8_t* base, uint32_t off, uint4 v) {
  __builtin_nontemporal_store(
      v4u{v.x, v.y, v.z, v.w},
      reinterpret_cast<__attribute__((address_space(1))) v4u*>(
          (__attribute__((address_space(1))) uint8_t*)base + off));
}
template <bool NT>
__device__ __forceinline__ void st16s(uint8_t* p, uint4 v) {
  if constexpr (NT) {
    __builtin_nontemporal_store(v4u{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u*>(p));
  } else {
    st16(p, v);
  }
}

template <int DS>
__device__ __forceinline__ typename ElemT<DS>::T ld1(const uint8_t* p) {
  return *reinterpret_cast<const typename ElemT<DS>::T*>(p);
}
template <int DS>
__device__ __forceinline__ void st1(uint8_t* p, typename ElemT<DS>::T v) {
  *reinterpret_cast<typename ElemT<DS>::T*>(p) = v;
}

__device__ __forceinline__ uint64_t ld_u64_unaligned(const uint8_t* p, int big) {
  uint64_t v = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
  return big ? __builtin_bswap64(v) : v;
}

// ---------------------------------------------------------------------------------
// per-item geometry (all values are wave-uniform).  Every per-dimension loop runs over
// the compile-time bound kMaxDims with a uniform `d < n` guard, so the arrays below
// are indexed by constants after unrolling and live in (scalar) registers, not scratch.
// ---------------------------------------------------------------------------------
enum ItemMode : int { kCopy = 0, kFill = 1, kSkip = 2 };

struct Item {
  const uint8_t* sbase;   // source bytes (payload for decode, region for encode)
  uint8_t* dbase;         // destination bytes
  int64_t s0, d0;         // element offsets of the box origin
  int32_t e[kMaxDims];    // box extents (elements written)
  int32_t v[kMaxDims];    // loadable extents (encode: array-domain clip; decode: == e)
  FastDiv ediv[kMaxDims]; // divisors for e[]
  uint64_t fill;          // constant for kFill
  int mode;
  uint32_t piece;
};

__device__ __forceinline__ int64_t find_shard(const ScatterArgs& a, int64_t citem) {
  int64_t lo = 0, hi = a.nshards - 1;
  while (lo < hi) {
    int64_t mid = (lo + hi + 1) >> 1;
    if (a.shards[mid].item_begin <= citem) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Index entry `lin` of shard S: the stored index (index_codecs endianness) or, for nested
// sharding, the flattened little-endian leaf index written by nested_index_kernel.
__device__ __forceinline__ void index_entry(const ScatterArgs& a, const DevShard& S, int64_t lin,
                                            uint64_t& off, uint64_t& nb) {
  if (S.flat) {
    const uint64_t* e = reinterpret_cast<const uint64_t*>(S.flat) + 2 * lin;
    off = e[0];
    nb = e[1];
    return;
  }
  const uint8_t* ent = S.data + S.index_off + 16 * lin;
  off = ld_u64_unaligned(ent, a.index_be);
  nb = ld_u64_unaligned(ent + 8, a.index_be);
}

__device__ __forceinline__ uint32_t rank_clamp(uint64_t r) {
  return r > 0xFFFFFFFEull ? 0xFFFFFFFEu : (uint32_t)r;
}

// The rank (RankGeom) of the inner chunk — the leaf, nested — at shard-grid coordinates ic.
__device__ __forceinline__ uint32_t chunk_rank(const RankGeom& g, const int32_t* ic) {
  uint64_t l1 = 0, k2 = 0;
#pragma unroll
  for (int d = 0; d < kMaxDims; d++) {
    if (d >= g.ndim) continue;
    if (g.r2 == 0) {
      l1 += (uint64_t)ic[d] * (uint64_t)g.cps_stride[d];
      continue;
    }
    const int32_t c1 = ic[d] / g.r[d];
    l1 += (uint64_t)c1 * (uint64_t)g.cps1_stride[d];
    k2 += (uint64_t)(ic[d] - c1 * g.r[d]) * (uint64_t)g.k2_stride[d];
  }
  return rank_clamp(g.r2 == 0 ? l1 : l1 * (uint64_t)g.r2 + 1 + k2);
}

// Records a chunk-level decode error in the shard's status words st: the lowest rank wins the
// key, and its details (a failed crc32c's stored and computed values, a short sub-shard's
// length) win the detail words, which are keyed by the same rank.
__device__ __forceinline__ void chunk_error(uint64_t* st, uint32_t rank, uint32_t kind,
                                            uint32_t da = 0, uint32_t db = 0) {
  const uint64_t hi = (uint64_t)(0xFFFFFFFFu - rank);
  atomicOr((unsigned long long*)(st + kStFlags),
           (unsigned long long)(kind & (kFlagRange | kFlagLength | kFlagChunkCrc | kFlagShort)));
  atomicMax((unsigned long long*)(st + kStBadChunk), (unsigned long long)((hi << 8) | kind));
  if (kind & (kFlagChunkCrc | kFlagShort)) {
    atomicMax((unsigned long long*)(st + kStDetailA), (unsigned long long)((hi << 32) | da));
    atomicMax((unsigned long long*)(st + kStDetailB), (unsigned long long)((hi << 32) | db));
  }
}

// Device address of the stored range [off, off + nb) of shard S (range-checked against the
// object size by the caller).  Without a piece table the object is whole at S.data.  With
// one (sub-shard reads: StoreHandleDataProvider.read(off, nb), ShardingIndexedCodec.java:
// 226-230, 353-356) the range must lie inside one piece; a host-decoded piece serves exactly
// its own range and *nb becomes its payload length.  false: no piece holds the range → the
// reference's "Could not load byte data for chunk".
__device__ __forceinline__ bool piece_src(const DevShard& S, uint64_t off, uint64_t& nb,
                                          const uint8_t*& src) {
  if (S.pieces == nullptr) {
    src = S.data + off;
    return true;
  }
  if (nb == 0) {  // an empty range is an empty buffer wherever it points (get(k, o, o)); the
    src = S.data;  // caller's length check then rejects it as the oracle does
    return true;
  }
  int64_t lo = 0, hi = S.npieces - 1;
  if (hi < 0 || S.pieces[0].off > off) return false;
  while (lo < hi) {  // last piece with p.off <= off
    const int64_t mid = (lo + hi + 1) >> 1;
    if (S.pieces[mid].off <= off) lo = mid;
    else hi = mid - 1;
  }
  const DevPiece P = S.pieces[lo];
  const uint64_t rel = off - P.off;
  if (P.dlen != P.len) {  // one host-decoded inner chunk
    if (rel != 0 || nb != P.len) return false;
    nb = P.dlen;
    src = P.src;
    return true;
  }
  if (rel > P.len || nb > P.len - rel) return false;
  src = P.src + rel;
  return true;
}

// Builds the geometry of work item `item` (returns the shard slot).  Decode (the generic
// kernel's clipped items): source, fill and mode come from the item's descriptor `D`, which
// the resolve kernel wrote after parsing and validating the index entry.
template <bool ENC>
__device__ __forceinline__ int64_t make_item(const ScatterArgs& a, int64_t item, Item& it,
                                             const ItemDesc* D = nullptr) {
  const int n = a.ndim;
  const int64_t citem = item >> a.piece_shift;
  it.piece = (uint32_t)(item & ((1ll << a.piece_shift) - 1));
  const int64_t s = find_shard(a, citem);
  const DevShard& S = a.shards[s];
  // inner-chunk coordinates: C-order unravel of the item inside the shard's box
  // (IndexingUtils.computeChunkCoords order, M/utils/IndexingUtils.java:36-49)
  uint32_t j = (uint32_t)(citem - S.item_begin);
  int32_t ic[kMaxDims];
#pragma unroll
  for (int d = kMaxDims - 1; d >= 0; --d) {
    ic[d] = 0;
    if (d < n) {
      const uint32_t c = (uint32_t)S.box_count[d];
      const uint32_t q = j / c;
      ic[d] = S.box_start[d] + (int32_t)(j - q * c);
      j = q;
    }
  }
  it.mode = kCopy;
  it.fill = 0;
  if constexpr (!ENC) {
    // kDescClip: src != 0 copies; src == 0 keeps the constant the resolve kernel chose
    // (fill_value for a missing shard, M/core/Array.java:400-402, 419-421; 0 for a missing
    // inner chunk, Q1, ShardingIndexedCodec.java:189, 219-221)
    if (D->src != 0) {
      it.sbase = (const uint8_t*)(uintptr_t)D->src;
    } else {
      it.mode = kFill;
      it.fill = D->fill;
      it.sbase = nullptr;
    }
    it.dbase = a.region;
    int64_t s0 = 0, d0 = S.out_base;
#pragma unroll
    for (int d = 0; d < kMaxDims; d++) {
      it.e[d] = 1;
      it.v[d] = 1;
      it.ediv[d] = a.inner_div[0];
      if (d < n) {
        const int32_t io = ic[d] * a.inner[d];
        const int32_t lo = max(io, S.part_lo[d]) - io;
        const int32_t hi = min(io + a.inner[d], S.part_hi[d]) - io;
        it.e[d] = hi - lo;
        it.v[d] = hi - lo;
        s0 += (int64_t)lo * a.pstride[d];
        d0 += (int64_t)(io + lo - S.part_lo[d]) * a.rstride[d];
        it.ediv[d] = (hi - lo == a.inner[d]) ? a.inner_div[d] : make_fastdiv((uint32_t)(hi - lo));
      }
    }
    it.s0 = s0;
    it.d0 = d0;
  } else {
    const int64_t off = a.item_off ? a.item_off[citem] : 0;
    if (off < 0) {
      it.mode = kSkip;
      return s;
    }
    it.sbase = a.region;
    it.dbase = S.wdata + off;
    int64_t s0 = S.out_base;
    bool empty = false;
#pragma unroll
    for (int d = 0; d < kMaxDims; d++) {
      it.e[d] = 1;
      it.v[d] = 1;
      it.ediv[d] = a.inner_div[0];
      if (d < n) {
        const int32_t io = ic[d] * a.inner[d];
        const int32_t vhi = min(io + a.inner[d], S.part_hi[d]) - io;
        it.e[d] = a.inner[d];
        it.v[d] = max(vhi, 0);
        empty |= vhi <= 0;
        s0 += (int64_t)(io - S.part_lo[d]) * a.rstride[d];
        it.ediv[d] = a.inner_div[d];
      }
    }
    it.s0 = s0;
    it.d0 = 0;
    // an inner chunk entirely in the boundary padding is all fill: never encoded, unless no
    // element equals the fill (a NaN fill): then it is stored as padding like any other
    if (empty && !a.fill_never) it.mode = kSkip;
  }
  return s;
}

// The write path's all-fill test (MultiArrayUtils.allValuesEqual, Java's ==): does an
// element differ from fill_value?  Bits compared under a.fill_mask, which drops the sign bit
// for a float ±0 fill (+0.0 == -0.0); every other fill compares every bit.  A NaN fill equals
// nothing: a.fill_never, the flags then start at 1 and every chunk is kept (engine.cpp).
__device__ __forceinline__ bool ne16(const uint4& v, const uint4& f, const uint4& m) {
  return (((v.x ^ f.x) & m.x) | ((v.y ^ f.y) & m.y) | ((v.z ^ f.z) & m.z) |
          ((v.w ^ f.w) & m.w)) != 0;
}
__device__ __forceinline__ bool ne4x4(const uint4& v, uint32_t f, uint32_t m) {
  return (((v.x ^ f) | (v.y ^ f) | (v.z ^ f) | (v.w ^ f)) & m) != 0;
}

// ---------------------------------------------------------------------------------
// row pass: rows along dim F, unit-stride on both sides (on the destination only for
// constant fills).  VEC: 16-byte granules; otherwise single elements with
// loadable-extent checks.  CHECK: compare against fill_value instead of storing.
// CLIP (encode, VEC only): the item is clipped by the array domain at a 16-byte granule
// boundary of F and/or in whole rows; granules outside the loadable extents store the
// encoded fill_value (boundary padding) instead of loading.  FLAG (encode, storing): also
// return whether a loaded element differs from fill_value (one read for test + encode).
// ---------------------------------------------------------------------------------
template <int DS, bool VEC, bool CHECK, bool CLIP = false, bool FLAG = false>
__device__ __forceinline__ bool row_pass(const ScatterArgs& a, const Item& it, int F,
                                         const int64_t* sstr, const int64_t* dstr,
                                         uint32_t nrows, const int32_t* ext,
                                         const FastDiv* ediv) {
  using T = typename ElemT<DS>::T;
  constexpr int U = 4;
  const int n = a.ndim;
  const bool fill = it.mode == kFill;
  int32_t eF = 1;
#pragma unroll
  for (int d = 0; d < kMaxDims; d++)
    if (d == F) eF = ext[d];
  const uint32_t gpr = VEC ? (uint32_t)(eF * DS / 16) : (uint32_t)eF;
  if (gpr == 0 || nrows == 0) return false;
  const FastDiv gdiv = make_fastdiv(gpr);
  const uint32_t pieces = 1u << a.piece_shift;
  const uint32_t r0 = (uint32_t)(((uint64_t)nrows * it.piece) / pieces);
  const uint32_t r1 = (uint32_t)(((uint64_t)nrows * (it.piece + 1)) / pieces);
  const uint32_t total = (r1 - r0) * gpr;
  const uint4 fv = fill16<DS>(CHECK ? a.fill : it.fill);
  const uint4 pad = fill16<DS>(a.fill);  // CLIP: raw fill_value granule (encoded on store)
  const uint4 fm = fill16<DS>(a.fill_mask);
  int64_t sF = 1, dF = 1;
  uint32_t vgF = 0;  // CLIP: loadable granules along F
#pragma unroll
  for (int d = 0; d < kMaxDims; d++)
    if (d == F) {
      sF = sstr[d];
      dF = dstr[d];
      vgF = (uint32_t)(it.v[d] * DS / 16);
    }
  bool diff = false;
  for (uint32_t base = threadIdx.x; base < total; base += kBlock * U) {
    uint4 vv[U];
    T sv[U];
    int64_t doff[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t g = base + u * kBlock;
      ok[u] = g < total;
      vv[u] = make_uint4(0, 0, 0, 0);
      sv[u] = 0;
      doff[u] = 0;
      if (!ok[u]) continue;
      uint32_t r = fdiv(g, gdiv);
      const uint32_t c = g - r * gpr;
      r += r0;
      int64_t so = it.s0, dof = it.d0;
      bool valid = true;
#pragma unroll
      for (int d = kMaxDims - 1; d >= 0; --d) {
        if (d >= n || d == F) continue;
        if (ext[d] <= 1) {  // one element along d: loadable unless the item lies beyond the
          valid &= it.v[d] > 0;  // array there (a padding-only item, kept for a NaN fill)
          continue;
        }
        const uint32_t q = fdiv(r, ediv[d]);
        const uint32_t m = r - q * (uint32_t)ext[d];
        so += (int64_t)m * sstr[d];
        dof += (int64_t)m * dstr[d];
        valid &= (int32_t)m < it.v[d];
        r = q;
      }
      if constexpr (VEC) {
        doff[u] = dof * DS + (int64_t)c * 16;
        if constexpr (CLIP) {
          valid &= c < vgF;
          vv[u] = valid ? ld16(it.sbase + so * DS + (int64_t)c * 16) : pad;
        } else if (!fill) {
          vv[u] = ld16(it.sbase + so * DS + (int64_t)c * 16);
        }
      } else {
        doff[u] = (dof + (int64_t)c * dF) * DS;
        bool vF = false;
#pragma unroll
        for (int d = 0; d < kMaxDims; d++)
          if (d == F) vF = (int32_t)c < it.v[d];
        valid &= vF;
        if (!fill) sv[u] = valid ? ld1<DS>(it.sbase + (so + (int64_t)c * sF) * DS) : (T)a.fill;
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      if (!ok[u]) continue;
      if constexpr (CHECK) {
        if constexpr (VEC) {
          diff |= ne16(vv[u], fv, fm);
        } else {
          diff |= ((sv[u] ^ (T)a.fill) & (T)a.fill_mask) != 0;
        }
      } else if constexpr (VEC) {
        st16(it.dbase + doff[u], fill ? fv : xform16<DS>(vv[u], a.swap, a.is_bool));
        if constexpr (FLAG) diff |= ne16(vv[u], pad, fm);
      } else {
        st1<DS>(it.dbase + doff[u], fill ? (T)it.fill : xform1<DS>(sv[u], a.swap, a.is_bool));
        if constexpr (FLAG) diff |= ((sv[u] ^ (T)a.fill) & (T)a.fill_mask) != 0;
      }
    }
  }
  return diff;
}

// Can the whole item move in 16-byte granules along F?  ENC: the destination is a shard
// payload, which may sit at 4 mod 16 (after a chunk's crc32c or a sub-shard index):
// dwordx4 stores, like loads, need dword alignment only in gfx9's unaligned mode.
template <int DS, bool ENC = false>
__device__ __forceinline__ bool vec_ok(const ScatterArgs& a, const Item& it, int F,
                                       const int64_t* sstr, const int64_t* dstr,
                                       const int32_t* ext, bool need_src) {
  const int n = a.ndim;
  bool ok = !(((uintptr_t)(it.dbase + it.d0 * DS)) & (ENC ? 3 : 15));
  // sources need dword alignment only: a chunk after a 4-byte crc32c or a sub-shard index
  // sits at 4 mod 16, and dwordx4 loads from dword-aligned addresses are legal on gfx950
  if (need_src) ok &= !(((uintptr_t)(it.sbase + it.s0 * DS)) & 3);
#pragma unroll
  for (int d = 0; d < kMaxDims; d++) {
    if (d >= n) continue;
    if (d == F) {
      ok &= !((ext[d] * DS) & 15);
      if (need_src) ok &= it.v[d] == ext[d];
      continue;
    }
    if (ext[d] > 1) {
      ok &= !((dstr[d] * DS) & 15);
      if (need_src) ok &= !((sstr[d] * DS) & 15);
    }
    if (need_src) ok &= it.v[d] == ext[d];
  }
  return ok;
}

// Encode: can a domain-clipped item move in 16-byte granules along F (row_pass CLIP)?  The
// loadable extent along F must end on a granule boundary; clipped rows are padded whole.
template <int DS>
__device__ __forceinline__ bool vec_clip_ok(const ScatterArgs& a, const Item& it, int F,
                                            const int64_t* sstr, const int64_t* dstr) {
  const int n = a.ndim;
  bool ok = !(((uintptr_t)(it.dbase + it.d0 * DS)) & 3) &&
            !(((uintptr_t)(it.sbase + it.s0 * DS)) & 3);
#pragma unroll
  for (int d = 0; d < kMaxDims; d++) {
    if (d >= n) continue;
    if (d == F) {
      ok &= !((it.e[d] * DS) & 15) && !((it.v[d] * DS) & 15);
    } else if (it.e[d] > 1) {
      ok &= !((dstr[d] * DS) & 15) && !((sstr[d] * DS) & 15);
    }
  }
  return ok;
}

// ---------------------------------------------------------------------------------
// tile pass: transpose between the src-fast dim fs and the dst-fast dim fd through
// 32x32-element LDS tiles (row pitch 33 elements: conflict-free on both sides).
// ---------------------------------------------------------------------------------
template <int DS>
__device__ __forceinline__ void tile_pass(const ScatterArgs& a, const Item& it,
                                          const int64_t* sstr, const int64_t* dstr,
                                          typename ElemT<DS>::T (*tile)[32][33]) {
  using T = typename ElemT<DS>::T;
  const int n = a.ndim, fs = a.fs, fd = a.fd;
  const int tid = threadIdx.x, l = tid >> 3, g = tid & 7;
  int32_t efs = 1, efd = 1, vfs = 1, vfd = 1;
  int64_t ss_fs = 1, ss_fd = 1, ds_fs = 1, ds_fd = 1;
  uint32_t nb = 1;
  bool vec = DS == 4 && !(((uintptr_t)(it.sbase + it.s0 * DS)) & 3) &&
             !(((uintptr_t)(it.dbase + it.d0 * DS)) & 15);
#pragma unroll
  for (int d = 0; d < kMaxDims; d++) {
    if (d >= n) continue;
    if (d == fs) {
      efs = it.e[d];
      vfs = it.v[d];
      ss_fs = sstr[d];
      ds_fs = dstr[d];
    }
    if (d == fd) {
      efd = it.e[d];
      vfd = it.v[d];
      ss_fd = sstr[d];
      ds_fd = dstr[d];
    }
    if (d != fs && d != fd) nb *= (uint32_t)it.e[d];
    if (d != fs && (sstr[d] & 3)) vec = false;
    if (d != fd && (dstr[d] & 3)) vec = false;
    if (it.v[d] != it.e[d]) vec = false;
  }
  const uint32_t ts = (uint32_t)(efs + 31) >> 5, td = (uint32_t)(efd + 31) >> 5;
  const uint32_t units = nb * ts * td;
  const uint32_t pieces = 1u << a.piece_shift;
  const uint32_t u0 = (uint32_t)(((uint64_t)units * it.piece) / pieces);
  const uint32_t u1 = (uint32_t)(((uint64_t)units * (it.piece + 1)) / pieces);
  const FastDiv tddiv = make_fastdiv(td), tsdiv = make_fastdiv(ts);
  for (uint32_t ub = u0; ub < u1; ub += kTileTPB) {
    int64_t so_t[kTileTPB], do_t[kTileTPB];
    uint32_t xs0[kTileTPB], xd0[kTileTPB];
    bool bval[kTileTPB], live[kTileTPB];
#pragma unroll
    for (int t = 0; t < kTileTPB; t++) {
      const uint32_t unit = ub + t;
      live[t] = unit < u1;
      const uint32_t q1 = fdiv(unit, tddiv);
      const uint32_t ud = unit - q1 * td;
      uint32_t b = fdiv(q1, tsdiv);
      const uint32_t us = q1 - b * ts;
      int64_t so = it.s0 + (int64_t)(us * 32) * ss_fs + (int64_t)(ud * 32) * ss_fd;
      int64_t dof = it.d0 + (int64_t)(us * 32) * ds_fs + (int64_t)(ud * 32) * ds_fd;
      bool bv = true;
#pragma unroll
      for (int d = kMaxDims - 1; d >= 0; --d) {
        if (d >= n || d == fs || d == fd) continue;
        if (it.e[d] <= 1) {  // see row_pass: a padding-only item loads nothing
          bv &= it.v[d] > 0;
          continue;
        }
        const uint32_t q = fdiv(b, it.ediv[d]);
        const uint32_t m = b - q * (uint32_t)it.e[d];
        so += (int64_t)m * sstr[d];
        dof += (int64_t)m * dstr[d];
        bv &= (int32_t)m < it.v[d];
        b = q;
      }
      so_t[t] = so;
      do_t[t] = dof;
      xs0[t] = us * 32;
      xd0[t] = ud * 32;
      bval[t] = bv;
    }
    // load phase: lane (l, g) reads 4 consecutive fs-elements of fd-row l
#pragma unroll
    for (int t = 0; t < kTileTPB; t++) {
      if (!live[t]) continue;
      const bool full = xs0[t] + 32 <= (uint32_t)efs && xd0[t] + 32 <= (uint32_t)efd;
      if (vec && full) {
        const uint4 x = ld16(it.sbase + (so_t[t] + (int64_t)l * ss_fd + g * 4) * 4);
        T* row = &tile[t][l][g * 4];
        row[0] = (T)xform1<4>(x.x, a.swap, 0);
        row[1] = (T)xform1<4>(x.y, a.swap, 0);
        row[2] = (T)xform1<4>(x.z, a.swap, 0);
        row[3] = (T)xform1<4>(x.w, a.swap, 0);
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t xs = xs0[t] + g * 4 + k, xd = xd0[t] + l;
          if (xs < (uint32_t)efs && xd < (uint32_t)efd) {
            const bool ld = bval[t] && (int32_t)xs < vfs && (int32_t)xd < vfd;
            const T x = ld ? ld1<DS>(it.sbase + (so_t[t] + (int64_t)l * ss_fd +
                                                 (int64_t)(g * 4 + k) * ss_fs) * DS)
                           : (T)a.fill;
            tile[t][l][g * 4 + k] = xform1<DS>(x, a.swap, a.is_bool);
          }
        }
      }
    }
    __syncthreads();
    // store phase: lane (l = fs-row, g) writes 4 consecutive fd-elements of fs-row l
#pragma unroll
    for (int t = 0; t < kTileTPB; t++) {
      if (!live[t]) continue;
      const bool full = xs0[t] + 32 <= (uint32_t)efs && xd0[t] + 32 <= (uint32_t)efd;
      if (vec && full) {
        uint4 y;
        y.x = (uint32_t)tile[t][g * 4 + 0][l];
        y.y = (uint32_t)tile[t][g * 4 + 1][l];
        y.z = (uint32_t)tile[t][g * 4 + 2][l];
        y.w = (uint32_t)tile[t][g * 4 + 3][l];
        st16(it.dbase + (do_t[t] + (int64_t)l * ds_fs + g * 4) * 4, y);
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t xs = xs0[t] + l, xd = xd0[t] + g * 4 + k;
          if (xs < (uint32_t)efs && xd < (uint32_t)efd)
            st1<DS>(it.dbase + (do_t[t] + (int64_t)l * ds_fs + (int64_t)(g * 4 + k) * ds_fd) * DS,
                    tile[t][g * 4 + k][l]);
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------
// resolve kernel (index parse): one thread per inner chunk → ItemDesc.  Validates the
// index entry (ShardingIndexedCodec.java:215-230) and classifies the item so that the
// scatter kernel's per-item work is a single 32-byte descriptor load, issued one item
// ahead.
// ---------------------------------------------------------------------------------
__device__ __forceinline__ ItemDesc resolve_one(const ScatterArgs& a, int64_t citem) {
  ItemDesc D;
  D.src = 0;
  D.d0 = 0;
  D.fill = 0;
  D.kind = kDescSkip;
  const int n = a.ndim;
  const int64_t s = find_shard(a, citem);
  const DevShard& S = a.shards[s];
  D.shard = (uint32_t)s;
  uint32_t j = (uint32_t)(citem - S.item_begin);
  int32_t ic[kMaxDims];
#pragma unroll
  for (int d = kMaxDims - 1; d >= 0; --d) {
    ic[d] = 0;
    if (d < n) {
      const uint32_t c = (uint32_t)S.box_count[d];
      const uint32_t q = j / c;
      ic[d] = S.box_start[d] + (int32_t)(j - q * c);
      j = q;
    }
  }
  bool full = true, row_clip = true;  // row_clip: cut only along the unit-stride dim
  int32_t hi_f = 0;
  int64_t d0 = S.out_base, lin = 0;
#pragma unroll
  for (int d = 0; d < kMaxDims; d++) {
    if (d >= n) continue;
    const int32_t io = ic[d] * a.inner[d];
    const int32_t lo = max(io, S.part_lo[d]) - io;
    const int32_t hi = min(io + a.inner[d], S.part_hi[d]) - io;
    full &= lo == 0 && hi == a.inner[d];
    row_clip &= lo == 0 && (d == a.fs || hi == a.inner[d]);
    if (d == a.fs) hi_f = hi;
    d0 += (int64_t)(io + lo - S.part_lo[d]) * a.rstride[d];
    lin += (int64_t)ic[d] * a.cps_stride[d];
  }
  D.d0 = d0;
  if (S.data == nullptr) {  // missing shard → fill_value (Array.java:400-402, 419-421)
    D.kind = full ? kDescFullFill : kDescClip;
    D.fill = a.fill;
    return D;
  }
  const uint8_t* src = S.data;
  if (a.sharded) {
    uint64_t off, nb;
    index_entry(a, S, lin, off, nb);
    if (off == ~0ull || nb == ~0ull) {  // Q1: zero-initialised part array
      D.kind = full ? kDescFullFill : kDescClip;
      D.fill = 0;
      return D;
    }
    const uint64_t total = (uint64_t)S.nbytes;
    bool range_ok = off <= total && nb <= total - off;
    if (range_ok) range_ok = piece_src(S, off, nb, src);  // sub-shard reads: the held pieces
    if (!range_ok || nb != (uint64_t)(a.inner_nbytes + a.crc_extra)) {
      const uint32_t kind = (range_ok ? kFlagLength : kFlagRange) | (a.rank.r2 ? kFlagLeaf : 0u);
      chunk_error(a.status + s * kStWords, chunk_rank(a.rank, ic), kind);
      D.kind = kDescSkip;
      return D;
    }
  }
  if (!a.sharded && (uint64_t)S.nbytes != (uint64_t)(a.inner_nbytes + a.crc_extra)) {
    // a whole chunk of the wrong length with a crc32c (the planner rejects the others): its
    // checksum decides first (zh_plan_wait, chunk_crc_detail_kernel)
    chunk_error(a.status + s * kStWords, 0, kFlagLength);
    D.kind = kDescSkip;
    return D;
  }
  D.src = (uint64_t)(uintptr_t)src;
  D.kind = full ? kDescFullCopy : kDescClip;
  if (!full && row_clip && !a.tile && a.crc_extra == 0 &&
      (a.fast_mode == kFastRowArith || a.fast_mode == kFastRowTable)) {
    // e.g. c2's boundary chunks (512 of 1024 z in bounds): the row kernel moves the row
    // prefix with the lanes remapped to its width (the chunk CRC, when fused, needs whole
    // payload rows: crc_extra == 0 only)
    const int64_t vb = (int64_t)hi_f * a.dsize;
    const int64_t vpr = vb / 16;
    if (vb % 16 == 0 && vpr > 0 && (vpr & (vpr - 1)) == 0 && vpr <= (1 << a.fast_vpr_shift)) {
      D.kind |= kDescClipRow;
      D.fill = (uint64_t)(63 - __clzll((unsigned long long)vpr));
    }
  }
  return D;
}

// Can the fast kernel take this item?  (table present, 16-byte aligned ends; the tile
// table path moves uint32 copies only)
__device__ __forceinline__ bool is_fast(const ScatterArgs& a, const ItemDesc& D) {
  const uint32_t mode = D.kind & kDescModeMask;
  const bool row_clip = mode == kDescClip && (D.kind & kDescClipRow) && a.row_group == 0;
  if (a.fast_mode == kFastNone ||
      (mode != kDescFullCopy && mode != kDescFullFill && !row_clip))
    return false;
  if ((((uintptr_t)a.region) + (uint64_t)D.d0 * a.dsize) & 15) return false;
  if (mode == kDescFullCopy && (D.src & 3)) return false;  // dword-aligned sources suffice
  if (a.tile && (a.dsize != 4 || mode != kDescFullCopy)) return false;
  return true;
}

__global__ __launch_bounds__(kBlock) void resolve_kernel(ScatterArgs a) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x; c < a.n_citems; c += stride) {
    ItemDesc D = resolve_one(a, c);
    if ((D.kind & kDescModeMask) != kDescSkip) {
      if (is_fast(a, D)) {
        D.kind |= kDescFast;
      } else {
        const uint32_t slot = atomicAdd(a.slow_count, 1u);
        a.slow_list[slot] = (uint32_t)c;
      }
    }
    a.desc[c] = D;
  }
}

// descriptor load into scalar registers (vector load + readfirstlane: tracked by vmcnt,
// so the one-item-ahead prefetch never forces an early lgkmcnt wait)
__device__ __forceinline__ uint32_t rfl(uint32_t v) {
  // readfirstlane is int-typed: keep it unsigned so 64-bit assembly never sign-extends
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

__device__ __forceinline__ ItemDesc ld_desc(const ItemDesc* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 x = q[0], y = q[1];
  ItemDesc D;
  D.src = ((uint64_t)rfl(x.y) << 32) | (uint64_t)rfl(x.x);
  D.d0 = (int64_t)(((uint64_t)rfl(x.w) << 32) | (uint64_t)rfl(x.z));
  D.fill = ((uint64_t)rfl(y.y) << 32) | (uint64_t)rfl(y.x);
  D.kind = rfl(y.z);
  D.shard = rfl(y.w);
  return D;
}

// Unclipped item as an Item (geometry is the launch-uniform inner chunk).
__device__ __forceinline__ void full_item(const ScatterArgs& a, const ItemDesc& D, uint32_t piece,
                                          Item& it) {
  it.sbase = (const uint8_t*)(uintptr_t)D.src;
  it.dbase = a.region;
  it.s0 = 0;
  it.d0 = D.d0;
  it.fill = D.fill;
  it.mode = (D.kind & kDescModeMask) == kDescFullFill ? kFill : kCopy;
  it.piece = piece;
#pragma unroll
  for (int d = 0; d < kMaxDims; d++) {
    it.e[d] = a.inner[d];
    it.v[d] = a.inner[d];
    it.ediv[d] = a.inner_div[d];
  }
}

// Row-interleaved tile path: a group of 8 tile units whose source rows are adjacent (the
// table's unit order puts batch-adjacent tiles next to each other, e.g. C4's x-neighbours)
// is moved so that one wave instruction covers the SAME row of all 8 tiles: lane (t, g)
// reads 16 bytes of row l of tile t, i.e. 1 KiB of contiguous payload per instruction
// (instead of 8 rows 4 KiB apart).  Tile pitch 1057 words (≡ 1 mod 32): lanes (t, g) hit
// banks t + 4g + j on both the write and the transposed read.
constexpr int kTG = 8;           // tiles per group
constexpr int kTilePitch = 1057; // words per LDS tile (32 x 33 + 1)

template <int DS, bool TILE>
__device__ __forceinline__ void generic_item(const ScatterArgs& a, Item& it,
                                             typename ElemT<DS>::T (*tile)[32][33]) {
  const int64_t* sstr = a.pstride;
  const int64_t* dstr = a.rstride;
  const int n = a.ndim;
  if (it.mode == kFill || !TILE) {
    const int F = it.mode == kFill ? a.fd : a.fs;
    uint32_t nrows = 1;
#pragma unroll
    for (int d = 0; d < kMaxDims; d++)
      if (d < n && d != F) nrows *= (uint32_t)it.e[d];
    const bool need_src = it.mode != kFill;
    if (vec_ok<DS>(a, it, F, sstr, dstr, it.e, need_src))
      row_pass<DS, true, false>(a, it, F, sstr, dstr, nrows, it.e, it.ediv);
    else
      row_pass<DS, false, false>(a, it, F, sstr, dstr, nrows, it.e, it.ediv);
  } else {
    tile_pass<DS>(a, it, sstr, dstr, tile);
  }
}

// ---------------------------------------------------------------------------------
// CRC-32C helpers (CRC32C.java:14-80, 119-125): GF(2) shift/combine, slicing tables,
// and the lane-interleaved update used by the chunk-CRC pass and the fused row kernel
// ---------------------------------------------------------------------------------
__constant__ uint32_t c_x2n[32] = {
    0x40000000u, 0x20000000u, 0x08000000u, 0x00800000u, 0x00008000u, 0x82F63B78u, 0x6EA2D55Cu,
    0x18B8EA18u, 0x510AC59Au, 0xB82BE955u, 0xB8FDB1E7u, 0x88E56F72u, 0x74C360A4u, 0xE4172B16u,
    0x0D65762Au, 0x35D73A62u, 0x28461564u, 0xBF455269u, 0xE2EA32DCu, 0xFE7740E6u, 0xF946610Bu,
    0x3C204F8Fu, 0x538586E3u, 0x59726915u, 0x734D5309u, 0xBC1AC763u, 0x7D0722CCu, 0xD289CABEu,
    0xE94CA9BCu, 0x05B74F3Fu, 0xA51E1F42u, 0x40000000u};

constexpr uint32_t kPoly = 0x82F63B78u;

// a(x) * b(x) mod P (reflected bit order).  The loop consumes a's bits from the top and stops
// once none is left (at most 32 steps for any a, 0 included).  The LDS tables the CRC kernels
// feed it from are laid out by compile-time constants checked with static_assert (kAln* below).
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (; a; a <<= 1) {
    if (a & 0x80000000u) p ^= b;
    b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

__device__ __forceinline__ uint32_t x2nmodp(uint64_t n, unsigned k) {
  uint32_t p = 1u << 31;
  while (n) {
    if (n & 1) p = multmodp(c_x2n[k & 31], p);
    n >>= 1;
    k++;
  }
  return p;
}

// crc(A || B) from crc(A), crc(B), |B|
__device__ __forceinline__ uint32_t crc_combine(uint32_t c1, uint32_t c2, uint64_t len2) {
  return multmodp(x2nmodp(len2, 3), c1) ^ c2;
}

// Compile-time CRC-32C constants (reflected Castagnoli polynomial, CRC32C.java:14-80):
// slicing-by-8 tables T, the zero-shift tables S of the lane-interleaved update
// (x^(8·4080)·b·x^(8k) for byte b at position k: the other 255 lanes' vectors of a 4 KiB
// round), the per-lane shift kfull[t] = x^(8·(4080 − 16t)) from a lane's last vector to the
// round's end, and x^(8·kCrcSpan).  Built by constexpr evaluation, read by every CRC kernel
// (before: every workgroup rebuilt them in LDS with 8 dependent rounds and x^n loops).
struct CrcTabs {
  uint32_t T[8][256];
  uint32_t S[4][256];
  uint32_t kfull[256];
  uint32_t kspan;
  uint32_t kidx[256];  // x^(8·kIdxSpan·j): span j of an index shifted past j later spans
};

constexpr uint32_t cx_mult(uint32_t a, uint32_t b) {  // a(x)·b(x) mod P, reflected
  uint32_t p = 0;
  for (int i = 0; i < 32; i++) {
    if (a & (1u << (31 - i))) p ^= b;
    b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

constexpr uint32_t cx_xpow8n(uint64_t n) {  // x^(8n) mod P
  uint32_t r = 1u << 31, b = 1u << 23;
  while (n) {
    if (n & 1) r = cx_mult(b, r);
    b = cx_mult(b, b);
    n >>= 1;
  }
  return r;
}

constexpr CrcTabs make_crc_tabs() {
  CrcTabs t{};
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
    t.T[0][i] = c;
  }
  for (int k = 1; k < 8; k++)
    for (int i = 0; i < 256; i++) t.T[k][i] = (t.T[k - 1][i] >> 8) ^ t.T[0][t.T[k - 1][i] & 0xFFu];
  const uint32_t k4080 = cx_xpow8n(4080);
  for (int b = 0; b < 4; b++)
    for (uint32_t i = 0; i < 256; i++) t.S[b][i] = cx_mult(k4080, i << (8 * b));
  const uint32_t x128 = cx_xpow8n(16);
  t.kfull[255] = 1u << 31;
  for (int i = 254; i >= 0; i--) t.kfull[i] = cx_mult(x128, t.kfull[i + 1]);
  t.kspan = cx_xpow8n(kCrcSpan);
  const uint32_t ki = cx_xpow8n(kIdxSpan);
  t.kidx[0] = 1u << 31;
  for (int j = 1; j < 256; j++) t.kidx[j] = cx_mult(ki, t.kidx[j - 1]);
  return t;
}

__device__ const CrcTabs g_crc = make_crc_tabs();

// slicing-by-8 tables into LDS (a copy of the compile-time table), per block
__device__ __forceinline__ void init_crc_tables(uint32_t (*T)[256]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 8; k++) T[k][tid] = g_crc.T[k][tid];
  __syncthreads();
}

// inner crc32c codec: CRC-32C of every resolved chunk payload, coalesced.  A workgroup
// takes one 64 KiB span of one chunk; lane l reads the 16-byte vectors l, l+256, ... (each
// wave load is 1 KiB contiguous) and keeps the raw register of its vectors as if the other
// lanes' bytes were zeros: acc = upd16(shift_4080(acc), v), with the constant zero-shift by
// four table lookups.  Each lane then shifts acc to the span end and the lanes XOR together
// (CRC linearity over GF(2)); the partial is the raw (init 0, no xorout) span register.
__device__ __forceinline__ uint32_t crc_upd16(uint32_t c, v4u v, const uint32_t (*T)[256]) {
  uint32_t lo = v.x ^ c, hi = v.y;
  c = T[7][lo & 0xFFu] ^ T[6][(lo >> 8) & 0xFFu] ^ T[5][(lo >> 16) & 0xFFu] ^ T[4][lo >> 24] ^
      T[3][hi & 0xFFu] ^ T[2][(hi >> 8) & 0xFFu] ^ T[1][(hi >> 16) & 0xFFu] ^ T[0][hi >> 24];
  lo = v.z ^ c;
  hi = v.w;
  return T[7][lo & 0xFFu] ^ T[6][(lo >> 8) & 0xFFu] ^ T[5][(lo >> 16) & 0xFFu] ^ T[4][lo >> 24] ^
         T[3][hi & 0xFFu] ^ T[2][(hi >> 8) & 0xFFu] ^ T[1][(hi >> 16) & 0xFFu] ^ T[0][hi >> 24];
}

__device__ __forceinline__ uint32_t crc_shift_tab(uint32_t c, const uint32_t (*S)[256]) {
  return S[0][c & 0xFFu] ^ S[1][(c >> 8) & 0xFFu] ^ S[2][(c >> 16) & 0xFFu] ^ S[3][c >> 24];
}

// Row offsets (payload, region) of row r of an unclipped inner chunk.
__device__ __forceinline__ void row_offsets(const ScatterArgs& a, const uint2* tab, uint32_t r,
                                            uint64_t& so, uint64_t& dof) {
  if (a.fast_mode == kFastRowTable) {
    const uint2 t = tab[r];
    so = t.x;
    dof = t.y;
    return;
  }
  so = 0;
  dof = 0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    if (i < a.rm_n) {
      const uint32_t m = i + 1 < a.rm_n ? (r & ((1u << a.rm_shift[i]) - 1)) : r;
      so += (uint64_t)m * (uint64_t)a.rm_sstr[i];
      dof += (uint64_t)m * (uint64_t)a.rm_dstr[i];
      r >>= a.rm_shift[i];
    }
  }
}

// Work order of the fast kernels: item i of the grid-stride walk is work item pitem(i).
__device__ __forceinline__ int64_t pitem(const ScatterArgs& a, int64_t i) {
  return a.item_mul ? (int64_t)(((uint64_t)i * a.item_mul) % (uint64_t)a.total_items) : i;
}

// decode, fast row kernel: unclipped aligned items whose rows (along the unit-stride dim)
// are whole 16-byte vectors.  Each lane owns one 16-byte column; the block walks
// (item, row batch) steps uniformly, and the loads of step k+1 are issued before the
// stores of step k, across item boundaries (vmcnt counts stores, so un-pipelined code
// would wait for the previous stores before every batch of loads).
//
// FLAGS (write path, encode view: source = region, destination = payload): also record
// whether each piece holds an element that differs from fill_value (the all-fill elision
// test of ShardingIndexedCodec.encode :129-133) in a.flags[piece], from the loaded vectors.
template <int DS, int U, int NT, bool CRC = false, bool FLAGS = false>
__global__ __launch_bounds__(kBlock) void decode_rows_kernel(ScatterArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint2* tab = reinterpret_cast<uint2*>(smem);
  for (int i = threadIdx.x; i < a.fast_n; i += kBlock)
    tab[i] = reinterpret_cast<const uint2*>(a.fast_tab)[i];
  // fused chunk CRC (inner crc32c): the lanes' loads of a piece are the payload vectors
  // tid + 256·m in order (rows sequential in the payload, host-checked), which is exactly
  // the chunk-CRC pass's lane pattern — the raw CRC needs no second read of the payload
  uint32_t(*T)[256] = reinterpret_cast<uint32_t(*)[256]>(smem + (((size_t)a.fast_n * 8 + 15) & ~(size_t)15));
  uint32_t(*S)[256] = T + 8;
  uint32_t kfull = 0, acc = 0;
  if constexpr (CRC) {
#pragma unroll
    for (int b = 0; b < 4; b++) S[b][threadIdx.x] = g_crc.S[b][threadIdx.x];
    init_crc_tables(T);
    kfull = g_crc.kfull[threadIdx.x];
  }
  __syncthreads();
  // lane geometry: one 16-byte column per lane, rows per step = kBlock / vectors per row;
  // per item, since a row-clipped item (kDescClipRow) moves narrower rows
  int vs = a.fast_vpr_shift;
  uint32_t col = (threadIdx.x & ((1u << vs) - 1)) * 16;
  uint32_t lr = threadIdx.x >> vs;
  uint32_t rstep = kBlock >> vs;
  const uint32_t nrows = (uint32_t)a.fast_rows, pieces = 1u << a.piece_shift;
  const uint32_t pmask = pieces - 1;
  const int64_t total = a.total_items;

  // block-uniform walk over this block's fast items
  int64_t item = blockIdx.x;
  ItemDesc D, Dn;
  if (item >= total) return;
  D = ld_desc(a.desc + (pitem(a, item) >> a.piece_shift));
  Dn = D;
  if (item + gridDim.x < total) Dn = ld_desc(a.desc + (pitem(a, item + gridDim.x) >> a.piece_shift));
  // seek to a fast item (item, D, Dn advance together)
  auto seek = [&]() -> bool {
    while (item < total && !(D.kind & kDescFast)) {
      item += gridDim.x;
      D = Dn;
      if (item + gridDim.x < total) Dn = ld_desc(a.desc + (pitem(a, item + gridDim.x) >> a.piece_shift));
    }
    return item < total;
  };
  if (!seek()) return;

  // current step
  const uint8_t* src;
  uint8_t* dst;
  bool fill;
  uint4 fv;
  uint32_t rbase, r1;
  auto start_item = [&]() {
    const uint32_t piece = (uint32_t)pitem(a, item) & pmask;
    rbase = (uint32_t)(((uint64_t)nrows * piece) / pieces);
    r1 = (uint32_t)(((uint64_t)nrows * (piece + 1)) / pieces);
    if constexpr (!FLAGS && !CRC) {
      const int v = (D.kind & kDescClipRow) ? (int)D.fill : a.fast_vpr_shift;
      if (v != vs) {  // uniform: the whole block moves to the item's row width
        vs = v;
        col = (threadIdx.x & ((1u << vs) - 1)) * 16;
        lr = threadIdx.x >> vs;
        rstep = kBlock >> vs;
      }
    }
    src = (const uint8_t*)(uintptr_t)D.src + col;
    dst = a.region + D.d0 * DS + col;
    fill = (D.kind & kDescModeMask) == kDescFullFill;
    fv = fill16<DS>(D.fill);
  };
  start_item();

  uint4 va[U];
  uint64_t da[U];
  bool differs = false;
  const uint4 ffill = fill16<DS>(a.fill);
  const uint4 fmask = fill16<DS>(a.fill_mask);
  auto load_step = [&](uint4* v, uint64_t* dd) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t r = rbase + lr + u * rstep;
      dd[u] = ~0ull;
      v[u] = fv;
      if (r < r1) {
        uint64_t so, dof;
        row_offsets(a, tab, r, so, dof);
        dd[u] = dof * DS;
        if (!fill) v[u] = ld16s<(NT & 1) != 0>(src + so * DS);
      }
    }
  };
  load_step(va, da);
  const uint8_t* dst_a = dst;
  bool fill_a = fill;
  uint4 fv_a = fv;
  int64_t item_a = item;
  for (;;) {
    // advance one step (uniform)
    rbase += rstep * U;
    bool more = true;
    const bool piece_end = rbase >= r1;
    if (piece_end) {
      item += gridDim.x;
      D = Dn;
      if (item + gridDim.x < total) Dn = ld_desc(a.desc + (pitem(a, item + gridDim.x) >> a.piece_shift));
      more = seek();
      if (more) start_item();
    }
    uint4 vb[U];
    uint64_t db[U];
    if (more) load_step(vb, db);
#pragma unroll
    for (int u = 0; u < U; u++)
      if (da[u] != ~0ull)
        st16s<(NT & 2) != 0>(const_cast<uint8_t*>(dst_a) + da[u],
                             fill_a ? fv_a : xform16<DS>(va[u], a.swap, a.is_bool));
    if constexpr (FLAGS) {
#pragma unroll
      for (int u = 0; u < U; u++)
        if (da[u] != ~0ull)
          differs |= ne16(va[u], ffill, fmask);
      if (piece_end) {  // uniform: one flag byte per piece, set by any wave that saw data
        if (__ballot(differs) != 0 && (threadIdx.x & 63) == 0)
          a.flags[pitem(a, item_a) >> a.piece_shift] = 1;
        differs = false;
      }
    }
    if constexpr (CRC) {
      if (!fill_a) {
#pragma unroll
        for (int u = 0; u < U; u++)
          if (da[u] != ~0ull) {
            // decode: the loaded payload vector; encode view (FLAGS): the stored one
            const uint4 cv = FLAGS ? xform16<DS>(va[u], a.swap, a.is_bool) : va[u];
            const v4u w = {cv.x, cv.y, cv.z, cv.w};
            acc = crc_upd16(crc_shift_tab(acc, S), w, T);
          }
        if (piece_end) {  // uniform: shift every lane to the piece end, XOR the wave
          uint32_t c = multmodp(kfull, acc);
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) c ^= (uint32_t)__shfl_xor((int)c, o, 64);
          if ((threadIdx.x & 63) == 0) atomicXor(a.crc_partials + pitem(a, item_a), c);
          acc = 0;
        }
      }
    }
    if (!more) break;
#pragma unroll
    for (int u = 0; u < U; u++) {
      va[u] = vb[u];
      da[u] = db[u];
    }
    dst_a = dst;
    fill_a = fill;
    fv_a = fv;
    item_a = item;
  }
}

// 4·(byte SEL of w) in one SDWA shift: the LDS byte offset of a 4-B table entry
template <int SEL>
__device__ __forceinline__ uint32_t byte_x4(uint32_t w) {
  uint32_t r;
  if constexpr (SEL == 0)
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(w));
  else if constexpr (SEL == 1)
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(w));
  else if constexpr (SEL == 2)
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(w));
  else
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(w));
  return r;
}

// a ^ b ^ c in one VALU op (v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Table lookups at a byte offset (4·index) from tables whose LDS position is a compile-time
// constant (the dynamic block's start plus a constant): base and table offsets fold into the
// ds_read immediate, so a lookup costs one SDWA op and the read.
__device__ __forceinline__ uint32_t tlook(const uint32_t (*T)[256], int k, uint32_t off4) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(T[k]) + off4);
}

// crc_upd16 / crc_shift_tab for tables at a constant LDS position (slicing-by-8 in two
// dependent halves; three-input XOR trees)
__device__ __forceinline__ uint32_t crc_upd8_k(uint32_t c, uint32_t w0, uint32_t w1,
                                               const uint32_t (*T)[256]) {
  const uint32_t lo = w0 ^ c, hi = w1;
  const uint32_t a0 = xor3(tlook(T, 7, byte_x4<0>(lo)), tlook(T, 6, byte_x4<1>(lo)),
                           tlook(T, 5, byte_x4<2>(lo)));
  const uint32_t a1 = xor3(tlook(T, 4, byte_x4<3>(lo)), tlook(T, 3, byte_x4<0>(hi)),
                           tlook(T, 2, byte_x4<1>(hi)));
  const uint32_t a2 = tlook(T, 1, byte_x4<2>(hi)) ^ tlook(T, 0, byte_x4<3>(hi));
  return xor3(a0, a1, a2);
}
__device__ __forceinline__ uint32_t crc_upd16_k(uint32_t c, v4u v, const uint32_t (*T)[256]) {
  return crc_upd8_k(crc_upd8_k(c, v.x, v.y, T), v.z, v.w, T);
}
__device__ __forceinline__ uint32_t crc_shift_k(uint32_t c, const uint32_t (*S)[256]) {
  return xor3(tlook(S, 0, byte_x4<0>(c)), tlook(S, 1, byte_x4<1>(c)), tlook(S, 2, byte_x4<2>(c))) ^
         tlook(S, 3, byte_x4<3>(c));
}

// encode, grouped row kernel (write path, narrow rows): a work item is G consecutive inner
// chunks — z-adjacent in the region when they sit in one shard row — and lane group q of
// every G·vpr lanes moves chunk q.  A wave load then covers G·(row bytes) of one region row
// instead of vpr-lane segments of 64/vpr different rows (region rows of a 32³ uint32 chunk
// are 128 B, 6 KiB apart in c3): +7 % in profiles/r02/enc_lab.json (G·row = 512 B).  Each
// lane group reads its own descriptor (not wave-uniform), so any item mix is correct;
// non-fast items idle their lane group (the slow kernel encodes them).  Rows per item and
// the row table are shared by every fast item (setup_fast); piece_shift == 0.
//
// CRC (inner crc32c fused; rows sequential in the payload, host-checked): chunk q's
// Lc = 256/G lanes store payload vectors j + Lc·m (j = the lane's index in the chunk), so a
// lane's raw register over its vectors is acc = shift_{16·Lc}(acc) ⊕ upd16(0, v) (table S),
// shifted to the payload end by x^(8·16·(Lc − 1 − j)); the chunk's lanes XOR their shares
// (CRC is linear over GF(2)) into its partial, one atomic per wave.
//
// FLAGS = false: the decode direction (payload rows → region rows; the planner's groups: with
// the fused chunk CRC by row length, without it 128-B rows whose row count is not a multiple
// of 8, rows_xpose_kernel taking the rest): full-fill
// items store their fill value, the CRC runs over the loaded payload vectors.
template <int DS, int G, int U, int NT, bool CRC, bool FLAGS>
__global__ __launch_bounds__(kBlock) void rows_group_kernel(ScatterArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // CRC: the tables first (a constant LDS position: crc_upd16_k / crc_shift_k), then the rows
  uint2* tab = reinterpret_cast<uint2*>(smem + (CRC ? 12 * 256 * 4 : 0));
  for (int i = threadIdx.x; i < a.fast_n; i += kBlock)
    tab[i] = reinterpret_cast<const uint2*>(a.fast_tab)[i];
  const int vs = a.fast_vpr_shift;
  const int GL = G << vs;  // lanes per group row (≤ 64, host-checked)
  const int tid = threadIdx.x, lane = tid & 63;
  const int q = (tid % GL) >> vs;
  const uint32_t col = (tid & ((1u << vs) - 1)) * 16;
  const uint32_t lr = tid / GL, rstep = kBlock / GL;
  uint32_t(*T)[256] = nullptr;
  uint32_t(*S)[256] = nullptr;
  uint32_t kl = 0;
  if constexpr (CRC) {
    T = reinterpret_cast<uint32_t(*)[256]>(smem);
    S = T + 8;
    init_crc_tables(T);
    constexpr uint32_t Lc = kBlock / G;
    const uint32_t kg = x2nmodp((uint64_t)(16 * Lc), 3);
#pragma unroll
    for (int b = 0; b < 4; b++) S[b][tid] = multmodp(kg, (uint32_t)tid << (8 * b));
    const uint32_t j = (lr << vs) + (uint32_t)(tid & ((1 << vs) - 1));
    kl = x2nmodp((uint64_t)(16 * (Lc - 1 - j)), 3);
  }
  __syncthreads();
  const uint32_t nrows = (uint32_t)a.fast_rows;
  const int64_t ngroups = (a.n_citems + G - 1) / G;
  // this lane's group leader (first lane of q's segment in the wave) and q's ballot mask
  uint64_t qmask = 0;
  for (int o = 0; o < 64; o += GL) qmask |= (((1ull << (1 << vs)) - 1) << (q << vs)) << o;
  const bool leader = lane == (q << vs);
  const uint4 ffill = fill16<DS>(a.fill);
  const uint4 fmask = fill16<DS>(a.fill_mask);
  for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int64_t pg = a.item_mul ? (int64_t)(((uint64_t)g * a.item_mul) % (uint64_t)ngroups) : g;
    const int64_t c = pg * G + q;
    bool on = false, fill = false;
    uint4 fv = ffill;
    const uint8_t* src = nullptr;
    uint8_t* dst = nullptr;
    if (c < a.n_citems) {
      const uint4* dp = reinterpret_cast<const uint4*>(a.desc + c);
      const uint4 x = dp[0], y = dp[1];
      on = (y.z & kDescFast) != 0;
      src = (const uint8_t*)(uintptr_t)(((uint64_t)x.y << 32) | x.x) + col;
      dst = a.region + (int64_t)(((uint64_t)x.w << 32) | x.z) * DS + col;
      if (!FLAGS) {
        fill = (y.z & kDescModeMask) == kDescFullFill;
        fv = fill16<DS>(((uint64_t)y.y << 32) | y.x);
      }
    }
    if (__syncthreads_or(on) == 0) continue;  // block-uniform: no fast chunk in the group
    bool differs = false;
    uint32_t acc = 0;
    // load U rows, then store them (no cross-step pipelining: the double-buffered form measured
    // 36.2 → 44.4 ms at G = 2, U = 4; profiles/r02/write/ab_enc4.txt)
#pragma unroll 1
    for (uint32_t r0 = 0; r0 < nrows; r0 += rstep * U) {
      uint4 v[U];
      uint64_t dd[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t r = r0 + lr + u * rstep;
        dd[u] = ~0ull;
        if (on && r < nrows) {
          uint64_t so, dof;
          row_offsets(a, tab, r, so, dof);
          dd[u] = dof * DS;
          v[u] = fv;
          if (!fill) v[u] = ld16s<(NT & 1) != 0>(src + so * DS);
        }
      }
#pragma unroll
      for (int u = 0; u < U; u++)
        if (dd[u] != ~0ull) {
          const uint4 w = fill ? fv : xform16<DS>(v[u], a.swap, a.is_bool);
          st16s<(NT & 2) != 0>(dst + dd[u], w);
          if (FLAGS)
            differs |= ne16(v[u], ffill, fmask);
          if constexpr (CRC) {  // the payload vector: stored (encode) or loaded (decode)
            const uint4 pv = FLAGS ? w : v[u];
            const v4u wv = {pv.x, pv.y, pv.z, pv.w};
            if (!fill) acc = crc_shift_k(acc, S) ^ crc_upd16_k(0u, wv, T);
          }
        }
    }
    // one flag byte per chunk, set by q's leader in any wave whose lanes saw data
    if (FLAGS && (__ballot(differs) & qmask) != 0 && leader && on) a.flags[c] = 1;
    if constexpr (CRC) {
      uint32_t cr = multmodp(kl, acc);
      for (int o = 1; o < (1 << vs); o <<= 1) cr ^= (uint32_t)__shfl_xor((int)cr, o, 64);
      for (int o = GL; o < 64; o <<= 1) cr ^= (uint32_t)__shfl_xor((int)cr, o, 64);
      if (leader && on && !fill) atomicXor(a.crc_partials + c, cr);
    }
  }
}

// Grouped row kernel with a lane exchange (decode, 128-B rows, 8 chunks per work item, no
// CRC).  rows_group_kernel at G = 8 moves 1 KiB of contiguous payload per wave instruction but
// stores each chunk's rows from 8 lanes, 128 B to each of 8 region rows.  Here every wave
// instruction is 1 KiB contiguous on both sides: a wave takes 8 rows of the 8 chunks, the
// payload side in layout B (lane = (row, 16-B column), register = chunk) and the region side
// in layout A (lane = (chunk q, column), register = row), and swaps layouts through LDS (8 KiB
// per wave; rows 72 vectors apart, so the 16-lane groups of ds_read_b128 and the 8-lane groups
// of ds_write_b128 hit distinct banks).  Full-fill chunks store their fill value.  Each lane
// group reads its own chunk's descriptor; the others come through readlane, so any chunk mix
// is correct (non-fast chunks stay on the slow list).  Host: fast_vpr_shift == 3,
// piece_shift == 0, item_mul over groups of 8.  (The encode-view form measured slower, 9.09 →
// 9.71 ms, and was removed in round 4.)
constexpr int kXRow = 72;  // 16-B vectors per exchange row (64 + 8)

template <int DS>
__global__ __launch_bounds__(kBlock) void rows_xpose_kernel(ScatterArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint2* tab = reinterpret_cast<uint2*>(smem);
  for (int i = threadIdx.x; i < a.fast_n; i += kBlock)
    tab[i] = reinterpret_cast<const uint2*>(a.fast_tab)[i];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hi = lane >> 3, col = lane & 7;  // layout A: hi = chunk; layout B: hi = row
  uint4* xw = reinterpret_cast<uint4*>(smem + (((size_t)a.fast_n * 8 + 15) & ~(size_t)15)) +
              wave * 8 * kXRow;
  __syncthreads();
  const uint32_t nrows = (uint32_t)a.fast_rows;
  const int64_t ngroups = (a.n_citems + 7) / 8;
  const uint4 ffill = fill16<DS>(a.fill);
  for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int64_t pg = a.item_mul ? (int64_t)(((uint64_t)g * a.item_mul) % (uint64_t)ngroups) : g;
    const int64_t c = pg * 8 + hi;
    bool on = false, fill = false;
    uint4 fv = ffill;
    uint64_t sb = 0, db = 0;  // this lane's chunk: source and destination bases
    if (c < a.n_citems) {
      const uint4* dp = reinterpret_cast<const uint4*>(a.desc + c);
      const uint4 x = dp[0], y = dp[1];
      on = (y.z & kDescFast) != 0;
      sb = ((uint64_t)x.y << 32) | x.x;
      db = (uint64_t)(uintptr_t)(a.region + (int64_t)(((uint64_t)x.w << 32) | x.z) * DS);
      fill = (y.z & kDescModeMask) == kDescFullFill;
      fv = fill16<DS>(((uint64_t)y.y << 32) | y.x);
    }
    if (__syncthreads_or(on) == 0) continue;  // block-uniform: no fast chunk in the group
    const uint64_t onm = __ballot(on), fillm = __ballot(on && fill);
    uint4 v[8];
    auto load = [&](uint32_t rb) {  // layout B loads: row rb + hi of chunk k
      uint64_t so, dof;
      row_offsets(a, tab, rb + hi, so, dof);
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint64_t s = ((uint64_t)__builtin_amdgcn_readlane((int)(sb >> 32), k * 8) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sb, k * 8);
        v[k] = make_uint4(0, 0, 0, 0);
        if (((onm & ~fillm) >> (k * 8)) & 1 && rb + hi < nrows)
          v[k] = ld16s<true>((const uint8_t*)s + so * DS + col * 16);
      }
    };
    load(wave * 8);
#pragma unroll 1
    for (uint32_t rb = wave * 8; rb < nrows; rb += 32) {
#pragma unroll
      for (int k = 0; k < 8; k++) xw[hi * kXRow + k * 8 + col] = v[k];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      uint4 y[8];  // layout A: chunk hi, row rb + r
#pragma unroll
      for (int r = 0; r < 8; r++) y[r] = xw[r * kXRow + hi * 8 + col];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (rb + 32 < nrows) load(rb + 32);  // the next step's loads before these stores
#pragma unroll
      for (int r = 0; r < 8; r++) {  // layout A stores into chunk hi's region rows
        uint64_t so, dof;
        row_offsets(a, tab, rb + r, so, dof);
        if (on && rb + r < nrows)
          st16s<true>((uint8_t*)db + dof * DS + col * 16,
                      fill ? fv : xform16<DS>(y[r], a.swap, a.is_bool));
      }
    }
  }
}

// Row-interleaved tile path (see kTG above).  With CRC (inner crc32c fused): lane (w, t, g)
// holds the payload vectors at bytes P_k = 4·tab[u].x + 4·(8w + k)·s_fd + 16g, k = 0..7,
// a constant gap G = 4·s_fd − 16 apart, so its raw register over [v0, G zeros, v1, …, v7]
// is acc = upd16(shift_G(acc), v_k).  Shifted to the payload end it contributes
// acc · x^(8(L − P_7 − 16)) to the chunk's raw CRC (CRC is linear over GF(2)), and
// L − P_7 − 16 = (L − E_u) + B_lane, E_u = the end of unit u's last payload row.  The host
// table gives K[u] = x^(8(L − E_u)); the caller applies the lane constant x^(8·B_lane) once
// per piece.  Returns the lane's share (zero without CRC).
//
// The lane's vector contributions c_k = upd16(0, v_k) are independent (no chain through the
// register: 16 lookups each); the register then folds them as acc = shift_{G+16}(acc) ⊕ c_k
// (S holds the shift by G + 16 bytes: upd16(c, v) = c·x^128 ⊕ upd16(0, v)), so the serial
// chain per vector is 4 lookups.  With a regular unit layout (crc_tile_step = x^(8Δ), host
// checked) the lane folds its groups as r = shift_Δ(r) ⊕ acc (table SD) and multiplies by its
// last unit's K once per piece, instead of one GF(2) multiply per group.
template <int NT, bool CRC, bool FLAGS = false>
__device__ __forceinline__ uint32_t fast_tiles_rows(const ScatterArgs& a, const uint2* tab,
                                                    const uint8_t* src, uint8_t* dst,
                                                    uint32_t piece, uint32_t* lds,
                                                    const uint32_t (*T)[256],
                                                    const uint32_t (*S)[256],
                                                    const uint32_t (*SD)[256],
                                                    const uint32_t* K, bool& differs) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = lane >> 3, g = lane & 7;
  const int64_t s_fd = a.pstride[a.fd], d_fs = a.rstride[a.fs];
  const uint32_t units = (uint32_t)a.fast_n, pieces = 1u << a.piece_shift;
  const uint32_t u0 = (uint32_t)(((uint64_t)units * piece) / pieces);
  const uint32_t u1 = (uint32_t)(((uint64_t)units * (piece + 1)) / pieces);
  uint32_t* mine = lds + t * kTilePitch;
  uint32_t share = 0, run = 0;
  uint32_t ulast = ~0u;  // the lane's last live unit (regular layout: one K multiply)
  const bool regular = CRC && a.crc_tile_step != 0;
  uint4 x[8];
  auto load = [&](uint32_t ub) {
    const uint32_t u = ub + t;
    if (u < u1) {
      const uint8_t* base = src + ((size_t)tab[u].x + g * 4) * 4;
#pragma unroll
      for (int k = 0; k < 8; k++)
        x[k] = ld16s<(NT & 1) != 0>(base + (size_t)(wave * 8 + k) * s_fd * 4);
    }
  };
  if (u0 < u1) load(u0);
  for (uint32_t ub = u0; ub < u1; ub += kTG) {
    const bool live = ub + t < u1;
    if constexpr (FLAGS) {  // write path: any element != fill_value (uint32 tiles)
      if (live) {
        const uint32_t f = (uint32_t)a.fill, fm = (uint32_t)a.fill_mask;
#pragma unroll
        for (int k = 0; k < 8; k++) differs |= ne4x4(x[k], f, fm);
      }
    }
    if (live) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        uint32_t* row = mine + (wave * 8 + k) * 33 + g * 4;
        row[0] = xform1<4>(x[k].x, a.swap, 0);
        row[1] = xform1<4>(x[k].y, a.swap, 0);
        row[2] = xform1<4>(x[k].z, a.swap, 0);
        row[3] = xform1<4>(x[k].w, a.swap, 0);
      }
    }
    __syncthreads();
    uint4 xc[8];  // raw payload vectors of this group, kept for the CRC (decode)
    if constexpr (CRC && !FLAGS) {
#pragma unroll
      for (int k = 0; k < 8; k++) xc[k] = x[k];
    }
    if (ub + kTG < u1) load(ub + kTG);
    uint32_t eacc = 0;  // encode view: raw register of the stored (payload) vectors
    if (live) {
      uint8_t* base = dst + ((size_t)tab[ub + t].y + g * 4) * 4;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int r = wave * 8 + k;
        uint4 y;
        y.x = mine[(g * 4 + 0) * 33 + r];
        y.y = mine[(g * 4 + 1) * 33 + r];
        y.z = mine[(g * 4 + 2) * 33 + r];
        y.w = mine[(g * 4 + 3) * 33 + r];
        st16s<(NT & 2) != 0>(base + (size_t)r * d_fs * 4, y);
        if constexpr (CRC && FLAGS) {  // the stored rows have the decode loads' geometry
          const v4u w = {y.x, y.y, y.z, y.w};
          const uint32_t ck = crc_upd16(0u, w, T);
          eacc = k ? crc_shift_tab(eacc, S) ^ ck : ck;
        }
      }
    }
    if constexpr (CRC) {
      if (live) {
        uint32_t acc = eacc;
        if constexpr (!FLAGS) {
#pragma unroll
          for (int k = 0; k < 8; k++) {  // c_k does not depend on the register
            const v4u w = {xc[k].x, xc[k].y, xc[k].z, xc[k].w};
            const uint32_t ck = crc_upd16(0u, w, T);
            acc = k ? crc_shift_tab(acc, S) ^ ck : ck;
          }
        }
        if (regular) {
          run = (ulast == ~0u ? 0u : crc_shift_tab(run, SD)) ^ acc;
          ulast = ub + t;
        } else {
          share ^= multmodp(K[ub + t], acc);
        }
      }
    }
    __syncthreads();
  }
  if (regular && ulast != ~0u) share = multmodp(K[ulast], run);
  return share;
}

// decode, fast tile kernel: unclipped aligned uint32 copies through 32x32 LDS tiles whose
// origins come from the LDS table.  CRC: the chunk CRC is fused (row-interleaved variant);
// each wave XORs its lanes' shares, already shifted to the payload end, into the chunk's
// partial, which data_crc_finalize_kernel compares with the stored value.
template <int NT, bool CRC, bool FLAGS>
__device__ __forceinline__ void decode_tiles_body(const ScatterArgs& a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint2* tab = reinterpret_cast<uint2*>(smem);
  uint8_t* after_tab = smem + (((size_t)a.fast_n * 8 + 15) & ~(size_t)15);
  uint32_t(*tile)[32][33] = reinterpret_cast<uint32_t(*)[32][33]>(after_tab);
  for (int i = threadIdx.x; i < a.fast_n; i += kBlock)
    tab[i] = reinterpret_cast<const uint2*>(a.fast_tab)[i];
  uint32_t(*T)[256] = nullptr;
  uint32_t(*S)[256] = nullptr;
  uint32_t(*SD)[256] = nullptr;
  uint32_t* K = nullptr;
  uint32_t kb = 0;
  if constexpr (CRC) {
    // slicing tables, the shift by the row pitch G + 16, the group step Δ, the per-unit end
    // shifts (host table after the (src, dst) pairs) and this lane's constant x^(8·B_lane)
    T = reinterpret_cast<uint32_t(*)[256]>(after_tab + (size_t)kTG * kTilePitch * 4);
    S = T + 8;
    SD = S + 4;
    K = reinterpret_cast<uint32_t*>(SD + 4);
    init_crc_tables(T);
    // payload row stride of the lane's vectors: the loaded rows (decode) or, on the encode
    // view, the stored rows (the same lane/row geometry on the destination side)
    const int64_t s_fd = FLAGS ? a.rstride[a.fs] : a.pstride[a.fd];
    const uint32_t kg = x2nmodp((uint64_t)(4 * s_fd), 3);
#pragma unroll
    for (int b = 0; b < 4; b++) {
      S[b][threadIdx.x] = multmodp(kg, (uint32_t)threadIdx.x << (8 * b));
      SD[b][threadIdx.x] =
          a.crc_tile_step ? multmodp(a.crc_tile_step, (uint32_t)threadIdx.x << (8 * b)) : 0u;
    }
    for (int i = threadIdx.x; i < a.fast_n; i += kBlock) K[i] = a.fast_tab[2 * a.fast_n + i];
    const int w = threadIdx.x >> 6, g = threadIdx.x & 7;
    kb = x2nmodp((uint64_t)(4 * (24 - 8 * w) * s_fd + 112 - 16 * g), 3);
  }
  __syncthreads();
  const int64_t total = a.total_items;
  const uint32_t pmask = (1u << a.piece_shift) - 1;
  int64_t item = blockIdx.x;
  if (item >= total) return;
  ItemDesc D = ld_desc(a.desc + (pitem(a, item) >> a.piece_shift));
  for (; item < total; item += gridDim.x) {
    const int64_t nxt = item + gridDim.x;
    ItemDesc Dn = D;
    if (nxt < total) Dn = ld_desc(a.desc + (pitem(a, nxt) >> a.piece_shift));
    if (D.kind & kDescFast) {
      const uint8_t* src = (const uint8_t*)(uintptr_t)D.src;
      uint8_t* dst = a.region + D.d0 * 4;
      const int64_t pi = pitem(a, item);
      bool differs = false;
      const uint32_t share = fast_tiles_rows<NT, CRC, FLAGS>(
          a, tab, src, dst, (uint32_t)pi & pmask, reinterpret_cast<uint32_t*>(tile), T, S, SD,
          K, differs);
      if constexpr (FLAGS) {
        if (__ballot(differs) != 0 && (threadIdx.x & 63) == 0) a.flags[pi >> a.piece_shift] = 1;
      }
      if constexpr (CRC) {
        uint32_t c = multmodp(kb, share);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c ^= (uint32_t)__shfl_xor((int)c, o, 64);
        if ((threadIdx.x & 63) == 0) atomicXor(a.crc_partials + (pi >> a.piece_shift), c);
      }
    }
    D = Dn;
  }
}

template <int NT, bool CRC = false, bool FLAGS = false>
__global__ __launch_bounds__(kBlock) void decode_tiles_kernel(ScatterArgs a) {
  decode_tiles_body<NT, CRC, FLAGS>(a);
}

// encode, grouped tile kernel (write path, uint32, transposed inner chunks): the tile path of
// the encode view reads region rows of 128 B, one per tile (the 8 tiles of a step are
// x-neighbours, a region row pitch apart), where the decode mirror reads 1 KiB of payload.
// Here a work item is G consecutive (z-adjacent) inner chunks and a step moves 8/G tiles of
// each: lane (t, g) with t = q·(8/G) + i moves tile i of chunk q, so a wave load covers
// G·128 B contiguous of each of 8/G region rows.  Same LDS tiles and bank layout as
// fast_tiles_rows; per-lane descriptors (any chunk mix is correct; non-fast chunks idle their
// lanes and stay on the slow list).  No CRC, piece_shift == 0 (host-checked).
//
// FLAGS = false: the decode direction (payload → region; every fast tile item is a full copy),
// the decode's tile groups (G = 4).  CRC: the chunk crc32c of the payload (encode: the stored vectors, which
// have the decode loads' geometry; decode: the loaded ones), fused as in fast_tiles_rows: a
// lane's 8 vectors
// fold with S, its units (u, u + 8/G, …) with SD = x^(8Δ) for that unit stride (host:
// tile_crc_step(ends, 8/G)), one K multiply per chunk, the lane constant kb, then an XOR over
// the chunk's lane segment and one atomic per wave.
//
// PF: the next step's loads are issued before this step's stores (decode_tiles_body's order).
//
// CRC tables: T[8][256], S[4][256], SD[4][256] (16 KiB; 50.5 KB per workgroup with the
// tiles, 3 per CU).  Compact slicing-by-4 tables (4 per CU) and conflict-free field tables
// measured slower or equal (round 3, profiles/r03/g, profiles/r03/l) and were removed.
//
// FLAGS (write path): 0 none, 1 the all-fill test by exact compares, 2 under a.fill_mask (a
// float ±0 fill); the masked form costs the CRC encode 2 % (42.1 vs 43.0 ms, c4crc,
// profiles/r05/wab/), so it gets kernels of its own.
//
template <int NT, int G, bool CRC, bool PF, int FLAGS>
__global__ __launch_bounds__(kBlock) void tiles_group_kernel(ScatterArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  // CRC: the tables first (T, S, SD: a constant LDS position for crc_upd16_k / crc_shift_k),
  // then K, the unit table and the tiles
  constexpr size_t kTabBytes = 16 * 256 * 4;
  uint8_t* tab_at = CRC ? smem + ((kTabBytes + (size_t)a.fast_n * 4 + 15) & ~(size_t)15) : smem;
  uint2* tab = reinterpret_cast<uint2*>(tab_at);
  uint8_t* after_tab = tab_at + (((size_t)a.fast_n * 8 + 15) & ~(size_t)15);
  uint32_t* lds = reinterpret_cast<uint32_t*>(after_tab);
  for (int i = threadIdx.x; i < a.fast_n; i += kBlock)
    tab[i] = reinterpret_cast<const uint2*>(a.fast_tab)[i];
  constexpr int TG = kTG / G;  // tiles of each chunk per step
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int t = lane >> 3, g = lane & 7, q = t / TG, ti = t % TG;
  const int64_t s_fd = a.pstride[a.fd], d_fs = a.rstride[a.fs];
  uint32_t(*T)[256] = nullptr;
  uint32_t(*S)[256] = nullptr;
  uint32_t(*SD)[256] = nullptr;
  uint32_t* K = nullptr;
  uint32_t kb = 0;
  if constexpr (CRC) {
    T = reinterpret_cast<uint32_t(*)[256]>(smem);
    // payload row pitch of the lane's vectors: the stored rows (encode) or the loaded rows
    const int64_t pitch = FLAGS ? d_fs : s_fd;
    const uint32_t kg = x2nmodp((uint64_t)(4 * pitch), 3);
    S = T + 8;
    SD = S + 4;
    K = reinterpret_cast<uint32_t*>(SD + 4);
    init_crc_tables(T);
#pragma unroll
    for (int b = 0; b < 4; b++) {
      S[b][threadIdx.x] = multmodp(kg, (uint32_t)threadIdx.x << (8 * b));
      SD[b][threadIdx.x] =
          a.crc_tile_step ? multmodp(a.crc_tile_step, (uint32_t)threadIdx.x << (8 * b)) : 0u;
    }
    for (int i = threadIdx.x; i < a.fast_n; i += kBlock) K[i] = a.fast_tab[2 * a.fast_n + i];
    kb = x2nmodp((uint64_t)(4 * (24 - 8 * wave) * pitch + 112 - 16 * g), 3);
  }
  __syncthreads();
  const bool regular = CRC && a.crc_tile_step != 0;
  const uint32_t units = (uint32_t)a.fast_n;
  // regular fold: a lane's last unit is the same in every fast chunk (ti + a multiple of TG),
  // so its two end multiplies (K of that unit, then kb) fold into one lane constant
  uint32_t kq = 0;
  if constexpr (CRC) {
    const uint32_t til = (uint32_t)ti;
    if (regular && til < units) kq = multmodp(kb, K[til + (units - 1 - til) / TG * TG]);
  }
  const int64_t ngroups = (a.n_citems + G - 1) / G;
  const uint64_t qmask = (TG * 8 == 64 ? ~0ull : ((1ull << (TG * 8)) - 1)) << (q * TG * 8);
  const bool leader = lane == q * TG * 8;
  const uint32_t f = (uint32_t)a.fill, fm = (uint32_t)a.fill_mask;
  uint32_t* mine = lds + t * kTilePitch;
  for (int64_t gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
    const int64_t pg = a.item_mul ? (int64_t)(((uint64_t)gi * a.item_mul) % (uint64_t)ngroups) : gi;
    const int64_t c = pg * G + q;
    bool on = false;
    const uint8_t* src = nullptr;
    uint8_t* dst = nullptr;
    if (c < a.n_citems) {
      const uint4* dp = reinterpret_cast<const uint4*>(a.desc + c);
      const uint4 x = dp[0], y = dp[1];
      on = (y.z & kDescFast) != 0;
      src = (const uint8_t*)(uintptr_t)(((uint64_t)x.y << 32) | x.x);
      dst = a.region + (int64_t)(((uint64_t)x.w << 32) | x.z) * 4;
    }
    if (__syncthreads_or(on) == 0) continue;  // block-uniform
    bool differs = false;
    uint32_t share = 0, run = 0, ulast = ~0u;
    uint4 x[8];
    auto load = [&](uint32_t ub_) {
      const uint32_t uu = ub_ + ti;
      if (on && uu < units) {
        const uint8_t* base = src + ((size_t)tab[uu].x + g * 4) * 4;
#pragma unroll
        for (int k = 0; k < 8; k++)
          x[k] = ld16s<(NT & 1) != 0>(base + (size_t)(wave * 8 + k) * s_fd * 4);
      }
    };
    // DEFER (encode CRC): step s's stored vectors stay in registers (yp) and fold into the CRC
    // after step s + 1 has issued its loads, so the lookups run under the load latency (c4crc
    // encode 41.87–41.93 → 41.54–41.84 ms in this form, 41.80–42.04 → 41.51–41.58 with the load
    // outside the live branch, profiles/r06/defer/; the same deferral in the grouped row kernels
    // cost them 2 waves per SIMD of registers and measured 13 % slower)
    constexpr bool DEFER = CRC && FLAGS && !PF;
    uint4 yp[8];
    bool lp = false;
    uint32_t up = 0;
    auto fold = [&]() {
      if constexpr (DEFER) {
        if (lp) {
          uint32_t eacc = 0;
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const v4u w = {yp[k].x, yp[k].y, yp[k].z, yp[k].w};
            const uint32_t ck = crc_upd16_k(0u, w, T);
            eacc = k ? crc_shift_k(eacc, S) ^ ck : ck;
          }
          if (regular) {
            run = (ulast != ~0u ? crc_shift_k(run, SD) : 0u) ^ eacc;
            ulast = up;
          } else {
            share ^= multmodp(K[up], eacc);
          }
        }
      }
    };
    if (PF) load(0);
#pragma unroll 1
    for (uint32_t ub = 0; ub < units; ub += TG) {
      const uint32_t u = ub + ti;
      const bool live = on && u < units;
      if (!live) fold();  // DEFER: the previous step's CRC (no loads to hide it under)
      if (live) {
        if (!PF) load(ub);  // inside the live branch: 46.3 → 42.3 ms on the c4crc encode
        fold();             // DEFER: the previous step's CRC, under these loads
#pragma unroll
        for (int k = 0; k < 8; k++) {
          if constexpr (FLAGS == 2) differs |= ne4x4(x[k], f, fm);
          if constexpr (FLAGS == 1)
            differs |= (x[k].x != f) | (x[k].y != f) | (x[k].z != f) | (x[k].w != f);
          uint32_t* row = mine + (wave * 8 + k) * 33 + g * 4;
          row[0] = xform1<4>(x[k].x, a.swap, 0);
          row[1] = xform1<4>(x[k].y, a.swap, 0);
          row[2] = xform1<4>(x[k].z, a.swap, 0);
          row[3] = xform1<4>(x[k].w, a.swap, 0);
        }
      }
      __syncthreads();
      uint4 xc[8];  // this step's payload vectors (decode CRC) while x takes the next step's
      if constexpr (CRC && !FLAGS) {
#pragma unroll
        for (int k = 0; k < 8; k++) xc[k] = x[k];
      }
      if (PF && ub + TG < units) load(ub + TG);
      if (live) {
        uint8_t* base = dst + ((size_t)tab[u].y + g * 4) * 4;
        uint32_t eacc = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const int r = wave * 8 + k;
          uint4 y;
          y.x = mine[(g * 4 + 0) * 33 + r];
          y.y = mine[(g * 4 + 1) * 33 + r];
          y.z = mine[(g * 4 + 2) * 33 + r];
          y.w = mine[(g * 4 + 3) * 33 + r];
          st16s<(NT & 2) != 0>(base + (size_t)r * d_fs * 4, y);
          if constexpr (DEFER) {
            yp[k] = y;
          } else if constexpr (CRC && FLAGS) {  // encode: the stored vectors
            const v4u w = {y.x, y.y, y.z, y.w};
            const uint32_t ck = crc_upd16_k(0u, w, T);
            eacc = k ? crc_shift_k(eacc, S) ^ ck : ck;
          }
        }
        if constexpr (CRC && !FLAGS) {  // decode: the loaded payload vectors, stores in flight
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const v4u w = {xc[k].x, xc[k].y, xc[k].z, xc[k].w};
            const uint32_t ck = crc_upd16_k(0u, w, T);
            eacc = k ? crc_shift_k(eacc, S) ^ ck : ck;
          }
        }
        if constexpr (CRC && !DEFER) {
          if (regular) {
            run = (ulast != ~0u ? crc_shift_k(run, SD) : 0u) ^ eacc;
            ulast = u;
          } else {
            share ^= multmodp(K[u], eacc);
          }
        }
      }
      lp = live;
      up = u;
      __syncthreads();
    }
    fold();  // DEFER: the last step's CRC
    if (FLAGS && (__ballot(differs) & qmask) != 0 && leader && on) a.flags[c] = 1;
    if constexpr (CRC) {
      uint32_t cr = regular ? (ulast != ~0u ? multmodp(kq, run) : 0u) : multmodp(kb, share);
#pragma unroll
      for (int o = TG * 4; o > 0; o >>= 1) cr ^= (uint32_t)__shfl_xor((int)cr, o, 64);
      if (leader && on) atomicXor(a.crc_partials + c, cr);
    }
  }
}

// a dword of LDS at a byte address known relative to LDS offset 0 (constant parts fold into
// the ds_read immediate)
__device__ __forceinline__ uint32_t lds_word(uint32_t byte_addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>((size_t)byte_addr);
}

// Slicing-by-8 step over the 8 raw payload bytes held by the words w0, w1 as they sit in the LDS
// tiles; the 8 tables T[7..0] are at LDS bytes 0, 1024, … (a kernel without static LDS, tables
// first in the dynamic block).  SWAP: the tiles hold byte-swapped words, so raw byte k of a word
// is its byte 3 − k; the tables then hold byte-swapped entries and the register is carried
// byte-swapped (c' = bswap(c): raw lo ^ c = bswap(w0 ^ c'), and the XOR of swapped entries is
// the swapped result).  Per 8 bytes: one XOR in, 8 SDWA offsets, 8 lookups, a 3-input XOR tree.
template <bool SWAP>
__device__ __forceinline__ uint32_t crc_upd8_lds(uint32_t c, uint32_t w0, uint32_t w1) {
  const uint32_t lo = w0 ^ c, hi = w1;
  constexpr int s0 = SWAP ? 3 : 0, s1 = SWAP ? 2 : 1, s2 = SWAP ? 1 : 2, s3 = SWAP ? 0 : 3;
  const uint32_t a0 = xor3(lds_word(byte_x4<s0>(lo) + 7 * 1024), lds_word(byte_x4<s1>(lo) + 6 * 1024),
                           lds_word(byte_x4<s2>(lo) + 5 * 1024));
  const uint32_t a1 = xor3(lds_word(byte_x4<s3>(lo) + 4 * 1024), lds_word(byte_x4<s0>(hi) + 3 * 1024),
                           lds_word(byte_x4<s1>(hi) + 2 * 1024));
  const uint32_t a2 = lds_word(byte_x4<s2>(hi) + 1 * 1024) ^ lds_word(byte_x4<s3>(hi));
  return xor3(a0, a1, a2);
}

// decode, grouped tile kernel with the chunk CRC over LDS rows.  The kernel
// must have no static LDS, since its tables are addressed from LDS offset 0: the host selects it
// only when rowcrc_lds_at_zero() confirms that for every instantiation.  The lanes
// move tiles as tiles_group_kernel<…, PF = true> does; for the CRC, lane i of the block takes
// payload row i & 31 of tile slot i >> 5 (128 contiguous payload bytes) from the LDS tiles after
// the stores of a step, and runs the plain slicing-by-8 update over it after the barrier: 16
// lookups per 16-B vector, no zero-shift (the fused kernel: 20), and no register copy of the
// loaded vectors.  A lane's CRC row and the tile it moves may belong to different chunks of
// the group; the CRC role reads its chunk's descriptor.  Row r of unit u ends (31 − r)·4·s_fd
// bytes before the unit end E_u, so the lane's share is K[u]·x^(8·(31 − r)·4·s_fd)·crc(row);
// its units u, u + 8/G, … fold with SD (regular layout) as in the fused kernels.
// SWAP (= a.swap, bytes(big) on uint32) is a template argument: the byte swap of the movers and
// the CRC's byte order cost no select per word.  LDS: T, S (unused), SD, K, table, tiles.
// (The same kernel on the encode view measured slower than the fused tile encode, 44.73 vs
// 43.57 ms, profiles/r03/v, and was removed in round 4.)
template <int G, bool SWAP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3)))
void tiles_rowcrc_kernel(ScatterArgs a) {
  static_assert(G == 1 || G == 2 || G == 4, "a wave's CRC rows must belong to one chunk");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t(*T)[256] = reinterpret_cast<uint32_t(*)[256]>(smem);
  uint32_t* flag = T[8];  // 8 words of the S area (no zero-shift table here)
  uint32_t(*SD)[256] = T + 12;
  uint32_t* K = reinterpret_cast<uint32_t*>(SD + 4);
  uint2* tab = reinterpret_cast<uint2*>(smem + ((16 * 1024 + (size_t)a.fast_n * 4 + 15) & ~(size_t)15));
  uint32_t* lds = reinterpret_cast<uint32_t*>(
      reinterpret_cast<uint8_t*>(tab) + (((size_t)a.fast_n * 8 + 15) & ~(size_t)15));
  const int tid = threadIdx.x;
  for (int i = tid; i < a.fast_n; i += kBlock) tab[i] = reinterpret_cast<const uint2*>(a.fast_tab)[i];
#pragma unroll
  for (int k = 0; k < 8; k++) T[k][tid] = SWAP ? __builtin_bswap32(g_crc.T[k][tid]) : g_crc.T[k][tid];
#pragma unroll
  for (int b = 0; b < 4; b++)
    SD[b][tid] = a.crc_tile_step ? multmodp(a.crc_tile_step, (uint32_t)tid << (8 * b)) : 0u;
  for (int i = tid; i < a.fast_n; i += kBlock) K[i] = a.fast_tab[2 * a.fast_n + i];
  __syncthreads();
  constexpr int TG = kTG / G;
  const int wave = tid >> 6, lane = tid & 63;
  const int t = lane >> 3, g = lane & 7, q = t / TG, ti = t % TG;  // mover role
  const int tc = tid >> 5, r = tid & 31, qc = tc / TG, tic = tc % TG;  // CRC role (wave-uniform qc)
  const int64_t s_fd = a.pstride[a.fd], d_fs = a.rstride[a.fs];
  const bool regular = a.crc_tile_step != 0;
  const uint32_t units = (uint32_t)a.fast_n;
  const int64_t ngroups = (a.n_citems + G - 1) / G;
  const uint32_t kr = x2nmodp((uint64_t)(31 - r) * 4 * (uint64_t)s_fd, 3);
  const uint32_t kq = regular && (uint32_t)tic < units
                          ? multmodp(kr, K[tic + (units - 1 - tic) / TG * TG]) : 0u;
  uint32_t* mine = lds + t * kTilePitch;
  const uint32_t* crow = lds + tc * kTilePitch + r * 33;
  auto sw = [](uint32_t x) { return SWAP ? __builtin_bswap32(x) : x; };
  for (int64_t gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
    const int64_t pg = a.item_mul ? (int64_t)(((uint64_t)gi * a.item_mul) % (uint64_t)ngroups) : gi;
    const int64_t c = pg * G + q, cc = pg * G + qc;
    bool on = false, onc = false;
    const uint8_t* src = nullptr;
    uint8_t* dst = nullptr;
    if (c < a.n_citems) {
      const uint4* dp = reinterpret_cast<const uint4*>(a.desc + c);
      const uint4 x = dp[0], y = dp[1];
      on = (y.z & kDescFast) != 0;
      src = (const uint8_t*)(uintptr_t)(((uint64_t)x.y << 32) | x.x);
      dst = a.region + (int64_t)(((uint64_t)x.w << 32) | x.z) * 4;
    }
    if (cc < a.n_citems) onc = (reinterpret_cast<const uint4*>(a.desc + cc)[1].z & kDescFast) != 0;
    // block-uniform skip; __syncthreads_or would add static LDS and move the tables off 0.
    // Per-wave flags in the unused S area, by iteration parity (every iteration has this
    // barrier, so no wave is more than one iteration ahead of another here).
    {
      const uint32_t any = __ballot(on) != 0 ? 1u : 0u;
      if (lane == 0) flag[((gi / gridDim.x) & 1) * 4 + wave] = any;
      __syncthreads();
      const uint32_t* f = flag + ((gi / gridDim.x) & 1) * 4;
      if ((f[0] | f[1] | f[2] | f[3]) == 0) continue;
    }
    uint32_t share = 0, run = 0, ulast = ~0u;
    uint4 x[8];
    auto load = [&](uint32_t ub_) {
      const uint32_t uu = ub_ + ti;
      if (on && uu < units) {
        const uint8_t* base = src + ((size_t)tab[uu].x + g * 4) * 4;
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = ld16s<true>(base + (size_t)(wave * 8 + k) * s_fd * 4);
      }
    };
    load(0);
#pragma unroll 1
    for (uint32_t ub = 0; ub < units; ub += TG) {
      const uint32_t u = ub + ti, uc = ub + tic;
      const bool live = on && u < units, livec = onc && uc < units;
      if (live) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
          uint32_t* row = mine + (wave * 8 + k) * 33 + g * 4;
          row[0] = sw(x[k].x);
          row[1] = sw(x[k].y);
          row[2] = sw(x[k].z);
          row[3] = sw(x[k].w);
        }
      }
      __syncthreads();
      if (ub + TG < units) load(ub + TG);
      if (live) {
        uint8_t* base = dst + ((size_t)tab[u].y + g * 4) * 4;
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const int rr = wave * 8 + k;
          uint4 y;
          y.x = mine[(g * 4 + 0) * 33 + rr];
          y.y = mine[(g * 4 + 1) * 33 + rr];
          y.z = mine[(g * 4 + 2) * 33 + rr];
          y.w = mine[(g * 4 + 3) * 33 + rr];
          st16s<true>(base + (size_t)rr * d_fs * 4, y);
        }
      }
      uint32_t w[32];
      if (livec) {
#pragma unroll
        for (int j = 0; j < 32; j++) w[j] = crow[j];
      }
      __syncthreads();
      if (livec) {
        uint32_t acc = 0;  // byte-swapped with SWAP
#pragma unroll
        for (int j = 0; j < 32; j += 2) acc = crc_upd8_lds<SWAP>(acc, w[j], w[j + 1]);
        if (SWAP) acc = __builtin_bswap32(acc);
        if (regular) {
          run = (ulast == ~0u ? 0u : crc_shift_tab(run, SD)) ^ acc;
          ulast = uc;
        } else {
          share ^= multmodp(K[uc], acc);
        }
      }
    }
    // regular fold: the CRC role's last unit is tic + a multiple of TG in every fast chunk,
    // so its two end multiplies fold into the lane constant kq
    uint32_t cr = regular ? (ulast != ~0u ? multmodp(kq, run) : 0u) : multmodp(kr, share);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cr ^= (uint32_t)__shfl_xor((int)cr, o, 64);
    if (lane == 0 && onc) atomicXor(a.crc_partials + cc, cr);
  }
}

// LDS layout of tiles_rowcrc_aln_kernel (bytes from the dynamic block's start, which is LDS 0:
// rowcrc_lds_at_zero).  A region overlapping the next one corrupts a table; round 3's aligned
// encode once put a ring row over K and spun a zero-K multiply, so the offsets are checked here
// and the host checks fast_n ≤ kAlnKMax before it selects the kernel.
constexpr int kAlnBoxAt = 8 * 256 * 4;                   // after T[8][256]
constexpr int kAlnBoxWords = 31 * 32;                    // rows 0-30 of a 32-word line each
constexpr int kAlnKAt = kAlnBoxAt + 4 * kAlnBoxWords;    // K[unit]
constexpr int kAlnKMax = kAlnUnitsMax;                   // units per chunk (host: fast_n ≤ 32)
constexpr int kAlnSDnAt = 12288;                         // SDn[8][16]
constexpr int kAlnSlotsAt = kAlnSDnAt + 8 * 16 * 4;      // 9 tile slots
static_assert(kAlnKAt + 4 * kAlnKMax <= kAlnSDnAt, "aligned row-CRC LDS: K overlaps SDn");
static_assert(kAlnSDnAt % 16 == 0 && kAlnSlotsAt % 16 == 0, "aligned row-CRC LDS alignment");
static_assert(kAlnSlotsAt + 9 * kTilePitch * 4 <= 160 * 1024 / 3,
              "aligned row-CRC LDS: 3 workgroups per CU (160 KiB)");

// decode, the row-CRC tile kernel over 128-B aligned lines (the default; host: a.tile_align,
// one chunk per work item, 16 ≤ fast_n ≤ 32 units, fast_n % 8 == 0, tab[u] = (32u, u·ystride)).
// The payload is then [32 rows][fast_n units][32 words]: step s of row r is the contiguous 1 KiB
// L(r, s) at 4096r·(fast_n/32) + 1024s.  A payload after a 4-byte crc32c starts δ = 4i mod 128
// bytes into a line, so a 1 KiB wave load of L(r, s) touched 9 lines, the first and last shared
// with other loads (the row-CRC kernel read ≈1.11× the payload bytes, PMC).  Here the movers
// load the aligned lines 1..8 of L(r, s) (lane λ: 16 B at 128 + 16λ from its first line) and
// write word j of lane λ, element e = 32 − δ/4 + 4λ + j of L(r, s), to tile e / 32, column
// e mod 32.  Elements e ≥ 256 (the start of L(r, s + 1), lanes 56-63) go to step s + 1's tile 0:
// the tiles live in a ring of 9 LDS slots (step s's tile t' in slot (8s + t') mod 9, so its
// "tile 8" IS the next step's tile 0, and that slot held the previous step's tile 7, already
// read).  Line 0 of L(r, 0) is the end of row r − 1: the head loads before step 0 (lane (t, g):
// 16 B of row 8w + t's first line) put its first δ bytes in the box (row r − 1's tail, taken by
// lanes 56-63 at the last step, which load line 7 again instead of line 8 for rows < 31) and
// the rest in tile 0.
// Per chunk 1025 line fetches, the minimum for a misaligned 128 KiB (1 shared with the previous
// chunk).  CRC as tiles_rowcrc_kernel (lane i: payload row i & 31 of tile i >> 5 from LDS).
// LDS (bytes): T[8][256] at 0 (byte-swapped entries with SWAP), the box (31 rows × 32 words)
// and K (≤ 32 words) in the S area at 8192, the unit-step shift as nibble tables SDn[8][16] at
// 12288 (8 lookups per step instead of 4; byte tables would take 4 KiB), the 9 slots at 12800:
// 50 852 B, 3 workgroups per CU (54 436 B, with byte tables, ran 2 per CU: 42.4 vs 36.4 ms, the
// same as the unaligned kernel padded to that size, profiles/r03/occ).  Every lane reads the
// same descriptor (G = 1): the skip is block-uniform.
template <bool SWAP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3)))
void tiles_rowcrc_aln_kernel(ScatterArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint32_t(*T)[256] = reinterpret_cast<uint32_t(*)[256]>(smem);
  uint32_t* const box = reinterpret_cast<uint32_t*>(smem + kAlnBoxAt);
  uint32_t* const K = reinterpret_cast<uint32_t*>(smem + kAlnKAt);
  uint32_t(*SDn)[16] = reinterpret_cast<uint32_t(*)[16]>(smem + kAlnSDnAt);
  uint32_t* const lds = reinterpret_cast<uint32_t*>(smem + kAlnSlotsAt);
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 8; k++) T[k][tid] = SWAP ? __builtin_bswap32(g_crc.T[k][tid]) : g_crc.T[k][tid];
  if (tid < 128)
    SDn[tid >> 4][tid & 15] =
        a.crc_tile_step ? multmodp(a.crc_tile_step, (uint32_t)(tid & 15) << (4 * (tid >> 4))) : 0u;
  for (int i = tid; i < a.fast_n; i += kBlock) K[i] = a.fast_tab[2 * a.fast_n + i];
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63, t = lane >> 3, g = lane & 7;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int tc = tid >> 5, r = tid & 31;  // CRC role
  const int64_t s_fd = a.pstride[a.fd], d_fs = a.rstride[a.fs];
  const bool regular = a.crc_tile_step != 0;
  const uint32_t units = (uint32_t)a.fast_n, ys = (uint32_t)a.tile_ystride;
  const uint32_t kr = x2nmodp((uint64_t)(31 - r) * 4 * (uint64_t)s_fd, 3);
  // units % 8 == 0 (host): every lane's last unit is units − 8 + tc in every chunk, so its
  // two end multiplies (K of that unit, then kr) fold into one lane constant
  const uint32_t kq = regular ? multmodp(kr, K[units - kTG + tc]) : 0u;
  auto sw = [](uint32_t v) { return SWAP ? __builtin_bswap32(v) : v; };
  auto rfl = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
  for (int64_t gi = blockIdx.x; gi < a.n_citems; gi += gridDim.x) {
    const int64_t c = a.item_mul ? (int64_t)(((uint64_t)gi * a.item_mul) % (uint64_t)a.n_citems) : gi;
    const uint4* dp = reinterpret_cast<const uint4*>(a.desc + c);
    const uint4 dx = dp[0], dy = dp[1];
    if ((rfl(dy.z) & kDescFast) == 0) continue;  // block-uniform
    const uint8_t* src = (const uint8_t*)(uintptr_t)(((uint64_t)rfl(dx.y) << 32) | rfl(dx.x));
    uint8_t* dst = a.region + (int64_t)(((uint64_t)rfl(dx.w) << 32) | rfl(dx.z)) * 4;
    const uint32_t dl = (uint32_t)(uintptr_t)src & 127u;
    const int Dp = dl ? (int)(dl >> 2) : 32;  // δ/4; 32: aligned (no head, carry or tail)
    const uint8_t* wsrc = dl ? src - dl + 128 : src;
    uint4 x[8];
    auto load = [&](uint32_t ub, bool last) {
      const uint8_t* base = wsrc + (size_t)ub * 128;
      // last step: lines 8 of rows < 31 are the next rows' head lines, already loaded: lanes
      // 56-63 then load line 7 again, in the same instruction as lanes 48-55 (no extra line,
      // no divergent branch; the box replaces the words)
      const uint32_t back = dl && last && t == 7 ? 128u : 0u;
#pragma unroll
      for (int k = 0; k < 8; k++)
        x[k] = ld16g(base + (size_t)(wv * 8 + k) * s_fd * 4,
                     (uint32_t)(16 * lane) - (wv * 8 + k < 31 ? back : 0u));
    };
    if (dl) {  // head lines: row hr − 1's tail | row hr's tile-0 head (slot 0)
      const uint4 h = ld16g(src - dl + (size_t)wv * 8 * s_fd * 4, (uint32_t)(t * s_fd * 4 + 16 * g));
      load(0, false);
      const int hr = wv * 8 + t;
      const uint32_t hv[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int d = 4 * g + j;
        if (d < Dp) {
          if (hr > 0) box[(hr - 1) * 32 + d] = sw(hv[j]);
        } else {
          lds[hr * 33 + d - Dp] = sw(hv[j]);
        }
      }
    } else {
      load(0, false);
    }
    uint32_t share = 0, run = 0, ulast = ~0u;
    int sb = 0;  // slot of this step's tile 0: (8s) mod 9
#pragma unroll 1
    for (uint32_t ub = 0; ub < units; ub += kTG) {
      const bool last = ub + kTG >= units;
      {
        int e0 = 32 - Dp + 4 * lane;  // element of L(r, s) held by word 0
        asm volatile("" : "+v"(e0));  // the word addresses stay per-step registers
        int wa[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int e = e0 + j;
          int sl = sb + (e >> 5);
          sl -= sl >= 9 ? 9 : 0;
          wa[j] = sl * kTilePitch + (e & 31);
        }
        if (dl && last) {  // the row tails of rows < 31 come from the box (lanes 56-63)
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const int rr = wv * 8 + k;
            uint32_t v[4] = {sw(x[k].x), sw(x[k].y), sw(x[k].z), sw(x[k].w)};
            if (t == 7 && rr < 31) {
              const uint4 bv = *reinterpret_cast<const uint4*>(box + rr * 32 + 4 * g);
              const uint32_t b4[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
              for (int j = 0; j < 4; j++)
                if (4 * g + j < Dp) v[j] = b4[j];
            }
#pragma unroll
            for (int j = 0; j < 4; j++) lds[wa[j] + rr * 33] = v[j];
          }
        } else {
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const int rr = wv * 8 + k;
            lds[wa[0] + rr * 33] = sw(x[k].x);
            lds[wa[1] + rr * 33] = sw(x[k].y);
            lds[wa[2] + rr * 33] = sw(x[k].z);
            lds[wa[3] + rr * 33] = sw(x[k].w);
          }
        }
      }
      __syncthreads();
      if (!last) load(ub + kTG, ub + 2 * kTG >= units);
      {  // movers: tile t (slot (sb + t) mod 9) to the region, scalar chunk base + row
        int st = sb + t;
        st -= st >= 9 ? 9 : 0;
        const uint32_t* mine = lds + st * kTilePitch;
        const uint32_t voff = ((ub + t) * ys + 4 * g) * 4;
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const int rr = wave * 8 + k;
          uint4 y;
          y.x = mine[(g * 4 + 0) * 33 + rr];
          y.y = mine[(g * 4 + 1) * 33 + rr];
          y.z = mine[(g * 4 + 2) * 33 + rr];
          y.w = mine[(g * 4 + 3) * 33 + rr];
          st16g(dst + (size_t)(wv * 8 + k) * d_fs * 4, voff, y);
        }
      }
      uint32_t w[32];
      {
        int sc = sb + tc;
        sc -= sc >= 9 ? 9 : 0;
        const uint32_t* crow = lds + sc * kTilePitch + r * 33;
#pragma unroll
        for (int j = 0; j < 32; j++) w[j] = crow[j];
      }
      __syncthreads();
      uint32_t acc = 0;  // byte-swapped with SWAP (byte tables)
#pragma unroll
      for (int j = 0; j < 32; j += 2) acc = crc_upd8_lds<SWAP>(acc, w[j], w[j + 1]);
      if (SWAP) acc = __builtin_bswap32(acc);
      const uint32_t uc = ub + tc;
      if (regular) {
        uint32_t sh = 0;  // run · x^(8Δ), nibble by nibble
#pragma unroll
        for (int i = 0; i < 8; i++) sh ^= SDn[i][(run >> (4 * i)) & 15];
        run = (ulast == ~0u ? 0u : sh) ^ acc;
        ulast = uc;
      } else {
        share ^= multmodp(K[uc], acc);
      }
      sb = sb == 0 ? 8 : sb - 1;
    }
    uint32_t cr = regular ? multmodp(kq, run) : multmodp(kr, share);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cr ^= (uint32_t)__shfl_xor((int)cr, o, 64);
    if (lane == 0) atomicXor(a.crc_partials + c, cr);
  }
}

// The CRC-fused decode variant held to 3 waves per SIMD (LDS allows 3 blocks of 4 waves per
// CU; unconstrained it takes 172 VGPRs and runs 2)
template <int NT, bool FLAGS>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3)))
void decode_tiles_crc_w3_kernel(ScatterArgs a) {
  decode_tiles_body<NT, true, FLAGS>(a);
}

// decode, slow kernel: the items the resolve kernel listed (clipped by the region,
// misaligned, or without a fast table), through the generic strided paths
__device__ void crc_index_block(const CrcIdxArgs& c, int64_t span, uint32_t* lds);  // below

// The first c.nspans workgroups run the index crc32c instead (crc_index_block; c.nspans = 0
// when the plan launched it on its own), in the same LDS.
template <int DS, bool TILE>
__global__ __launch_bounds__(kBlock) void decode_slow_kernel(ScatterArgs a, CrcIdxArgs c) {
  using T = typename ElemT<DS>::T;
  constexpr int kTileWords = ((TILE ? kTileTPB : 1) * 32 * 33 * DS + 7) / 8 * 2;
  __shared__ uint64_t sm[(kTileWords > kCrcLdsWords ? kTileWords : kCrcLdsWords) / 2 + 1];
  if (blockIdx.x < c.nspans) {  // uniform per workgroup
    crc_index_block(c, blockIdx.x, reinterpret_cast<uint32_t*>(sm));
    return;
  }
  T (*tile)[32][33] = reinterpret_cast<T (*)[32][33]>(sm);
  const int64_t total = (int64_t)(*a.slow_count) << a.piece_shift;
  const uint32_t pmask = (1u << a.piece_shift) - 1;
  const int64_t nb = (int64_t)gridDim.x - c.nspans;
  for (int64_t k = (int64_t)blockIdx.x - c.nspans; k < total; k += nb) {
    const uint32_t citem = a.slow_list[k >> a.piece_shift];
    const uint32_t piece = (uint32_t)k & pmask;
    const ItemDesc D = ld_desc(a.desc + citem);
    Item it;
    if ((D.kind & kDescModeMask) == kDescClip) {
      make_item<false>(a, ((int64_t)citem << a.piece_shift) | piece, it, &D);
    } else {
      full_item(a, D, piece, it);
    }
    generic_item<DS, TILE>(a, it, tile);
  }
}

// decode, small plans in one launch (zh_plan::small_one): the index crc32c workgroups first
// (c.nspans, as in the slow kernel), then one workgroup per item piece resolves its item's
// index entry (resolve_one, the resolve kernel's per-item body, on one lane; its status writes
// are idempotent across an item's pieces) and moves it through the generic paths the slow
// kernel uses.  A 64³ region of a c4 shard (27 inner chunks, 26 clipped) took four dependent
// launches: the index CRC, resolve, the fast kernel for its one whole chunk, the slow list.
template <int DS, bool TILE>
__global__ __launch_bounds__(kBlock) void decode_small_kernel(ScatterArgs a, CrcIdxArgs c) {
  using T = typename ElemT<DS>::T;
  constexpr int kTileWords = ((TILE ? kTileTPB : 1) * 32 * 33 * DS + 7) / 8 * 2;
  __shared__ uint64_t sm[(kTileWords > kCrcLdsWords ? kTileWords : kCrcLdsWords) / 2 + 1];
  __shared__ ItemDesc sd;
  if (blockIdx.x < c.nspans) {  // uniform per workgroup
    crc_index_block(c, blockIdx.x, reinterpret_cast<uint32_t*>(sm));
    return;
  }
  T (*tile)[32][33] = reinterpret_cast<T (*)[32][33]>(sm);
  const int64_t total = a.total_items;
  const uint32_t pmask = (1u << a.piece_shift) - 1;
  const int64_t nb = (int64_t)gridDim.x - c.nspans;
  for (int64_t k = (int64_t)blockIdx.x - c.nspans; k < total; k += nb) {
    const int64_t citem = k >> a.piece_shift;
    if (threadIdx.x == 0) sd = resolve_one(a, citem);
    __syncthreads();
    const ItemDesc D = sd;
    __syncthreads();
    const uint32_t mode = D.kind & kDescModeMask;
    if (mode == kDescSkip) continue;  // uniform
    Item it;
    if (mode == kDescClip) {
      make_item<false>(a, k, it, &D);
    } else {
      full_item(a, D, (uint32_t)k & pmask, it);
    }
    generic_item<DS, TILE>(a, it, tile);
  }
}

// encode one (piece of an) item through the generic paths: source = region, destination =
// shard payload, boundary padding written as fill_value.  FLAG (row paths): returns this
// thread's share of the all-fill test from the same loads.
template <int DS, bool TILE, bool FLAG = false>
__device__ __forceinline__ bool encode_item(const ScatterArgs& a, Item& it,
                                            typename ElemT<DS>::T (*tile)[32][33]) {
  const int64_t* sstr = a.rstride;
  const int64_t* dstr = a.pstride;
  const int n = a.ndim;
  if constexpr (!TILE) {
    const int F = a.fs;  // == a.fd
    uint32_t nrows = 1;
    bool clipped = false;
#pragma unroll
    for (int d = 0; d < kMaxDims; d++) {
      if (d < n && d != F) nrows *= (uint32_t)it.e[d];
      if (d < n) clipped |= it.v[d] != it.e[d];
    }
    if (!clipped && vec_ok<DS, true>(a, it, F, sstr, dstr, it.e, true))
      return row_pass<DS, true, false, false, FLAG>(a, it, F, sstr, dstr, nrows, it.e, it.ediv);
    if (clipped && vec_clip_ok<DS>(a, it, F, sstr, dstr))
      return row_pass<DS, true, false, true, FLAG>(a, it, F, sstr, dstr, nrows, it.e, it.ediv);
    return row_pass<DS, false, false, false, FLAG>(a, it, F, sstr, dstr, nrows, it.e, it.ediv);
  } else {
    tile_pass<DS>(a, it, sstr, dstr, tile);
    return false;
  }
}

// Does this thread's share of the loadable part of an (encode) item differ from fill_value?
template <int DS>
__device__ __forceinline__ bool flag_item(const ScatterArgs& a, const Item& it) {
  const int64_t* sstr = a.rstride;
  const int n = a.ndim, F = n - 1;
  int32_t ext[kMaxDims];
  FastDiv ediv[kMaxDims];
  uint32_t nrows = 1;
  bool vec = !(((uintptr_t)(it.sbase + it.s0 * DS)) & 15);
#pragma unroll
  for (int d = 0; d < kMaxDims; d++) {
    ext[d] = it.v[d];
    ediv[d] = it.ediv[d];
    if (d >= n) continue;
    if (ext[d] != a.inner[d] && ext[d] > 0) ediv[d] = make_fastdiv((uint32_t)ext[d]);
    if (d != F) {
      nrows *= (uint32_t)ext[d];
      if (ext[d] > 1 && ((sstr[d] * DS) & 15)) vec = false;
    } else if ((ext[d] * DS) & 15) {
      vec = false;
    }
  }
  if (vec) return row_pass<DS, true, true>(a, it, F, sstr, sstr, nrows, ext, ediv);
  return row_pass<DS, false, true>(a, it, F, sstr, sstr, nrows, ext, ediv);
}

// ---------------------------------------------------------------------------------
// write path, one pass (zh_array_write fast path): the layout assumes every in-bounds
// inner chunk is kept, the fast decode kernels run on an "encode view" (source = region,
// destination = payloads) and record the all-fill test per piece; when some chunk turns out
// to be all fill_value, the host runs a second pass with the true layout over those shards.
// ---------------------------------------------------------------------------------
// per inner chunk: its payload offset under the one-pass layout (every in-bounds inner chunk
// kept, C order: the chunk's rank in the shard's in-bounds box × stored chunk bytes, after the
// index when it is at the start; -1 for chunks wholly in the boundary padding; item_off ==
// nullptr: a.item_off was uploaded by the host), then the
// encode-view descriptor (src = the chunk's origin in the region, d0 = its payload position
// relative to vbase, in elements) or a slow-list entry (clipped by the array boundary,
// misaligned)
// Nested sharding: a leaf's cell (C order over the shard's cells), its position in the cell
// (C order over the cell's leaf grid) and its rank in the cell's in-bounds leaf box.
__device__ __forceinline__ void nest_coords(const ScatterArgs& a, const EncNest& nz,
                                            const DevShard& S, int64_t c, int64_t& cell,
                                            int64_t& k2, int64_t& rank, bool& in) {
  uint32_t j = (uint32_t)(c - S.item_begin);
  int64_t mc = 1, mk = 1, mr = 1;
  cell = k2 = rank = 0;
  in = true;
#pragma unroll
  for (int d = kMaxDims - 1; d >= 0; --d) {
    if (d >= a.ndim) continue;
    const uint32_t bc = (uint32_t)S.box_count[d];
    const uint32_t q = j / bc;
    const int32_t lc = (int32_t)(j - q * bc);
    j = q;
    const int32_t c1 = lc / nz.r[d], w = lc - c1 * nz.r[d];
    const int32_t cnt = a.fill_never ? nz.r[d]
                                     : min(nz.r[d], (S.part_hi[d] - c1 * nz.r[d] * a.inner[d] +
                                                     a.inner[d] - 1) / a.inner[d]);
    in &= w < cnt;
    cell += c1 * mc;
    mc *= nz.g1[d];
    k2 += w * mk;
    mk *= nz.r[d];
    rank += w * mr;
    mr *= max(cnt, 1);
  }
}

__global__ __launch_bounds__(kBlock) void encode_resolve_kernel(ScatterArgs a, EncNest nz,
                                                                int64_t* item_off,
                                                                int64_t base_off, int64_t cn,
                                                                const uint8_t* vbase,
                                                                int vfast) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x; c < a.n_citems; c += stride) {
    if (!item_off) {  // offsets uploaded by the host (second pass after a fallback)
    } else if (nz.cell) {  // nested: the cell's offset + the sub-index (at the start) + the rank
      const int64_t s = find_shard(a, c);
      int64_t cell, k2, rank;
      bool in;
      nest_coords(a, nz, a.shards[s], c, cell, k2, rank, in);
      const int64_t co = nz.cell[2 * (s * nz.ncell + cell)];
      item_off[c] = in && co >= 0 ? co + (nz.sub_start ? nz.sub_isz : 0) + rank * cn : -1;
    } else {
      const DevShard& S = a.shards[find_shard(a, c)];
      uint32_t j = (uint32_t)(c - S.item_begin);
      int64_t rank = 0, mul = 1;
      bool in = true;
#pragma unroll
      for (int d = kMaxDims - 1; d >= 0; --d) {
        if (d >= a.ndim) continue;
        const uint32_t bc = (uint32_t)S.box_count[d];
        const uint32_t q = j / bc;
        const int64_t icd = (int64_t)(j - q * bc);
        j = q;
        const int64_t cnt = a.fill_never ? (int64_t)bc : (S.part_hi[d] + a.inner[d] - 1) / a.inner[d];
        in &= icd < cnt;
        rank += icd * mul;
        mul *= cnt;
      }
      item_off[c] = in ? base_off + rank * cn : -1;
    }
    Item it;
    make_item<true>(a, c << a.piece_shift, it);
    ItemDesc D;
    D.src = 0;
    D.d0 = 0;
    D.fill = 0;
    D.shard = 0;
    D.kind = kDescSkip;
    if (it.mode != kSkip) {
      bool full = true;
#pragma unroll
      for (int d = 0; d < kMaxDims; d++)
        if (d < a.ndim) full &= it.v[d] == it.e[d];
      const uint64_t saddr = (uint64_t)(uintptr_t)(it.sbase + it.s0 * a.dsize);
      const int64_t doff = it.dbase - vbase;
      D.src = saddr;
      D.d0 = doff / a.dsize;
      D.kind = kDescFullCopy;
      const bool fast = vfast && full && (saddr & 3) == 0 &&
                        (((uintptr_t)it.dbase) & 3) == 0 && doff >= 0 && doff % a.dsize == 0 &&
                        (!a.tile || a.dsize == 4);
      if (fast) {
        D.kind |= kDescFast;
      } else {
        const uint32_t slot = atomicAdd(a.slow_count, 1u);
        a.slow_list[slot] = (uint32_t)c;
      }
    }
    a.desc[c] = D;
  }
}

// the slow-list chunks: generic encode + the all-fill test of each piece
template <int DS, bool TILE>
__global__ __launch_bounds__(kBlock) void encode_slow_kernel(ScatterArgs a) {
  using T = typename ElemT<DS>::T;
  __shared__ T tile[TILE ? kTileTPB : 1][32][33];
  const int64_t total = (int64_t)(*a.slow_count) << a.piece_shift;
  const uint32_t pmask = (1u << a.piece_shift) - 1;
  for (int64_t k = blockIdx.x; k < total; k += gridDim.x) {
    const int64_t item = ((int64_t)a.slow_list[k >> a.piece_shift] << a.piece_shift) |
                         ((uint32_t)k & pmask);
    Item it;
    make_item<true>(a, item, it);
    if (it.mode == kSkip) continue;
    // row paths test the loaded vectors on the way; the tile path reads the piece twice
    const bool diff = TILE ? flag_item<DS>(a, it) : encode_item<DS, false, true>(a, it, tile);
    if constexpr (TILE) encode_item<DS, TILE>(a, it, tile);
    const int any = __syncthreads_or(diff ? 1 : 0);
    if (threadIdx.x == 0 && any) a.flags[item >> a.piece_shift] = 1;
  }
}

// after the one-pass encode, per inner chunk: count a kept chunk none of whose pieces holds a
// non-fill element (the layout assumed it kept; the reference elides it, :129-133 → the host
// falls back), build its chunk-CRC store descriptor (inner crc32c), and write the index entry
// (ShardingIndexedCodec.encode :135-160): (offset, nbytes) or (-1, -1), in the index codecs'
// byte order, at S.index_off of the shard's buffer
__global__ __launch_bounds__(kBlock) void encode_finish_kernel(ScatterArgs a, EncNest nz,
                                                               int64_t chunk_nbytes,
                                                               uint32_t* bad, ItemDesc* crc_desc) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x; c < a.n_citems; c += stride) {
    const int64_t s = find_shard(a, c);
    const DevShard& S = a.shards[s];
    const int64_t off = a.item_off[c];
    if (off >= 0 && a.flags[c] == 0) atomicAdd(bad, 1u);
    if (crc_desc) {
      ItemDesc D;
      D.src = off >= 0 ? (uint64_t)(uintptr_t)(S.wdata + off) : 0;
      D.d0 = 0;
      D.fill = 0;
      // the fast bit tells the CRC pass which chunks the row kernel already hashed
      D.kind = off >= 0 ? kDescFullCopy | (a.desc[c].kind & kDescFast) : kDescSkip;
      D.shard = (uint32_t)s;
      crc_desc[c] = D;
    }
    uint64_t eo = off >= 0 ? (uint64_t)off : ~0ull;
    const uint64_t en = off >= 0 ? (uint64_t)chunk_nbytes : ~0ull;
    uint8_t* e;
    int be;
    if (nz.cell) {  // nested: the leaf's entry in its cell's sub-shard index, offset relative
      int64_t cell, k2, rank;  // to the cell (ShardingIndexedCodec.encode of the sub-shard)
      bool in;
      nest_coords(a, nz, S, c, cell, k2, rank, in);
      const int64_t* ci = nz.cell + 2 * (s * nz.ncell + cell);
      if (ci[0] < 0) continue;  // elided cell: no sub-index (the host wrote (-1, -1) above it)
      if (off >= 0) eo = (uint64_t)(off - ci[0]);
      e = S.wdata + ci[1] + 16 * k2;
      be = nz.sub_be;
    } else {
      if (!a.sharded || S.index_off < 0) continue;
      e = S.wdata + S.index_off + 16 * (c - S.item_begin);
      be = a.index_be;
    }
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const int sh = be ? 56 - 8 * b : 8 * b;
      e[b] = (uint8_t)(eo >> sh);
      e[8 + b] = (uint8_t)(en >> sh);
    }
  }
}

// ---------------------------------------------------------------------------------
// CRC-32C of the shard index (helpers: "CRC-32C helpers" above the row kernel)
// ---------------------------------------------------------------------------------
// Standard CRC-32C of a span of slen bytes from the lanes' raw registers c (init 0, no final
// xor) of their segments [lb, lb + llen): shift each to the span end, XOR the block, add the
// init/xorout terms.  Uniform call; every lane returns the result.
__device__ uint32_t lanes_to_span_crc(uint32_t c, int64_t lb, int64_t llen, int64_t slen,
                                      uint32_t* red) {
  const int tid = threadIdx.x;
  uint32_t v = llen > 0 ? multmodp(x2nmodp((uint64_t)(slen - lb - llen), 3), c) : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  uint32_t raw = 0;
#pragma unroll
  for (int w = 0; w < kBlock / 64; w++) raw ^= red[w];
  const uint32_t r = multmodp(x2nmodp((uint64_t)slen, 3), 0xFFFFFFFFu) ^ raw ^ 0xFFFFFFFFu;
  __syncthreads();
  return r;
}


// Index CRC, one workgroup per 4 KiB span of a job (a shard index, or a sub-shard index on
// the write path), finished in the same launch: each span's raw register (init 0, no xorout)
// goes to partials[span]; the job's last workgroup to finish (a self-resetting counter per
// job, after partials[nspans + job]) shifts every span's register to the job end in parallel
// (one lane per span, x^(8·4096·j) from a table), XORs them, adds the init/xorout terms, and
// compares
// with the stored little-endian crc32c (decode: Crc32cCodec.decode :24-48, status) or stores
// it (status == nullptr: Crc32cCodec.encode :50-60).  A dword-aligned span is read as
// coalesced 16-byte vectors (lane l: vectors l, l+256, ...) with the lane-interleaved update;
// otherwise with a per-lane slicing-by-8 byte loop.
// The combine of one job's span partials (the last workgroup of crc_index_kernel): shift every
// span register to the index end, XOR, finish the CRC, then compare it with the stored one
// (read) or store it (write path).  (A second launch for the combine, without the per-workgroup
// device-scope release of the completion counter, measured slower: 74.2 vs 69.7 µs per small
// read, profiles/r03/q; removed in round 4.)
__device__ __forceinline__ void crc_index_finish(const CrcJob& J, const uint32_t* partials,
                                                 int sshift, uint64_t* status, uint32_t* red) {
  const int tid = threadIdx.x;
  const int64_t SPAN = (int64_t)kIdxSpan << sshift;
  const int64_t njs = (J.len + SPAN - 1) / SPAN;
  // span k ends at min((k+1)·SPAN, len); the bytes after it are (njs−1−k)·SPAN when the last
  // span is full, else (njs−2−k)·SPAN + tail (the last span itself: 0)
  const int64_t tail = J.len - (njs - 1) * SPAN;
  const uint32_t xtail = tail == SPAN ? g_crc.kidx[1 << sshift] : x2nmodp((uint64_t)tail, 3);
  uint32_t r = 0;
  for (int64_t k = tid; k < njs; k += kBlock) {
    const uint32_t pk = __hip_atomic_load(partials + J.span_begin + k, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
    const int64_t j = (njs - 2 - k) << sshift;  // 4 KiB units of the full spans after span k
    uint32_t sh;
    if (k == njs - 1) sh = 1u << 31;
    else if (j < 256) sh = multmodp(g_crc.kidx[j], xtail);
    else sh = x2nmodp((uint64_t)(J.len - (k + 1) * SPAN), 3);
    r ^= multmodp(sh, pk);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) r ^= (uint32_t)__shfl_xor((int)r, o, 64);
  __syncthreads();
  if ((tid & 63) == 0) red[tid >> 6] = r;
  __syncthreads();
  if (tid != 0) return;
  r = red[0] ^ red[1] ^ red[2] ^ red[3];
  const uint32_t c = multmodp(x2nmodp((uint64_t)J.len, 3), 0xFFFFFFFFu) ^ r ^ 0xFFFFFFFFu;
  const uint8_t* sp = J.base + J.len;  // stored little-endian (Crc32cCodec.java:121,130)
  if (!status) {  // write path: store it after the index (Crc32cCodec.encode :50-60)
    uint8_t* w = const_cast<uint8_t*>(sp);
    w[0] = (uint8_t)c;
    w[1] = (uint8_t)(c >> 8);
    w[2] = (uint8_t)(c >> 16);
    w[3] = (uint8_t)(c >> 24);
    return;
  }
  const uint32_t stored =
      (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) | ((uint32_t)sp[2] << 16) | ((uint32_t)sp[3] << 24);
  uint64_t* st = status + (int64_t)J.shard * kStWords;
  if (c != stored) {  // bit 32 marks the pair as set (nested sub-shard checks come later)
    st[kStCrcStored] = (1ull << 32) | stored;
    st[kStCrcComputed] = c;
    atomicOr((unsigned long long*)(st + kStFlags), (unsigned long long)kFlagCrc);
  }
}

// One workgroup's share of the index CRC launch: span `span` of the jobs, in LDS scratch of
// kCrcLdsWords words (the tables, the wave reduction, the last-workgroup flag).  Its own
// launch (crc_index_kernel, the write path) or the first c.nspans workgroups of the decode's
// slow kernel (decode_slow_kernel): the index check then runs beside the clipped chunks'
// decode instead of ahead of the resolve kernel — it only writes status words.
__device__ void crc_index_block(const CrcIdxArgs& c, int64_t span, uint32_t* lds) {
  uint32_t (*T)[256] = reinterpret_cast<uint32_t (*)[256]>(lds);
  uint32_t (*S)[256] = reinterpret_cast<uint32_t (*)[256]>(lds + 8 * 256);
  uint32_t* red = lds + 12 * 256;
  uint32_t* last = red + kBlock;
  const int sshift = c.sshift;
  const int64_t SPAN = (int64_t)kIdxSpan << sshift;
  const int tid = threadIdx.x;
  int64_t lo = 0, hi = c.njobs - 1;
  while (lo < hi) {
    int64_t mid = (lo + hi + 1) >> 1;
    if (c.jobs[mid].span_begin <= span) lo = mid;
    else hi = mid - 1;
  }
  const CrcJob J = c.jobs[lo];
  const int64_t sb = (span - J.span_begin) * SPAN;
  const int64_t slen = min(SPAN, J.len - sb);
  const uint8_t* base = J.base + sb;
  const bool aligned = (((uintptr_t)base) & 3) == 0;
  const int nblk = (int)(slen >> 4);
  // the span's first vectors are in flight while the tables are copied into LDS
  v4u v[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int j = tid + u * kBlock;
    if (aligned && j < nblk) v[u] = *reinterpret_cast<const v4u*>(base + 16 * (int64_t)j);
  }
#pragma unroll
  for (int b = 0; b < 4; b++) S[b][tid] = g_crc.S[b][tid];
  init_crc_tables(T);
  uint32_t raw;
  if (aligned) {
    uint32_t acc = 0;
    int nb = 0;
    for (int j0 = 0; j0 < nblk; j0 += kBlock * 4) {
      if (j0 > 0) {
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int j = j0 + tid + u * kBlock;
          if (j < nblk) v[u] = *reinterpret_cast<const v4u*>(base + 16 * (int64_t)j);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (j0 + tid + u * kBlock < nblk) {
          acc = crc_upd16(crc_shift_tab(acc, S), v[u], T);
          nb++;
        }
    }
    uint32_t contrib = 0;
    if (nb > 0) {
      const int64_t e = 16 * (int64_t)(tid + kBlock * (nb - 1)) + 16;
      contrib = multmodp((slen & 4095) == 0 ? g_crc.kfull[tid] : x2nmodp((uint64_t)(slen - e), 3),
                         acc);
    }
    if (tid == 0) {  // tail bytes (span length not a multiple of 16) end the span
      uint32_t t = 0;
      for (int64_t i = (int64_t)nblk * 16; i < slen; i++) t = T[0][(t ^ base[i]) & 0xFFu] ^ (t >> 8);
      contrib ^= t;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) contrib ^= (uint32_t)__shfl_xor((int)contrib, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = contrib;
    __syncthreads();
    raw = red[0] ^ red[1] ^ red[2] ^ red[3];
  } else {
    const int64_t kLane = SPAN / kBlock;  // bytes per lane
    const int64_t lb = (int64_t)tid * kLane;
    const int64_t llen = max((int64_t)0, min((int64_t)kLane, slen - lb));
    uint32_t cr = 0;
    for (int64_t i = 0; i < llen; i++) cr = T[0][(cr ^ base[lb + i]) & 0xFFu] ^ (cr >> 8);
    uint32_t w = llen > 0 ? multmodp(x2nmodp((uint64_t)(slen - lb - llen), 3), cr) : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) w ^= (uint32_t)__shfl_xor((int)w, o, 64);
    if ((tid & 63) == 0) red[tid >> 6] = w;
    __syncthreads();
    raw = red[0] ^ red[1] ^ red[2] ^ red[3];
  }
  uint32_t* counter = c.partials + c.nspans + lo;
  const int64_t njs = (J.len + SPAN - 1) / SPAN;
  // Publish the span's register write-through (an agent-scope store: sc1, past this XCD's L2)
  // and wait for it before the ticket; the last workgroup reads every partial with agent-scope
  // loads.  No release / acquire fence: __threadfence() here wrote back the whole XCD L2 in
  // every workgroup (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility").
  if (tid == 0) {
    __hip_atomic_store(c.partials + span, raw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (uint32_t)(njs - 1);
  }
  __syncthreads();
  if (!*last) return;  // uniform
  // ready for the next launch (every other workgroup has counted)
  if (tid == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  crc_index_finish(J, c.partials, sshift, c.status, red);
}

__global__ __launch_bounds__(kBlock) void crc_index_kernel(CrcIdxArgs c) {
  __shared__ uint32_t lds[kCrcLdsWords];
  crc_index_block(c, blockIdx.x, lds);
}

// (crc_upd16 / crc_shift_tab: see "CRC-32C helpers" above the row kernel)

constexpr int kDcBatch = 8;  // vectors in flight per lane

__global__ __launch_bounds__(kBlock) void data_crc_partial_kernel(DataCrcArgs a) {
  __shared__ uint32_t T[8][256];
  __shared__ uint32_t S[4][256];
  __shared__ uint32_t wred[kBlock / 64];
  const int tid = threadIdx.x;
#pragma unroll
  for (int b = 0; b < 4; b++) S[b][tid] = g_crc.S[b][tid];  // the other lanes' 255 vectors
  init_crc_tables(T);
  // a span of whole 4 KiB rounds: this lane's last vector ends 4080 - 16*tid bytes before
  // the span end
  const uint32_t kfull = g_crc.kfull[tid];
  const int64_t total = a.n_items * a.nspan;
  for (int64_t blk = blockIdx.x; blk < total; blk += gridDim.x) {
    const int64_t item = blk / a.nspan;
    const int64_t span = blk - item * a.nspan;
    const ItemDesc D = ld_desc(a.desc + item);
    const uint32_t mode = D.kind & kDescModeMask;
    // missing shards / inner chunks are clip or fill descriptors without a source
    if ((mode != kDescFullCopy && mode != kDescClip) || D.src == 0) continue;  // uniform
    if (a.skip_fast && (D.kind & kDescFast)) continue;  // fused into the row kernel
    const uint8_t* base = (const uint8_t*)(uintptr_t)D.src + span * a.span;
    const int64_t slen = min(a.span, a.len - span * a.span);
    const int nblk = (int)(slen >> 4);
    uint32_t acc = 0;
    int nb = 0;
    for (int j0 = 0; j0 < nblk; j0 += kBlock * kDcBatch) {
      v4u v[kDcBatch];
#pragma unroll
      for (int u = 0; u < kDcBatch; u++) {
        const int j = j0 + tid + u * kBlock;
        if (j < nblk) v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(base + 16 * (int64_t)j));
      }
#pragma unroll
      for (int u = 0; u < kDcBatch; u++) {
        if (j0 + tid + u * kBlock < nblk) {
          acc = crc_upd16(crc_shift_tab(acc, S), v[u], T);
          nb++;
        }
      }
    }
    uint32_t contrib = 0;
    if (nb > 0) {
      const int64_t e = 16 * (int64_t)(tid + kBlock * (nb - 1)) + 16;
      const uint32_t k = (slen & 4095) == 0 ? kfull : x2nmodp((uint64_t)(slen - e), 3);
      contrib = multmodp(k, acc);
    }
    if (tid == 0) {  // tail bytes (payload length not a multiple of 16) end the span
      uint32_t t = 0;
      for (int64_t i = (int64_t)nblk * 16; i < slen; i++) t = T[0][(t ^ base[i]) & 0xFFu] ^ (t >> 8);
      contrib ^= t;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) contrib ^= (uint32_t)__shfl_xor((int)contrib, o, 64);
    if ((tid & 63) == 0) wred[tid >> 6] = contrib;
    __syncthreads();
    if (tid == 0) a.partials[blk] = wred[0] ^ wred[1] ^ wred[2] ^ wred[3];
    __syncthreads();
  }
}

// combine the raw span registers into the standard CRC; decode: compare with the stored
// little-endian value (mismatch → Crc32cCodec.java:39-44 via the shard's status); encode:
// write it after the payload (Crc32cCodec.java:50-60)
__global__ void data_crc_finalize_kernel(DataCrcArgs a) {
  const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= a.n_items) return;
  const ItemDesc D = a.desc[item];
  const uint32_t mode = D.kind & kDescModeMask;
  if ((mode != kDescFullCopy && mode != kDescClip) || D.src == 0) return;
  uint32_t raw = 0;
  const uint32_t kspan = x2nmodp((uint64_t)a.span, 3);
  for (int64_t k = 0; k < a.nspan; k++) {
    const int64_t slen = min(a.span, a.len - k * a.span);
    raw = multmodp(slen == a.span ? kspan : x2nmodp((uint64_t)slen, 3), raw) ^
          a.partials[item * a.nspan + k];
  }
  const uint32_t c = multmodp(x2nmodp((uint64_t)a.len, 3), 0xFFFFFFFFu) ^ raw ^ 0xFFFFFFFFu;
  uint8_t* s = (uint8_t*)(uintptr_t)D.src + a.len;
  if (a.store) {
    s[0] = (uint8_t)c;
    s[1] = (uint8_t)(c >> 8);
    s[2] = (uint8_t)(c >> 16);
    s[3] = (uint8_t)(c >> 24);
    return;
  }
  const uint32_t stored =
      (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24);
  if (c != stored) {  // the chunk's shard-grid coordinates (the resolve kernel's unravel)
    const DevShard& S = a.shards[D.shard];
    uint32_t j = (uint32_t)(item - S.item_begin);
    int32_t ic[kMaxDims];
#pragma unroll
    for (int d = kMaxDims - 1; d >= 0; --d) {
      ic[d] = 0;
      if (d < a.rank.ndim) {
        const uint32_t cnt = (uint32_t)S.box_count[d];
        const uint32_t q = j / cnt;
        ic[d] = S.box_start[d] + (int32_t)(j - q * cnt);
        j = q;
      }
    }
    chunk_error(a.status + (int64_t)D.shard * kStWords, chunk_rank(a.rank, ic),
                kFlagChunkCrc | (a.rank.r2 ? kFlagLeaf : 0u), stored, c);
  }
}


// ---------------------------------------------------------------------------------
// nested sharding: flatten the two-level index (ShardingIndexedCodec.decodeInternal :183-243
// applied twice — the outer codec's inner pipeline is the level-2 sharding codec, whose
// decode(ByteBuffer) :97-103 reads its own index from the sub-shard bytes)
// ---------------------------------------------------------------------------------
// rank of level-1 cell lin1 (k2 < 0) or of its leaf k2 (RankGeom)
__device__ __forceinline__ uint32_t nest_rank(const NestArgs& a, int64_t lin1, int64_t k2) {
  return rank_clamp((uint64_t)lin1 * (uint64_t)(a.cps2 + 1) + (uint64_t)(k2 + 1));
}

// CRC-32C of p[0, len) by the whole workgroup (kBlock lanes, kCrcLane-byte segments per
// lane, kCrcSpan bytes per round); result valid in every lane.
__device__ uint32_t block_crc(const uint8_t* p, int64_t len, const uint32_t (*T)[256],
                              uint32_t* red) {
  const int tid = threadIdx.x;
  uint32_t total = 0;
  for (int64_t sb = 0; sb < len; sb += kCrcSpan) {
    const int64_t slen = min((int64_t)kCrcSpan, len - sb);
    const int64_t lb = (int64_t)tid * kCrcLane;
    const int64_t llen = max((int64_t)0, min((int64_t)kCrcLane, slen - lb));
    const uint8_t* q = p + sb + lb;
    uint32_t c = 0;
    for (int64_t i = 0; i < llen; i++) c = T[0][(c ^ q[i]) & 0xFFu] ^ (c >> 8);
    total = crc_combine(total, lanes_to_span_crc(c, lb, llen, slen, red), (uint64_t)slen);
  }
  return total;
}

__global__ __launch_bounds__(kBlock) void nested_index_kernel(NestArgs a) {
  __shared__ uint32_t T[1][256];
  __shared__ uint32_t red[kBlock];
  const int tid = threadIdx.x;
  {
    uint32_t c = (uint32_t)tid;
#pragma unroll
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
    T[0][tid] = c;
  }
  __syncthreads();
  const int n = a.ndim;
  for (int64_t it = blockIdx.x; it < a.n_l1; it += gridDim.x) {
    int64_t lo = 0, hi = a.nshards - 1;  // shard of this level-1 cell (uniform)
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (a.shards[mid].l1_begin <= it) lo = mid;
      else hi = mid - 1;
    }
    const DevShard& S = a.shards[lo];
    if (S.data == nullptr || S.flat == nullptr) continue;
    int64_t j = it - S.l1_begin, lin1 = 0, fbase = 0;
    int32_t c1[kMaxDims];
#pragma unroll
    for (int d = kMaxDims - 1; d >= 0; --d) {
      c1[d] = 0;
      if (d < n) {
        const int64_t cnt = S.l1_box_count[d];
        c1[d] = S.l1_box_start[d] + (int32_t)(j % cnt);
        j /= cnt;
        lin1 += (int64_t)c1[d] * a.cps1_stride[d];
        fbase += (int64_t)c1[d] * a.r[d] * a.flat_stride[d];
      }
    }
    const uint8_t* ent = S.data + S.index_off + 16 * lin1;
    const uint64_t off1 = ld_u64_unaligned(ent, a.index_be);
    const uint64_t nb1 = ld_u64_unaligned(ent + 8, a.index_be);
    const uint64_t total = (uint64_t)S.nbytes;
    bool ok = !(off1 == ~0ull || nb1 == ~0ull);  // missing sub-shard: zeros (Q1)
    const uint8_t* sub = nullptr;
    uint64_t held = nb1;  // the sub-shard must be held whole (sub-shard reads: one piece)
    uint64_t* st = a.status + lo * kStWords;
    if (ok && !(off1 <= total && nb1 <= total - off1 && piece_src(S, off1, held, sub) &&
                held == nb1)) {
      if (tid == 0) chunk_error(st, nest_rank(a, lin1, -1), kFlagRange | kFlagL1);
      ok = false;
    } else if (ok && nb1 < (uint64_t)a.sub_isz) {  // the level-2 decode's index read fails
      if (tid == 0) chunk_error(st, nest_rank(a, lin1, -1), kFlagShort | kFlagL1, (uint32_t)nb1);
      ok = false;
    }
    const uint8_t* ib = ok ? (a.sub_start ? sub : sub + nb1 - a.sub_isz) : nullptr;
    if (ok && a.sub_crc) {  // Crc32cCodec.decode on the sub-shard index (:24-48)
      const int64_t len = a.sub_isz - 4;
      const uint32_t c = block_crc(ib, len, T, red);
      const uint8_t* s = ib + len;
      const uint32_t stored =
          (uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24);
      if (c != stored && tid == 0)
        chunk_error(st, nest_rank(a, lin1, -1), kFlagChunkCrc | kFlagL1, stored, c);
      ok = ok && c == stored;
    }
    uint64_t* flat = reinterpret_cast<uint64_t*>(S.flat);
    for (int64_t k2 = tid; k2 < a.cps2; k2 += kBlock) {
      int64_t q = k2, f = fbase;
#pragma unroll
      for (int d = kMaxDims - 1; d >= 0; --d)
        if (d < n) {
          f += (q % a.r[d]) * a.flat_stride[d];
          q /= a.r[d];
        }
      uint64_t eo = ~0ull, en = ~0ull;
      if (ok) {
        const uint64_t off2 = ld_u64_unaligned(ib + 16 * k2, a.sub_be);
        const uint64_t nb2 = ld_u64_unaligned(ib + 16 * k2 + 8, a.sub_be);
        if (!(off2 == ~0ull || nb2 == ~0ull)) {
          if (!(off2 <= nb1 && nb2 <= nb1 - off2)) {
            chunk_error(st, nest_rank(a, lin1, k2), kFlagRange | kFlagLeaf);
          } else if (nb2 != (uint64_t)a.leaf_nbytes) {
            // with a leaf crc32c the checksum comes first (below)
            if (!a.leaf_crc) chunk_error(st, nest_rank(a, lin1, k2), kFlagLength | kFlagLeaf);
          } else {
            eo = off1 + off2;
            en = nb2;
          }
        }
      }
      flat[2 * f] = eo;
      flat[2 * f + 1] = en;
    }
    if (!ok || !a.leaf_crc) continue;
    // Crc32cCodec.decode (:24-48) of the cell's leaves outside the requested part, and of every
    // leaf whose stored length is wrong: the level-2 decode reads every leaf of the sub-shard
    // (:97-103), the crc32c stage before the bytes codec (so a wrong length fails the checksum
    // unless it happens to match, then the length, Q12).  The data-CRC pass checks the
    // well-formed leaves inside the part.  Uniform over the workgroup (block_crc).
    for (int64_t k2 = 0; k2 < a.cps2; k2++) {
      int64_t q = k2;
      bool inside = true;
#pragma unroll
      for (int d = kMaxDims - 1; d >= 0; --d)
        if (d < n) {
          const int64_t lo_e = ((int64_t)c1[d] * a.r[d] + q % a.r[d]) * a.leaf[d];
          q /= a.r[d];
          inside = inside && lo_e < S.part_hi[d] && lo_e + a.leaf[d] > S.part_lo[d];
        }
      const uint64_t off2 = ld_u64_unaligned(ib + 16 * k2, a.sub_be);
      const uint64_t nb2 = ld_u64_unaligned(ib + 16 * k2 + 8, a.sub_be);
      const bool len_ok = nb2 == (uint64_t)a.leaf_nbytes;
      if ((inside && len_ok) || off2 == ~0ull || nb2 == ~0ull ||
          !(off2 <= nb1 && nb2 <= nb1 - off2))
        continue;  // the data-CRC pass's, missing, or reported above
      const uint32_t rk = nest_rank(a, lin1, k2);
      if (nb2 < 4) {  // no room for the checksum
        if (tid == 0) chunk_error(st, rk, kFlagLength | kFlagLeaf);
        continue;
      }
      const uint8_t* lp = sub + off2;
      const uint32_t c = block_crc(lp, (int64_t)nb2 - 4, T, red);
      const uint8_t* sp = lp + nb2 - 4;
      const uint32_t stored = (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) |
                              ((uint32_t)sp[2] << 16) | ((uint32_t)sp[3] << 24);
      if (c != stored && tid == 0)
        chunk_error(st, rk, kFlagChunkCrc | kFlagLeaf, stored, c);
      else if (!len_ok && tid == 0)
        chunk_error(st, rk, kFlagLength | kFlagLeaf);
    }
  }
}

// Error path of a single-level chain with a chunk crc32c (zh_plan_wait): the chunk of shard
// `shard`, index entry `lin`, was rejected for its length.  The reference's pipeline runs the
// crc32c stage before the bytes codec, so the checksum over its stored bytes decides first:
// out = {1 + (mismatch ? 2 : 0), stored, computed, stored length} (out[0] = 0: under 4 bytes).
// Unsharded chains: the whole chunk object.  One workgroup.
__global__ __launch_bounds__(kBlock) void chunk_crc_detail_kernel(ScatterArgs a, int64_t shard,
                                                                  int64_t lin, uint64_t* out) {
  __shared__ uint32_t T[1][256];
  __shared__ uint32_t red[kBlock];
  const int tid = threadIdx.x;
  {
    uint32_t c = (uint32_t)tid;
#pragma unroll
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
    T[0][tid] = c;
  }
  __syncthreads();
  const DevShard& S = a.shards[shard];
  uint64_t off = 0, nb = (uint64_t)S.nbytes;
  if (a.sharded) index_entry(a, S, lin, off, nb);
  const uint8_t* src = nullptr;
  const uint64_t total = (uint64_t)S.nbytes;
  if (!(off <= total && nb <= total - off) || nb < 4 || !piece_src(S, off, nb, src)) {
    if (tid == 0) {
      out[0] = 0;
      out[3] = nb;
    }
    return;
  }
  const uint32_t c = block_crc(src, (int64_t)nb - 4, T, red);
  if (tid != 0) return;
  const uint8_t* sp = src + nb - 4;
  const uint32_t stored = (uint32_t)sp[0] | ((uint32_t)sp[1] << 8) | ((uint32_t)sp[2] << 16) |
                          ((uint32_t)sp[3] << 24);
  out[0] = 1 | (c != stored ? 2 : 0);
  out[1] = stored;
  out[2] = c;
  out[3] = nb;
}

hipError_t launch_chunk_crc_detail(const ScatterArgs& a, int64_t shard, int64_t lin,
                                   uint64_t* out, hipStream_t stream) {
  hipLaunchKernelGGL(chunk_crc_detail_kernel, dim3(1), dim3(kBlock), 0, stream, a, shard, lin,
                     out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// synthetic data
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <int DS>
__global__ __launch_bounds__(kBlock) void synth_fill_kernel(uint8_t* dst, int64_t n, int64_t first,
                                                             uint64_t seed) {
  using T = typename ElemT<DS>::T;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i * 4 < n; i += stride) {
    const int64_t e0 = i * 4;
    if (e0 + 4 <= n && !(((uintptr_t)(dst + e0 * DS)) & (4 * DS - 1)) && DS == 4) {
      uint4 v;
      v.x = (uint32_t)splitmix64((uint64_t)(first + e0 + 0) ^ seed);
      v.y = (uint32_t)splitmix64((uint64_t)(first + e0 + 1) ^ seed);
      v.z = (uint32_t)splitmix64((uint64_t)(first + e0 + 2) ^ seed);
      v.w = (uint32_t)splitmix64((uint64_t)(first + e0 + 3) ^ seed);
      st16(dst + e0 * DS, v);
    } else {
      for (int k = 0; k < 4 && e0 + k < n; k++)
        st1<DS>(dst + (e0 + k) * DS, (T)splitmix64((uint64_t)(first + e0 + k) ^ seed));
    }
  }
}

struct VerifyArgs {
  const uint8_t* region;
  int32_t ndim;
  int64_t rows;               // prod(shape[0..n-2])
  int64_t rowlen;             // shape[n-1]
  int64_t shape[kMaxDims];
  int64_t offset[kMaxDims];
  int64_t astride[kMaxDims];  // array C-order strides
  uint64_t seed;
  unsigned long long* count;
};

template <int DS>
__global__ __launch_bounds__(kBlock) void synth_verify_kernel(VerifyArgs a) {
  using T = typename ElemT<DS>::T;
  __shared__ unsigned long long wsum[kBlock / 64];
  unsigned long long bad = 0;
  const int n = a.ndim;
  for (int64_t r = blockIdx.x; r < a.rows; r += gridDim.x) {
    // global index of the row start
    int64_t rr = r, g = 0;
    for (int d = n - 2; d >= 0; --d) {
      const int64_t m = rr % a.shape[d];
      rr /= a.shape[d];
      g += (a.offset[d] + m) * a.astride[d];
    }
    g += a.offset[n - 1];
    const uint8_t* row = a.region + r * a.rowlen * DS;
    for (int64_t c = threadIdx.x; c < a.rowlen; c += kBlock) {
      const T want = (T)splitmix64((uint64_t)(g + c) ^ a.seed);
      bad += ld1<DS>(row + c * DS) != want;
    }
  }
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_down(bad, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = bad;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
    for (int w = 0; w < kBlock / 64; w++) s += wsum[w];
    if (s) atomicAdd(a.count, s);
  }
}

// ---------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------
hipError_t launch_nested_index(const NestArgs& a, int grid, hipStream_t stream) {
  if (a.n_l1 <= 0) return hipSuccess;
  hipLaunchKernelGGL(nested_index_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_data_crc_partial(const DataCrcArgs& a, int grid, hipStream_t stream) {
  if (a.n_items <= 0) return hipSuccess;
  hipLaunchKernelGGL(data_crc_partial_kernel, dim3((unsigned)grid), dim3(kBlock), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_data_crc_finalize(const DataCrcArgs& a, hipStream_t stream) {
  if (a.n_items <= 0) return hipSuccess;
  hipLaunchKernelGGL(data_crc_finalize_kernel, dim3((unsigned)((a.n_items + 255) / 256)),
                     dim3(256), 0, stream, a);
  return hipGetLastError();
}

hipError_t launch_data_crc(const DataCrcArgs& a, int grid, hipStream_t stream) {
  hipError_t e = launch_data_crc_partial(a, grid, stream);
  return e == hipSuccess ? launch_data_crc_finalize(a, stream) : e;
}

hipError_t launch_crc(const CrcJob* jobs, int64_t njobs, int64_t nspans, int span_shift,
                      uint32_t* partials, uint64_t* status, hipStream_t stream) {
  if (njobs == 0) return hipSuccess;
  const CrcIdxArgs c{jobs, njobs, nspans, partials, status, span_shift, 0};
  hipLaunchKernelGGL(crc_index_kernel, dim3((unsigned)nspans), dim3(kBlock), 0, stream, c);
  return hipGetLastError();
}

hipError_t launch_resolve(const ScatterArgs& a, hipStream_t stream) {
  if (a.n_citems == 0) return hipSuccess;
  const int grid = (int)std::min<int64_t>((a.n_citems + kBlock - 1) / kBlock, 8192);
  hipLaunchKernelGGL(resolve_kernel, dim3(grid), dim3(kBlock), 0, stream, a);
  return hipGetLastError();
}

template <int DS>
static void launch_scatter_ds(const ScatterArgs& a, int grid, hipStream_t s) {
  // Every decode fast kernel streams non-temporal loads and stores (host: nt & 3 == 3); the
  // host picks the kernel (tile_variant, row_group, crc_fused, tile_align) and checks the LDS
  // layout each one assumes (check_lds_layouts).
  size_t lds = ((size_t)a.fast_n * 8 + 15) & ~(size_t)15;
  if (a.fast_mode == kFastTileTable) {
    if constexpr (DS == 4) {
      const int v = a.tile_variant;
      lds += (size_t)kTG * kTilePitch * 4;
      if (v == 51 && a.crc_fused) {  // the row-CRC tile kernel, one chunk per work item
        if (a.tile_align) {  // LDS: tables 12.5 KiB + 9 slots (the host checked the rest)
          const size_t la = kAlnSlotsAt + (size_t)9 * kTilePitch * 4;
          if (a.swap) hipLaunchKernelGGL((tiles_rowcrc_aln_kernel<true>), dim3(grid), dim3(kBlock), la, s, a);
          else hipLaunchKernelGGL((tiles_rowcrc_aln_kernel<false>), dim3(grid), dim3(kBlock), la, s, a);
          return;
        }
        const size_t lc = lds + 16 * 256 * 4 + (size_t)a.fast_n * 4 + 64;
        if (a.swap) hipLaunchKernelGGL((tiles_rowcrc_kernel<1, true>), dim3(grid), dim3(kBlock), lc, s, a);
        else hipLaunchKernelGGL((tiles_rowcrc_kernel<1, false>), dim3(grid), dim3(kBlock), lc, s, a);
        return;
      }
      if (v == 24 && !a.crc_fused) {  // 4 chunks per work item, next step's loads prefetched
        hipLaunchKernelGGL((tiles_group_kernel<3, 4, false, true, 0>), dim3(grid), dim3(kBlock), lds, s, a);
        return;
      }
      if (a.crc_fused) {
        lds += 16 * 256 * 4 + (size_t)a.fast_n * 4;  // T[8][256] + S, SD[4][256] + K[fast_n]
        hipLaunchKernelGGL((decode_tiles_crc_w3_kernel<3, false>), dim3(grid), dim3(kBlock), lds, s, a);
      } else {
        hipLaunchKernelGGL((decode_tiles_kernel<3>), dim3(grid), dim3(kBlock), lds, s, a);
      }
    }
  } else if (a.fast_mode != kFastNone && a.row_group == 8) {  // host: 128-B rows, no CRC
    hipLaunchKernelGGL((rows_xpose_kernel<DS>), dim3(grid), dim3(kBlock),
                       lds + 4 * 8 * kXRow * 16, s, a);
  } else if (a.fast_mode != kFastNone && a.row_group > 0) {  // host: piece_shift 0
    // with the chunk CRC the payload loads go through the cache (NT = 2): a payload after a
    // 4-byte crc32c sits at 4 mod 16 and the line two wave loads share then hits in L2
    // (c3crc reads 1.085× → 1.0016× algorithmic, profiles/r03/c3crc_summary.json)
    const size_t lc = lds + (a.crc_fused ? 12 * 256 * 4 : 0);
    // host: with the fused chunk CRC G·row = 256 B (G = 1, 2, 4); without it G = 4 for 128-B
    // rows whose row count is not a multiple of 8 (the lane exchange needs that)
    switch (a.row_group * 2 + (a.crc_fused ? 1 : 0)) {
      case 3: hipLaunchKernelGGL((rows_group_kernel<DS, 1, 4, 2, true, false>), dim3(grid), dim3(kBlock), lc, s, a); break;
      case 5: hipLaunchKernelGGL((rows_group_kernel<DS, 2, 4, 2, true, false>), dim3(grid), dim3(kBlock), lc, s, a); break;
      case 8: hipLaunchKernelGGL((rows_group_kernel<DS, 4, 4, 3, false, false>), dim3(grid), dim3(kBlock), lc, s, a); break;
      case 9: hipLaunchKernelGGL((rows_group_kernel<DS, 4, 4, 2, true, false>), dim3(grid), dim3(kBlock), lc, s, a); break;
      default: break;  // no other combination is planned
    }
  } else if (a.fast_mode != kFastNone && a.crc_fused) {
    lds += 12 * 256 * 4;  // slicing tables T[8][256] + zero-shift tables S[4][256]
    hipLaunchKernelGGL((decode_rows_kernel<DS, 4, 3, true>), dim3(grid), dim3(kBlock), lds, s, a);
  } else if (a.fast_mode != kFastNone) {
    hipLaunchKernelGGL((decode_rows_kernel<DS, 4, 3>), dim3(grid), dim3(kBlock), lds, s, a);
  }
}

// tiles_rowcrc_kernel and tiles_rowcrc_aln_kernel address their CRC tables from LDS offset 0:
// true when no instantiation has static LDS (the dynamic block then starts at 0)
bool rowcrc_lds_at_zero() {
  static const bool ok = [] {
    const void* fns[] = {(const void*)tiles_rowcrc_kernel<1, false>, (const void*)tiles_rowcrc_kernel<1, true>,
                         (const void*)tiles_rowcrc_aln_kernel<false>,
                         (const void*)tiles_rowcrc_aln_kernel<true>};
    for (const void* f : fns) {
      hipFuncAttributes at;
      if (hipFuncGetAttributes(&at, f) != hipSuccess || at.sharedSizeBytes != 0) return false;
    }
    return true;
  }();
  return ok;
}

// the fast-path selection of the last decode scatter launch (diagnostic: zh_debug_last_fast_path)
std::atomic<int64_t> g_last_fast_path{-1};
// the encode view's fast-path selection of the last write: fast_mode·10⁶ + group·10³
std::atomic<int64_t> g_last_encode_path{-1};

hipError_t launch_scatter(const ScatterArgs& a, int dsize, int grid, hipStream_t stream) {
  if (a.total_items == 0) return hipSuccess;
  g_last_fast_path.store((int64_t)a.tile_align * 1000000000 + (int64_t)a.fast_mode * 1000000 +
                         (int64_t)a.tile_variant * 1000 +
                         (int64_t)(a.row_group & 0xFF) * 4 + (a.piece_shift ? 1 : 0));
  switch (dsize) {
    case 1: launch_scatter_ds<1>(a, grid, stream); break;
    case 2: launch_scatter_ds<2>(a, grid, stream); break;
    case 4: launch_scatter_ds<4>(a, grid, stream); break;
    case 8: launch_scatter_ds<8>(a, grid, stream); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int DS>
static void launch_slow_ds(const ScatterArgs& a, int grid, const CrcIdxArgs& c, hipStream_t s) {
  if (a.tile)
    hipLaunchKernelGGL((decode_slow_kernel<DS, true>), dim3(grid), dim3(kBlock), 0, s, a, c);
  else
    hipLaunchKernelGGL((decode_slow_kernel<DS, false>), dim3(grid), dim3(kBlock), 0, s, a, c);
}

template <int DS>
static void launch_small_ds(const ScatterArgs& a, int grid, const CrcIdxArgs& c, hipStream_t s) {
  if (a.tile)
    hipLaunchKernelGGL((decode_small_kernel<DS, true>), dim3(grid), dim3(kBlock), 0, s, a, c);
  else
    hipLaunchKernelGGL((decode_small_kernel<DS, false>), dim3(grid), dim3(kBlock), 0, s, a, c);
}

hipError_t launch_decode_small(const ScatterArgs& a, int grid, const CrcIdxArgs& crc,
                               hipStream_t stream) {
  g_last_fast_path.store(-1);  // zh_debug_last_fast_path: the one-launch small decode
  const CrcIdxArgs c = crc.njobs > 0 ? crc : CrcIdxArgs{};
  grid = std::max(grid, 1) + (int)c.nspans;
  switch (a.dsize) {
    case 1: launch_small_ds<1>(a, grid, c, stream); break;
    case 2: launch_small_ds<2>(a, grid, c, stream); break;
    case 4: launch_small_ds<4>(a, grid, c, stream); break;
    case 8: launch_small_ds<8>(a, grid, c, stream); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_decode_slow(const ScatterArgs& a, int grid, const CrcIdxArgs& crc,
                              hipStream_t stream) {
  const CrcIdxArgs c = crc.njobs > 0 ? crc : CrcIdxArgs{};
  grid = std::max(grid, 1) + (int)c.nspans;
  switch (a.dsize) {
    case 1: launch_slow_ds<1>(a, grid, c, stream); break;
    case 2: launch_slow_ds<2>(a, grid, c, stream); break;
    case 4: launch_slow_ds<4>(a, grid, c, stream); break;
    case 8: launch_slow_ds<8>(a, grid, c, stream); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// the encode view through the fast kernels (FLAGS).  Returns false when a grouped launch
// (group > 0) found no kernel for its combination: the host set the visit order and grid over
// groups, so no ungrouped kernel may run instead.  Region loads and payload stores stream
// non-temporally, except the grouped row encode with the chunk CRC, which stores its payloads
// through the cache: a payload after a 4-byte crc32c sits at 4 mod 16, and L2 merges the line two
// stores share (c3crc write 41.04 → 39.77 ms, writes 1.079× → 1.007×; the tile encode measured
// 43.28 → 43.66 ms that way and keeps non-temporal stores).
// The chunk-CRC tile encode (c4crc write) stores its payloads non-temporally too.  Its
// payloads after each 4-byte crc32c sit at 4 mod 16 and split 32-B sectors (writes 1.059× the
// payload); round 6 measured the alternatives on the GPU and removed them (DESIGN §4 "The
// chunk-CRC encode", profiles/r06/{enc,aln,occ}/; the code is in git history, commit 7ab15c4):
// stores through the cache (writes 1.089×, 42.6 vs 41.8 ms), sector-aligned stores (writes
// 1.024×, 47.7 ms), 2 workgroups per CU (47.8 vs 42.2 ms at 3) and two sub-groups per workgroup
// sharing one table set (48.2–49.9 vs 41.7 ms).

template <int DS>
static bool launch_encode_fast_ds(const ScatterArgs& v, int grid, int group, hipStream_t s) {
  const size_t lds = ((size_t)v.fast_n * 8 + 15) & ~(size_t)15;
  if (v.fast_mode != kFastTileTable) {
    if (group > 0 && v.crc_fused) {  // host: rows sequential in the payload, whole chunks
      const size_t lc = lds + 12 * 256 * 4;  // + slicing tables T[8][256], shift table S[4][256]
      switch (group) {
        case 1: hipLaunchKernelGGL((rows_group_kernel<DS, 1, 4, 1, true, true>), dim3(grid), dim3(kBlock), lc, s, v); return true;
        case 2: hipLaunchKernelGGL((rows_group_kernel<DS, 2, 4, 1, true, true>), dim3(grid), dim3(kBlock), lc, s, v); return true;
        case 4: hipLaunchKernelGGL((rows_group_kernel<DS, 4, 4, 1, true, true>), dim3(grid), dim3(kBlock), lc, s, v); return true;
        default: return false;
      }
    }
    if (group > 0) {  // host: G·vpr ≤ 64 lanes, piece_shift == 0, v.item_mul over groups
      switch (group) {
        case 1: hipLaunchKernelGGL((rows_group_kernel<DS, 1, 4, 3, false, true>), dim3(grid), dim3(kBlock), lds, s, v); return true;
        case 2: hipLaunchKernelGGL((rows_group_kernel<DS, 2, 4, 3, false, true>), dim3(grid), dim3(kBlock), lds, s, v); return true;
        case 4: hipLaunchKernelGGL((rows_group_kernel<DS, 4, 4, 3, false, true>), dim3(grid), dim3(kBlock), lds, s, v); return true;
        case 8: hipLaunchKernelGGL((rows_group_kernel<DS, 8, 4, 3, false, true>), dim3(grid), dim3(kBlock), lds, s, v); return true;
        default: return false;
      }
    }
    if (v.crc_fused) {  // chunk crc32c of the stored payload, fused (rows sequential in the payload)
      hipLaunchKernelGGL((decode_rows_kernel<DS, 4, 3, true, true>), dim3(grid), dim3(kBlock),
                         lds + 12 * 256 * 4, s, v);
      return true;
    }
    // uint32 rows: 8 rows in flight per lane (+2.4 % on c3, profiles/r01/experiments/)
    if constexpr (DS == 4)
      hipLaunchKernelGGL((decode_rows_kernel<DS, 8, 3, false, true>), dim3(grid), dim3(kBlock), lds, s, v);
    else
      hipLaunchKernelGGL((decode_rows_kernel<DS, 4, 3, false, true>), dim3(grid), dim3(kBlock), lds, s, v);
    return true;
  }
  if constexpr (DS == 4) {
    const size_t l = lds + (size_t)kTG * kTilePitch * 4;
    if (group > 0 && v.crc_fused) {  // host: crc_tile_step for 8/G units
      const size_t lc = l + 16 * 256 * 4 + (size_t)v.fast_n * 4 + 64;  // + alignment
      const bool m = v.fill_mask != ~0ull;  // a float ±0 fill: the masked all-fill test
      if (group != 2) return false;  // host: 2 chunks per work item
      if (m)
        hipLaunchKernelGGL((tiles_group_kernel<3, 2, true, false, 2>), dim3(grid), dim3(kBlock), lc, s, v);
      else
        hipLaunchKernelGGL((tiles_group_kernel<3, 2, true, false, 1>), dim3(grid), dim3(kBlock), lc, s, v);
      return true;
    }
    if (group > 0) {  // host: piece_shift == 0, item_mul
      if (group != 2) return false;  // host: 2 chunks per work item
      hipLaunchKernelGGL((tiles_group_kernel<3, 2, false, false, 2>), dim3(grid), dim3(kBlock), l, s, v);
      return true;
    }
    if (v.crc_fused)  // chunk crc32c of the stored payload: tables + per-unit shifts
      hipLaunchKernelGGL((decode_tiles_crc_w3_kernel<3, true>), dim3(grid), dim3(kBlock),
                         l + 16 * 256 * 4 + (size_t)v.fast_n * 4, s, v);
    else
      hipLaunchKernelGGL((decode_tiles_kernel<3, false, true>), dim3(grid), dim3(kBlock), l, s, v);
    return true;
  }
  return group == 0;
}

hipError_t launch_encode_fast(const ScatterArgs& view, int grid, int group, hipStream_t stream) {
  if (view.total_items == 0 || view.fast_mode == kFastNone) return hipSuccess;
  g_last_encode_path.store((int64_t)view.fast_mode * 1000000 + (int64_t)group * 1000);
  bool ok = false;
  switch (view.dsize) {
    case 1: ok = launch_encode_fast_ds<1>(view, grid, group, stream); break;
    case 2: ok = launch_encode_fast_ds<2>(view, grid, group, stream); break;
    case 4: ok = launch_encode_fast_ds<4>(view, grid, group, stream); break;
    case 8: ok = launch_encode_fast_ds<8>(view, grid, group, stream); break;
    default: return hipErrorInvalidValue;
  }
  if (!ok) return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_encode_resolve(const ScatterArgs& a, const EncNest& nz, int64_t* item_off,
                                 int64_t base_off, int64_t cn, const uint8_t* vbase, int vfast,
                                 hipStream_t stream) {
  if (a.n_citems == 0) return hipSuccess;
  const int grid = (int)std::min<int64_t>((a.n_citems + kBlock - 1) / kBlock, 8192);
  hipLaunchKernelGGL(encode_resolve_kernel, dim3(grid), dim3(kBlock), 0, stream, a, nz, item_off,
                     base_off, cn, vbase, vfast);
  return hipGetLastError();
}

template <int DS>
static void launch_encode_slow_ds(const ScatterArgs& a, int grid, hipStream_t s) {
  if (a.tile)
    hipLaunchKernelGGL((encode_slow_kernel<DS, true>), dim3(grid), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((encode_slow_kernel<DS, false>), dim3(grid), dim3(kBlock), 0, s, a);
}

hipError_t launch_encode_slow(const ScatterArgs& a, int grid, hipStream_t stream) {
  switch (a.dsize) {
    case 1: launch_encode_slow_ds<1>(a, grid, stream); break;
    case 2: launch_encode_slow_ds<2>(a, grid, stream); break;
    case 4: launch_encode_slow_ds<4>(a, grid, stream); break;
    case 8: launch_encode_slow_ds<8>(a, grid, stream); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_encode_finish(const ScatterArgs& a, const EncNest& nz, int64_t chunk_nbytes,
                                uint32_t* bad, ItemDesc* crc_desc, hipStream_t stream) {
  if (a.n_citems == 0) return hipSuccess;
  const int grid = (int)std::min<int64_t>((a.n_citems + kBlock - 1) / kBlock, 8192);
  hipLaunchKernelGGL(encode_finish_kernel, dim3(grid), dim3(kBlock), 0, stream, a, nz,
                     chunk_nbytes, bad, crc_desc);
  return hipGetLastError();
}

// dst block b ← src block idx[b] (blocks of bb bytes, bb % 16 == 0, 16-B aligned): one
// workgroup per block, 16-B vectors (bench / tests: shards re-laid out in another order)
__global__ __launch_bounds__(kBlock) void gather_blocks_kernel(uint8_t* dst, const uint8_t* src,
                                                               const int64_t* idx, int64_t n,
                                                               int64_t bb) {
  for (int64_t b = blockIdx.x; b < n; b += gridDim.x) {
    const uint4* s = reinterpret_cast<const uint4*>(src + idx[b] * bb);
    uint4* d = reinterpret_cast<uint4*>(dst + b * bb);
    for (int64_t v = threadIdx.x; v < bb / 16; v += kBlock) d[v] = s[v];
  }
}

hipError_t launch_gather_blocks(void* dst, const void* src, const int64_t* d_idx, int64_t n,
                                int64_t bb, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  const int grid = (int)std::min<int64_t>(n, 65536);
  hipLaunchKernelGGL(gather_blocks_kernel, dim3(grid), dim3(kBlock), 0, stream, (uint8_t*)dst,
                     (const uint8_t*)src, d_idx, n, bb);
  return hipGetLastError();
}

// Write-bandwidth probe of a large output buffer (allocation calibration, DESIGN §4
// "Placement"): non-temporal 16-B stores, no loads.
//   pattern 0: contiguous, 4 KiB per workgroup step
//   pattern 1: the decode kernels' store pattern: a work item is 1024 lines of 128 B, 6 KiB
//              apart (one 32x32x32 uint32 chunk of a region with 1536-element rows); a wave
//              stores 8 lines per instruction
__global__ __launch_bounds__(kBlock) void write_probe_kernel(uint8_t* __restrict__ dst,
                                                              int64_t bytes, int pattern) {
  const uint4 v = make_uint4(0x5A5A5A5Au, 0xA5A5A5A5u, 0x0F0F0F0Fu, 0xF0F0F0F0u);
  if (pattern == 0) {
    const int64_t nv = bytes >> 4;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nv;
         i += (int64_t)gridDim.x * kBlock)
      st16s<true>(dst + (i << 4), v);
    return;
  }
  constexpr int64_t kLine = 128, kPitch = 6144, kLines = 1024;
  constexpr int64_t kGroup = kPitch * kLines;           // 48 items share 6 MiB
  const int64_t items = bytes / kGroup * (kPitch / kLine);
  const int t = threadIdx.x, c = t & 7, r0 = t >> 3;    // 16-B column, line within step
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
    uint8_t* base = dst + (it / (kPitch / kLine)) * kGroup + (it % (kPitch / kLine)) * kLine;
    for (int64_t l = r0; l < kLines; l += kBlock / 8) st16s<true>(base + l * kPitch + c * 16, v);
  }
}

hipError_t launch_write_probe(void* dst, int64_t bytes, int pattern, hipStream_t stream) {
  if (bytes <= 0) return hipSuccess;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = cus * 32;
  hipLaunchKernelGGL(write_probe_kernel, dim3(grid), dim3(kBlock), 0, stream, (uint8_t*)dst,
                     bytes, pattern);
  return hipGetLastError();
}

// Copy ceiling of a (source, destination) pair (bench evidence, DESIGN §4 "Ceilings"): the
// fastest plain stream measured in tools/copy_lab.hip — a 32-bit byte-swapping copy, each
// workgroup owning 128 KiB spans, 4 non-temporal 16-B loads in flight per lane, then their
// non-temporal stores.  Same bytes moved per output byte as the decode (one read, one write).
__global__ __launch_bounds__(kBlock) void copy_probe_kernel(const uint8_t* __restrict__ src,
                                                             uint8_t* __restrict__ dst,
                                                             int64_t bytes) {
  constexpr int64_t kSpan = 128 << 10, kU = 4;
  const int64_t spans = bytes / kSpan;
  for (int64_t sp = blockIdx.x; sp < spans; sp += gridDim.x) {
    const uint8_t* s = src + sp * kSpan;
    uint8_t* d = dst + sp * kSpan;
    for (int64_t i = threadIdx.x * 16; i < kSpan; i += kBlock * 16 * kU) {
      uint4 v[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) v[u] = ld16s<true>(s + i + u * kBlock * 16);
#pragma unroll
      for (int u = 0; u < kU; u++)
        st16s<true>(d + i + u * kBlock * 16,
                    make_uint4(__builtin_bswap32(v[u].x), __builtin_bswap32(v[u].y),
                               __builtin_bswap32(v[u].z), __builtin_bswap32(v[u].w)));
    }
  }
}

hipError_t launch_copy_probe(void* dst, const void* src, int64_t bytes, hipStream_t stream) {
  bytes = bytes / (128 << 10) * (128 << 10);
  if (bytes <= 0) return hipSuccess;
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = (int)std::min<int64_t>(bytes / (128 << 10), (int64_t)cus * 32);
  hipLaunchKernelGGL(copy_probe_kernel, dim3(grid), dim3(kBlock), 0, stream,
                     (const uint8_t*)src, (uint8_t*)dst, bytes);
  return hipGetLastError();
}

hipError_t launch_synth_fill(void* dst, int64_t n, int dsize, int64_t first, uint64_t seed,
                             hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int64_t vecs = (n + 3) / 4;
  int grid = (int)std::min<int64_t>((vecs + kBlock - 1) / kBlock, 65536);
  uint8_t* p = (uint8_t*)dst;
  switch (dsize) {
    case 1: hipLaunchKernelGGL(synth_fill_kernel<1>, dim3(grid), dim3(kBlock), 0, stream, p, n, first, seed); break;
    case 2: hipLaunchKernelGGL(synth_fill_kernel<2>, dim3(grid), dim3(kBlock), 0, stream, p, n, first, seed); break;
    case 4: hipLaunchKernelGGL(synth_fill_kernel<4>, dim3(grid), dim3(kBlock), 0, stream, p, n, first, seed); break;
    case 8: hipLaunchKernelGGL(synth_fill_kernel<8>, dim3(grid), dim3(kBlock), 0, stream, p, n, first, seed); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_synth_verify(const void* region, int ndim, const int64_t* array_shape,
                               const int64_t* offset, const int64_t* shape, int dsize,
                               uint64_t seed, unsigned long long* d_count, hipStream_t stream) {
  VerifyArgs a;
  a.region = (const uint8_t*)region;
  a.ndim = ndim;
  a.seed = seed;
  a.count = d_count;
  int64_t st = 1;
  for (int d = ndim - 1; d >= 0; --d) {
    a.astride[d] = st;
    st *= array_shape[d];
    a.shape[d] = shape[d];
    a.offset[d] = offset[d];
  }
  a.rows = 1;
  for (int d = 0; d < ndim - 1; d++) a.rows *= shape[d];
  a.rowlen = shape[ndim - 1];
  if (a.rows <= 0 || a.rowlen <= 0) return hipSuccess;
  int grid = (int)std::min<int64_t>(a.rows, 65536);
  switch (dsize) {
    case 1: hipLaunchKernelGGL(synth_verify_kernel<1>, dim3(grid), dim3(kBlock), 0, stream, a); break;
    case 2: hipLaunchKernelGGL(synth_verify_kernel<2>, dim3(grid), dim3(kBlock), 0, stream, a); break;
    case 4: hipLaunchKernelGGL(synth_verify_kernel<4>, dim3(grid), dim3(kBlock), 0, stream, a); break;
    case 8: hipLaunchKernelGGL(synth_verify_kernel<8>, dim3(grid), dim3(kBlock), 0, stream, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace zh
