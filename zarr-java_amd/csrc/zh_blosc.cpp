// zh_blosc.cpp — host decompression of blosc1 frames (the `blosc` codec of v3 and v2
// arrays, M/v3/codec/core/BloscCodec.java / M/v2/codec/core/BloscCodec.java, which call the
// blosc-java JNI library).  Compressors stay on the host (north star); this restates the
// blosc1 frame and its BloscLZ / LZ4 / zlib payloads so that the raw chunk bytes can be
// handed to the device, without the blosc library (absent from this image).
//
// Frame (16-byte header, little-endian): version, versionlz, flags, typesize, nbytes,
// blocksize, cbytes; then one int32 start offset per block.  flags: 0x01 byte shuffle,
// 0x02 memcpyed (raw bytes follow the header), 0x04 bit shuffle, 0x10 blocks not split into
// typesize streams, bits 5-7 compressor (0 BloscLZ, 1 LZ4/LZ4HC, 3 zlib, 4 zstd through
// zh_zstd.cpp; 2 snappy is not available).  A split block is typesize streams of blocksize/typesize bytes; each stream is
// int32 csize + payload (csize == stream size: stored raw).  The last (short) block is never
// split.  Pinned by the reference's v2_sample fixtures (BloscLZ split + shuffle, LZ4
// unsplit + shuffle, memcpyed), tests/test_blosc.py.
#include <zlib.h>

#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/zarrhip.h"

namespace {

void set_err(char* err, size_t errlen, const char* msg) {
  if (err && errlen) {
    strncpy(err, msg, errlen - 1);
    err[errlen - 1] = 0;
  }
}

uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// LZ4 block format: token (literal length << 4 | match length - 4), 255-continued lengths,
// literals, 16-bit LE offset, overlapping match copy.  Returns bytes written or -1.
int64_t lz4_block(const uint8_t* s, size_t n, uint8_t* d, size_t cap) {
  size_t i = 0, o = 0;
  while (i < n) {
    const uint8_t tok = s[i++];
    size_t lit = tok >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (i >= n) return -1;
        b = s[i++];
        lit += b;
      } while (b == 255);
    }
    if (lit > n - i || lit > cap - o) return -1;
    memcpy(d + o, s + i, lit);
    i += lit;
    o += lit;
    if (i >= n) break;  // the last sequence has literals only
    if (n - i < 2) return -1;
    const size_t off = (size_t)s[i] | ((size_t)s[i + 1] << 8);
    i += 2;
    size_t ml = tok & 15;
    if (ml == 15) {
      uint8_t b;
      do {
        if (i >= n) return -1;
        b = s[i++];
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (off == 0 || off > o || ml > cap - o) return -1;
    for (size_t k = 0; k < ml; k++, o++) d[o] = d[o - off];
  }
  return (int64_t)o;
}

// BloscLZ (FastLZ-derived): ctrl < 32 → ctrl+1 literals; else match of (ctrl >> 5) + 2
// bytes (7 → 255-continued), distance ((ctrl & 31) << 8) + next byte + 1, with the 16-bit
// far form (+8191) when that byte is 255 and the high part is 31.
int64_t blosclz_block(const uint8_t* s, size_t n, uint8_t* d, size_t cap) {
  constexpr size_t kMaxDistance = 8191;
  if (n == 0) return 0;
  size_t ip = 0, o = 0;
  uint32_t ctrl = s[ip++] & 31u;
  for (;;) {
    if (ctrl >= 32) {
      size_t len = (ctrl >> 5) - 1;
      size_t dist = (size_t)(ctrl & 31) << 8;
      if (len == 6) {
        uint8_t c;
        do {
          if (ip >= n) return -1;
          c = s[ip++];
          len += c;
        } while (c == 255);
      }
      if (ip >= n) return -1;
      const uint8_t code = s[ip++];
      if (code == 255 && dist == (31u << 8)) {
        if (n - ip < 2) return -1;
        dist = (((size_t)s[ip] << 8) | s[ip + 1]) + kMaxDistance;
        ip += 2;
      } else {
        dist += code;
      }
      len += 3;
      if (dist + 1 > o || len > cap - o) return -1;
      for (size_t k = 0; k < len; k++, o++) d[o] = d[o - dist - 1];
    } else {
      const size_t lit = ctrl + 1;
      if (lit > n - ip || lit > cap - o) return -1;
      memcpy(d + o, s + ip, lit);
      ip += lit;
      o += lit;
    }
    if (ip >= n) break;
    ctrl = s[ip++];
  }
  return (int64_t)o;
}

int64_t zlib_block(const uint8_t* s, size_t n, uint8_t* d, size_t cap) {
  uLongf dl = (uLongf)cap;
  if (uncompress(d, &dl, s, (uLong)n) != Z_OK) return -1;
  return (int64_t)dl;
}

int64_t zstd_block(const uint8_t* s, size_t n, uint8_t* d, size_t cap) {
  size_t got = 0;
  if (zh_zstd_decompress(s, n, nullptr, 0, &got, nullptr, 0) != ZH_OK || got != cap) return -1;
  if (zh_zstd_decompress(s, n, d, cap, &got, nullptr, 0) != ZH_OK) return -1;
  return (int64_t)got;
}

// Bit unshuffle of ne elements (ne % 8 == 0) of ts bytes: the shuffled block holds, for
// each byte position j and bit k, a row of ne/8 bytes whose bit m of byte q is bit k of byte
// j of element 8q+m (bitshuffle's bshuf_trans_bit_elem layout, which blosc's bitshuffle()
// applies per block).
void bit_unshuffle(const uint8_t* in, uint8_t* out, size_t ne, size_t ts) {
  const size_t rowb = ne / 8;
  memset(out, 0, ne * ts);
  for (size_t j = 0; j < ts; j++)
    for (size_t k = 0; k < 8; k++) {
      const uint8_t* row = in + (j * 8 + k) * rowb;
      for (size_t q = 0; q < rowb; q++) {
        const uint8_t b = row[q];
        if (!b) continue;
        for (size_t m = 0; m < 8; m++)
          out[(8 * q + m) * ts + j] |= (uint8_t)(((b >> m) & 1) << k);
      }
    }
}

}  // namespace

extern "C" {

int zh_blosc_decompress(const void* src_v, size_t srclen, void* dst_v, size_t dstcap,
                        size_t* nbytes_out, char* err, size_t errlen) {
  const uint8_t* src = (const uint8_t*)src_v;
  uint8_t* dst = (uint8_t*)dst_v;
  if (!src || srclen < 16) {
    set_err(err, errlen, "blosc frame shorter than its 16-byte header");
    return ZH_EDATA;
  }
  const uint8_t flags = src[2], ts = src[3];
  const size_t nbytes = rd32(src + 4), bsize = rd32(src + 8), cbytes = rd32(src + 12);
  // The header is validated before the size query answers: callers allocate nbytes, and a
  // corrupt frame must not make them allocate gigabytes first.
  if (cbytes > srclen) {
    set_err(err, errlen, "blosc frame truncated");
    return ZH_EDATA;
  }
  const bool memcpyed = (flags & 0x02) != 0;
  if (memcpyed && 16 + nbytes > srclen) {
    set_err(err, errlen, "blosc frame truncated");
    return ZH_EDATA;
  }
  size_t nblocks = 0;
  if (!memcpyed && nbytes > 0) {
    // no codec here expands a stream by more than ~1032x (deflate), so a larger nbytes is a
    // corrupt header
    if (bsize == 0 || ts == 0 || nbytes > 2048 * (size_t)cbytes + 65536) {
      set_err(err, errlen, "corrupt blosc header");
      return ZH_EDATA;
    }
    nblocks = (nbytes + bsize - 1) / bsize;
    if (16 + 4 * nblocks > srclen) {
      set_err(err, errlen, "blosc frame truncated");
      return ZH_EDATA;
    }
  }
  if (nbytes_out) *nbytes_out = nbytes;
  if (!dst) return ZH_OK;  // size query
  if (nbytes > dstcap) {
    set_err(err, errlen, "blosc destination too small");
    return ZH_EINVAL;
  }
  if (memcpyed) {
    memcpy(dst, src + 16, nbytes);
    return ZH_OK;
  }
  const bool bitshuf = (flags & 0x04) && !(flags & 0x01);
  const int comp = flags >> 5;
  if (comp != 0 && comp != 1 && comp != 3 && comp != 4) {
    set_err(err, errlen, "blosc compressor (snappy) not available on this host");
    return ZH_EUNSUPPORTED;
  }
  if (nbytes == 0) return ZH_OK;
  std::vector<uint8_t> tmp(std::min(bsize, nbytes));  // one (shuffled) block
  for (size_t k = 0; k < nblocks; k++) {
    const size_t bs = k + 1 < nblocks ? bsize : nbytes - k * bsize;
    const bool leftover = bs < bsize;
    const size_t nsplit = ((flags & 0x10) || leftover) ? 1 : ts;
    const size_t neb = bs / nsplit;
    if (nsplit > 1 && bs % nsplit != 0) {  // split streams must tile the block exactly
      set_err(err, errlen, "blosc frame header corrupt (block not a multiple of the typesize)");
      return ZH_EDATA;
    }
    size_t p = rd32(src + 16 + 4 * k);
    uint8_t* blk = ((flags & 0x01) && ts > 1) || bitshuf ? tmp.data() : dst + k * bsize;
    for (size_t sidx = 0; sidx < nsplit; sidx++) {
      if (p + 4 > srclen) {
        set_err(err, errlen, "blosc frame truncated");
        return ZH_EDATA;
      }
      const size_t cs = rd32(src + p);
      p += 4;
      if (cs > srclen - p) {
        set_err(err, errlen, "blosc frame truncated");
        return ZH_EDATA;
      }
      uint8_t* out = blk + sidx * neb;
      int64_t got;
      if (cs == neb) {
        memcpy(out, src + p, neb);
        got = (int64_t)neb;
      } else if (comp == 0) {
        got = blosclz_block(src + p, cs, out, neb);
      } else if (comp == 1) {
        got = lz4_block(src + p, cs, out, neb);
      } else if (comp == 3) {
        got = zlib_block(src + p, cs, out, neb);
      } else {
        got = zstd_block(src + p, cs, out, neb);
      }
      if (got != (int64_t)neb) {
        set_err(err, errlen, "corrupt blosc block");
        return ZH_EDATA;
      }
      p += cs;
    }
    if (bitshuf) {
      // c-blosc 1.x (frame version <= 2): whole block bit-shuffled when its element count is
      // a multiple of 8, else stored as is; later formats shuffle the multiple-of-8 prefix and
      // keep the leftover bytes
      uint8_t* d = dst + k * bsize;
      size_t ne = ts ? bs / ts : 0;
      if (src[0] <= 2 && ne % 8 != 0) ne = 0;
      ne -= ne % 8;
      if (ne) bit_unshuffle(tmp.data(), d, ne, ts);
      memcpy(d + ne * ts, tmp.data() + ne * ts, bs - ne * ts);
    } else if (blk == tmp.data()) {  // byte unshuffle: stream j holds byte j of every element
      uint8_t* d = dst + k * bsize;
      const size_t ne = bs / ts;
      for (size_t e = 0; e < ne; e++)
        for (size_t j = 0; j < ts; j++) d[e * ts + j] = tmp[j * ne + e];
      memcpy(d + ne * ts, tmp.data() + ne * ts, bs - ne * ts);
    }
  }
  return ZH_OK;
}

}  // extern "C"
