// zh_zstd.cpp — Zstandard frame decoder (RFC 8878), host side, written from the format
// specification.  It backs the host decompression hand-off of the device pipeline (SURVEY §8(f)
// rank 3): ZstdCodec.decode (M/core/codec/core/ZstdCodec.java:14-22, zstd-jni 1.5.x in the
// reference) and blosc frames whose compressor is zstd (BloscCodec.java; withBlosc() defaults
// to cname "zstd", M/v3/codec/CodecBuilder.java:58-60).  The decoded bytes then go to the
// device `bytes` / transpose / scatter stages.
//
// Covered: zstd frames (single or concatenated) and skippable frames; raw, RLE and compressed
// blocks; raw / RLE / Huffman-compressed / treeless literals with 1 or 4 streams; Huffman trees
// with direct or FSE-compressed weights; sequences with predefined / RLE / FSE / repeat tables;
// repeat offsets; the optional XXH64 content checksum.  Dictionaries are not (zarr's zstd codec
// has none): a frame naming one is rejected as unsupported.  The encoder side writes valid
// frames of raw blocks (content size and, if asked, the checksum), which every zstd decoder
// reads; it does not compress.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/zarrhip.h"

namespace {

void set_err(char* err, size_t errlen, const char* msg) {
  if (err && errlen) snprintf(err, errlen, "%s", msg);
}

constexpr uint32_t kMagic = 0xFD2FB528u;
constexpr int kMaxHufBits = 11;

struct Fail {
  int status;
  const char* msg;
};

[[noreturn]] void fail(const char* msg, int status = ZH_EDATA) { throw Fail{status, msg}; }

int highbit(uint64_t v) {  // index of the highest set bit (v > 0)
  int r = 0;
  while (v >>= 1) r++;
  return r;
}

uint64_t rd_le(const uint8_t* p, int n) {
  uint64_t v = 0;
  for (int i = n - 1; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}

// ---- XXH64 (content checksum: low 32 bits of XXH64(content, seed 0)) -----------------
constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull,
                   P3 = 1609587929392839161ull, P4 = 9650029242287828579ull,
                   P5 = 2870177450012600261ull;
inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t xround(uint64_t acc, uint64_t in) {
  acc += in * P2;
  acc = rotl(acc, 31);
  return acc * P1;
}
inline uint64_t xmerge(uint64_t acc, uint64_t v) {
  acc ^= xround(0, v);
  return acc * P1 + P4;
}

}  // namespace

extern "C" uint64_t zh_xxh64(const void* data, size_t len, uint64_t seed) {
  const uint8_t* p = (const uint8_t*)data;
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* lim = end - 32;
    do {
      v1 = xround(v1, rd_le(p, 8));
      v2 = xround(v2, rd_le(p + 8, 8));
      v3 = xround(v3, rd_le(p + 16, 8));
      v4 = xround(v4, rd_le(p + 24, 8));
      p += 32;
    } while (p <= lim);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = xmerge(h, v1);
    h = xmerge(h, v2);
    h = xmerge(h, v3);
    h = xmerge(h, v4);
  } else {
    h = seed + P5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    h ^= xround(0, rd_le(p, 8));
    h = rotl(h, 27) * P1 + P4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= rd_le(p, 4) * P1;
    h = rotl(h, 23) * P2 + P3;
    p += 4;
  }
  while (p < end) {
    h ^= (*p++) * P5;
    h = rotl(h, 11) * P1;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

namespace {

// ---- bit streams ----------------------------------------------------------------------
// Forward, LSB-first (FSE table descriptions).
struct FwdBits {
  const uint8_t* p;
  size_t len;
  size_t bit = 0;  // absolute bit position
  uint32_t read(int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; i++, bit++) {
      if (bit / 8 >= len) fail("zstd: table description overruns its section");
      v |= (uint32_t)((p[bit / 8] >> (bit % 8)) & 1) << i;
    }
    return v;
  }
  void rewind(int n) { bit -= n; }
  size_t bytes_used() const { return (bit + 7) / 8; }
};

// Backward (FSE / Huffman payloads): read from the end; the last byte's highest set bit is
// the end marker.  Reading past the start yields zero bits (offset goes negative).
struct BackBits {
  const uint8_t* p;
  int64_t off;  // bits left above position 0
  BackBits(const uint8_t* src, size_t len) : p(src) {
    if (len == 0) fail("zstd: empty bitstream");
    const uint8_t last = src[len - 1];
    if (last == 0) fail("zstd: bitstream without its end marker");
    off = (int64_t)len * 8 - (8 - highbit(last));
  }
  uint64_t read(int n) {
    if (n == 0) return 0;
    off -= n;
    int64_t o = off;
    int nb = n;
    if (o < 0) {
      nb += (int)o;
      o = 0;
    }
    uint64_t v = 0;
    for (int i = 0; i < nb; i++) {
      const int64_t b = o + i;
      v |= (uint64_t)((p[b >> 3] >> (b & 7)) & 1) << i;
    }
    if (off < 0) v = -off >= 64 ? 0 : v << (-off);
    return v;
  }
};

// ---- FSE ---------------------------------------------------------------------------------
struct Fse {
  int log = -1;  // -1: no table yet
  std::vector<uint8_t> sym, nbits;
  std::vector<uint16_t> base;

  void build(const int16_t* norm, int nsym, int acc) {
    const int size = 1 << acc;
    log = acc;
    sym.assign(size, 0);
    nbits.assign(size, 0);
    base.assign(size, 0);
    std::vector<uint16_t> next(nsym > 0 ? nsym : 1, 0);
    int high = size;
    for (int s = 0; s < nsym; s++)
      if (norm[s] == -1) {
        sym[--high] = (uint8_t)s;
        next[s] = 1;
      }
    const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    int pos = 0;
    for (int s = 0; s < nsym; s++) {
      if (norm[s] <= 0) continue;
      next[s] = (uint16_t)norm[s];
      for (int i = 0; i < norm[s]; i++) {
        sym[pos] = (uint8_t)s;
        do pos = (pos + step) & mask;
        while (pos >= high);
      }
    }
    if (pos != 0) fail("zstd: FSE table spread does not close");
    for (int i = 0; i < size; i++) {
      const uint16_t d = next[sym[i]]++;
      nbits[i] = (uint8_t)(acc - highbit(d));
      base[i] = (uint16_t)(((uint32_t)d << nbits[i]) - size);
    }
  }
  void rle(uint8_t s) {
    log = 0;
    sym.assign(1, s);
    nbits.assign(1, 0);
    base.assign(1, 0);
  }
  // Reads a table description; returns the bytes it used.
  size_t read_header(const uint8_t* src, size_t len, int max_log, int max_sym) {
    FwdBits in{src, len};
    const int acc = 5 + (int)in.read(4);
    if (acc > max_log) fail("zstd: FSE accuracy log too large");
    int remaining = 1 << acc;
    int16_t norm[256];
    int s = 0;
    while (remaining > 0 && s < max_sym) {
      const int bits = highbit((uint64_t)remaining + 1) + 1;
      uint32_t val = in.read(bits);
      const uint32_t lower = (1u << (bits - 1)) - 1;
      const uint32_t threshold = (1u << bits) - 1 - ((uint32_t)remaining + 1);
      if ((val & lower) < threshold) {
        in.rewind(1);
        val &= lower;
      } else if (val > lower) {
        val -= threshold;
      }
      const int proba = (int)val - 1;
      remaining -= proba < 0 ? -proba : proba;
      norm[s++] = (int16_t)proba;
      if (proba == 0) {
        int rep = (int)in.read(2);
        for (;;) {
          for (int i = 0; i < rep && s < max_sym; i++) norm[s++] = 0;
          if (rep != 3) break;
          rep = (int)in.read(2);
        }
      }
    }
    if (remaining != 0) fail("zstd: FSE probabilities do not sum to the table size");
    build(norm, s, acc);
    return in.bytes_used();
  }
  uint32_t init(BackBits& b) const { return (uint32_t)b.read(log); }
  uint8_t peek(uint32_t st) const { return sym[st]; }
  void update(uint32_t& st, BackBits& b) const { st = base[st] + (uint32_t)b.read(nbits[st]); }
};

// ---- Huffman -----------------------------------------------------------------------------
struct Huf {
  int max_bits = 0;  // 0: no table yet
  std::vector<uint8_t> sym, nbits;

  void from_weights(const uint8_t* w, int n) {  // n transmitted weights; the last is implied
    if (n + 1 > 256) fail("zstd: too many Huffman symbols");
    uint64_t sum = 0;
    for (int i = 0; i < n; i++) {
      if (w[i] > kMaxHufBits) fail("zstd: Huffman weight too large");
      sum += w[i] ? (1ull << (w[i] - 1)) : 0;
    }
    if (sum == 0) fail("zstd: Huffman weights all zero");
    const int mb = highbit(sum) + 1;
    const uint64_t left = (1ull << mb) - sum;
    if (left & (left - 1)) fail("zstd: Huffman weights do not complete a tree");
    if (mb > kMaxHufBits) fail("zstd: Huffman tree too deep");
    uint8_t bits[256];
    for (int i = 0; i < n; i++) bits[i] = w[i] ? (uint8_t)(mb + 1 - w[i]) : 0;
    bits[n] = (uint8_t)(mb + 1 - (highbit(left) + 1));
    const int ns = n + 1;
    max_bits = 0;
    int count[kMaxHufBits + 2] = {0};
    for (int i = 0; i < ns; i++) {
      max_bits = bits[i] > max_bits ? bits[i] : max_bits;
      count[bits[i]]++;
    }
    const int size = 1 << max_bits;
    sym.assign(size, 0);
    nbits.assign(size, 0);
    uint32_t idx[kMaxHufBits + 2];
    idx[max_bits] = 0;
    for (int i = max_bits; i >= 1; i--) {
      idx[i - 1] = idx[i] + (uint32_t)count[i] * (1u << (max_bits - i));
      for (uint32_t k = idx[i]; k < idx[i - 1]; k++) nbits[k] = (uint8_t)i;
    }
    if (idx[0] != (uint32_t)size) fail("zstd: Huffman code space not filled");
    for (int i = 0; i < ns; i++) {
      if (!bits[i]) continue;
      const uint32_t len = 1u << (max_bits - bits[i]);
      for (uint32_t k = 0; k < len; k++) sym[idx[bits[i]] + k] = (uint8_t)i;
      idx[bits[i]] += len;
    }
  }
  // Tree description at src; returns the bytes it used.
  size_t read_tree(const uint8_t* src, size_t len) {
    if (len < 1) fail("zstd: missing Huffman tree description");
    const uint8_t hb = src[0];
    uint8_t w[256];
    int n = 0;
    if (hb >= 128) {  // direct 4-bit weights
      n = hb - 127;
      const size_t nb = ((size_t)n + 1) / 2;
      if (1 + nb > len) fail("zstd: Huffman weights truncated");
      for (int i = 0; i < n; i++) w[i] = (uint8_t)(i % 2 == 0 ? src[1 + i / 2] >> 4 : src[1 + i / 2] & 15);
      from_weights(w, n);
      return 1 + nb;
    }
    const size_t cs = hb;  // FSE-compressed weights: two interleaved states
    if (1 + cs > len || cs == 0) fail("zstd: Huffman weights truncated");
    Fse f;
    const size_t hl = f.read_header(src + 1, cs, 6, 256);
    if (hl >= cs) fail("zstd: Huffman weight stream empty");
    BackBits b(src + 1 + hl, cs - hl);
    uint32_t s1 = f.init(b), s2 = f.init(b);
    for (;;) {
      if (n >= 255) fail("zstd: too many Huffman weights");
      w[n++] = f.peek(s1);
      f.update(s1, b);
      if (b.off < 0) {
        w[n++] = f.peek(s2);
        break;
      }
      if (n >= 255) fail("zstd: too many Huffman weights");
      w[n++] = f.peek(s2);
      f.update(s2, b);
      if (b.off < 0) {
        if (n >= 255) fail("zstd: too many Huffman weights");
        w[n++] = f.peek(s1);
        break;
      }
    }
    from_weights(w, n);
    return 1 + cs;
  }
  void decode_stream(const uint8_t* src, size_t len, uint8_t* out, size_t nout) const {
    BackBits b(src, len);
    uint32_t st = (uint32_t)b.read(max_bits);
    const uint32_t mask = (1u << max_bits) - 1;
    for (size_t i = 0; i < nout; i++) {
      out[i] = sym[st];
      const int nb = nbits[st];
      st = ((st << nb) + (uint32_t)b.read(nb)) & mask;
    }
    if (b.off != -max_bits) fail("zstd: Huffman stream not consumed exactly");
  }
};

// ---- sequences: code tables ---------------------------------------------------------------
const uint32_t kLLBase[36] = {0,  1,  2,   3,   4,   5,    6,    7,    8,    9,     10,    11,
                              12, 13, 14,  15,  16,  18,   20,   22,   24,   28,    32,    40,
                              48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
const uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  1,  1,
                             1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
const uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10,  11,  12,   13,   14,   15,   16,
                              17, 18, 19, 20, 21, 22, 23, 24,  25,  26,   27,   28,   29,   30,
                              31, 32, 33, 34, 35, 37, 39, 41,  43,  47,   51,   59,   67,   83,
                              99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
const uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                             0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                             2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
const int16_t kLLDefault[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
const int16_t kMLDefault[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
const int16_t kOFDefault[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// ---- frame decoder -----------------------------------------------------------------------
struct FrameState {
  Huf huf;
  Fse ll, of, ml;
  uint64_t rep[3] = {1, 4, 8};
};

struct Out {
  uint8_t* dst;   // may be null (size query)
  size_t cap;
  size_t pos;     // bytes produced overall (all frames)
  size_t frame0;  // where the current frame's content starts
  void need(size_t n) {
    if (n > cap - pos) fail("zstd: decoded data exceeds the output buffer", ZH_EINVAL);
  }
};

size_t read_seq_table(Fse& t, int mode, const uint8_t* p, size_t len, const int16_t* dflt,
                      int ndflt, int dlog, int max_log, int max_sym) {
  switch (mode) {
    case 0:
      t.build(dflt, ndflt, dlog);
      return 0;
    case 1:
      if (len < 1) fail("zstd: RLE sequence table truncated");
      if (p[0] >= max_sym) fail("zstd: RLE sequence code out of range");
      t.rle(p[0]);
      return 1;
    case 2:
      return t.read_header(p, len, max_log, max_sym);
    default:
      if (t.log < 0) fail("zstd: repeat sequence table without a previous table");
      return 0;
  }
}

void decode_block(const uint8_t* src, size_t len, FrameState& fs, Out& out,
                  std::vector<uint8_t>& lit) {
  // -- literals section
  if (len < 1) fail("zstd: empty compressed block");
  const int ltype = src[0] & 3, sf = (src[0] >> 2) & 3;
  size_t regen = 0, hsz = 0, lsec = 0;
  const uint8_t* lits = nullptr;
  if (ltype <= 1) {
    if (sf == 0 || sf == 2) {
      hsz = 1;
      regen = src[0] >> 3;
    } else if (sf == 1) {
      hsz = 2;
      if (len < 2) fail("zstd: literals header truncated");
      regen = (src[0] >> 4) + ((size_t)src[1] << 4);
    } else {
      hsz = 3;
      if (len < 3) fail("zstd: literals header truncated");
      regen = (src[0] >> 4) + ((size_t)src[1] << 4) + ((size_t)src[2] << 12);
    }
    if (ltype == 0) {
      if (hsz + regen > len) fail("zstd: raw literals truncated");
      lits = src + hsz;
      lsec = hsz + regen;
    } else {
      if (hsz + 1 > len) fail("zstd: RLE literals truncated");
      lit.assign(regen, src[hsz]);
      lits = lit.data();
      lsec = hsz + 1;
    }
  } else {
    size_t csz;
    int nstreams = sf == 0 ? 1 : 4;
    if (sf <= 1) {
      hsz = 3;
      if (len < 3) fail("zstd: literals header truncated");
      const uint64_t h = rd_le(src, 3);
      regen = (h >> 4) & 1023;
      csz = (h >> 14) & 1023;
    } else if (sf == 2) {
      hsz = 4;
      if (len < 4) fail("zstd: literals header truncated");
      const uint64_t h = rd_le(src, 4);
      regen = (h >> 4) & 16383;
      csz = (h >> 18) & 16383;
    } else {
      hsz = 5;
      if (len < 5) fail("zstd: literals header truncated");
      const uint64_t h = rd_le(src, 5);
      regen = (h >> 4) & 262143;
      csz = (h >> 22) & 262143;
    }
    if (hsz + csz > len) fail("zstd: compressed literals truncated");
    const uint8_t* p = src + hsz;
    size_t rem = csz;
    if (ltype == 2) {
      const size_t t = fs.huf.read_tree(p, rem);
      p += t;
      rem -= t;
    } else if (fs.huf.max_bits == 0) {
      fail("zstd: treeless literals without a previous Huffman table");
    }
    lit.resize(regen);
    if (nstreams == 1) {
      fs.huf.decode_stream(p, rem, lit.data(), regen);
    } else {
      if (rem < 6) fail("zstd: literals jump table truncated");
      const size_t s1 = rd_le(p, 2), s2 = rd_le(p + 2, 2), s3 = rd_le(p + 4, 2);
      if (6 + s1 + s2 + s3 > rem) fail("zstd: literals streams truncated");
      const size_t s4 = rem - 6 - s1 - s2 - s3;
      const size_t per = (regen + 3) / 4;
      if (3 * per > regen) fail("zstd: literals too short for four streams");
      const uint8_t* q = p + 6;
      fs.huf.decode_stream(q, s1, lit.data(), per);
      fs.huf.decode_stream(q + s1, s2, lit.data() + per, per);
      fs.huf.decode_stream(q + s1 + s2, s3, lit.data() + 2 * per, per);
      fs.huf.decode_stream(q + s1 + s2 + s3, s4, lit.data() + 3 * per, regen - 3 * per);
    }
    lits = lit.data();
    lsec = hsz + csz;
  }
  // -- sequences section
  const uint8_t* p = src + lsec;
  size_t rem = len - lsec;
  if (rem < 1) fail("zstd: sequences section missing");
  size_t nseq;
  if (p[0] < 128) {
    nseq = p[0];
    p += 1;
    rem -= 1;
  } else if (p[0] < 255) {
    if (rem < 2) fail("zstd: sequence count truncated");
    nseq = ((size_t)(p[0] - 128) << 8) + p[1];
    p += 2;
    rem -= 2;
  } else {
    if (rem < 3) fail("zstd: sequence count truncated");
    nseq = rd_le(p + 1, 2) + 0x7F00;
    p += 3;
    rem -= 3;
  }
  size_t lpos = 0;
  if (nseq > 0) {
    if (rem < 1) fail("zstd: sequence modes missing");
    const uint8_t modes = p[0];
    if (modes & 3) fail("zstd: reserved bits set in the sequence modes");
    p += 1;
    rem -= 1;
    size_t u = read_seq_table(fs.ll, (modes >> 6) & 3, p, rem, kLLDefault, 36, 6, 9, 36);
    p += u;
    rem -= u;
    u = read_seq_table(fs.of, (modes >> 4) & 3, p, rem, kOFDefault, 29, 5, 8, 32);
    p += u;
    rem -= u;
    u = read_seq_table(fs.ml, (modes >> 2) & 3, p, rem, kMLDefault, 53, 6, 9, 53);
    p += u;
    rem -= u;
    BackBits b(p, rem);
    uint32_t sll = fs.ll.init(b), sof = fs.of.init(b), sml = fs.ml.init(b);
    for (size_t k = 0; k < nseq; k++) {
      const uint8_t ofc = fs.of.peek(sof), llc = fs.ll.peek(sll), mlc = fs.ml.peek(sml);
      if (llc > 35 || mlc > 52 || ofc > 31) fail("zstd: sequence code out of range");
      const uint64_t ofv = (1ull << ofc) + b.read(ofc);
      const size_t ml = kMLBase[mlc] + (size_t)b.read(kMLBits[mlc]);
      const size_t ll = kLLBase[llc] + (size_t)b.read(kLLBits[llc]);
      if (k + 1 < nseq) {
        fs.ll.update(sll, b);
        fs.ml.update(sml, b);
        fs.of.update(sof, b);
      }
      uint64_t offset;  // repeat offsets (RFC 8878 §3.1.2.5)
      if (ofv > 3) {
        offset = ofv - 3;
        fs.rep[2] = fs.rep[1];
        fs.rep[1] = fs.rep[0];
        fs.rep[0] = offset;
      } else {
        unsigned idx = (unsigned)ofv - 1 + (ll == 0 ? 1u : 0u);
        if (idx == 0) {
          offset = fs.rep[0];
        } else {
          offset = idx < 3 ? fs.rep[idx] : fs.rep[0] - 1;
          if (idx > 1) fs.rep[2] = fs.rep[1];
          fs.rep[1] = fs.rep[0];
          fs.rep[0] = offset;
        }
      }
      if (lpos + ll > regen) fail("zstd: sequence reads past the literals");
      out.need(ll + ml);
      if (out.dst && ll) memcpy(out.dst + out.pos, lits + lpos, ll);
      lpos += ll;
      out.pos += ll;
      if (offset == 0 || offset > out.pos - out.frame0) fail("zstd: match offset before the frame");
      if (out.dst) {
        uint8_t* d = out.dst + out.pos;
        const uint8_t* s = d - offset;
        for (size_t i = 0; i < ml; i++) d[i] = s[i];
      }
      out.pos += ml;
    }
    if (b.off != 0) fail("zstd: sequence bitstream not consumed exactly");
  }
  const size_t tail = regen - lpos;  // remaining literals
  out.need(tail);
  if (out.dst && tail) memcpy(out.dst + out.pos, lits + lpos, tail);
  out.pos += tail;
}

// One frame at src (magic already checked by the caller); returns bytes consumed.
size_t decode_frame(const uint8_t* src, size_t len, Out& out, int64_t* content_size) {
  if (len < 5) fail("zstd: frame header truncated");
  const uint8_t fhd = src[4];
  const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, csum = (fhd >> 2) & 1,
            did_flag = fhd & 3;
  if (fhd & 0x08) fail("zstd: reserved frame header bit set");
  size_t p = 5;
  if (!single) p += 1;  // window descriptor (the whole output is one buffer)
  const int did_size[4] = {0, 1, 2, 4};
  if (p + did_size[did_flag] > len) fail("zstd: frame header truncated");
  if (did_flag && rd_le(src + p, did_size[did_flag]) != 0)
    fail("zstd: frames that need a dictionary are not supported", ZH_EUNSUPPORTED);
  p += did_size[did_flag];
  const int fcs_size = fcs_flag == 0 ? (single ? 1 : 0) : (fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8);
  if (p + fcs_size > len) fail("zstd: frame header truncated");
  int64_t fcs = -1;
  if (fcs_size) {
    fcs = (int64_t)rd_le(src + p, fcs_size);
    if (fcs_size == 2) fcs += 256;
  }
  p += fcs_size;
  if (content_size) *content_size = fcs;
  out.frame0 = out.pos;
  const bool size_only = !out.dst && fcs >= 0;  // size query: the header says it all
  FrameState fs;
  std::vector<uint8_t> lit;
  for (;;) {
    if (p + 3 > len) fail("zstd: block header truncated");
    const uint32_t bh = (uint32_t)rd_le(src + p, 3);
    p += 3;
    const int last = bh & 1, type = (bh >> 1) & 3;
    const size_t bsz = bh >> 3;
    if (type == 3) fail("zstd: reserved block type");
    if (size_only) {
      p += type == 1 ? 1 : bsz;
      if (p > len) fail("zstd: block truncated");
    } else if (type == 1) {  // RLE: one byte, bsz copies
      if (p + 1 > len) fail("zstd: block truncated");
      out.need(bsz);
      if (out.dst && bsz) memset(out.dst + out.pos, src[p], bsz);
      out.pos += bsz;
      p += 1;
    } else {
      if (p + bsz > len) fail("zstd: block truncated");
      if (bsz > (128u << 10)) fail("zstd: block larger than 128 KiB");
      if (type == 0) {
        out.need(bsz);
        if (out.dst && bsz) memcpy(out.dst + out.pos, src + p, bsz);
        out.pos += bsz;
      } else {
        decode_block(src + p, bsz, fs, out, lit);
      }
      p += bsz;
    }
    if (last) break;
  }
  if (size_only) out.pos += (size_t)fcs;
  const size_t produced = out.pos - out.frame0;
  if (fcs >= 0 && (uint64_t)fcs != produced) fail("zstd: frame content size mismatch");
  if (csum) {
    if (p + 4 > len) fail("zstd: content checksum truncated");
    if (out.dst) {
      const uint32_t want = (uint32_t)rd_le(src + p, 4);
      const uint32_t got = (uint32_t)zh_xxh64(out.dst + out.frame0, produced, 0);
      if (want != got) fail("zstd: content checksum mismatch");
    }
    p += 4;
  }
  return p;
}

int run(const uint8_t* s, size_t n, Out& out, char* err, size_t errlen) {
  try {
    size_t p = 0;
    int frames = 0;
    while (p < n) {
      if (n - p < 4) fail("zstd: trailing bytes after the last frame");
      const uint32_t magic = (uint32_t)rd_le(s + p, 4);
      if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
        if (n - p < 8) fail("zstd: skippable frame truncated");
        const uint64_t sz = rd_le(s + p + 4, 4);
        if (sz > n - p - 8) fail("zstd: skippable frame truncated");
        p += 8 + sz;
        continue;
      }
      if (magic != kMagic) fail("zstd: unknown frame magic");
      p += decode_frame(s + p, n - p, out, nullptr);
      frames++;
    }
    if (!frames) fail("zstd: no frame");
    return ZH_OK;
  } catch (const Fail& f) {
    set_err(err, errlen, f.msg);
    return f.status;
  } catch (const std::bad_alloc&) {
    set_err(err, errlen, "zstd: out of memory");
    return ZH_ENOMEM;
  }
}

}  // namespace

extern "C" {

// Size query (dst == NULL): the sum of the frames' declared content sizes, or, when a frame
// omits its size, a full decode pass without output.  Decode: dstcap must hold the content.
int zh_zstd_decompress(const void* src, size_t srclen, void* dst, size_t dstcap, size_t* dstlen,
                       char* err, size_t errlen) {
  if (!src || !dstlen) return ZH_EINVAL;
  Out out{(uint8_t*)dst, dst ? dstcap : SIZE_MAX, 0, 0};
  const int st = run((const uint8_t*)src, srclen, out, err, errlen);
  *dstlen = out.pos;
  return st;
}

// A frame of raw blocks (no compression): content size in the header, XXH64 checksum when
// `checksum` is set.  dst NULL: returns the frame size in *dstlen.
int zh_zstd_compress_raw(const void* src, size_t srclen, int checksum, void* dst, size_t dstcap,
                         size_t* dstlen) {
  if (!dstlen || (!src && srclen)) return ZH_EINVAL;
  const size_t maxb = (size_t)128 << 10;
  const size_t nblk = srclen == 0 ? 1 : (srclen + maxb - 1) / maxb;
  const size_t need = 4 + 1 + 8 + nblk * 3 + srclen + (checksum ? 4 : 0);
  *dstlen = need;
  if (!dst) return ZH_OK;
  if (dstcap < need) return ZH_EINVAL;
  uint8_t* d = (uint8_t*)dst;
  size_t p = 0;
  auto put = [&](uint64_t v, int n) {
    for (int i = 0; i < n; i++) d[p++] = (uint8_t)(v >> (8 * i));
  };
  put(kMagic, 4);
  put((3u << 6) | (1u << 5) | (checksum ? 4u : 0u), 1);  // 8-byte FCS, single segment
  put(srclen, 8);
  for (size_t k = 0; k < nblk; k++) {
    const size_t o = k * maxb, b = srclen - o < maxb ? srclen - o : maxb;
    put(((uint32_t)b << 3) | (k + 1 == nblk ? 1u : 0u), 3);  // raw block
    if (b) memcpy(d + p, (const uint8_t*)src + o, b);
    p += b;
  }
  if (checksum) put((uint32_t)zh_xxh64(src, srclen, 0), 4);
  return ZH_OK;
}

}  // extern "C"
