// zh_files.cpp — region reads whose chunks are files of a FilesystemStore.
//
// core.Array.read over a FilesystemStore (M/core/Array.java:378-441) reads every chunk key
// through FilesystemStore (M/store/FilesystemStore.java:43-102): `exists` (a regular file),
// then for a whole chunk `get(keys)`, and for a shard the StoreHandleDataProvider reads of
// decodeInternal (ShardingIndexedCodec.java:190-230, 333-357) — the index by a prefix or suffix
// read, then one range read per referenced inner chunk.  zh_array_read_files takes the files'
// paths and does those reads itself: the index on the calling thread (it decides the ranges),
// the ranges inside the pipelined read's in lanes, each pread landing in a page-locked ring slot
// that is DMA'd to the device (zh_pipeline.cpp).  The bytes are copied once on the host, not
// read into a store buffer first and copied into the ring after, and the reads of slab r + 1
// overlap the decode and D2H of slab r.  Sources name the file bytes by file addresses
// (zh_ctx.h): the planner lays them out like any host bytes and never dereferences them.
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "zh_ctx.h"

namespace zh {

std::string file_fetch(const zh_ctx* ctx, void* dst, const void* src, int64_t n) {
  const uint64_t a = (uint64_t)(uintptr_t)src & ~kFileTag;
  const size_t slot = (size_t)(a >> kFileOffBits);
  int64_t off = (int64_t)(a & ((1ull << kFileOffBits) - 1));
  if (slot >= ctx->files.size()) return "file source outside the read's file table";
  const int fd = ctx->files[slot];
  uint8_t* d = (uint8_t*)dst;
  while (n > 0) {
    const ssize_t r = pread(fd, d, (size_t)std::min<int64_t>(n, (int64_t)1 << 30), (off_t)off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) {  // an error, or the file ended (it shrank after its size was taken)
      std::string why = r < 0 ? strerror(errno) : "unexpected end of file";
      return "Failed to read from store at '" + ctx->file_paths[slot] + "': " + why;
    }
    d += r;
    off += r;
    n -= r;
  }
  return "";
}

}  // namespace zh

using namespace zh;

namespace {

// The open files of one zh_array_read_files call, registered on the context for the read
// (ctx->mu held) and closed on every exit.
struct FileTable {
  zh_ctx* ctx;
  explicit FileTable(zh_ctx* c) : ctx(c) {
    ctx->files.clear();
    ctx->file_paths.clear();
  }
  ~FileTable() {
    for (int fd : ctx->files)
      if (fd >= 0) close(fd);
    ctx->files.clear();
    ctx->file_paths.clear();
  }
};

// Reads [off, off + n) of file slot into dst; ZH_EIO with the message on failure.
int read_range(zh_ctx* ctx, int64_t slot, int64_t off, int64_t n, uint8_t* dst, char* err,
               size_t errlen) {
  const std::string m = file_fetch(ctx, dst, file_addr(slot, off), n);
  if (m.empty()) return ZH_OK;
  set_err(err, errlen, "%s", m.c_str());
  return ZH_EIO;
}

// A read that does not run pipelined (small, or not splittable): the file bytes the sources
// name are read into host buffers first and the sources pointed at them (one plan then
// stages them as it stages any host bytes).
int file_materialize(zh_ctx* ctx, std::vector<SrcDesc>& srcs,
                     std::vector<std::vector<zh_shard_piece>>& pieces,
                     std::vector<std::vector<uint8_t>>& keep, char* err, size_t errlen) {
  auto fetch = [&](const void* a, int64_t n, const uint8_t** out) -> int {
    keep.emplace_back((size_t)std::max<int64_t>(n, 1));
    const std::string m = file_fetch(ctx, keep.back().data(), a, n);
    if (!m.empty()) {
      set_err(err, errlen, "%s", m.c_str());
      return ZH_EIO;
    }
    *out = keep.back().data();
    return ZH_OK;
  };
  for (size_t i = 0; i < srcs.size(); i++) {
    SrcDesc& s = srcs[i];
    if (s.data && is_file_addr(s.data)) {
      int st = fetch(s.data, s.nbytes, &s.data);
      if (st != ZH_OK) return st;
    }
    for (zh_shard_piece& q : pieces[i]) {
      if (!q.data || !is_file_addr(q.data) || q.data_nbytes <= 0) continue;
      const uint8_t* p = nullptr;
      int st = fetch(q.data, q.data_nbytes, &p);
      if (st != ZH_OK) return st;
      q.data = p;
    }
  }
  return ZH_OK;
}

}  // namespace

extern "C" {

int zh_array_read_files(zh_ctx* ctx, const zh_array_meta* meta, const char* const* paths,
                        int64_t npaths, const int64_t* offset, const int64_t* shape, void* out,
                        uint32_t flags, char* err, size_t errlen) {
  if (!ctx || !meta || !offset || !shape || !out || (npaths > 0 && !paths)) return ZH_EINVAL;
  if (flags & ZH_SRC_DEVICE) {
    set_err(err, errlen, "zh_array_read_files reads host files: ZH_SRC_DEVICE is not allowed");
    return ZH_EINVAL;
  }
  int st = zh_validate_meta(meta, err, errlen);
  if (st != ZH_OK) return st;
  const int n = meta->ndim;
  for (int d = 0; d < n; d++) {  // M/core/Array.java:386-390 (the planner's check, early)
    if (offset[d] < 0 || offset[d] + shape[d] > meta->shape[d]) {
      set_err(err, errlen, "Requested data is outside of the array's domain.");
      return ZH_EDATA;
    }
    if (shape[d] <= 0) {
      set_err(err, errlen, "empty selection at dimension %d", d);
      return ZH_EINVAL;
    }
  }
  int64_t cstart[kMaxDims], ccount[kMaxDims];
  const int64_t ncoords = chunk_coords(n, meta->chunk_shape, offset, shape, cstart, ccount);
  if (ncoords > kIntMax) {
    set_err(err, errlen, "Number of chunks exceeds Integer.MAX_VALUE");
    return ZH_EARITH;
  }
  if (ncoords != npaths) {
    set_err(err, errlen, "expected %lld chunk paths (computeChunkCoords order), got %lld",
            (long long)ncoords, (long long)npaths);
    return ZH_EINVAL;
  }
  if (npaths > kFileMaxSlots) return ZH_EUNSUPPORTED;
  std::lock_guard<std::mutex> lk(ctx->mu);
  FileTable table(ctx);
  const zh_codec_chain& c = meta->chain;
  const int64_t isz = c.sharded ? zh_shard_index_size(meta) : 0;
  std::vector<SrcDesc> srcs((size_t)npaths);
  std::vector<std::vector<uint8_t>> index((size_t)npaths);
  std::vector<std::vector<zh_shard_piece>> pieces((size_t)npaths);
  int64_t cur[kMaxDims] = {0};
  for (int64_t i = 0; i < npaths; i++) {
    int64_t cc[kMaxDims];
    for (int d = 0; d < n; d++) cc[d] = cstart[d] + cur[d];
    for (int d = n - 1; d >= 0; d--) {
      if (++cur[d] < ccount[d]) break;
      cur[d] = 0;
    }
    const char* path = paths[i];
    ctx->files.push_back(-1);
    ctx->file_paths.push_back(path ? path : "");
    if (!path) continue;  // missing key
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) {
      const int oe = errno;
      // FilesystemStore.exists is Files.isRegularFile (false when the file is absent, is no
      // regular file, or cannot be stat'ed); an existing regular file that cannot be opened is
      // a failed read (readAllBytes / newByteChannel → StoreException.readFailed)
      struct stat sb;
      if (oe == ENOENT || oe == ENOTDIR || stat(path, &sb) != 0 || !S_ISREG(sb.st_mode)) continue;
      set_err(err, errlen, "Failed to read from store at '%s': %s", path, strerror(oe));
      return ZH_EIO;
    }
    ctx->files.back() = fd;
    struct stat sb;
    if (fstat(fd, &sb) != 0) {
      set_err(err, errlen, "Failed to read from store at '%s': %s", path, strerror(errno));
      return ZH_EIO;
    }
    if (!S_ISREG(sb.st_mode)) continue;  // Files.isRegularFile (FilesystemStore.java:44-46)
    const int64_t size = (int64_t)sb.st_size;
    if (size >= kFileMaxBytes) return ZH_EUNSUPPORTED;
    SrcDesc& s = srcs[(size_t)i];
    if (!c.sharded) {  // get(keys): the whole object
      s.data = file_addr(i, 0);
      s.nbytes = size;
      continue;
    }
    // the stored index: a prefix read (index_location start) or a suffix read of isz bytes
    // (get(keys, -isz)); a file shorter than the index gives what it holds, and the planner
    // reports "Shard [...] is smaller than its index"
    const int64_t ilen = std::min(size, isz);
    auto& ib = index[(size_t)i];
    ib.resize((size_t)std::max<int64_t>(ilen, 1));
    const int64_t ioff = c.index_location == ZH_INDEX_START ? 0 : size - ilen;
    if ((st = read_range(ctx, i, ioff, ilen, ib.data(), err, errlen)) != ZH_OK) return st;
    s.index = ib.data();
    s.index_nbytes = ilen;
    s.shard_nbytes = size;
    if (ilen < isz) continue;  // no ranges: the planner reports the short index
    int32_t co[kMaxDims], oo[kMaxDims], ps[kMaxDims];
    if (projection(n, cc, meta->shape, meta->chunk_shape, offset, shape, co, oo, ps) != ZH_OK) {
      set_err(err, errlen, "projection exceeds Integer.MAX_VALUE");
      return ZH_EARITH;
    }
    int64_t lo[kMaxDims], hi[kMaxDims];
    for (int d = 0; d < n; d++) {
      lo[d] = co[d];
      hi[d] = (int64_t)co[d] + ps[d];
    }
    // the referenced inner chunks' ranges, adjacent ones merged (one pread per run); entries
    // beyond the file are left out and read as "Could not load byte data" on the device
    std::vector<std::pair<int64_t, int64_t>> rs;
    if (shard_ranges(meta, ib.data(), size, lo, hi, INT64_MAX, rs) != ZH_OK) continue;
    for (auto& r : rs) pieces[(size_t)i].push_back({r.first, r.second, file_addr(i, r.first), r.second});
    s.pieces = pieces[(size_t)i].data();
    s.npieces = (int64_t)pieces[(size_t)i].size();
  }
  const uint32_t f = flags & ZH_OUT_DEVICE;
  if (env_int("ZH_PIPE", 1) != 0) {
    st = read_pipelined(ctx, meta, srcs.data(), npaths, offset, shape, out, f, nullptr, err,
                        errlen);
    if (st != ZH_EUNSUPPORTED) return st;
  }
  std::vector<std::vector<uint8_t>> keep;
  if ((st = file_materialize(ctx, srcs, pieces, keep, err, errlen)) != ZH_OK) return st;
  for (size_t i = 0; i < srcs.size(); i++)
    if (srcs[i].pieces) srcs[i].pieces = pieces[i].data();
  return read_one_plan(ctx, meta, srcs.data(), npaths, offset, shape, out, f, nullptr, err,
                       errlen);
}

}  // extern "C"
