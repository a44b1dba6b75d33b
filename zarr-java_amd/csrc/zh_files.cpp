// zh_files.cpp — region reads and writes whose chunks are files of a FilesystemStore.
//
// core.Array.read over a FilesystemStore (M/core/Array.java:378-441) reads every chunk key
// through FilesystemStore (M/store/FilesystemStore.java:42-102): `exists` (a regular file),
// then for a whole chunk `get(keys)`, and for a part of a shard the StoreHandleDataProvider
// reads of decodeInternal (ShardingIndexedCodec.java:190-230, 333-357) — the index by a prefix
// or suffix read, then one range read per referenced inner chunk.  zh_array_read_files takes
// the files' paths and does those reads itself: the indexes on the calling thread (they decide
// the ranges), the ranges inside the pipelined read's in lanes, each pread landing in a
// page-locked ring slot that is DMA'd to the device (zh_pipeline.cpp).  Sources name file
// bytes as SrcRef::file(slot, offset) into a process-wide table of the files of the reads in
// flight, so one read may span several contexts (zh_array_read_files_multi).
//
// Range semantics follow get(keys, start, end) (:84-102): a buffer of end - start bytes holding
// what the file has, zeros after its end (file_fetch).  A whole-shard part is the reference's
// chunkHandle.read() + ByteBufferDataProvider (ShardingIndexedCodec.java:246-251, 301-331):
// slices of the file as it is, where an index or entry beyond the file is an error.
//
// zh_array_write_files is the write side: the device encode, then writeChunk's store calls
// (FilesystemStore.set / delete) here, the encoded bytes D2H'd through the page-locked ring in
// windows that the copy lanes pwrite into a temporary file per chunk, renamed over the chunk's
// file once all its bytes are in.
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <limits.h>
#include <signal.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "zh_ctx.h"

namespace {

using zh::SrcRef;

// ---- store names (StoreException's text) ----------------------------------------------

// FilesystemStore.toString() of a store (its file: URI without the trailing '/'), or the
// caller's name for it; the filesystem root when no store is given.
std::string store_name(const zh_file_store* st) {
  if (st && st->name) return st->name;
  std::string r = st && st->root ? st->root : "/";
  while (r.size() > 1 && r.back() == '/') r.pop_back();
  if (r == "/") r.clear();
  return "file://" + r;
}

// The key of `path` in the store: the path below the store's directory ('/'-joined keys,
// String.join("/", keys) in StoreException), or the path itself outside it.
std::string store_key(const zh_file_store* st, const char* path) {
  std::string root = st && st->root ? st->root : "/";
  while (root.size() > 1 && root.back() == '/') root.pop_back();
  const std::string p(path);
  size_t k = 0;
  if (root == "/") {
    if (p.empty() || p[0] != '/') return p;
  } else {
    if (p.compare(0, root.size(), root) != 0 || p.size() <= root.size() || p[root.size()] != '/')
      return p;
    k = root.size();
  }
  while (k < p.size() && p[k] == '/') k++;
  return p.substr(k);
}

std::string failed(const char* what, const std::string& store, const std::string& key,
                   const std::string& cause) {
  return std::string("Failed to ") + what + " store '" + store + "' at key '" + key + "': " + cause;
}

// IOException.getMessage() of a failed open of `path` as the JDK words it (UnixException:
// AccessDeniedException carries just the file; other errors "file: reason").
std::string open_cause(const std::string& path, int e) {
  if (e == EACCES || e == EPERM) return path;
  return path + ": " + strerror(e);
}

// ---- the file table --------------------------------------------------------------------

struct FileEnt {
  std::string path, store, key;
  int fd = -1;
  int pins = 0;       // file_fetch calls reading it now (its descriptor stays open)
  bool live = false;
  // range reads past the end read as zeros (a part's reads, get(keys, start, end)); otherwise
  // the file is read as it was when its size was taken (a whole object or shard), and a read
  // that meets the end (the file shrank meanwhile) fails
  bool pad = false;
};

struct FileTable {
  std::mutex mu;
  std::vector<FileEnt> ent;
  std::vector<int32_t> free;
  std::deque<int32_t> opened;  // slots in the order their descriptors were opened (may be stale)
  int open = 0;  // descriptors open (and slots reserved for an open in progress)
};

FileTable& table() {
  static FileTable t;
  return t;
}

int32_t slot_take(const std::string& path, const std::string& store, const std::string& key,
                  bool pad) {
  FileTable& t = table();
  std::lock_guard<std::mutex> lk(t.mu);
  int32_t k;
  if (!t.free.empty()) {
    k = t.free.back();
    t.free.pop_back();
  } else {
    k = (int32_t)t.ent.size();
    t.ent.emplace_back();
  }
  FileEnt& e = t.ent[(size_t)k];
  e.path = path;
  e.store = store;
  e.key = key;
  e.fd = -1;
  e.pins = 0;
  e.live = true;
  e.pad = pad;
  return k;
}

void slot_give(int32_t k) {
  FileTable& t = table();
  std::lock_guard<std::mutex> lk(t.mu);
  FileEnt& e = t.ent[(size_t)k];
  if (e.fd >= 0) {
    close(e.fd);
    t.open--;
  }
  e = FileEnt();
  t.free.push_back(k);
  // the queue of opens keeps an entry per open until close_lru meets it: drop the stale ones
  // at its front now (all of them once nothing is open), so a long-running process doing
  // reads of few files keeps it bounded
  if (t.open == 0) {
    t.opened.clear();
  } else {
    while (!t.opened.empty()) {
      const FileEnt& f = t.ent[(size_t)t.opened.front()];
      if (f.live && f.fd >= 0) break;
      t.opened.pop_front();
    }
  }
}

// Closes the oldest open descriptor nobody is reading (caller holds t.mu): the queue of opens
// in order, stale entries (closed since, or a slot given back) dropped, pinned ones moved to
// the back; false when every open descriptor is being read.  O(1) per close but for the few
// pinned ones (at most one per lane), so a read of many files costs no scan of the table.
bool close_lru(FileTable& t) {
  for (size_t tries = t.opened.size(); tries > 0; tries--) {
    const int32_t k = t.opened.front();
    t.opened.pop_front();
    FileEnt& e = t.ent[(size_t)k];
    if (!e.live || e.fd < 0) continue;
    if (e.pins > 0) {
      t.opened.push_back(k);
      continue;
    }
    close(e.fd);
    e.fd = -1;
    t.open--;
    return true;
  }
  return false;
}

// The open descriptor of slot k, pinned until file_unpin (opened by path when closed), or -1
// with *msg set.  At most kFileMaxOpen descriptors are open: beyond that the oldest idle one is
// closed first.  The open itself runs outside the table's lock.
int file_pin(int32_t k, std::string* msg) {
  FileTable& t = table();
  std::string path;
  {
    std::lock_guard<std::mutex> lk(t.mu);
    FileEnt& e = t.ent[(size_t)k];
    if (!e.live) {
      *msg = "a store file that no read has open";
      return -1;
    }
    if (e.fd >= 0) {
      e.pins++;
      return e.fd;
    }
    while (t.open >= zh::kFileMaxOpen && close_lru(t)) {
    }
    t.open++;  // reserved for this open
    path = e.path;
  }
  int fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0 && (errno == EMFILE || errno == ENFILE)) {  // other descriptors of the process
    {
      std::lock_guard<std::mutex> lk(t.mu);
      while (close_lru(t)) {
      }
    }
    fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  }
  const int oe = errno;
  std::lock_guard<std::mutex> lk(t.mu);
  FileEnt& e = t.ent[(size_t)k];
  if (fd < 0) {
    t.open--;
    *msg = failed("read from", e.store, e.key, open_cause(e.path, oe));
    return -1;
  }
  if (e.fd >= 0) {  // another lane opened it meanwhile
    close(fd);
    t.open--;
  } else {
    e.fd = fd;
    t.opened.push_back(k);
  }
  e.pins++;
  return e.fd;
}

void file_unpin(int32_t k) {
  FileTable& t = table();
  std::lock_guard<std::mutex> lk(t.mu);
  t.ent[(size_t)k].pins--;
}

bool slot_pads(int32_t k) {
  FileTable& t = table();
  std::lock_guard<std::mutex> lk(t.mu);
  return t.ent[(size_t)k].pad;
}

std::string slot_read_failed(int32_t k, const std::string& cause) {
  FileTable& t = table();
  std::lock_guard<std::mutex> lk(t.mu);
  const FileEnt& e = t.ent[(size_t)k];
  return failed("read from", e.store, e.key, cause);
}

}  // namespace

namespace zh {

std::string file_fetch(void* dst, const SrcRef& src, int64_t n) {
  const int32_t k = src.slot();
  int64_t off = src.file_offset();
  std::string msg;
  const int fd = file_pin(k, &msg);
  if (fd < 0) return msg;
  uint8_t* d = (uint8_t*)dst;
  while (n > 0) {
    const ssize_t r = pread(fd, d, (size_t)std::min<int64_t>(n, (int64_t)1 << 30), (off_t)off);
    if (r < 0 && errno == EINTR) continue;
    if (r < 0) {
      msg = slot_read_failed(k, strerror(errno));
      break;
    }
    if (r == 0) {  // the end of the file: the rest of a part's range reads as zeros
      if (slot_pads(k)) memset(d, 0, (size_t)n);
      else msg = slot_read_failed(k, "unexpected end of file");
      break;
    }
    d += r;
    off += r;
    n -= r;
  }
  file_unpin(k);
  return msg;
}

std::string file_fetch_all(const std::vector<FileRead>& reads) {
  for (const FileRead& r : reads) {
    const std::string m = file_fetch(r.dst, r.src, r.n);
    if (!m.empty()) return m;
  }
  return "";
}

}  // namespace zh

using namespace zh;

namespace {

// The files of one read: their slots go back (and their descriptors are closed) on every exit.
struct FileSet {
  std::vector<int32_t> taken;
  ~FileSet() {
    for (int32_t k : taken) slot_give(k);
  }
};

// What one read of files holds for the planner: the sources and the memory they point into.
struct FileSources {
  FileSet set;
  std::vector<SrcDesc> srcs;
  std::vector<std::vector<uint8_t>> index;
  std::vector<std::vector<Piece>> pieces;
};

// Sources for a read of the files `paths` (computeChunkCoords order of [offset, offset+shape)):
// per file the reference's store reads up to the ranges (exists, the stored index), the ranges
// as file sources.
int file_sources(const zh_array_meta* meta, const zh_file_store* store, const char* const* paths,
                 int64_t npaths, const int64_t* offset, const int64_t* shape, FileSources& fs,
                 char* err, size_t errlen) {
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
  const zh_codec_chain& c = meta->chain;
  const int64_t isz = c.sharded ? zh_shard_index_size(meta) : 0;
  const std::string sname = store_name(store);
  fs.srcs.assign((size_t)npaths, SrcDesc());
  fs.index.assign((size_t)npaths, {});
  fs.pieces.assign((size_t)npaths, {});
  std::vector<FileRead> ireads;
  std::vector<int32_t> slot_of((size_t)npaths, -1);
  std::vector<std::array<int64_t, kMaxDims>> lo((size_t)npaths), hi((size_t)npaths);
  int64_t cur[kMaxDims] = {0};
  for (int64_t i = 0; i < npaths; i++) {
    int64_t cc[kMaxDims];
    for (int d = 0; d < n; d++) cc[d] = cstart[d] + cur[d];
    for (int d = n - 1; d >= 0; d--) {
      if (++cur[d] < ccount[d]) break;
      cur[d] = 0;
    }
    const char* path = paths[i];
    if (!path) continue;  // missing key
    // FilesystemStore.exists is Files.isRegularFile (:42-45): false when the file is absent,
    // is no regular file, or cannot be stat'ed
    struct stat sb;
    if (stat(path, &sb) != 0 || !S_ISREG(sb.st_mode)) continue;
    const int64_t size = (int64_t)sb.st_size;
    SrcDesc& s = fs.srcs[(size_t)i];
    if (!c.sharded) {  // get(keys): the whole object
      const int32_t k = slot_take(path, sname, store_key(store, path), false);
      fs.set.taken.push_back(k);
      s.data = SrcRef::file(k, 0);
      s.nbytes = size;
      continue;
    }
    int32_t co[kMaxDims], oo[kMaxDims], ps[kMaxDims];
    if (projection(n, cc, meta->shape, meta->chunk_shape, offset, shape, co, oo, ps) != ZH_OK) {
      set_err(err, errlen, "projection exceeds Integer.MAX_VALUE");
      return ZH_EARITH;
    }
    bool full = true;  // decodePartial: Arrays.equals(shape, chunkShape) (:246)
    for (int d = 0; d < n; d++) {
      full = full && ps[d] == meta->chunk_shape[d];
      lo[(size_t)i][(size_t)d] = co[d];
      hi[(size_t)i][(size_t)d] = (int64_t)co[d] + ps[d];
    }
    const int32_t k = slot_take(path, sname, store_key(store, path), !full);
    fs.set.taken.push_back(k);
    slot_of[(size_t)i] = k;
    // the stored index: a suffix read (get(keys, -isz)) or a prefix read (get(keys, 0, isz)).
    // A suffix of a file shorter than the index, or any index past the end of a whole shard's
    // bytes, is short: the planner reports "Shard [...] of N bytes is smaller than its index".
    // A part's prefix read is zero-padded like any range (get(keys, start, end)).
    const bool start = c.index_location == ZH_INDEX_START;
    const int64_t ilen = start && !full ? isz : std::min(size, isz);
    auto& ib = fs.index[(size_t)i];
    ib.resize((size_t)std::max<int64_t>(ilen, 1));
    ireads.push_back({ib.data(), SrcRef::file(k, start ? 0 : size - ilen), ilen});
    s.index = ib.data();
    s.index_nbytes = ilen;
    // a whole shard resolves its entries against the file's size; a part's range reads are
    // zero-padded, so no entry is out of reach by its offset (shard size unknown)
    s.shard_nbytes = full ? size : -1;
  }
  // every shard's index, then the ranges from each
  const std::string m = file_fetch_all(ireads);
  if (!m.empty()) {
    set_err(err, errlen, "%s", m.c_str());
    return ZH_EIO;
  }
  for (int64_t i = 0; c.sharded && i < npaths; i++) {
    SrcDesc& s = fs.srcs[(size_t)i];
    if (!s.index || s.index_nbytes < isz) continue;  // missing, or the planner reports it short
    const int32_t k = slot_of[(size_t)i];
    const uint8_t* ib = s.index + (c.index_location == ZH_INDEX_START ? 0 : s.index_nbytes - isz);
    // the referenced inner chunks' ranges, adjacent ones merged (one pread per run).  Entries
    // beyond a whole shard's file, or longer than a Java buffer (2^31 - 1 bytes: the
    // reference's (int) allocation fails) are left out and read as "Could not load byte data"
    // on the device.
    std::vector<std::pair<int64_t, int64_t>> rs;
    if (shard_ranges(meta, ib, s.shard_nbytes, lo[(size_t)i].data(), hi[(size_t)i].data(),
                     INT64_MAX, rs, kIntMax) != ZH_OK)
      continue;
    auto& pv = fs.pieces[(size_t)i];
    for (auto& r : rs) {
      if (r.first > INT64_MAX - r.second) continue;  // the range's end is not a file offset
      pv.push_back({r.first, r.second, SrcRef::file(k, r.first), r.second});
    }
    s.pieces = pv.data();
    s.npieces = (int64_t)pv.size();
  }
  return ZH_OK;
}

// Files.createDirectories(parent) (FilesystemStore.set, M/store/FilesystemStore.java:107-115):
// every missing directory above `path`.  "" or the failing directory.
std::string make_parents(const std::string& path, int* why) {
  for (size_t k = 1; k < path.size(); k++) {
    if (path[k] != '/') continue;
    const std::string dir = path.substr(0, k);
    if (mkdir(dir.c_str(), 0777) != 0 && errno != EEXIST) {
      const int me = errno;  // mkdir's reason, before stat can change errno
      struct stat sb;
      if (stat(dir.c_str(), &sb) == 0 && S_ISDIR(sb.st_mode)) continue;
      *why = me;
      return dir;
    }
  }
  return "";
}

std::string parent_of(const std::string& path) {
  const size_t k = path.find_last_of('/');
  return k == std::string::npos || k == 0 ? std::string(k == 0 ? "/" : "") : path.substr(0, k);
}

// pwrite of n bytes at off, retried on EINTR / short writes; 0 or the errno.
int write_all(int fd, const uint8_t* p, int64_t n, int64_t off) {
  while (n > 0) {
    const ssize_t w = pwrite(fd, p, (size_t)std::min<int64_t>(n, (int64_t)1 << 30), (off_t)off);
    if (w < 0 && errno == EINTR) continue;
    if (w < 0) return errno;
    if (w == 0) return EIO;
    p += w;
    off += w;
    n -= w;
  }
  return 0;
}

std::atomic<uint64_t> g_tmp_seq{0};

// Where a chunk's bytes go: the chunk's path, or a symlink's target, so that
// the rename replaces the file the link names and not the link (FilesystemStore.set writes
// through it).
std::string write_target(const std::string& path) {
  struct stat sb;
  if (lstat(path.c_str(), &sb) == 0 && S_ISLNK(sb.st_mode)) {
    char buf[PATH_MAX];
    if (realpath(path.c_str(), buf)) return buf;
  }
  return path;
}

// Temporary files "<target>.zhtmp<pid>.<n>" left by a writer process that died part-way: a
// crash would otherwise leave them for FilesystemStore.list to report as keys.  Removed when
// the next write of the same chunk starts (the name's pid no longer runs).
void sweep_stale_tmp(const std::string& target) {
  const size_t slash = target.find_last_of('/');
  const std::string dir = slash == std::string::npos ? "." : target.substr(0, slash);
  const std::string pre =
      (slash == std::string::npos ? target : target.substr(slash + 1)) + ".zhtmp";
  DIR* d = opendir(dir.c_str());
  if (!d) return;
  while (dirent* e = readdir(d)) {
    const std::string name = e->d_name;
    if (name.compare(0, pre.size(), pre) != 0) continue;
    const long pid = strtol(name.c_str() + pre.size(), nullptr, 10);
    if (pid <= 0 || pid == (long)getpid()) continue;
    if (kill((pid_t)pid, 0) != 0 && errno == ESRCH) (void)unlink((dir + "/" + name).c_str());
  }
  closedir(d);
}

}  // namespace

extern "C" {

int zh_array_write_files(zh_ctx* ctx, const zh_array_meta* m, const void* src,
                         const int64_t* offset, const int64_t* shape, const zh_file_store* store,
                         const char* const* paths, int64_t npaths, uint32_t flags,
                         int64_t* nbytes, char* err, size_t errlen) {
  if (!ctx || !m || !src || !offset || !shape || (npaths > 0 && !paths)) return ZH_EINVAL;
  int st = zh_validate_meta(m, err, errlen);
  if (st != ZH_OK) return st;
  for (int64_t i = 0; i < npaths; i++)
    if (!paths[i]) {
      set_err(err, errlen, "chunk path %lld is null", (long long)i);
      return ZH_EINVAL;
    }
  (void)hipSetDevice(ctx->device);
  const std::string sname = store_name(store);
  int64_t rbytes = m->dtype_size;
  for (int d = 0; d < m->ndim; d++) rbytes *= std::max<int64_t>(0, shape[d]);
  const int64_t bound = zh_array_encoded_bound(m);
  void* dsrc = nullptr;
  void* ddst = nullptr;
  size_t gsrc = 0, gdst = 0;
  hipError_t e = hipSuccess;
  if (!(flags & ZH_SRC_DEVICE)) {  // the region to the device (pageable or page-locked)
    e = ctx_alloc(ctx, (size_t)std::max<int64_t>(1, rbytes), &dsrc, &gsrc);
    if (e == hipSuccess) e = hipMemcpy(dsrc, src, (size_t)rbytes, hipMemcpyHostToDevice);
  }
  if (e == hipSuccess)
    e = ctx_alloc(ctx, (size_t)std::max<int64_t>(1, bound * npaths), &ddst, &gdst);
  std::vector<zh_chunk_dst> dsts((size_t)std::max<int64_t>(1, npaths));
  if (e == hipSuccess) {
    for (int64_t i = 0; i < npaths; i++) {
      dsts[(size_t)i].data = (uint8_t*)ddst + i * bound;
      dsts[(size_t)i].capacity = bound;
      dsts[(size_t)i].nbytes = 0;
    }
    // ShardingIndexedCodec.encode of every chunk on the device (all-fill chunks: nbytes 0)
    st = zh_array_write(ctx, m, dsrc ? dsrc : src, offset, shape, dsts.data(), npaths, nullptr,
                        err, errlen);
  }
  if (e == hipSuccess && st == ZH_OK) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    // writeChunk per chunk (M/core/Array.java:143-156): all fill → delete the key
    // (FilesystemStore.delete, :130-143: a missing file is fine); otherwise set (:105-128):
    // the parent directories first (here, for every chunk, before any byte is written)
    std::string last_parent;
    for (int64_t i = 0; st == ZH_OK && i < npaths; i++) {
      const int64_t nb = dsts[(size_t)i].nbytes;
      if (nbytes) nbytes[i] = nb;
      const std::string key = store_key(store, paths[i]);
      if (nb == 0) {
        if (unlink(paths[i]) != 0 && errno != ENOENT) {
          const std::string cause = std::string("Failed to delete file: ") + paths[i];
          set_err(err, errlen, "%s", failed("delete from", sname, key, cause).c_str());
          st = ZH_EIO;
        }
        continue;
      }
      const std::string parent = parent_of(paths[i]);
      if (parent == last_parent) continue;
      int why = 0;
      if (!make_parents(paths[i], &why).empty()) {
        (void)why;
        const std::string cause = "Failed to create parent directories for path: " + parent;
        set_err(err, errlen, "%s", failed("write to", sname, key, cause).c_str());
        st = ZH_EIO;
        break;
      }
      last_parent = parent;
    }
    // the encoded bytes out: windows of the ring size, the copy lanes each D2H'ing one window
    // into a page-locked slot of their own while pwrite-ing the previous one
    int lanes = 1;
    int64_t win = 16 << 20;
    if (st == ZH_OK && (st = pipe_out_ring(ctx, &lanes, &win)) != ZH_OK)
      set_err(err, errlen, "page-locked staging rings: allocation failed");
    struct Job {
      int64_t chunk, off, len;
    };
    // windows taken round-robin over groups of `lanes` chunks: buffered writes to one file
    // serialize on its inode lock, so the lanes spread over the files of a group; a chunk's
    // file is open from its first window's write to its last, so at most 3 * lanes files are
    // open (two undrained windows per lane, plus the group being taken)
    std::vector<Job> jobs;
    for (int64_t g0 = 0; st == ZH_OK && g0 < npaths; g0 += lanes) {
      const int64_t g1 = std::min<int64_t>(npaths, g0 + lanes);
      int64_t most = 0;
      for (int64_t i = g0; i < g1; i++) most = std::max(most, dsts[(size_t)i].nbytes);
      for (int64_t o = 0; o < most; o += win)
        for (int64_t i = g0; i < g1; i++)
          if (o < dsts[(size_t)i].nbytes)
            jobs.push_back({i, o, std::min(win, dsts[(size_t)i].nbytes - o)});
    }
    lanes = (int)std::max<int64_t>(1, std::min<int64_t>(lanes, (int64_t)jobs.size()));
    // per chunk: its temporary file (created by its first write) and the windows still due
    struct Out {
      std::mutex mu;
      int fd = -1;
      std::string tmp, target;  // the temporary file; the file it is renamed over
      int64_t left = 0;
      bool done = false;
    };
    std::unique_ptr<Out[]> outs(new Out[(size_t)std::max<int64_t>(1, npaths)]);
    for (const Job& J : jobs) outs[(size_t)J.chunk].left++;
    std::atomic<size_t> next{0};
    std::atomic<int> fail{ZH_OK};
    std::mutex fmu;
    std::string fmsg;
    auto lane_fail = [&](int code, const std::string& m2) {
      std::lock_guard<std::mutex> g(fmu);
      if (fail.load() == ZH_OK) {
        fail = code;
        fmsg = m2;
      }
    };
    auto write_failed = [&](int64_t i, int eno) {
      (void)eno;
      const std::string cause = "Failed to write " + std::to_string(dsts[(size_t)i].nbytes) +
                                " bytes to file: " + paths[i];
      lane_fail(ZH_EIO, failed("write to", sname, store_key(store, paths[i]), cause));
    };
    // one window into chunk J.chunk's temporary file; the chunk's last window renames it over
    // the chunk's file
    auto put = [&](const Job& J, const uint8_t* bytes) {
      Out& O = outs[(size_t)J.chunk];
      int fd;
      {
        std::lock_guard<std::mutex> g(O.mu);
        if (O.fd < 0) {
          O.target = write_target(paths[J.chunk]);
          sweep_stale_tmp(O.target);
          O.tmp = O.target + ".zhtmp" + std::to_string(getpid()) + "." +
                  std::to_string(g_tmp_seq.fetch_add(1));
          O.fd = open(O.tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
          if (O.fd < 0) {
            write_failed(J.chunk, errno);
            return;
          }
          struct stat old;  // an existing chunk file keeps its permission bits
          if (stat(O.target.c_str(), &old) == 0) (void)fchmod(O.fd, old.st_mode & 07777);
        }
        fd = O.fd;
      }
      const int we = write_all(fd, bytes, J.len, J.off);
      if (we != 0) {
        write_failed(J.chunk, we);
        return;
      }
      std::lock_guard<std::mutex> g(O.mu);
      if (--O.left > 0) return;
      const int ce = close(O.fd) != 0 ? errno : 0;
      O.fd = -1;
      if (ce != 0 || rename(O.tmp.c_str(), O.target.c_str()) != 0) {
        write_failed(J.chunk, ce ? ce : errno);
        unlink(O.tmp.c_str());
        return;
      }
      O.done = true;
    };
    auto lane = [&](int L) {
      (void)hipSetDevice(ctx->device);
      hipEvent_t ev[2] = {nullptr, nullptr};
      for (auto& x : ev)
        if (hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess) {
          lane_fail(ZH_EHIP, "hipEventCreate failed");
          return;
        }
      const Job* pend = nullptr;
      int pslot = 0, flip = 0;
      auto drain = [&]() {
        if (!pend) return;
        if (hipEventSynchronize(ev[pslot]) != hipSuccess)
          lane_fail(ZH_EHIP, "device-to-host copy of an encoded chunk failed");
        else if (fail.load() == ZH_OK)
          put(*pend, (const uint8_t*)ctx->ring_out[(size_t)(2 * L + pslot)]);
        pend = nullptr;
      };
      for (;;) {
        const size_t j = next.fetch_add(1);
        if (j >= jobs.size() || fail.load() != ZH_OK) break;
        const Job& J = jobs[j];
        const int k = flip;
        flip ^= 1;
        void* slot = ctx->ring_out[(size_t)(2 * L + k)];
        if (hipMemcpyAsync(slot, (const uint8_t*)dsts[(size_t)J.chunk].data + J.off,
                           (size_t)J.len, hipMemcpyDeviceToHost, ctx->pipe_out) != hipSuccess ||
            hipEventRecord(ev[k], ctx->pipe_out) != hipSuccess) {
          lane_fail(ZH_EHIP, "device-to-host copy of an encoded chunk failed");
          break;
        }
        drain();  // the previous window (the other slot) while this one copies
        pend = &J;
        pslot = k;
      }
      drain();
      for (auto& x : ev)
        if (x) (void)hipEventDestroy(x);
    };
    if (st == ZH_OK && !jobs.empty()) {
      std::vector<std::thread> th;
      for (int L = 0; L < lanes; L++) th.emplace_back(lane, L);
      for (auto& t : th) t.join();
      if (fail.load() != ZH_OK) {
        st = fail.load();
        set_err(err, errlen, "%s", fmsg.c_str());
      }
    }
    // chunks a failure left unfinished: their temporary files go, their files stay as they were
    for (int64_t i = 0; i < npaths; i++) {
      Out& O = outs[(size_t)i];
      if (O.fd >= 0) close(O.fd);
      if (!O.tmp.empty() && !O.done) unlink(O.tmp.c_str());
    }
  }
  if (dsrc) ctx_release(ctx, dsrc, gsrc);
  if (ddst) ctx_release(ctx, ddst, gdst);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_err(err, errlen, "HIP error %s (%s)", hipGetErrorName(e), hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? ZH_ENOMEM : ZH_EHIP;
  }
  return st;
}

int zh_debug_file_table(int64_t* out) {
  if (!out) return ZH_EINVAL;
  FileTable& t = table();
  std::lock_guard<std::mutex> lk(t.mu);
  out[0] = (int64_t)(t.ent.size() - t.free.size());
  out[1] = t.open;
  out[2] = (int64_t)t.opened.size();
  return ZH_OK;
}

int64_t zh_debug_file_reads(const zh_array_meta* meta, const zh_file_store* store,
                            const char* const* paths, int64_t npaths, const int64_t* offset,
                            const int64_t* shape, int64_t* reads, int64_t cap, char* err,
                            size_t errlen) {
  if (!meta || !offset || !shape || (npaths > 0 && !paths)) return -ZH_EINVAL;
  int st = zh_validate_meta(meta, err, errlen);
  if (st != ZH_OK) return -st;
  FileSources fs;
  st = file_sources(meta, store, paths, npaths, offset, shape, fs, err, errlen);
  if (st != ZH_OK) return -st;
  int64_t k = 0;
  auto put = [&](int64_t i, int64_t off, int64_t n) {
    if (reads && k < cap) {
      reads[3 * k] = i;
      reads[3 * k + 1] = off;
      reads[3 * k + 2] = n;
    }
    k++;
  };
  for (int64_t i = 0; i < npaths; i++) {
    const SrcDesc& s = fs.srcs[(size_t)i];
    if (s.data.is_file()) put(i, 0, s.nbytes);  // a whole object
    if (s.index) {  // the index read: a prefix, or a suffix of the file
      struct stat sb;
      const int64_t size = stat(paths[i], &sb) == 0 ? (int64_t)sb.st_size : 0;
      put(i, meta->chain.index_location == ZH_INDEX_START ? 0 : size - s.index_nbytes,
          s.index_nbytes);
    }
    for (int64_t q = 0; q < s.npieces; q++) put(i, s.pieces[q].offset, s.pieces[q].nbytes);
  }
  return k;
}

int zh_array_read_files(zh_ctx* ctx, const zh_array_meta* meta, const zh_file_store* store,
                        const char* const* paths, int64_t npaths, const int64_t* offset,
                        const int64_t* shape, void* out, uint32_t flags, char* err,
                        size_t errlen) {
  if (!ctx || !meta || !offset || !shape || !out || (npaths > 0 && !paths)) return ZH_EINVAL;
  if (flags & ZH_SRC_DEVICE) {
    set_err(err, errlen, "zh_array_read_files reads host files: ZH_SRC_DEVICE is not allowed");
    return ZH_EINVAL;
  }
  int st = zh_validate_meta(meta, err, errlen);
  if (st != ZH_OK) return st;
  FileSources fs;
  st = file_sources(meta, store, paths, npaths, offset, shape, fs, err, errlen);
  if (st != ZH_OK) return st;
  std::lock_guard<std::mutex> lk(ctx->mu);
  // large reads pipelined (the in lanes pread the ranges into the ring); otherwise one plan,
  // which reads the file bytes into host buffers first
  return read_region(ctx, meta, fs.srcs.data(), npaths, offset, shape, out, flags & ZH_OUT_DEVICE,
                     nullptr, err, errlen);
}

int zh_array_read_files_multi(zh_ctx* const* ctxs, int ndev, int root, const zh_array_meta* meta,
                              const zh_file_store* store, const char* const* paths,
                              int64_t npaths, const int64_t* offset, const int64_t* shape,
                              void* out, uint32_t flags, int32_t* slab_route, char* err,
                              size_t errlen) {
  if (!ctxs || ndev <= 0 || !meta || !offset || !shape || !out || (npaths > 0 && !paths))
    return ZH_EINVAL;
  if (flags & ZH_SRC_DEVICE) {
    set_err(err, errlen, "zh_array_read_files reads host files: ZH_SRC_DEVICE is not allowed");
    return ZH_EINVAL;
  }
  int st = zh_validate_meta(meta, err, errlen);
  if (st != ZH_OK) return st;
  FileSources fs;
  st = file_sources(meta, store, paths, npaths, offset, shape, fs, err, errlen);
  if (st != ZH_OK) return st;
  return read_multi_impl(ctxs, ndev, root, meta, fs.srcs.data(), npaths, offset, shape, out,
                         flags & ZH_OUT_DEVICE, slab_route, err, errlen);
}

}  // extern "C"
