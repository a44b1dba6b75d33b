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
// (zh_ctx.h) into a process-wide table of open files, so one read may span several contexts
// (zh_array_read_files_multi); the planner lays file bytes out like any host bytes and reads
// them itself only for a plan that stages its own copies (not pipelined).
//
// zh_array_write_files is the write side: the device encode, then writeChunk's store calls
// (FilesystemStore.set / delete) here, the encoded bytes D2H'd through the page-locked ring in
// windows that the copy lanes pwrite straight into the chunk files.
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "zh_ctx.h"

namespace {

// The process-wide table of the store files open for reads in flight: slot → (fd, path).
// Slots are taken and given back per read; file addresses name a slot.
struct FileSlots {
  std::mutex mu;
  std::vector<int> fd;
  std::vector<std::string> path;
  std::vector<int64_t> free;
};

FileSlots& slots() {
  static FileSlots s;
  return s;
}

int64_t slot_take(int fd, const char* path) {
  FileSlots& s = slots();
  std::lock_guard<std::mutex> lk(s.mu);
  int64_t k;
  if (!s.free.empty()) {
    k = s.free.back();
    s.free.pop_back();
    s.fd[(size_t)k] = fd;
    s.path[(size_t)k] = path;
  } else {
    if ((int64_t)s.fd.size() >= zh::kFileMaxSlots) return -1;
    k = (int64_t)s.fd.size();
    s.fd.push_back(fd);
    s.path.push_back(path);
  }
  return k;
}

void slot_give(int64_t k) {
  FileSlots& s = slots();
  std::lock_guard<std::mutex> lk(s.mu);
  if (s.fd[(size_t)k] >= 0) close(s.fd[(size_t)k]);
  s.fd[(size_t)k] = -1;
  s.path[(size_t)k].clear();
  s.free.push_back(k);
}

}  // namespace

namespace zh {

std::string file_fetch(void* dst, const void* src, int64_t n) {
  const uint64_t a = (uint64_t)(uintptr_t)src & ~kFileTag;
  const size_t k = (size_t)(a >> kFileOffBits);
  int64_t off = (int64_t)(a & ((1ull << kFileOffBits) - 1));
  int fd = -1;
  {
    FileSlots& s = slots();
    std::lock_guard<std::mutex> lk(s.mu);
    if (k < s.fd.size()) fd = s.fd[k];
  }
  if (fd < 0) return "a file source that no read has open";
  uint8_t* d = (uint8_t*)dst;
  while (n > 0) {
    const ssize_t r = pread(fd, d, (size_t)std::min<int64_t>(n, (int64_t)1 << 30), (off_t)off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) {  // an error, or the file ended (it shrank after its size was taken)
      const std::string why = r < 0 ? strerror(errno) : "unexpected end of file";
      FileSlots& s = slots();
      std::lock_guard<std::mutex> lk(s.mu);
      return "Failed to read from store at '" + s.path[k] + "': " + why;
    }
    d += r;
    off += r;
    n -= r;
  }
  return "";
}

namespace {

// A small pool of reader threads for file_fetch_all, created on first use and kept: a read
// below the pipeline threshold would otherwise pay a thread start per call.
struct ReadPool {
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::vector<std::thread> th;
  std::vector<FileRead> q;
  size_t next = 0, finished = 0, total = 0;
  std::string fail;
  bool stop = false;
  ~ReadPool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  void worker() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stop || next < q.size(); });
      if (stop) return;
      const FileRead r = q[next++];
      lk.unlock();
      const std::string m = file_fetch(r.dst, r.src, r.n);
      lk.lock();
      if (!m.empty() && fail.empty()) fail = m;
      if (++finished == total) done_cv.notify_all();
    }
  }
};

ReadPool& read_pool(int want) {
  static ReadPool p;
  std::lock_guard<std::mutex> lk(p.mu);
  while ((int)p.th.size() < want) p.th.emplace_back([] { read_pool(0).worker(); });
  return p;
}

std::mutex g_pool_call;  // one batch at a time

}  // namespace

std::string file_fetch_all(const std::vector<FileRead>& reads) {
  constexpr int64_t kPiece = 512 << 10;
  std::vector<FileRead> pieces;
  for (const FileRead& r : reads)
    for (int64_t o = 0; o < r.n; o += kPiece)
      pieces.push_back({(uint8_t*)r.dst + o, (const uint8_t*)r.src + o, std::min(kPiece, r.n - o)});
  const int threads = std::min(32, std::max(1, env_int("ZH_FILE_THREADS", 1)));
  if (pieces.size() <= 1 || threads <= 1) {
    for (const FileRead& r : pieces) {
      const std::string m = file_fetch(r.dst, r.src, r.n);
      if (!m.empty()) return m;
    }
    return "";
  }
  std::lock_guard<std::mutex> call(g_pool_call);
  ReadPool& p = read_pool(threads);
  std::unique_lock<std::mutex> lk(p.mu);
  p.q = std::move(pieces);
  p.next = p.finished = 0;
  p.total = p.q.size();
  p.fail.clear();
  p.cv.notify_all();
  p.done_cv.wait(lk, [&] { return p.finished == p.total; });
  std::string m = p.fail;
  p.q.clear();
  p.next = p.total = p.finished = 0;
  return m;
}

}  // namespace zh

using namespace zh;

namespace {

// The files of one read, open for its duration: their slots go back (and the files are closed)
// on every exit.
struct FileSet {
  std::vector<int64_t> taken;
  ~FileSet() {
    for (int64_t k : taken) slot_give(k);
  }
};

// Sources for a read of the files `paths` (computeChunkCoords order of [offset, offset+shape)):
// per file the reference's store reads up to the ranges (open / exists, the stored index), the
// ranges as file addresses.  index / pieces hold what the sources point into.
int file_sources(const zh_array_meta* meta, const char* const* paths, int64_t npaths,
                 const int64_t* offset, const int64_t* shape, FileSet& set,
                 std::vector<SrcDesc>& srcs, std::vector<std::vector<uint8_t>>& index,
                 std::vector<std::vector<zh_shard_piece>>& pieces, char* err, size_t errlen) {
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
  srcs.assign((size_t)npaths, SrcDesc());
  index.assign((size_t)npaths, {});
  pieces.assign((size_t)npaths, {});
  int64_t cur[kMaxDims] = {0};
  std::vector<FileRead> ireads;
  std::vector<int64_t> slot_of((size_t)npaths, -1);  // the file's slot in the table
  for (int64_t i = 0; i < npaths; i++) {
    const char* path = paths[i];
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
    struct stat sb;
    if (fstat(fd, &sb) != 0) {
      const int fe = errno;
      close(fd);
      set_err(err, errlen, "Failed to read from store at '%s': %s", path, strerror(fe));
      return ZH_EIO;
    }
    if (!S_ISREG(sb.st_mode)) {  // Files.isRegularFile (FilesystemStore.java:44-46)
      close(fd);
      continue;
    }
    const int64_t size = (int64_t)sb.st_size;
    const int64_t k = size < kFileMaxBytes ? slot_take(fd, path) : -1;
    if (k < 0) {
      close(fd);
      set_err(err, errlen, "'%s': %s", path,
              size < kFileMaxBytes ? "too many store files open for reads at once"
                                   : "file larger than a file address can name");
      return ZH_EUNSUPPORTED;
    }
    set.taken.push_back(k);
    slot_of[(size_t)i] = k;
    SrcDesc& s = srcs[(size_t)i];
    if (!c.sharded) {  // get(keys): the whole object
      s.data = file_addr(k, 0);
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
    ireads.push_back({ib.data(), file_addr(k, ioff), ilen});
    s.index = ib.data();
    s.index_nbytes = ilen;
    s.shard_nbytes = size;
  }
  // every shard's index in one batch (file_fetch_all), then the ranges from each
  const std::string m = file_fetch_all(ireads);
  if (!m.empty()) {
    set_err(err, errlen, "%s", m.c_str());
    return ZH_EIO;
  }
  std::fill(cur, cur + kMaxDims, 0);
  for (int64_t i = 0; c.sharded && i < npaths; i++) {
    int64_t cc[kMaxDims];
    for (int d = 0; d < n; d++) cc[d] = cstart[d] + cur[d];
    for (int d = n - 1; d >= 0; d--) {
      if (++cur[d] < ccount[d]) break;
      cur[d] = 0;
    }
    SrcDesc& s = srcs[(size_t)i];
    if (!s.index || s.index_nbytes < isz) continue;  // missing, or the planner reports it short
    const int64_t k = slot_of[(size_t)i];
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
    if (shard_ranges(meta, s.index, s.shard_nbytes, lo, hi, INT64_MAX, rs) != ZH_OK) continue;
    for (auto& r : rs) pieces[(size_t)i].push_back({r.first, r.second, file_addr(k, r.first), r.second});
    s.pieces = pieces[(size_t)i].data();
    s.npieces = (int64_t)pieces[(size_t)i].size();
  }
  return ZH_OK;
}

// Files.createDirectories(parent) (FilesystemStore.set, M/store/FilesystemStore.java:106-115):
// every missing directory above `path`.  "" or the failure's message.
std::string make_parents(const char* path) {
  std::string p(path);
  for (size_t k = 1; k < p.size(); k++) {
    if (p[k] != '/') continue;
    const std::string dir = p.substr(0, k);
    if (mkdir(dir.c_str(), 0777) != 0 && errno != EEXIST) {
      struct stat sb;
      if (stat(dir.c_str(), &sb) == 0 && S_ISDIR(sb.st_mode)) continue;
      return "Failed to create parent directories for path: " + dir + ": " + strerror(errno);
    }
  }
  return "";
}

// pwrite of n bytes at off, retried on EINTR / short writes; "" or strerror.
std::string write_all(int fd, const uint8_t* p, int64_t n, int64_t off) {
  while (n > 0) {
    const ssize_t w = pwrite(fd, p, (size_t)std::min<int64_t>(n, (int64_t)1 << 30), (off_t)off);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return w < 0 ? strerror(errno) : "no progress";
    p += w;
    off += w;
    n -= w;
  }
  return "";
}

}  // namespace

extern "C" {

int zh_array_write_files(zh_ctx* ctx, const zh_array_meta* m, const void* src,
                         const int64_t* offset, const int64_t* shape, const char* const* paths,
                         int64_t npaths, uint32_t flags, int64_t* nbytes, char* err,
                         size_t errlen) {
  if (!ctx || !m || !src || !offset || !shape || (npaths > 0 && !paths)) return ZH_EINVAL;
  int st = zh_validate_meta(m, err, errlen);
  if (st != ZH_OK) return st;
  for (int64_t i = 0; i < npaths; i++)
    if (!paths[i]) {
      set_err(err, errlen, "chunk path %lld is null", (long long)i);
      return ZH_EINVAL;
    }
  (void)hipSetDevice(ctx->device);
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
  std::vector<int> fds((size_t)std::max<int64_t>(1, npaths), -1);
  if (e == hipSuccess && st == ZH_OK) {
    std::lock_guard<std::mutex> lk(ctx->mu);
    // writeChunk per chunk (M/core/Array.java:143-156): all fill → delete the key
    // (FilesystemStore.delete: a missing file is fine), else set: the parent directories, then
    // the file created or truncated and written
    for (int64_t i = 0; st == ZH_OK && i < npaths; i++) {
      const int64_t nb = dsts[(size_t)i].nbytes;
      if (nbytes) nbytes[i] = nb;
      if (nb == 0) {
        if (unlink(paths[i]) != 0 && errno != ENOENT) {
          set_err(err, errlen, "Failed to delete from store at '%s': %s", paths[i],
                  strerror(errno));
          st = ZH_EIO;
        }
        continue;
      }
      std::string msg = make_parents(paths[i]);
      int fd = -1;
      if (msg.empty()) {
        fd = open(paths[i], O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
        if (fd < 0) msg = strerror(errno);
      }
      if (!msg.empty()) {
        set_err(err, errlen, "Failed to write to store at '%s': %s", paths[i], msg.c_str());
        st = ZH_EIO;
        break;
      }
      fds[(size_t)i] = fd;
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
    // windows taken round-robin over the chunks: buffered writes to one file serialize on its
    // inode lock, so the lanes spread over as many files as the write has
    std::vector<Job> jobs;
    int64_t most = 0;
    for (int64_t i = 0; st == ZH_OK && i < npaths; i++)
      most = std::max(most, dsts[(size_t)i].nbytes);
    for (int64_t o = 0; st == ZH_OK && o < most; o += win)
      for (int64_t i = 0; i < npaths; i++)
        if (o < dsts[(size_t)i].nbytes)
          jobs.push_back({i, o, std::min(win, dsts[(size_t)i].nbytes - o)});
    lanes = (int)std::max<int64_t>(1, std::min<int64_t>(lanes, (int64_t)jobs.size()));
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
        if (hipEventSynchronize(ev[pslot]) != hipSuccess) {
          lane_fail(ZH_EHIP, "device-to-host copy of an encoded chunk failed");
        } else {
          const std::string w = write_all(fds[(size_t)pend->chunk],
                                          (const uint8_t*)ctx->ring_out[(size_t)(2 * L + pslot)],
                                          pend->len, pend->off);
          if (!w.empty())
            lane_fail(ZH_EIO, std::string("Failed to write to store at '") + paths[pend->chunk] +
                                  "': " + w);
        }
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
    for (size_t i = 0; i < fds.size(); i++) {
      if (fds[i] < 0) continue;
      if (close(fds[i]) != 0 && st == ZH_OK) {
        set_err(err, errlen, "Failed to write to store at '%s': %s", paths[i], strerror(errno));
        st = ZH_EIO;
      }
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

int64_t zh_debug_file_reads(const zh_array_meta* meta, const char* const* paths, int64_t npaths,
                            const int64_t* offset, const int64_t* shape, int64_t* reads,
                            int64_t cap, char* err, size_t errlen) {
  if (!meta || !offset || !shape || (npaths > 0 && !paths)) return -ZH_EINVAL;
  int st = zh_validate_meta(meta, err, errlen);
  if (st != ZH_OK) return -st;
  FileSet set;
  std::vector<SrcDesc> srcs;
  std::vector<std::vector<uint8_t>> index;
  std::vector<std::vector<zh_shard_piece>> pieces;
  st = file_sources(meta, paths, npaths, offset, shape, set, srcs, index, pieces, err, errlen);
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
    const SrcDesc& s = srcs[(size_t)i];
    if (s.data) put(i, 0, s.nbytes);  // a whole object
    if (s.index)  // the index read: a prefix, or the last index_nbytes bytes
      put(i, meta->chain.index_location == ZH_INDEX_START ? 0 : s.shard_nbytes - s.index_nbytes,
          s.index_nbytes);
    for (int64_t q = 0; q < s.npieces; q++) put(i, s.pieces[q].offset, s.pieces[q].nbytes);
  }
  return k;
}

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
  FileSet set;
  std::vector<SrcDesc> srcs;
  std::vector<std::vector<uint8_t>> index;
  std::vector<std::vector<zh_shard_piece>> pieces;
  st = file_sources(meta, paths, npaths, offset, shape, set, srcs, index, pieces, err, errlen);
  if (st != ZH_OK) return st;
  std::lock_guard<std::mutex> lk(ctx->mu);
  // large reads pipelined (the in lanes pread the ranges into the ring); otherwise one plan,
  // which reads the file bytes into host buffers first
  return read_region(ctx, meta, srcs.data(), npaths, offset, shape, out, flags & ZH_OUT_DEVICE,
                     nullptr, err, errlen);
}

int zh_array_read_files_multi(zh_ctx* const* ctxs, int ndev, int root, const zh_array_meta* meta,
                              const char* const* paths, int64_t npaths, const int64_t* offset,
                              const int64_t* shape, void* out, uint32_t flags,
                              int32_t* slab_route, char* err, size_t errlen) {
  if (!ctxs || ndev <= 0 || !meta || !offset || !shape || !out || (npaths > 0 && !paths))
    return ZH_EINVAL;
  if (flags & ZH_SRC_DEVICE) {
    set_err(err, errlen, "zh_array_read_files reads host files: ZH_SRC_DEVICE is not allowed");
    return ZH_EINVAL;
  }
  int st = zh_validate_meta(meta, err, errlen);
  if (st != ZH_OK) return st;
  FileSet set;
  std::vector<SrcDesc> srcs;
  std::vector<std::vector<uint8_t>> index;
  std::vector<std::vector<zh_shard_piece>> pieces;
  st = file_sources(meta, paths, npaths, offset, shape, set, srcs, index, pieces, err, errlen);
  if (st != ZH_OK) return st;
  return read_multi_impl(ctxs, ndev, root, meta, srcs.data(), npaths, offset, shape, out,
                         flags & ZH_OUT_DEVICE, slab_route, err, errlen);
}

}  // extern "C"
