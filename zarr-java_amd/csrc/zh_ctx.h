// zh_ctx.h — host-side state shared by the planner (zh_engine.cpp), the sub-shard source
// forms (zh_pieces.cpp) and the pipelined host read (zh_pipeline.cpp).  Not public ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "zh_internal.h"

// =====================================================================================
// context
// =====================================================================================
struct zh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int cu_count = 256;
  std::mutex mu;
  // write-path scratch (grow-only, under mu; zh_array_write synchronises before it returns)
  uint8_t* wscratch = nullptr;
  size_t wscratch_cap = 0;
  // device blocks released by finished plans, reused by later plans of this context: fresh
  // device memory pays for its first touch (a 2 GiB staging buffer cost ~30 ms in page
  // setup on every one-shot host-output read) and small allocations pay per call
  std::mutex cache_mu;
  std::multimap<size_t, void*> cache;  // block bytes → block
  size_t cache_bytes = 0;
  // pipelined host reads (zh_pipeline.cpp): the copy streams and the page-locked rings the
  // pageable sources / outputs pass through, created on first use and kept
  hipStream_t pipe_in = nullptr, pipe_out = nullptr;
  std::vector<void*> ring_in, ring_out;  // pinned slots
  size_t ring_slot = 0;
  // zh_host_staging: page-locked staging for bindings (the JNI shim)
  void* staging = nullptr;
  size_t staging_cap = 0;
  bool staging_oneoff = false;
  // page-locked slots for the plans' status read-back (zh_plan_wait: one async copy on the
  // plan's stream and one synchronise, instead of a synchronise and a blocking copy)
  std::mutex status_mu;
  uint64_t* status_pin = nullptr;  // kStatusSlots × kStatusSlotWords, created on first use
  std::vector<int> status_free;
  bool status_failed = false;
  // page-locked slots for small plans' table uploads (deferred to the first execute as an
  // async copy on its stream, instead of a blocking pageable copy at plan creation)
  uint8_t* upload_pin = nullptr;   // kUploadSlots × kUploadSlotBytes, created on first use
  std::vector<int> upload_free;
  bool upload_failed = false;
  // page-locked buffer a one-plan read of store files (zh_array_read_files) reads its bytes
  // into, so that the plan's H2D is one DMA; grow-only, used under mu by plans that are
  // created, run and freed while mu is held (read_region, read_multi_impl)
  uint8_t* file_pin = nullptr;
  size_t file_pin_cap = 0;
  // page-locked landing buffer of a small one-plan read into pageable host memory:
  // the D2H goes here as a DMA and one memcpy moves it out; used under mu, created on first use
  uint8_t* hout_pin = nullptr;
  bool hout_pin_failed = false;
};

namespace zh {
constexpr int kStatusSlots = 64;
constexpr int kStatusSlotWords = 192;  // 32 shards × kStWords
constexpr int kUploadSlots = 16;
constexpr size_t kUploadSlotBytes = 64 << 10;
}  // namespace zh

namespace zh {

[[noreturn]] void src_ref_misuse(const char* what);

// Where the bytes of a source range are: memory (a host address, or a device address under
// ZH_SRC_DEVICE), or byte `offset` of a store file open for the read (zh_array_read_files:
// `slot` in zh_files.cpp's file table).  The planner lays both out alike (offsets add,
// adjacent ranges merge); only memory can be dereferenced or DMA'd, and mem() is the one way
// to the address: it refuses a file source, so no host-pointer use can receive one.
class SrcRef {
 public:
  SrcRef() = default;
  static SrcRef memory(const void* p) {
    SrcRef r;
    r.p_ = (const uint8_t*)p;
    return r;
  }
  static SrcRef file(int32_t slot, int64_t offset) {
    SrcRef r;
    r.slot_ = slot;
    r.off_ = offset;
    return r;
  }
  bool is_file() const { return slot_ >= 0; }
  bool empty() const { return slot_ < 0 && p_ == nullptr; }
  const uint8_t* mem() const {
    if (slot_ >= 0) src_ref_misuse("a store file range used as memory");
    return p_;
  }
  int32_t slot() const {
    if (slot_ < 0) src_ref_misuse("memory used as a store file range");
    return slot_;
  }
  int64_t file_offset() const { return off_; }
  SrcRef operator+(int64_t d) const {
    SrcRef r = *this;
    if (slot_ >= 0) r.off_ += d;
    else r.p_ += d;
    return r;
  }
  // this range starts where `prev` (prev_len bytes) ends, in the same memory or file
  bool follows(const SrcRef& prev, int64_t prev_len) const {
    if (slot_ != prev.slot_) return false;
    return slot_ >= 0 ? off_ == prev.off_ + prev_len : p_ == prev.p_ + prev_len;
  }

 private:
  const uint8_t* p_ = nullptr;
  int32_t slot_ = -1;
  int64_t off_ = 0;
};

// One held byte range of a stored shard (zh_shard_piece with a typed source).
struct Piece {
  int64_t offset = 0, nbytes = 0;
  SrcRef data;
  int64_t data_nbytes = 0;
};

// One stored chunk / shard as the planner takes it: a whole object (data, nbytes), or a
// sub-shard form (the stored index + the byte ranges held, zh_shard_src); data empty and
// index == nullptr: the key is missing.  The index is always memory; pieces point into
// storage the entry point owns for the call.
struct SrcDesc {
  SrcRef data;
  int64_t nbytes = 0;
  const uint8_t* index = nullptr;
  int64_t index_nbytes = 0;
  int64_t shard_nbytes = -1;
  const Piece* pieces = nullptr;
  int64_t npieces = 0;
};

}  // namespace zh

struct zh_plan {
  zh_ctx* ctx = nullptr;
  zh_array_meta meta{};
  uint32_t flags = 0;
  int64_t nshards = 0;
  int64_t n_items = 0;          // inner-chunk items (without pieces)
  int64_t in_bytes = 0, out_bytes = 0;
  std::vector<int64_t> coords;  // chunk coords (for messages)
  // device state
  std::vector<std::pair<void*, size_t>> blocks;  // context-cache blocks owned by the plan
  hipEvent_t done_ev = nullptr;  // recorded after every execute (plan_free waits on it)
  uint8_t* d_tables = nullptr;   // one allocation holding the tables below
  zh::DevShard* d_shards = nullptr;
  uint64_t* d_status = nullptr;
  int status_slot = -1;         // the context's page-locked status slot (−1: blocking copy)
  int upload_slot = -1;         // page-locked copy of the tables' prefix (−1: uploaded at create)
  size_t upload_bytes = 0;      // bytes of that prefix: the tables, then zeroed status words
  bool upload_pending = false;  // the next enqueue copies it (and skips the status memset)
  zh::CrcJob* d_crc_jobs = nullptr;
  uint32_t* d_crc_partials = nullptr;
  int64_t n_crc_jobs = 0, n_crc_spans = 0;
  int crc_shift = 0;            // index-CRC span = kIdxSpan << crc_shift
  bool idx_crc_fused = true;    // the index CRC runs in the slow kernel's launch (ZH_IDX_CRC_FUSE)
  bool small_one = false;       // resolve + decode in one launch (ZH_SMALL_ONE, small plans)
  int small_grid = 0;
  uint8_t* d_input = nullptr;   // staged host sources
  std::vector<std::pair<int64_t, zh::SrcRef>> h2d;  // (offset in d_input, host source)
  std::vector<int64_t> h2d_len;
  std::vector<std::unique_ptr<uint8_t[]>> h2d_keep;  // file bytes read for its own h2d copies
  bool external_h2d = false;    // the pipelined read does the h2d copies (plan_enqueue skips)
  bool early_h2d = false;       // plan_create queued the h2d copies on the context's stream
  uint8_t* d_out = nullptr;     // staging when the output is host memory
  zh::ScatterArgs args{};
  zh::ItemDesc* d_desc = nullptr;   // per inner-chunk descriptors (resolve kernel)
  uint32_t* d_slow = nullptr;   // [count, list...] of items for the generic kernel
  uint32_t* d_fast_tab = nullptr;
  uint8_t* d_flat = nullptr;    // nested sharding: flattened leaf indexes
  uint32_t* d_dcrc = nullptr;   // inner crc32c: span partials per chunk
  zh::DataCrcArgs dcrc{};
  int dcrc_grid = 0;
  zh::NestArgs nest{};
  int nest_grid = 0;
  int tile_mode = 0;
  int grid = 0;
  int slow_grid = 0;
  hipStream_t last_stream = nullptr;
  // zh_plan_wait's device-detected data error: its shard (index into coords) and the key
  // that orders it within the shard (~0: the shard index crc32c; else the kStBadChunk key)
  int64_t err_shard = -1;
  uint64_t err_key = 0;
  // hipGraph replay of execute (zh_plan_set_graph)
  bool use_graph = false;
  hipGraphExec_t graph_exec = nullptr;
  void* graph_out = nullptr;
  hipStream_t graph_stream = nullptr;
  // timing
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::array<hipEvent_t, 3>> ev_pending;
};

namespace zh {

constexpr int64_t kIntMax = 2147483647LL;

void set_err(char* err, size_t errlen, const char* fmt, ...);
int env_int(const char* name, int def);
std::string fmt_ints(const int64_t* v, int n);
uint64_t ld_u64_host(const uint8_t* p, bool be);
int64_t chunk_coords(int n, const int32_t* chunk, const int64_t* off, const int64_t* shp,
                     int64_t* start, int64_t* count);
const int32_t* leaf_shape(const zh_array_meta* m);
hipError_t ctx_alloc(zh_ctx* ctx, size_t bytes, void** p, size_t* got);
void ctx_release(zh_ctx* ctx, void* p, size_t bytes);

// Planner over generic sources (zh_plan_create / zh_array_read_pieces); external_h2d: the
// caller copies p->h2d itself (the pipelined read).
int plan_create(zh_ctx* ctx, const zh_array_meta* m, const SrcDesc* srcs, int64_t nchunks,
                const int64_t* offset, const int64_t* shape, uint32_t flags, bool external_h2d,
                zh_plan** out, char* err, size_t errlen);
void plan_free(zh_plan* p);

// The byte ranges of one stored shard a part [part_lo, part_hi) needs (zh_shard_ranges):
// (offset, nbytes) pairs sorted by offset, adjacent runs merged up to max_run bytes; entries
// longer than max_entry bytes are left out.
int shard_ranges(const zh_array_meta* m, const uint8_t* index, int64_t shard_nbytes,
                 const int64_t* part_lo, const int64_t* part_hi, int64_t max_run,
                 std::vector<std::pair<int64_t, int64_t>>& out, int64_t max_entry = INT64_MAX);

// Region read over generic sources: the pipelined path for large host reads (zh_pipeline.cpp),
// else one plan.  Caller holds ctx->mu.
// Where the last data error reported on this thread sits in the oracle's order (DESIGN §3
// Q17): the failing chunk's coords and its key in the shard (zh_plan::err_key).  Set by
// zh_plan_wait and by the pipelined read's pick, cleared by read_region; the multi-device
// read orders its slabs' data errors by it.
struct DataErrPos {
  bool set = false;
  std::vector<int64_t> cc;
  uint64_t key = 0;
};
extern thread_local DataErrPos g_data_err;
// is (a, ka) before (b, kb) in that order?
inline bool data_err_before(const std::vector<int64_t>& a, uint64_t ka,
                            const std::vector<int64_t>& b, uint64_t kb) {
  return a < b || (a == b && ka > kb);
}

int read_region(zh_ctx* ctx, const zh_array_meta* meta, const SrcDesc* srcs, int64_t nsrc,
                const int64_t* offset, const int64_t* shape, void* out, uint32_t flags,
                void* stream, char* err, size_t errlen);
// One plan: create, execute, wait, free.
int read_one_plan(zh_ctx* ctx, const zh_array_meta* meta, const SrcDesc* srcs, int64_t nsrc,
                  const int64_t* offset, const int64_t* shape, void* out, uint32_t flags,
                  void* stream, char* err, size_t errlen);
// Pipelined host read; ZH_EUNSUPPORTED when the region does not qualify or split.
int read_pipelined(zh_ctx* ctx, const zh_array_meta* meta, const SrcDesc* srcs, int64_t nsrc,
                   const int64_t* offset, const int64_t* shape, void* out, uint32_t flags,
                   void* stream, char* err, size_t errlen);
void pipeline_release(zh_ctx* ctx);  // zh_ctx_destroy: streams and rings
// The pipelined read's copy lanes (ZH_PIPE_THREADS) and ring window (ZH_PIPE_CHUNK_KB), with
// both rings holding two slots per lane and the copy streams created (caller holds ctx->mu).
int pipe_out_ring(zh_ctx* ctx, int* lanes, int64_t* window);
// One region over several contexts (zh_array_read_multi_routed / zh_array_read_pieces_multi).
int read_multi_impl(zh_ctx* const* ctxs, int ndev, int root, const zh_array_meta* meta,
                    const SrcDesc* chunks, int64_t nchunks, const int64_t* offset,
                    const int64_t* shape, void* out, uint32_t flags, int32_t* slab_route,
                    char* err, size_t errlen);

// Enqueue one execution of a plan (kernels; the h2d copies unless external_h2d; the d2h copy
// for host outputs) on stream s.
int plan_enqueue_impl(zh_plan* p, void* out, hipStream_t s);
int plan_mark_done_impl(zh_plan* p, hipStream_t s);

int projection(int n, const int64_t* cc, const int64_t* ashape, const int32_t* chunk,
               const int64_t* soff, const int64_t* sshape, int32_t* co, int32_t* oo, int32_t* ps);

// Store files of a read (zh_array_read_files, zh_files.cpp).  A process-wide table holds, per
// file of the reads in flight, its path, the store and key its errors name, and — while a read
// needs it — an open descriptor: at most kFileMaxOpen are open at once (a read of thousands of
// chunk files stays under the process's descriptor limit; a closed one is reopened by path when
// its next range is read).  Sources name file bytes as SrcRef::file(slot, offset).
constexpr int kFileMaxOpen = 64;
// the largest extent a one-plan file read stages in zh_ctx::file_pin
constexpr int64_t kFilePinMax = (int64_t)256 << 20;
// Reads the n bytes at `src` (a file SrcRef) into dst: pread, retried on EINTR and short reads.
// Bytes past the end of the file read as zeros, as FilesystemStore.get(keys, start, end)
// returns a buffer of end - start bytes holding what the file has (M/store/FilesystemStore.java:
// 84-102).  Returns "" or StoreException.readFailed's text (StoreException.java:17-21).
std::string file_fetch(void* dst, const SrcRef& src, int64_t n);
struct FileRead {
  void* dst;
  SrcRef src;
  int64_t n;
};
// file_fetch of every read in order: the small reads a plan stages itself and the shards'
// indexes.  "" or the first failure's message.
std::string file_fetch_all(const std::vector<FileRead>& reads);

}  // namespace zh
