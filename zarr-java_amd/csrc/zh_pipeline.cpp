// zh_pipeline.cpp — pipelined host-terminated region reads.
//
// The reference's read starts and ends in host memory: store bytes in, a ucar.ma2.Array on
// the Java heap out (M/core/Array.java:397-441, HipArray.read).  A one-plan read runs its
// copies and its decode back to back: H2D of every source, then the kernels, then the D2H,
// each through the runtime's pageable staging when the caller's memory is not page-locked.
// Here the region is split into C-order slabs along its first axis of extent >= 2 (all
// earlier axes of extent 1, so a slab is one contiguous part of the output), at inner-chunk
// boundaries so that no stored chunk is read by two slabs, and three stages run concurrently:
//
//   in lanes   pageable sources: memcpy (several host threads) into page-locked ring slots,
//              one DMA per slot-sized window of the slab's device staging; page-locked
//              sources: DMA straight from them                        (stream pipe_in)
//   decode     slab r's plan (index crc32c, resolve, scatter) once its copies are in; into
//              the output (device) or a device slot (host output)     (the call's stream)
//   out lanes  DMA of the decoded slab into ring slots and memcpy into the caller's pageable
//              output, or straight into a page-locked output           (stream pipe_out)
//
// so both PCIe directions, the host copies and the kernels overlap.  Each slab is planned
// over only the chunks it touches, and a sub-shard part stages only the ranges it references
// (zh_engine.cpp caller_pieces / compact_pieces).  At most 4 slab plans are
// alive, so their device staging cycles through the context's block cache.  Errors: a data
// error the device finds (a checksum, an index entry) does not stop the read; of all of them
// the one reported is the first in the oracle's order — the chunk first in C order, then the
// error the one-plan read would report in it — since slabs can cut a shard
// into parts.  A planning failure at slab r runs slabs < r and reports a data error among
// them first, as the one-plan read would; HIP and store-read failures stop the read.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "zh_ctx.h"

namespace zh {
namespace {

struct PipeCfg {
  int64_t min_bytes;   // host bytes (sources + output) below which one plan is used
  int64_t dout_min_bytes;  // the same for device sources and a host output
  int64_t slab_bytes;  // output (or input) bytes per slab
  int64_t chunk;       // bytes per ring slot / DMA window
  int threads;         // memcpy lanes per direction
  int dslots;          // device output slots (host outputs)
};

PipeCfg pipe_cfg() {
  PipeCfg c;
  const int min_kb = std::max(0, env_int("ZH_PIPE_MIN_KB", 64 << 10));
  c.min_bytes = (int64_t)min_kb << 10;
  // device sources, host output: only the D2H has anything to overlap with, and one plan (its
  // D2H a DMA into pinned memory or the runtime's pageable copy, ~49 GiB/s) measured faster up
  // to 512 MiB (46.6 vs 30.7 GiB/s at 64 MiB, 49.1 vs 43.9 at 512 MiB, profiles/r05/mid/)
  c.dout_min_bytes = c.min_bytes * 16;
  c.slab_bytes = (int64_t)std::max(4, env_int("ZH_PIPE_SLAB_KB", 128 << 10)) << 10;
  c.chunk = (int64_t)std::max(64, env_int("ZH_PIPE_CHUNK_KB", 16 << 10)) << 10;
  c.threads = std::min(16, std::max(1, env_int("ZH_PIPE_THREADS", 6)));
  c.dslots = 3;
  return c;
}

// Page-locked host memory (hipHostMalloc'd or hipHostRegister'd) can be DMA'd directly.
bool host_pinned(const void* p) {
  hipPointerAttribute_t a;
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Per-slab completion flags the stages wait on; abort() wakes every waiter (a failed stage).
struct Flags {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<char> v;
  bool aborted = false;
  explicit Flags(size_t n) : v(n, 0) {}
  void set(size_t i) {
    std::lock_guard<std::mutex> lk(mu);
    v[i] = 1;
    cv.notify_all();
  }
  bool wait(size_t i) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return v[i] || aborted; });
    return v[i] && !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
};

// One host → device copy job: a direct DMA from page-locked memory, or a window of a plan's
// device staging assembled in a ring slot from (offset in window, source, bytes) parts.
struct InJob {
  int64_t slab;
  uint8_t* dst;
  int64_t len;
  const void* direct;  // non-null: DMA from here
  std::vector<std::pair<int64_t, std::pair<SrcRef, int64_t>>> parts;
};

// One device → host copy job of a decoded slab.
struct OutJob {
  int64_t slab;
  const uint8_t* src;  // device
  uint8_t* dst;        // caller's host output
  int64_t len;
};

// Splits the plan's h2d list into jobs: page-locked entries of at least kDirectMin (1 MiB) go
// as their own DMA; the rest is packed into windows of at most `chunk` bytes of the staging.
void in_jobs(zh_plan* p, int64_t slab, int64_t chunk, std::vector<InJob>& jobs,
             bool* any_pageable) {
  constexpr int64_t kDirectMin = 1 << 20;
  InJob cur;
  cur.slab = slab;
  cur.dst = nullptr;
  cur.len = 0;
  cur.direct = nullptr;
  int64_t wstart = 0;
  auto flush = [&] {
    if (cur.dst) jobs.push_back(std::move(cur));
    cur = InJob();
    cur.slab = slab;
    cur.dst = nullptr;
    cur.len = 0;
    cur.direct = nullptr;
  };
  for (size_t k = 0; k < p->h2d.size(); k++) {
    const int64_t off = p->h2d[k].first, len = p->h2d_len[k];
    const SrcRef& src = p->h2d[k].second;
    if (len <= 0) continue;
    if (len >= kDirectMin && !src.is_file() && host_pinned(src.mem())) {
      flush();  // a window must not span (and overwrite) a directly copied range
      jobs.push_back(InJob{slab, p->d_input + off, len, src.mem(), {}});
      continue;
    }
    *any_pageable = true;
    int64_t done = 0;
    while (done < len) {
      const int64_t at = off + done;
      if (cur.dst && at - wstart >= chunk) flush();
      if (!cur.dst) {
        wstart = at;
        cur.dst = p->d_input + at;
      }
      const int64_t take = std::min(len - done, chunk - (at - wstart));
      cur.parts.push_back({at - wstart, {src + done, take}});
      cur.len = at - wstart + take;
      done += take;
    }
  }
  flush();
}

// memcpy over `n` bytes split between the calling lane only (each lane is one thread; the
// lanes run their jobs concurrently).
inline void copy_bytes(void* dst, const void* src, int64_t n) { memcpy(dst, src, (size_t)n); }

int ensure_pipe(zh_ctx* ctx, int slots, size_t slot_bytes) {
  if (!ctx->pipe_in && hipStreamCreateWithFlags(&ctx->pipe_in, hipStreamNonBlocking) != hipSuccess)
    return ZH_EHIP;
  if (!ctx->pipe_out && hipStreamCreateWithFlags(&ctx->pipe_out, hipStreamNonBlocking) != hipSuccess)
    return ZH_EHIP;
  if (ctx->ring_slot != slot_bytes) {  // a new slot size (ZH_PIPE_CHUNK_KB changed): rebuild
    for (void* q : ctx->ring_in) (void)hipHostFree(q);
    for (void* q : ctx->ring_out) (void)hipHostFree(q);
    ctx->ring_in.clear();
    ctx->ring_out.clear();
    ctx->ring_slot = slot_bytes;
  }
  for (auto* ring : {&ctx->ring_in, &ctx->ring_out}) {
    while ((int)ring->size() < slots) {
      void* q = nullptr;
      if (hipHostMalloc(&q, slot_bytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return ZH_ENOMEM;
      }
      ring->push_back(q);
    }
  }
  return ZH_OK;
}

}  // namespace

int pipe_out_ring(zh_ctx* ctx, int* lanes, int64_t* window) {
  const PipeCfg c = pipe_cfg();
  *lanes = c.threads;
  *window = c.chunk;
  return ensure_pipe(ctx, 2 * c.threads, (size_t)c.chunk);
}

void pipeline_release(zh_ctx* ctx) {
  if (!ctx) return;
  for (void* q : ctx->ring_in) (void)hipHostFree(q);
  for (void* q : ctx->ring_out) (void)hipHostFree(q);
  ctx->ring_in.clear();
  ctx->ring_out.clear();
  if (ctx->pipe_in) (void)hipStreamDestroy(ctx->pipe_in);
  if (ctx->pipe_out) (void)hipStreamDestroy(ctx->pipe_out);
  ctx->pipe_in = ctx->pipe_out = nullptr;
  if (ctx->staging) (void)hipHostFree(ctx->staging);
  ctx->staging = nullptr;
  ctx->staging_cap = 0;
}

int read_pipelined(zh_ctx* ctx, const zh_array_meta* meta, const SrcDesc* srcs, int64_t nsrc,
                   const int64_t* offset, const int64_t* shape, void* out, uint32_t flags,
                   void* stream_v, char* err, size_t errlen) {
  const int n = meta->ndim;
  if (n <= 0 || n > kMaxDims || zh_validate_meta(meta, nullptr, 0) != ZH_OK)
    return ZH_EUNSUPPORTED;
  const bool host_out = !(flags & ZH_OUT_DEVICE), host_in = !(flags & ZH_SRC_DEVICE);
  if (!host_out && !host_in) return ZH_EUNSUPPORTED;
  int64_t nel = 1;
  for (int d = 0; d < n; d++) {
    if (offset[d] < 0 || shape[d] <= 0 || offset[d] + shape[d] > meta->shape[d])
      return ZH_EUNSUPPORTED;  // the one-plan path reports it
    nel *= shape[d];
  }
  const int64_t obytes = nel * meta->dtype_size;
  int64_t ibytes = 0;
  if (host_in)
    for (int64_t i = 0; i < nsrc && srcs; i++) {
      ibytes += srcs[i].nbytes + srcs[i].index_nbytes;
      for (int64_t k = 0; k < srcs[i].npieces; k++) ibytes += srcs[i].pieces[k].data_nbytes;
    }
  const PipeCfg cfg = pipe_cfg();
  const int64_t host_bytes = (host_out ? obytes : 0) + ibytes;
  if (host_bytes < (host_in ? cfg.min_bytes : cfg.dout_min_bytes)) return ZH_EUNSUPPORTED;
  {
    int64_t cs[kMaxDims], cc[kMaxDims];  // the caller's list must match the whole region
    if (chunk_coords(n, meta->chunk_shape, offset, shape, cs, cc) != nsrc || !srcs)
      return ZH_EUNSUPPORTED;
  }
  // split axis: the first of extent >= 2, all earlier of extent 1 (contiguous output slabs)
  int ax = -1;
  for (int d = 0; d < n; d++) {
    if (shape[d] >= 2) {
      ax = d;
      break;
    }
  }
  if (ax < 0) return ZH_EUNSUPPORTED;
  // slab boundaries on the chunks the outer index addresses (the inner chunk; a level-1 cell
  // with nested sharding; the chunk unsharded), so no stored chunk is read by two slabs
  const int64_t unit =
      meta->chain.sharded ? meta->chain.inner_chunk_shape[ax] : meta->chunk_shape[ax];
  const int64_t a0 = offset[ax], a1 = offset[ax] + shape[ax];
  const int64_t u0 = a0 / unit, u1 = (a1 + unit - 1) / unit, nu = u1 - u0;
  const int64_t big = std::max(host_out ? obytes : 0, ibytes);
  int64_t want = (big + cfg.slab_bytes - 1) / cfg.slab_bytes;
  // at least 8 slabs of >= 8 MiB: a read of a few hundred MiB (the JNI shim's bounded slabs,
  // §1 "The JNI shim") otherwise ran as 2 slabs with H2D, decode and D2H barely overlapped
  want = std::max(want, std::min<int64_t>(8, big / ((int64_t)8 << 20)));
  const int64_t nslab = std::min<int64_t>(std::max<int64_t>(want, 2), nu);
  if (nslab < 2) return ZH_EUNSUPPORTED;
  std::vector<int64_t> bound((size_t)nslab + 1);
  for (int64_t r = 0; r <= nslab; r++)
    bound[(size_t)r] = std::min(a1, std::max(a0, (u0 + nu * r / nslab) * unit));
  int64_t rstride[kMaxDims], cstart[kMaxDims], ccount[kMaxDims], cstride[kMaxDims];
  {
    int64_t s1 = 1, s2 = 1;
    chunk_coords(n, meta->chunk_shape, offset, shape, cstart, ccount);
    for (int d = n - 1; d >= 0; d--) {
      rstride[d] = s1;
      s1 *= shape[d];
      cstride[d] = s2;
      s2 *= ccount[d];
    }
  }
  (void)hipSetDevice(ctx->device);
  hipStream_t sdec = stream_v ? (hipStream_t)stream_v : ctx->stream;
  // ---- slab geometry: offset, shape, output byte range, sources (host work only)
  struct Slab {
    int64_t o[kMaxDims], s[kMaxDims];
    int64_t obase, obytes;
    std::vector<SrcDesc> sub;
  };
  std::vector<Slab> slabs((size_t)nslab);
  int64_t max_slab = 0;
  for (int64_t r = 0; r < nslab; r++) {
    Slab& S = slabs[(size_t)r];
    for (int d = 0; d < n; d++) {
      S.o[d] = offset[d];
      S.s[d] = shape[d];
    }
    S.o[ax] = bound[(size_t)r];
    S.s[ax] = bound[(size_t)r + 1] - bound[(size_t)r];
    int64_t st0[kMaxDims], cnt[kMaxDims];
    const int64_t m = chunk_coords(n, meta->chunk_shape, S.o, S.s, st0, cnt);
    S.sub.resize((size_t)m);
    int64_t cur[kMaxDims] = {0};
    for (int64_t i = 0; i < m; i++) {
      int64_t lin = 0;
      for (int d = 0; d < n; d++) lin += (st0[d] + cur[d] - cstart[d]) * cstride[d];
      S.sub[(size_t)i] = srcs[lin];
      for (int d = n - 1; d >= 0; d--) {
        if (++cur[d] < cnt[d]) break;
        cur[d] = 0;
      }
    }
    int64_t base = 0, sb = meta->dtype_size;
    for (int d = 0; d < n; d++) {
      base += (S.o[d] - offset[d]) * rstride[d];
      sb *= S.s[d];
    }
    S.obase = base * meta->dtype_size;
    S.obytes = sb;
    max_slab = std::max(max_slab, sb);
  }
  // At most `W` slab plans are alive: each holds its device staging, which then comes back
  // from the context's block cache for the next slab and the next call (fresh device memory
  // pays for its first touch: all slabs' staging at once cost ~15 ms per GiB on every call).
  const int W = 4;
  std::vector<zh_plan*> plans((size_t)nslab, nullptr);
  int st = ZH_OK;
  hipError_t he = hipSuccess;
  const bool out_pinned = host_out && host_pinned(out);
  std::vector<void*> dslot;
  std::vector<size_t> dslot_got;
  const int nds = host_out ? (int)std::min<int64_t>(cfg.dslots, nslab) : 0;
  for (int k = 0; k < nds && he == hipSuccess; k++) {
    void* q = nullptr;
    size_t got = 0;
    he = ctx_alloc(ctx, (size_t)max_slab, &q, &got);
    if (he == hipSuccess) {
      dslot.push_back(q);
      dslot_got.push_back(got);
    }
  }
  std::vector<OutJob> ojobs;
  std::vector<int64_t> out_total((size_t)nslab, 0);
  if (nds > 0 && he == hipSuccess)
    for (int64_t r = 0; r < nslab; r++) {
      const Slab& S = slabs[(size_t)r];
      const uint8_t* dsrc = (const uint8_t*)dslot[(size_t)(r % nds)];
      const int64_t step = out_pinned ? S.obytes : cfg.chunk;
      for (int64_t o = 0; o < S.obytes; o += step) {
        ojobs.push_back(OutJob{r, dsrc + o, (uint8_t*)out + S.obase + o, std::min(step, S.obytes - o)});
        out_total[(size_t)r]++;
      }
    }
  const int lanes_in = host_in ? cfg.threads : 0;
  const int lanes_out = ojobs.empty() ? 0 : (out_pinned ? 1 : cfg.threads);
  if (he == hipSuccess && (lanes_in || lanes_out)) {
    st = ensure_pipe(ctx, 2 * std::max(lanes_in, lanes_out), (size_t)cfg.chunk);
    if (st != ZH_OK) set_err(err, errlen, "page-locked staging rings: allocation failed");
  }
  std::vector<hipEvent_t> in_ev((size_t)nslab, nullptr), dec_ev((size_t)nslab, nullptr),
      out_ev((size_t)nslab, nullptr);
  std::vector<hipEvent_t> slot_ev;
  auto mk = [&](hipEvent_t* e) {
    if (he == hipSuccess) he = hipEventCreateWithFlags(e, hipEventDisableTiming);
  };
  for (int64_t r = 0; r < nslab; r++) {
    mk(&in_ev[(size_t)r]);
    mk(&dec_ev[(size_t)r]);
    mk(&out_ev[(size_t)r]);
  }
  // ring slot events: in lanes use [0, E), out lanes [E, 2E) (slot k of each ring)
  const int E = 2 * std::max(lanes_in, lanes_out);
  slot_ev.assign((size_t)(2 * E), nullptr);
  for (auto& e : slot_ev) mk(&e);
  Flags fin((size_t)nslab), fdec((size_t)nslab), fout((size_t)nslab);
  std::atomic<int> lane_err{ZH_OK};
  std::string lane_msg;
  std::mutex lane_mu;
  // the in lanes' job queue, filled as plans are created (deque: stable references)
  std::deque<InJob> ijobs;
  std::vector<int64_t> in_total((size_t)nslab, 0);
  std::mutex qmu;
  std::condition_variable qcv;
  size_t next_in = 0;
  bool all_published = false, q_abort = false;
  auto abort_all = [&] {
    fin.abort();
    fdec.abort();
    fout.abort();
    std::lock_guard<std::mutex> lk(qmu);
    q_abort = true;
    qcv.notify_all();
  };
  auto lane_fail = [&](hipError_t e, const char* what) {
    {
      std::lock_guard<std::mutex> lk(lane_mu);
      if (lane_err.load() == ZH_OK) {
        lane_err = e == hipErrorOutOfMemory ? ZH_ENOMEM : ZH_EHIP;
        lane_msg = std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")";
      }
    }
    abort_all();
  };
  auto lane_fail_io = [&](const std::string& msg) {  // a store file read failed (ZH_EIO)
    {
      std::lock_guard<std::mutex> lk(lane_mu);
      if (lane_err.load() == ZH_OK) {
        lane_err = ZH_EIO;
        lane_msg = msg;
      }
    }
    abort_all();
  };
  std::vector<std::thread> th;
  std::atomic<int64_t> next_out{0};
  std::vector<std::atomic<int64_t>> in_done((size_t)nslab), out_done((size_t)nslab);
  for (auto& x : in_done) x = 0;
  for (auto& x : out_done) x = 0;
  // status of the slabs, in C order: planning failure (from slab plan_fail on), device errors
  int plan_st = ZH_OK, dev_st = ZH_OK;
  std::string plan_msg, dev_msg;
  // the data error first in the oracle's order: its chunk coords, its key in the shard
  bool data_err = false;
  std::vector<int64_t> data_cc;
  uint64_t data_key = 0;
  std::string data_msg;
  int64_t nplan = nslab;  // slabs that got a plan
  const bool go = st == ZH_OK && he == hipSuccess;
  if (go) {
    // ---- in lanes
    for (int L = 0; L < lanes_in; L++)
      th.emplace_back([&, L] {
        (void)hipSetDevice(ctx->device);
        int flip = 0;
        for (;;) {
          InJob* Jp = nullptr;
          {
            std::unique_lock<std::mutex> lk(qmu);
            qcv.wait(lk, [&] { return next_in < ijobs.size() || all_published || q_abort; });
            if (q_abort || next_in >= ijobs.size()) break;
            Jp = &ijobs[next_in++];
          }
          InJob& J = *Jp;
          hipError_t e = hipSuccess;
          if (J.direct) {
            e = hipMemcpyAsync(J.dst, J.direct, (size_t)J.len, hipMemcpyHostToDevice, ctx->pipe_in);
          } else {
            const int k = 2 * L + flip;
            flip ^= 1;
            e = hipEventSynchronize(slot_ev[(size_t)k]);  // the slot's previous DMA is done
            uint8_t* slot = (uint8_t*)ctx->ring_in[(size_t)k];
            std::string io;
            for (auto& part : J.parts) {
              if (!part.second.first.is_file()) {
                copy_bytes(slot + part.first, part.second.first.mem(), part.second.second);
                continue;
              }
              // a store file's range (zh_array_read_files): read straight into the slot
              io = file_fetch(slot + part.first, part.second.first, part.second.second);
              if (!io.empty()) break;
            }
            if (!io.empty()) {
              lane_fail_io(io);
              break;
            }
            if (e == hipSuccess)
              e = hipMemcpyAsync(J.dst, slot, (size_t)J.len, hipMemcpyHostToDevice, ctx->pipe_in);
            if (e == hipSuccess) e = hipEventRecord(slot_ev[(size_t)k], ctx->pipe_in);
          }
          if (e != hipSuccess) {
            lane_fail(e, "pipelined read: host-to-device copy");
            break;
          }
          // the lane that issues a slab's last copy marks the slab's input as enqueued
          if (in_done[(size_t)J.slab].fetch_add(1) + 1 == in_total[(size_t)J.slab]) {
            e = hipEventRecord(in_ev[(size_t)J.slab], ctx->pipe_in);
            if (e != hipSuccess) {
              lane_fail(e, "pipelined read: event");
              break;
            }
            fin.set((size_t)J.slab);
          }
        }
      });
    // ---- out lanes
    for (int L = 0; L < lanes_out; L++)
      th.emplace_back([&, L] {
        (void)hipSetDevice(ctx->device);
        int flip = 0;
        int64_t waited = -1;
        const OutJob* pend = nullptr;  // a copied-out window whose memcpy is still due
        int pend_slot = -1;
        auto drain = [&]() -> bool {
          if (!pend) return true;
          const hipError_t e = hipEventSynchronize(slot_ev[(size_t)(E + pend_slot)]);
          if (e != hipSuccess) {
            lane_fail(e, "pipelined read: device-to-host copy");
            return false;
          }
          copy_bytes(pend->dst, ctx->ring_out[(size_t)pend_slot], pend->len);
          pend = nullptr;
          return true;
        };
        for (;;) {
          const int64_t j = next_out.fetch_add(1);
          if (j >= (int64_t)ojobs.size() || lane_err.load() != ZH_OK) break;
          const OutJob& J = ojobs[(size_t)j];
          if (waited != J.slab) {
            if (!fdec.wait((size_t)J.slab)) break;
            waited = J.slab;
          }
          hipError_t e = hipStreamWaitEvent(ctx->pipe_out, dec_ev[(size_t)J.slab], 0);
          if (out_pinned) {
            if (e == hipSuccess)
              e = hipMemcpyAsync(J.dst, J.src, (size_t)J.len, hipMemcpyDeviceToHost, ctx->pipe_out);
          } else {
            const int k = 2 * L + flip;
            flip ^= 1;
            // slot k was last used two windows ago; its memcpy ran when the next one was issued
            if (e == hipSuccess)
              e = hipMemcpyAsync(ctx->ring_out[(size_t)k], J.src, (size_t)J.len,
                                 hipMemcpyDeviceToHost, ctx->pipe_out);
            if (e == hipSuccess) e = hipEventRecord(slot_ev[(size_t)(E + k)], ctx->pipe_out);
            if (e == hipSuccess && !drain()) break;
            pend = &J;
            pend_slot = k;
          }
          if (e != hipSuccess) {
            lane_fail(e, "pipelined read: device-to-host copy");
            break;
          }
          if (out_done[(size_t)J.slab].fetch_add(1) + 1 == out_total[(size_t)J.slab]) {
            e = hipEventRecord(out_ev[(size_t)J.slab], ctx->pipe_out);
            if (e != hipSuccess) {
              lane_fail(e, "pipelined read: event");
              break;
            }
            fout.set((size_t)J.slab);
          }
        }
        if (lane_err.load() == ZH_OK) drain();
      });
    // ---- this thread: plans (at most W alive), decode, status
    int64_t created = 0, retired = 0;
    auto publish_done = [&] {
      std::lock_guard<std::mutex> lk(qmu);
      all_published = true;
      qcv.notify_all();
    };
    auto create = [&](int64_t r) -> bool {
      Slab& S = slabs[(size_t)r];
      char e[1024] = {0};
      zh_plan* p = nullptr;
      const int rc = plan_create(ctx, meta, S.sub.data(), (int64_t)S.sub.size(), S.o, S.s,
                                 (flags & ZH_SRC_DEVICE) | ZH_OUT_DEVICE, true, &p, e, sizeof e);
      if (rc != ZH_OK) {
        plan_st = rc;
        plan_msg = e;
        return false;
      }
      plans[(size_t)r] = p;
      std::vector<InJob> js;
      bool pg = false;
      in_jobs(p, r, cfg.chunk, js, &pg);
      {
        std::lock_guard<std::mutex> lk(qmu);
        in_total[(size_t)r] = (int64_t)js.size();
        for (auto& j : js) ijobs.push_back(std::move(j));
        qcv.notify_all();
      }
      if (js.empty()) fin.set((size_t)r);
      return true;
    };
    // retire: the plan's status (deferred device errors, C order), then its blocks go back
    auto retire = [&](int64_t k) {
      zh_plan* p = plans[(size_t)k];
      if (!p) return;
      char e[1024] = {0};
      // its own decode only (the stream holds later slabs' work)
      if (p->done_ev) (void)hipEventSynchronize(p->done_ev);
      p->last_stream = nullptr;
      if (dev_st == ZH_OK && lane_err.load() == ZH_OK) {
        const int rc = zh_plan_wait(p, e, sizeof e);
        if (rc == ZH_EDATA && p->err_shard >= 0) {
          const int n = p->meta.ndim;
          std::vector<int64_t> cc(p->coords.begin() + p->err_shard * n,
                                  p->coords.begin() + (p->err_shard + 1) * n);
          if (!data_err || data_err_before(cc, p->err_key, data_cc, data_key)) {
            data_cc = cc;
            data_key = p->err_key;
            data_msg = e;
          }
          data_err = true;
        } else if (rc != ZH_OK) {
          dev_st = rc;
          dev_msg = e;
        }
      }
      plan_free(p);
      plans[(size_t)k] = nullptr;
    };
    auto top_up = [&](int64_t upto) {  // plans for slabs < upto
      while (created < upto && created < nplan) {
        if (created - retired >= W) retire(retired++);
        if (dev_st != ZH_OK) return;
        if (!create(created)) {
          nplan = created;
          return;
        }
        created++;
      }
    };
    top_up(W);
    if (created >= nplan) publish_done();
    for (int64_t r = 0; r < nplan && dev_st == ZH_OK; r++) {
      if (!fin.wait((size_t)r)) break;
      hipError_t e = hipSuccess;
      if (in_total[(size_t)r] > 0) e = hipStreamWaitEvent(sdec, in_ev[(size_t)r], 0);
      void* dst = (uint8_t*)out + slabs[(size_t)r].obase;
      if (host_out) {
        dst = dslot[(size_t)(r % nds)];
        if (r >= nds) {  // the slot's previous slab has been copied out
          if (!fout.wait((size_t)(r - nds))) break;
          if (e == hipSuccess) e = hipStreamWaitEvent(sdec, out_ev[(size_t)(r - nds)], 0);
        }
      }
      if (e != hipSuccess) {
        lane_fail(e, "pipelined read: stream wait");
        break;
      }
      zh_plan* p = plans[(size_t)r];
      int rc = plan_enqueue_impl(p, dst, sdec);
      if (rc == ZH_OK) rc = plan_mark_done_impl(p, sdec);
      if (rc == ZH_OK) p->last_stream = sdec;
      e = rc == ZH_OK ? hipEventRecord(dec_ev[(size_t)r], sdec) : hipErrorLaunchFailure;
      if (e != hipSuccess) {
        lane_fail(e, "pipelined read: kernel launch");
        break;
      }
      fdec.set((size_t)r);
      // the next plan (its input copies start while this slab decodes); the slab W back is
      // retired first: its decode was enqueued before this one
      top_up(r + W + 1);
      if (created >= nplan) publish_done();
    }
    if (dev_st != ZH_OK || lane_err.load() != ZH_OK || nplan < nslab) {
      // stop: no further slab is decoded, so nothing waits for the lanes' remaining jobs
      if (dev_st != ZH_OK || lane_err.load() != ZH_OK) abort_all();
    }
    publish_done();
    // out lanes wait for slabs that were never decoded (a planning failure): release them
    if (nplan < nslab) fdec.abort();
    for (auto& t : th) t.join();
    (void)hipStreamSynchronize(sdec);
    if (ctx->pipe_in) (void)hipStreamSynchronize(ctx->pipe_in);
    if (ctx->pipe_out) (void)hipStreamSynchronize(ctx->pipe_out);
    while (retired < created) retire(retired++);
  }
  // ---- status: the first failing slab in C order
  if (st == ZH_OK && he != hipSuccess) {
    set_err(err, errlen, "HIP error %s (%s)", hipGetErrorName(he), hipGetErrorString(he));
    st = he == hipErrorOutOfMemory ? ZH_ENOMEM : ZH_EHIP;
  }
  if (st == ZH_OK && lane_err.load() != ZH_OK) {
    set_err(err, errlen, "%s", lane_msg.c_str());
    st = lane_err.load();
  }
  if (st == ZH_OK && dev_st != ZH_OK) {
    set_err(err, errlen, "%s", dev_msg.c_str());
    st = dev_st;
  }
  g_data_err.set = false;
  if (st == ZH_OK && data_err) {
    set_err(err, errlen, "%s", data_msg.c_str());
    st = ZH_EDATA;
    g_data_err.set = true;
    g_data_err.cc = data_cc;
    g_data_err.key = data_key;
  }
  if (st == ZH_OK && plan_st != ZH_OK) {
    set_err(err, errlen, "%s", plan_msg.c_str());
    st = plan_st;
  }
  for (zh_plan* p : plans)
    if (p) plan_free(p);
  for (size_t k = 0; k < dslot.size(); k++) ctx_release(ctx, dslot[k], dslot_got[k]);
  for (auto* v : {&in_ev, &dec_ev, &out_ev, &slot_ev})
    for (hipEvent_t e : *v)
      if (e) (void)hipEventDestroy(e);
  return st;
}

}  // namespace zh
