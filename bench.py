#!/usr/bin/env python3
"""Headline benchmark: device-resident Zarr v3 chunk decode on MI355X.

Workload (default c4 = BASELINE.json configs[3], the chain the metric names:
"sharding+bytes+transpose", 32^3 sharding, 1 GPU):
  uint32 array 1x4096x4096x1536 (96 GiB decoded), chunk (= shard) 1x1024x1024x1024,
  codecs [sharding_indexed{chunk_shape [1,32,32,32], codecs [transpose [0,3,2,1],
          bytes(big)], index_codecs [bytes(little), crc32c], index_location end}].
c3 (configs[2], no transpose) and c2 (configs[1], unsharded bytes) are the other
single-GPU configs.  One step = one full-array core.Array.read (M/core/Array.java:378-441)
of all 32 shards / 786,432 in-bounds inner chunks: index CRC + index parse + byte swap
(+ transpose) + scatter, inputs already resident in HBM.  Synthetic data v(g) =
lo32(splitmix64(g ^ 0x5A5A2026)) is written on the device and encoded by the product's own
write path (zh_array_write); after warmup the decoded array is verified element-by-element
on the device against the generator.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c3|c2|...]

N=1 prints the headline line (weak scaling of one full array per GPU, which at N=1 is the
single-GPU number), plus `extra_configs` (c3, c2 and c4 little-endian timed in the same
process), a one-shot `zh_array_read` time and the CPU baseline.

N>1 (BASELINE.json configs[4]): ONE full array partitioned across the GPUs in
contiguous y-slabs (512 rows at N=8, aligned to inner chunks), strong scaling.  Each rank
holds the shards its slab touches, decodes its slab (value = decode-only aggregate GiB/s =
array bytes / max-over-ranks time), then the root assembles the whole region over RCCL
(grouped send/recv into one buffer on the root, re-verified there: `gather`), and every rank
copies its slab into its slice of one host region buffer (`host_terminated`).  Launched by
torch.distributed.run (one process per GPU), or, when WORLD_SIZE is unset, bench.py launches
the N ranks itself before anything touches the GPU.  --mode weak keeps the older
one-array-per-GPU run.
"""
import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zarr-java_amd"))

SEED = 0x5A5A2026
GiB = 1 << 30
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "GiB/s device-resident chunk decode (sharding+bytes+transpose), uint32 1024³"

CONFIGS = {
    # name: (description, sharded, transpose order[, extra make_meta keywords])
    "c2": ("bytes(big) only, chunk 1x1024x1024x1024", False, None),
    "c3": ("sharding 1x32x32x32 + bytes(big), index [bytes(little), crc32c] at end", True, None),
    "c4": ("c3 + transpose [0,3,2,1] inside the shard", True, [0, 3, 2, 1]),
    "c4le": ("c4 with bytes(little) inner codec (the endian-neutral copy, §8(d))", True,
             [0, 3, 2, 1], dict(little=True)),
    # §8(f) rank-2 workloads (not the headline): same array and shards
    "c3crc": ("c3 with inner codecs [bytes(big), crc32c] (per-chunk checksum verified)", True,
              None, dict(inner_crc32c=True)),
    "c4crc": ("c4 with inner codecs [transpose [0,3,2,1], bytes(big), crc32c] (per-chunk "
              "checksum verified)", True, [0, 3, 2, 1], dict(inner_crc32c=True)),
    "c3nest": ("nested sharding: shard 1x1024^3 -> 1x256x256x256 sub-shards -> 1x32x32x32 "
               "leaves, bytes(big); both indexes [bytes(little), crc32c] at end", True, None,
               dict(nested=True)),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def self_launch(nproc):
    """`--gpus N` without a launcher: start N ranks under torch.distributed.run as CHILD
    processes (this process has touched neither torch nor HIP, and it is not replaced by an
    exec) and return their exit status.  Rank 0's stdout is the one JSON line."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    log(f"[launcher] {nproc} ranks: {' '.join(cmd[1:6])} ...")
    return subprocess.call(cmd, env=env)


class Dist:
    """Barrier / max over ranks.  torch.distributed (gloo on CPU tensors) only when N>1;
    torch is imported before libzarrhip so both share one HIP runtime."""

    def __init__(self, ws, need_torch=False):
        self.ws = ws
        if need_torch or ws > 1:
            import torch  # noqa: F401  (load torch's HIP runtime first)
        if ws > 1:
            import torch
            import torch.distributed as dist
            # gloo prints its connection lines on stdout: keep stdout for the one JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo")
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.torch, self.dist = torch, dist

    def barrier(self):
        if self.ws > 1:
            self.dist.barrier()

    def max(self, v):
        if self.ws == 1:
            return v
        t = self.torch.tensor([float(v)], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.ws > 1:
            self.dist.destroy_process_group()


def build_meta(A, cfg, ydiv=1):
    _, sharded, order = CONFIGS[cfg][:3]
    extra = dict(CONFIGS[cfg][3]) if len(CONFIGS[cfg]) > 3 else {}
    inner = [1, 32, 32, 32]
    if extra.pop("nested", False):
        inner = [1, 256, 256, 256]
        extra["nested_chunk_shape"] = [1, 32, 32, 32]
    endian = A.ZH_ENDIAN_LITTLE if extra.pop("little", False) else A.ZH_ENDIAN_BIG
    return A.make_meta([1, 4096 // ydiv, 4096, 1536], [1, 1024, 1024, 1024], 4,
                       endian=endian, sharded=sharded, **extra,
                       inner_chunk_shape=inner if sharded else None,
                       transpose_order=order, index_endian=A.ZH_ENDIAN_LITTLE,
                       index_crc32c=True, index_location=A.ZH_INDEX_END)


def chunk_capacities(meta, coords):
    """Exact encoded sizes for synthetic data (every in-bounds inner chunk is non-fill;
    inner chunks wholly in the boundary padding are elided as all-fill)."""
    n = meta.ndim
    ch = meta.chain
    sharded = ch.sharded
    l1 = [ch.inner_chunk_shape[d] if sharded else meta.chunk_shape[d] for d in range(n)]
    leaf = [ch.nested_chunk_shape[d] for d in range(n)] if ch.nested else l1

    def prod(v):
        r = 1
        for x in v:
            r *= x
        return r

    leaf_bytes = 4 * prod(leaf) + (4 if ch.inner_crc32c else 0)
    isz = sub_isz = 0
    if sharded:
        isz = 16 * prod([meta.chunk_shape[d] // l1[d] for d in range(n)]) + 4
    if ch.nested:
        sub_isz = 16 * prod([l1[d] // leaf[d] for d in range(n)]) + 4
    caps = []
    for c in coords:
        valid = cells = 1
        for d in range(n):
            lo = c[d] * meta.chunk_shape[d]
            hi = min(lo + meta.chunk_shape[d], meta.shape[d])
            valid *= -(-(hi - lo) // leaf[d])
            cells *= -(-(hi - lo) // l1[d])
        caps.append(valid * leaf_bytes + isz + (cells * sub_isz if ch.nested else 0))
    return caps


def all_coords(L, meta, off=None, shp=None):
    n = meta.ndim
    shape = [meta.shape[d] for d in range(n)]
    off = [0] * n if off is None else off
    shp = shape if shp is None else shp
    cs = (C.c_int32 * 8)(*[meta.chunk_shape[d] for d in range(n)])
    num = L.zh_compute_chunk_coords(n, (C.c_int64 * 8)(*shape), cs, (C.c_int64 * 8)(*off),
                                    (C.c_int64 * 8)(*shp), None, 0)
    buf = (C.c_int64 * (num * n))()
    L.zh_compute_chunk_coords(n, (C.c_int64 * 8)(*shape), cs, (C.c_int64 * 8)(*off),
                              (C.c_int64 * 8)(*shp), buf, num)
    return [tuple(buf[i * n + d] for d in range(n)) for i in range(num)]


def slab_layout(caps):
    offs, tot = [], 0
    for cap in caps:
        offs.append(tot)
        tot += (cap + 255) // 256 * 256
    return offs, tot


def pmc_traffic(config):
    """HBM bytes per launch of the scatter kernel from the newest committed PMC summary for
    this config (profiles/rNN/<config>_summary.json, made by profiles/pmc_summary.py from
    separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes, FETCH_SIZE x2 per the gfx950 note)."""
    import glob
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"{config}_summary.json")))
    if not cands:
        return None, None
    d = json.load(open(cands[-1]))
    info = {"path": os.path.relpath(cands[-1], ROOT),
            "note": "PMC passes of another process (rocprofv3 wraps the whole program), on "
                    "the box of that closing run",
            "profile_kernel_ms": round(d["kernel_trace"]["avg_ns"] / 1e6, 3)}
    return int(d["pmc"]["traffic_bytes_per_launch"]), info


def kernel_name(meta):
    # tile chains: tiles_group_kernel; with the chunk crc32c the row-CRC tile kernel over
    # 128-B aligned payload windows (c4crc's layout)
    if meta.chain.has_transpose:
        return "tiles_rowcrc_aln_kernel" if meta.chain.inner_crc32c else "tiles_group_kernel"
    # row chains with 128-B rows and no chunk CRC: the lane-exchange kernel
    c = meta.chain
    if c.sharded and not c.inner_crc32c and \
            c.inner_chunk_shape[meta.ndim - 1] * meta.dtype_size == 128:
        return "rows_xpose_kernel"
    # with the chunk crc32c: the grouped row-CRC kernel
    if c.sharded and c.inner_crc32c:
        return "rows_group_kernel"
    return "decode_rows_kernel<4,4>"


def roofline_of(plan, st, config=None):
    kt = plan.kernel_time()
    scatter_ms = kt["scatter_ms"] / max(1, kt["launches"])
    index_ms = kt["index_ms"] / max(1, kt["launches"])
    alg = st["in_bytes"] + st["out_bytes"]
    achieved = alg / (scatter_ms / 1000.0) / 1e9
    traffic, src = pmc_traffic(config) if config else (None, None)
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_over_alg": round(traffic / alg, 4) if traffic else None,
            "traffic_source": src, "kernel": kernel_name(plan._meta),
            "kernel_ms": round(scatter_ms, 3), "index_kernels_ms": round(index_ms, 4),
            "alg_bytes_per_launch": alg}


def ceiling_probe(dev, out, src, nbytes):
    """What this box allows for this output buffer, measured on the line's own buffers before
    its decode: the copy ceiling — a streaming byte-swapping copy of the
    shard slab into the output (zh_device_copy_rate; the decode's own traffic: one read and one
    write per output byte; tools/copy_lab.hip's fastest form) — and the contiguous store probe
    of the output (zh_device_write_rate pattern 0), both GB/s (1e9 B/s)."""
    return {"copy_ceiling_GBps": round(dev.copy_rate(out, src, nbytes, 3), 1),
            "store_probe_GBps": round(dev.write_rate(out, nbytes, 0, 3), 1)}


def reallocate(dev, out, nbytes, k):
    """A fresh output allocation (the k-th): free the old one, hold a k x 16 GiB spacer while
    allocating so the allocator hands out other physical memory (freed and allocated again, a
    buffer comes back on the same pages: DESIGN §4 "Placement"), then drop the spacer."""
    dev.free(out)
    spacer = None
    try:
        spacer = dev.malloc(k * 16 * GiB)
    except Exception:  # not enough room beside the slab: allocate without one
        spacer = None
    try:
        return dev.malloc(nbytes)
    finally:
        if spacer:
            dev.free(spacer)


def _amd_smi(cmd, device):
    r = subprocess.run(["amd-smi", cmd, "-g", str(device), "--json"], capture_output=True,
                       text=True, timeout=60)
    d = json.loads(r.stdout)
    if isinstance(d, dict) and "gpu_data" in d:
        d = d["gpu_data"]
    return d[0] if isinstance(d, list) and d else d


def _val(x):
    return x.get("value") if isinstance(x, dict) else x


def gpu_state(device=0, static=False):
    """The box the line ran on, from amd-smi (or the error): memory / fabric / SoC clocks, the
    range of the XCD clocks, socket power, temperatures and the throttle counters — plus, with
    static, the HBM vendor, size and rated bandwidth and the power cap.  A box whose memory runs
    slower shows here and in the copy ceiling, not in the kernel (DESIGN §4 "Placement")."""
    out = {}
    try:
        m = _amd_smi("metric", device)
        clk = m.get("clock", {})
        gfx = [_val(v.get("clk")) for k, v in clk.items() if k.startswith("gfx_")]
        gfx = [g for g in gfx if isinstance(g, (int, float))]
        out["clock_MHz"] = {k: _val(clk[k].get("clk")) for k in ("mem_0", "fclk_0", "socclk_0")
                            if k in clk}
        if gfx:
            out["clock_MHz"]["gfx_min_max"] = [min(gfx), max(gfx)]
        out["socket_power_W"] = _val(m.get("power", {}).get("socket_power"))
        t = m.get("temperature", {})
        out["temperature_C"] = {k: _val(t.get(k)) for k in ("hotspot", "mem")}
        th = m.get("throttle", {})
        out["throttle"] = {k: th.get(k) for k in (
            "ppt_accumulated", "hbm_thermal_accumulated", "socket_thermal_accumulated",
            "prochot_accumulated", "ppt_violation_status", "hbm_thermal_violation_status")}
    except Exception as e:  # no amd-smi, or no JSON: say so in the line
        out["metric_error"] = repr(e)[:200]
    if static:
        try:
            st = _amd_smi("static", device)
            v = st.get("vram", {})
            out["vram"] = {"type": v.get("type"), "vendor": v.get("vendor"),
                           "size_MB": _val(v.get("size")),
                           "max_bandwidth_GBps": _val(v.get("max_bandwidth"))}
            out["power_cap_W"] = _val(st.get("limit", {}).get("ppt0", {}).get("socket_power_limit"))
        except Exception as e:  # noqa: BLE001
            out["static_error"] = repr(e)[:200]
    return out


# ------------------------------------------------------------------------------------------
# host-inclusive readChunk pipeline
# ------------------------------------------------------------------------------------------
def host_inclusive(dev, A, meta, coords, offs, sizes, shard_slab, scratch, reps=3):
    """Host-resident bytes in, host-resident decoded array out, through the library's own
    read: one zh_array_read of the region [1,1024,4096,1024] (the four interior shards
    (0,0,k,0): 16 GiB of stored shards in, 16 GiB out) from host sources into a host output.
    The library pipelines it (zh_pipeline.cpp: 512 MiB C-order slabs, H2D | decode | D2H
    overlapped, page-locked sources and output by direct DMA, pageable ones through its pinned
    rings and host copy lanes).  Two forms, timed the same way (min of `reps`):
      pinned   — shards and output in page-locked host memory (hipHostMalloc);
      pageable — ordinary host memory touched once before (the JVM heap's state).
    Each output is checked element by element against the generator on the device."""
    import numpy as np
    n = meta.ndim
    cs = [meta.chunk_shape[d] for d in range(n)]
    off, shp = [0, 0, 0, 0], [1, cs[1], 4 * cs[2], cs[3]]
    pos = {c: i for i, c in enumerate(coords)}
    sel = [pos[(0, 0, k, 0)] for k in range(4)]
    in_sz = [sizes[i] for i in sel]
    out_sz = 4
    for v in shp:
        out_sz *= v
    res = {"region_offset": off, "region_shape": shp, "h2d_bytes": sum(in_sz),
           "d2h_bytes": out_sz,
           "call": "zh_array_read(host shards, host output): the library's pipelined host read"}
    chk = scratch  # device room for the check (the headline's output buffer, rewritten later)
    hin = dev.malloc_pinned(sum(in_sz))
    hout = dev.malloc_pinned(out_sz)
    pin_ptrs, p = [], 0
    for k, i in enumerate(sel):  # stage the encoded shards into host memory
        pin_ptrs.append(hin + p)
        dev.memcpy(hin + p, shard_slab + offs[i], in_sz[k], 1, None, True)
        p += in_sz[k]
    try:
        page_in = [np.empty(sz, np.uint8) for sz in in_sz]
        for buf, ptr, sz in zip(page_in, pin_ptrs, in_sz):
            C.memmove(buf.ctypes.data, ptr, sz)
        page_out = np.empty(out_sz, np.uint8)
        page_out[:] = 1  # touched once, as a warm heap is
        for name, srcs, outp in (
                ("pinned", [(q, sz) for q, sz in zip(pin_ptrs, in_sz)], hout),
                ("pageable", [(b.ctypes.data, sz) for b, sz in zip(page_in, in_sz)],
                 page_out.ctypes.data)):
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                dev.array_read(meta, srcs, off, shp, outp, 0)
                ts.append(time.perf_counter() - t0)
            dev.memcpy(chk, outp, out_sz, 0, None, True)
            bad = int(dev.synth_verify(chk, [meta.shape[d] for d in range(n)], off, shp, 4, SEED))
            ts.sort()
            res[name] = {"value": round(out_sz / ts[0] / GiB, 2), "unit": "GiB/s",
                         "ms_min": round(ts[0] * 1e3, 1),
                         "ms_median": round(ts[len(ts) // 2] * 1e3, 1),
                         "verify_mismatches": bad}
            log(f"host-inclusive {name}: {json.dumps(res[name])}")
        del page_in, page_out
    finally:
        dev.free_pinned(hin)
        dev.free_pinned(hout)
    res["value"] = res["pinned"]["value"]
    res["unit"] = "GiB/s"
    return res


# ------------------------------------------------------------------------------------------
# CPU baseline
# ------------------------------------------------------------------------------------------
def host_cpu_info():
    """Threads this process may use (affinity ∩ cgroup CPU quota), nproc and the CPU model."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, -(-int(q) // int(per)))
        except (OSError, ValueError):
            pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(aff, quota) if quota else aff
    return {"threads": usable, "nproc": os.cpu_count(), "affinity": aff, "cgroup_quota": quota,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cpu_model": model}


def _store_dir(need_bytes):
    for d in ("/dev/shm", os.environ.get("TMPDIR", "/tmp")):
        try:
            v = os.statvfs(d)
            if v.f_bavail * v.f_frsize >= need_bytes + (2 << 30):
                return d
        except OSError:
            pass
    return None


def cpu_baseline(dev, A, L, meta, shard_ptr, shard_nbytes, budget_s=12.0):
    """The C oracle (the restated reference path, oracle/zh_oracle.c) on this host's cores,
    over BASELINE.md §3's workload: Array.read of [1,1024,1024,512] regions (2 GiB out each),
    each inside one shard, from a FilesystemStore on tmpfs, so each goes through the partial
    path — suffix read of the index, then one open + range read + close per inner chunk
    (StoreHandleDataProvider, ShardingIndexedCodec.java:253,333-357) — and the part array's
    second copy into the output (M/core/Array.java:422-426).  All usable threads, then one;
    plus the c2 "scaled chunk" proxy (1 GiB bytes(big) chunks, 2 per region).  k is sized to
    the budget.  The reference Java is not timed: there is no JDK on the box."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    info = host_cpu_info()
    threads = info["threads"]
    n = meta.ndim
    region = [1, 1024, 1024, 512]
    rbytes = 4 * 1024 * 1024 * 512
    d = _store_dir(shard_nbytes + 2 * GiB)
    if d is None:
        return {"value": None, "unit": "GiB/s", "cores": threads, "kind": "port",
                "sample": "skipped: no tmpfs room for a 4 GiB shard file", **info}
    base = os.path.join(d, f"zh_cpu_store_{os.getpid()}")
    os.makedirs(os.path.join(base, "c", "0", "0", "0"), exist_ok=True)
    shard_path = os.path.join(base, "c", "0", "0", "0", "0")
    pin = dev.malloc_pinned(shard_nbytes)
    dev.memcpy(pin, shard_ptr, shard_nbytes, 1, None, True)
    with open(shard_path, "wb") as f:   # the store file, written from the device encode
        f.write((C.c_char * shard_nbytes).from_address(pin))
    out = dev.malloc_pinned(rbytes)
    chk = dev.malloc(rbytes)
    res = {"unit": "GiB/s", "kind": "port", "cores": threads, **info,
           "reference_java": "not timed (no JDK on the box)"}
    try:
        def timed(paths_meta, paths, off, shp, nthreads, budget, max_reps):
            t, reps = 0.0, 0
            while reps < max_reps and (reps == 0 or t < budget):
                o = list(off(reps))
                t0 = time.perf_counter()
                O.array_read_store(paths_meta, paths, o, shp, out_addr=out, nthreads=nthreads)
                t += time.perf_counter() - t0
                reps += 1
            return t, reps

        zoff = lambda r: [0, 0, 0, 512 * (r % 2)]   # noqa: E731  z ∈ {0, 512} inside shard 0
        # first read checked element-by-element against the generator (on the device)
        O.array_read_store(meta, [shard_path], [0] * n, region, out_addr=out, nthreads=threads)
        dev.memcpy(chk, out, rbytes, 0, None, True)
        bad = dev.synth_verify(chk, [meta.shape[d] for d in range(n)], [0] * n, region, 4, SEED)
        if bad:
            raise SystemExit(f"cpu baseline read differs from the generator: {bad}")
        t, r = timed(meta, [shard_path], zoff, region, threads, budget_s * 0.6, 48)
        res["value"] = round(r * rbytes / t / GiB, 4)
        res["sample"] = (f"{r} x Array.read [1,1024,1024,512] (2 GiB out each) from a "
                         f"FilesystemStore shard file on {d} through the partial path "
                         f"(C oracle, OpenMP over inner chunks, {threads} threads), {t:.1f} s; "
                         f"first read verified vs the generator")
        t1, r1 = timed(meta, [shard_path], zoff, region, 1, budget_s * 0.2, 48)
        res["single_core"] = {"value": round(r1 * rbytes / t1 / GiB, 4), "unit": "GiB/s",
                              "cores": 1, "sample": f"{r1} x the same read, 1 thread, {t1:.1f} s"}
    finally:
        os.unlink(shard_path)
    # c2 "scaled chunk" proxy: bytes(big) chunks [1,1024,1024,256] (1 GiB
    # objects); the region spans 2 chunks, so the fill + copyRegion scatter path runs
    pm = A.make_meta([1, 1024, 1024, 512], [1, 1024, 1024, 256], 4, endian=A.ZH_ENDIAN_BIG)
    src = dev.malloc(rbytes)
    dev.synth_fill(src, rbytes // 4, 4, 0, SEED)
    cb = [dev.malloc(rbytes // 2) for _ in range(2)]
    sizes = dev.array_write(pm, src, [0] * 4, region, [(b, rbytes // 2) for b in cb])
    paths = []
    for i, (b, sz) in enumerate(zip(cb, sizes)):
        p = os.path.join(base, f"c2_{i}")
        dev.memcpy(pin, b, sz, 1, None, True)
        with open(p, "wb") as f:
            f.write((C.c_char * sz).from_address(pin))
        paths.append(p)
    try:
        t2, r2 = timed(pm, paths, lambda r: [0] * 4, region, threads, budget_s * 0.2, 48)
        dev.memcpy(chk, out, rbytes, 0, None, True)
        bad = dev.synth_verify(chk, region, [0] * 4, region, 4, SEED)
        res["c2_scaled_chunk"] = {
            "value": round(r2 * rbytes / t2 / GiB, 4), "unit": "GiB/s", "cores": threads,
            "verify_mismatches": int(bad),
            "sample": f"{r2} x Array.read [1,1024,1024,512] of a bytes(big) array with "
                      f"[1,1024,1024,256] chunks (1 GiB files, 2 per read: fill + scatter), "
                      f"{t2:.1f} s"}
    finally:
        for p in paths:
            os.unlink(p)
        import shutil
        shutil.rmtree(base, ignore_errors=True)
        for b in cb + [src, chk]:
            dev.free(b)
        dev.free_pinned(out)
        dev.free_pinned(pin)
    return res


# ------------------------------------------------------------------------------------------
# N > 1: one array split over the GPUs (strong scaling)
# ------------------------------------------------------------------------------------------
def _mem_available():
    """Host memory this job may still use: MemAvailable, capped by the cgroup's limit
    (memory.max − memory.current), which /proc/meminfo does not show."""
    avail = 0
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                avail = int(line.split()[1]) * 1024
    except OSError:
        pass
    try:
        lim = open("/sys/fs/cgroup/memory.max").read().strip()
        if lim != "max":
            cur = int(open("/sys/fs/cgroup/memory.current").read().strip())
            avail = min(avail, int(lim) - cur)
    except (OSError, ValueError):
        pass
    return avail


def host_terminated(args, dist, dev, plan, out, out_bytes, shape, so, ss, rank, ws, align):
    """Host-terminated read (no gather) through the product's
    zarrhip.parallel.SharedHostRegion: one host buffer holding the whole region in /dev/shm,
    mapped by every rank, each rank page-locking only its own slice and decoding its slab
    straight into it (here: its plan into device memory, then one D2H into the slice), so N
    GPUs drive N PCIe links at once.  When the host cannot hold the region (tmpfs or
    MemAvailable short by the region + 32 GiB), each rank streams its slab through a private
    2 GiB pinned ring instead (same links, nothing kept), and says so.  Timed: barrier, reps x
    (decode + D2H), sync, max over ranks; then the slices are verified against the generator."""
    from zarrhip.parallel import SharedHostRegion
    full = 4
    for s in shape:
        full *= s
    reps = max(1, min(args.steps, 3))
    ring = 2 << 30
    region = None
    # this job's region file (SharedHostRegion creates it exclusively): one a killed earlier run
    # on the same port left behind is removed first, so it neither blocks the name nor holds
    # the host memory the check below counts
    name = f"/dev/shm/zh_region_{os.environ.get('MASTER_PORT', 'solo')}_{os.getuid()}"
    if rank == 0:
        try:
            os.unlink(name)
        except OSError:
            pass
    dist.barrier()
    if int(dist.max(0 if _mem_available() >= full + (32 << 30) else 1)) == 0:
        try:
            region = SharedHostRegion([0] * len(shape), shape, 4, dev=dev, align=align, name=name)
        except (MemoryError, OSError):  # no room, or the file cannot be made: the bounded form
            region = None
    if region is not None:
        assert region.slab_offset == list(so) and region.slab_shape == list(ss)
        dst = region.slice_addr()
        kind = ("zarrhip.parallel.SharedHostRegion: one region buffer in /dev/shm shared by the "
                "ranks; each pins its slice")

        def copy_out():
            dev.memcpy(dst, out, out_bytes, 1, None, False)

        def decode(po, ps, addr):  # the slab's plan, then its D2H into the slice
            plan.execute(out)
            dev.memcpy(addr, out, out_bytes, 1, None, False)
            plan.wait()
            dev.sync()
        region.read(decode)
    else:
        dst = dev.malloc_pinned(min(ring, out_bytes))
        kind = "bounded: each rank streams its slab through a private 2 GiB pinned ring"

        def copy_out():
            for o in range(0, out_bytes, ring):
                dev.memcpy(dst, out + o, min(ring, out_bytes - o), 1, None, False)
        plan.execute(out)
        copy_out()
        plan.wait()
    dev.sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.execute(out)
        copy_out()
    plan.wait()
    dev.sync()
    t = dist.max(time.perf_counter() - t0)
    dist.barrier()
    t1 = time.perf_counter()
    for _ in range(reps):
        copy_out()
    dev.sync()
    t_copy = dist.max(time.perf_counter() - t1)
    bad = 0
    if region is not None:  # the host slice must hold this rank's slab of the generator's array
        dev.memset(out, 0, out_bytes)
        dev.memcpy(out, dst, out_bytes, 0, None, True)
        bad = dist.max(dev.synth_verify(out, shape, so, ss, 4, SEED))
        region.close()
    else:
        dev.free_pinned(dst)
    if bad:
        raise SystemExit(f"[rank {rank}] host-terminated slab verification FAILED: {bad}")
    return {"buffer": kind, "reps": reps, "ms_per_step": round(t * 1e3 / reps, 3),
            "value": round(full * reps / t / GiB, 2), "unit": "GiB/s",
            "d2h_only_ms_per_step": round(t_copy * 1e3 / reps, 3),
            "d2h_GBps_per_rank": round(out_bytes * reps / t_copy / 1e9, 2),
            "region_bytes": full, "verified": region is not None}


def gpus_shared(dist, device, ndev, ws):
    """Do two ranks drive the same physical GPU?  Compared by device UUID / PCI address over
    the process group (a launcher may give each rank one visible device); without either,
    fewer visible devices than ranks means sharing."""
    import torch
    ident = None
    try:
        pr = torch.cuda.get_device_properties(device)
        for attr in ("uuid", "pci_bus_id"):
            v = getattr(pr, attr, None)
            if v is not None and str(v):
                ident = f"{attr}:{v}:{getattr(pr, 'pci_domain_id', '')}:{getattr(pr, 'pci_device_id', '')}"
                break
    except Exception:
        ident = None
    ids = [None] * ws
    dist.dist.all_gather_object(ids, ident)
    if all(i is not None for i in ids):
        return len(set(ids)) < ws
    return ndev < ws


def visible_devices():
    """GPUs this rank can see (torch.cuda.device_count does not initialise HIP here)."""
    import torch
    return torch.cuda.device_count()


def strong_slab(L, meta, ws, rank):
    """Rank `rank`'s part of the strong-scaling read: the region's y-slabs on the
    inner-chunk grid (slab_partition; 512 rows at N=8 on the full array), this rank's slab, and
    the shard-aligned box `lo`/`ext` whose shards it must hold (`cover`, computeChunkCoords
    order).  Pure geometry: tests/test_multigpu_plan.py runs it at full size and at world 8 on
    a scaled array."""
    from zarrhip.parallel import slab_partition
    n = meta.ndim
    shape = [meta.shape[d] for d in range(n)]
    cs = [meta.chunk_shape[d] for d in range(n)]
    inner_y = meta.chain.inner_chunk_shape[1] if meta.chain.sharded else 1
    parts = slab_partition([0] * n, shape, ws, align=inner_y)
    so, ss = parts[rank]
    lo = [(so[d] // cs[d]) * cs[d] for d in range(n)]
    hi = [min(-(-(so[d] + ss[d]) // cs[d]) * cs[d], shape[d]) for d in range(n)]
    ext = [h - l for l, h in zip(lo, hi)]
    for d in range(2, n):
        assert lo[d] == 0 and ext[d] == shape[d]
    nel_cover = 1
    for e in ext:
        nel_cover *= e
    full_bytes = meta.dtype_size
    for s_ in shape:
        full_bytes *= s_
    slab_bytes = meta.dtype_size
    for s_ in ss:
        slab_bytes *= s_
    return {"parts": parts, "so": so, "ss": ss, "lo": lo, "ext": ext, "align": inner_y,
            "cover": all_coords(L, meta, lo, ext), "nel_cover": nel_cover,
            "cover_bytes": nel_cover * meta.dtype_size, "slab_bytes": slab_bytes,
            "full_bytes": full_bytes}


def strong_memory_plan(geo, shard_bytes, rank, backend, headroom=4 << 30):
    """Device memory one rank of the strong-scaling read holds at once, checked before anything
    is allocated: the decode's output (the shard-aligned cover box, also the encode source of
    the rank's shards), its shards, on the root with RCCL the assembled region (torch), on a
    peer with RCCL its send buffer, and headroom for plan tables and staging."""
    region = geo["full_bytes"] if rank == 0 and backend == "nccl" else 0
    send = geo["slab_bytes"] if rank != 0 and backend == "nccl" else 0
    out = {"output": geo["cover_bytes"], "shards": int(shard_bytes), "region": region,
           "send_buffer": send, "headroom": headroom}
    out["total"] = sum(out.values())
    return out


def run_strong(args, dist, A, meta, rank, ws, local):
    """Strong scaling: ONE full array split into per-rank y-slabs (512 rows at
    N=8, aligned to inner chunks); each rank holds only the shards its slab touches (encoded
    on its own GPU), decodes its slab, the root assembles the region over RCCL, and every
    rank copies its slab to its slice of one host buffer."""
    import torch
    from zarrhip._lib import DeviceContext, lib
    from zarrhip.parallel import slab_byte_offset
    L = lib()
    ndev = visible_devices()
    device = local % max(1, ndev)
    backend = args.gather_backend
    shared_gpu = gpus_shared(dist, device, ndev, ws)
    if backend == "nccl" and shared_gpu:
        backend = "gloo"   # rehearsal with several ranks on one GPU: RCCL needs distinct GPUs
    if backend == "nccl":
        torch.cuda.set_device(device)
    dev = DeviceContext(device)
    info = dev.info()
    n = meta.ndim
    shape = [meta.shape[d] for d in range(n)]
    geo = strong_slab(L, meta, ws, rank)
    parts, so, ss, lo, ext, cover = (geo[k] for k in ("parts", "so", "ss", "lo", "ext", "cover"))
    inner_y = geo["align"]
    caps = chunk_capacities(meta, cover)
    nel_cover = geo["nel_cover"]
    first = lo[1] * shape[2] * shape[3] if n == 4 else 0
    t0 = time.perf_counter()
    offs, tot = slab_layout(caps)
    full_bytes = geo["full_bytes"]
    plan_mem = strong_memory_plan(geo, tot, rank, backend)
    need = plan_mem["total"]
    if need > info["total_mem"]:
        raise SystemExit(f"[rank {rank}] memory plan: {need / GiB:.1f} GiB needed "
                         f"({json.dumps(plan_mem)}) > {info['total_mem'] / GiB:.1f} GiB on "
                         f"device {device}; use more ranks")
    log(f"[rank {rank}] memory plan: {need / GiB:.1f} of {info['total_mem'] / GiB:.1f} GiB")
    # zh_device_malloc's default (1 GiB VMM chunks at these sizes), as at N = 1
    src = dev.malloc(nel_cover * 4, 0)
    dev.synth_fill(src, nel_cover, 4, first, SEED)
    slab_buf = dev.malloc(tot, 0)
    sizes = dev.array_write(meta, src, lo, ext, [(slab_buf + o, c) for o, c in zip(offs, caps)])
    log(f"[rank {rank}/{ws}] device {device} of {ndev} ({info['arch']}): slab y "
        f"[{so[1]}, {so[1] + ss[1]}), {len(cover)} shards encoded in "
        f"{time.perf_counter() - t0:.2f}s")
    where = {c: (slab_buf + o, s) for c, o, s in zip(cover, offs, sizes)}
    mine = all_coords(L, meta, so, ss)
    nel = 1
    for s in ss:
        nel *= s
    out_bytes = nel * 4
    # the decode's write target: the encode source (it is done with); RCCL only ever sees
    # torch-allocated buffers: a send buffer on every rank and the assembled region on the root
    out = src
    region_t = out_t = None
    if backend == "nccl":
        if rank == 0:
            region_t = torch.empty(full_bytes, dtype=torch.uint8, device=f"cuda:{device}")
            base = slab_byte_offset(shape, so, 4)
            out_t = region_t[base:base + out_bytes]
        else:
            out_t = torch.empty(out_bytes, dtype=torch.uint8, device=f"cuda:{device}")
    plan = dev.plan(meta, [where[c] for c in mine], so, ss, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    st = plan.stats()
    for _ in range(max(1, args.warmup)):
        plan.execute(out)
    plan.wait()
    bad = dev.synth_verify(out, shape, so, ss, 4, SEED)
    if bad:
        raise SystemExit(f"[rank {rank}] slab verification FAILED: {bad} mismatches")
    # this rank's box: the copy ceiling of its own buffers (shards -> output), as at N = 1
    ceil = ceiling_probe(dev, out, slab_buf, min(out_bytes, tot))
    plan.set_timing(True)
    dist.barrier()
    dev.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.execute(out)
    plan.wait()
    dev.sync()
    t_rank = time.perf_counter() - t0
    t_dec = dist.max(t_rank)
    dist.barrier()
    roof = roofline_of(plan, st)
    # each rank's decode against its own copy ceiling (collectives on every rank)
    own = (roof.get("achieved") or 0.0) / max(ceil["copy_ceiling_GBps"], 1e-9)
    roof["frac_of_copy_ceiling_min_over_ranks"] = round(-dist.max(-own), 4)
    roof["frac_of_copy_ceiling_max_over_ranks"] = round(dist.max(own), 4)
    roof["copy_ceiling_GBps_min_over_ranks"] = round(-dist.max(-ceil["copy_ceiling_GBps"]), 1)
    roof["copy_ceiling_GBps_max_over_ranks"] = round(dist.max(ceil["copy_ceiling_GBps"]), 1)
    kern_max = dist.max(roof["kernel_ms"])
    if roof.get("kernel_ms"):  # the line's roofline: the slowest rank's kernel time
        roof["kernel_ms_rank0"] = roof["kernel_ms"]
        roof["achieved"] = round(roof["achieved"] * roof["kernel_ms"] / kern_max, 1)
        roof["frac"] = round(roof["achieved"] / roof["peak"], 4)
        roof["kernel_ms"] = round(kern_max, 3)
        roof["kernel_ms_is"] = "max over ranks"
    gather = None
    if backend in ("nccl", "gloo"):
        def sources(po, ps):  # the chunk sources of one piece of this rank's slab
            return [where[c] for c in all_coords(L, meta, po, ps)]
        gather = gather_to_root(args, dist, dev, backend, plan, out, out_t, region_t, out_bytes,
                                full_bytes, parts, shape, rank, ws, device, t_dec, sources,
                                meta, inner_y)
    host_out = None
    if not args.no_host_out:
        host_out = host_terminated(args, dist, dev, plan, out, out_bytes, shape, so, ss, rank,
                                   ws, inner_y)
    res = {"slab_offset": so, "slab_shape": ss, "device": device, "shared_gpu": shared_gpu,
           "decode_ms_per_step": round(t_dec * 1e3 / args.steps, 3),
           "rank_ms_per_step": round(t_rank * 1e3 / args.steps, 3),
           "value": round(full_bytes * args.steps / t_dec / GiB, 2), "roofline": roof,
           "kernel_ms_max_over_ranks": round(kern_max, 3), "gather": gather,
           "host_terminated": host_out, "info": info}
    plan.close()
    dev.free(out)
    del out_t, region_t
    dev.free(slab_buf)
    return res


def gather_to_root(args, dist, dev, backend, plan, out, out_t, region_t, out_bytes, full_bytes,
                   parts, shape, rank, ws, device, t_dec, sources, meta, align):
    """Assemble the region on rank 0 with the product's gather,
    zarrhip.parallel.RegionGather: every rank's slab is cut into pieces of at most
    --gather-piece-mb (1 GiB) along y at inner-chunk rows; each piece is decoded by a plan of its
    own (zarrhip.parallel.PlanDecoder) straight into the rank's RCCL send buffer (the root: into
    its slice of the region) and sent point-to-point into its place in the root's region as soon
    as its own decode is done, so the decode of piece k+1 runs while piece k is on the wire.  The
    root then re-verifies every element of the assembled region against the generator.
    Reported: the overlapped timeline (value_incl_gather), and for comparison the decode into
    the send buffer followed by the same bounded pieces sent back to back (gather_ms; run(None)
    on buffers the headline plan filled).  gloo (ranks sharing one GPU, rehearsal): through host
    tensors, verified per slab."""
    import torch
    import torch.distributed as tdist
    from zarrhip.parallel import PlanDecoder, RegionGather, gather_pieces
    sizes = [4 * int(__import__("numpy").prod(s)) for _, s in parts]
    cap = int(args.gather_piece_mb) << 20
    sched = gather_pieces(shape, parts, 4, cap, align=align)
    if backend == "nccl":
        grp = tdist.new_group(backend="nccl")
        g = RegionGather([0] * len(shape), shape, 4, group=grp, align=align, piece_bytes=cap,
                         device=device, region=region_t, send=out_t if rank else None)
        world = g.world
        decoder = PlanDecoder(dev, meta, sources)
        # decode straight into this rank's RCCL send buffer (the root: its slice of the
        # region), timed as the headline loop: no staging copy between decode and send
        reps_d = max(1, min(args.steps, 5))
        plan.execute(g.send_buf.data_ptr())
        plan.wait()
        dist.barrier()
        dev.sync()
        tc = time.perf_counter()
        for _ in range(reps_d):
            plan.execute(g.send_buf.data_ptr())
        plan.wait()
        t_dec_send = dist.max(time.perf_counter() - tc) / reps_d
        g.run(None)  # warm the communicator and the P2P channels
        g.run(decoder)
        reps = max(1, min(args.steps, 3))
        dist.barrier()
        t1 = time.perf_counter()
        for _ in range(reps):
            g.run(None)  # the decoded slab sent in bounded pieces, back to back
        t_g = dist.max(time.perf_counter() - t1) / reps
        if rank == 0:
            torch.cuda.synchronize(device)
            region_t.zero_()  # the overlapped timeline must fill every byte again
            torch.cuda.synchronize(device)
        dist.barrier()
        t2 = time.perf_counter()
        for _ in range(reps):
            g.run(decoder)
        t_ov = dist.max(time.perf_counter() - t2) / reps
        bad = 0
        if rank == 0:
            bad = dev.synth_verify(region_t.data_ptr(), shape, [0] * len(shape), shape, 4, SEED)
        bad = int(dist.max(bad))
        if bad:
            raise SystemExit(f"gathered region verification FAILED: {bad}")
        decoder.close()
        how = ("zarrhip.parallel.RegionGather: RCCL point-to-point into the root's region buffer "
               f"(xGMI) in pieces of at most {args.gather_piece_mb} MiB, each sent as soon as its "
               "own plan (PlanDecoder) has decoded it into the send buffer (the root's own slab on "
               "a side stream); gather_ms: the decoded slab sent in the same pieces back to back")
        return {"backend": backend, "how": how, "world_size": world,
                "piece_cap_bytes": cap, "pieces_per_rank": [len(p) for p in sched],
                "max_piece_bytes": max(nb for p in sched for _, _, _, nb in p),
                "gather_ms": round(t_g * 1e3, 3),
                "decode_into_send_ms": round(t_dec_send * 1e3, 3),
                "overlapped_ms": round(t_ov * 1e3, 3),
                "root_ingress_GBps": round((full_bytes - sizes[0]) / t_g / 1e9, 1),
                "value_incl_gather": round(full_bytes / t_ov / GiB, 2),
                "value_incl_gather_sequential": round(full_bytes / (t_dec_send + t_g) / GiB, 2),
                "unit": "GiB/s", "root_verified_elements": full_bytes // 4}
    # gloo (ranks sharing one GPU): a rehearsal through host tensors
    if backend != "nccl":
        world = ws
        mx = max(sizes)
        # host memory on this one box: every rank's slab copy plus the root's receive buffers
        if int(dist.max(0 if _mem_available() >= 2 * ws * mx + (8 << 30) else 1)):
            return {"backend": backend, "world_size": world,
                    "skipped": f"gloo rehearsal gather needs {2 * ws * mx / GiB:.0f} GiB of host "
                               "memory beyond what this box has free (use --ydiv)"}
        host = (C.c_char * out_bytes)()
        dev.memcpy(C.addressof(host), out, out_bytes, 1, None, True)
        send = torch.frombuffer(host, dtype=torch.uint8)
        if out_bytes < mx:
            send = torch.cat([send, torch.zeros(mx - out_bytes, dtype=torch.uint8)])
        recv = [torch.empty(mx, dtype=torch.uint8) for _ in range(ws)] if rank == 0 else None
        dist.barrier()
        t1 = time.perf_counter()
        tdist.gather(send, recv, dst=0)
        t_g = dist.max(time.perf_counter() - t1)
        bad = 0
        if rank == 0:
            chk = dev.malloc(mx)
            for r in range(ws):
                dev.memcpy(chk, recv[r].data_ptr(), sizes[r], 0, None, True)
                bad += dev.synth_verify(chk, shape, parts[r][0], parts[r][1], 4, SEED)
            dev.free(chk)
        bad = int(dist.max(bad))
        if bad:
            raise SystemExit(f"gathered region verification FAILED: {bad}")
        how = "gloo gather through host memory (ranks share one GPU: rehearsal only)"
        t_dec_send = t_dec / args.steps  # the headline decode; the copy out is in t_g
    return {"backend": backend, "how": how, "world_size": world,
            "gather_ms": round(t_g * 1e3, 3),
            "decode_into_send_ms": round(t_dec_send * 1e3, 3),
            "root_ingress_GBps": round((full_bytes - sizes[0]) / t_g / 1e9, 1),
            "value_incl_gather": round(full_bytes / (t_dec_send + t_g) / GiB, 2),
            "unit": "GiB/s", "root_verified_elements": full_bytes // 4}


def dry_run(args, dist, rank, ws):
    """--dry-run: the N>1 harness without a GPU (launch, process group, slab partition,
    barrier, max over ranks, one JSON line); no decode runs, so there is no value."""
    from zarrhip.parallel import gather_pieces, slab_partition
    shape = [1, 4096, 4096, 1536]
    parts = slab_partition([0] * 4, shape, ws, align=32)
    so, ss = parts[rank]
    sched = gather_pieces(shape, parts, 4, int(args.gather_piece_mb) << 20, align=32)
    dist.barrier()
    rows = int(dist.max(ss[1]))
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": ws,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": None,
                          "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
                          "dtype": "u32", "data": "synthetic", "dry_run": True,
                          "config": {"workload": "dry run (no GPU): harness only",
                                     "slab_rows_max": rows,
                                     "gather_pieces_per_rank": [len(p) for p in sched],
                                     "gather_max_piece_bytes": max(
                                         nb for p in sched for _, _, _, nb in p),
                                     "parallelism": f"slab-parallel x{ws}"}}), flush=True)


# ------------------------------------------------------------------------------------------
# write path
# ------------------------------------------------------------------------------------------
def run_write(args, dist, dev, A, meta, shape, region, out_bytes, shard_slab, offs, caps, rank,
              ws):
    """Write path: zh_array_write of the full array = core.Array.write
    + ShardingIndexedCodec.encode of every shard (one pass: speculative C-order layout with
    the all-fill test fused, index + crc32c on the device) from the device-resident region
    into device shard buffers.  The call synchronises internally, so it is timed by wall
    clock; the written shards are verified by decoding them and checking every element.
    --sparse zeroes (= fill_value) the first row of inner chunks along y, so that 1/128 of the
    chunks are elided and every call takes the second pass (the reference's layout)."""
    n = len(shape)
    dsts = [(shard_slab + o, c) for o, c in zip(offs, caps)]
    zbytes = 0
    if args.sparse:
        ch = meta.chain
        leaf = (ch.nested_chunk_shape if ch.nested else ch.inner_chunk_shape) if ch.sharded \
            else meta.chunk_shape
        zy = int(leaf[1])
        zbytes = zy * shape[2] * shape[3] * 4
        dev.memset(region, 0, zbytes)
    for _ in range(max(1, args.warmup)):
        sizes = dev.array_write(meta, region, [0] * n, shape, dsts)
    dist.barrier()
    dev.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sizes = dev.array_write(meta, region, [0] * n, shape, dsts)
    dev.sync()
    elapsed = dist.max(time.perf_counter() - t0)
    in_bytes = sum(sizes)
    # a deleted (all fill_value) chunk is a missing key: the read fills it
    plan = dev.plan(meta, [(shard_slab + o, s) if s else (None, 0) for o, s in zip(offs, sizes)],
                    [0] * n, shape, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    dev.memset(region, 0, out_bytes)
    plan.execute(region)
    plan.wait()
    plan.close()
    if zbytes:
        rest = [shape[0], shape[1] - zy] + list(shape[2:])
        bad = dev.synth_verify(region + zbytes, shape, [0, zy] + [0] * (n - 2), rest, 4, SEED)
        import numpy as np
        step = 1 << 30
        for o in range(0, zbytes, step):
            blk = np.frombuffer(dev.d2h(region + o, min(step, zbytes - o)), np.uint8)
            bad += int(np.count_nonzero(blk))
    else:
        bad = dev.synth_verify(region, shape, [0] * n, shape, 4, SEED)
    if bad:
        raise SystemExit(f"write round trip FAILED: {bad} mismatching elements")
    log(f"[rank {rank}] write path verified: decode of the written shards == generator")
    ms = elapsed * 1000.0 / args.steps
    achieved = (in_bytes + out_bytes) / (ms / 1000.0) / 1e9
    if rank == 0:
        print(json.dumps({
            "metric": "GiB/s device-resident chunk encode (sharding+bytes+transpose), "
                      "uint32 1024³ — write path",
            "value": round(ws * args.steps * out_bytes / elapsed / GiB, 2), "unit": "GiB/s",
            "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": f"{args.config}: Array.write of the full "
                                   f"{'sparse (first y-row of inner chunks = fill_value) ' if zbytes else ''}"
                                   f"{'x'.join(map(str, shape))} uint32 array, "
                                   f"{CONFIGS[args.config][0]}",
                       "encoded_bytes": in_bytes, "decoded_bytes_per_gpu": out_bytes,
                       "parallelism": f"shard-parallel x{ws}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None, "kernel": "zh_array_write (whole call, wall clock)",
                         "alg_bytes_per_launch": in_bytes + out_bytes}}), flush=True)


# ------------------------------------------------------------------------------------------
# N = 1 extras: other configs, one-shot read
# ------------------------------------------------------------------------------------------
def time_steps(dev, plan, out, steps):
    """Per-step wall times (execute + wait each) → (min, median) ms."""
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        plan.execute(out)
        plan.wait()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts.sort()
    return ts[0], ts[len(ts) // 2]


def extra_config(dev, A, L, cfg, out, shape, steps, slab=None):
    """Re-encode the resident decoded array (= the generator's values) with config `cfg`,
    decode it `steps` times, verify every element, and report its rate and roofline.
    Reuses `slab` when it holds the encoded size; returns (result, slab, slab_bytes)."""
    meta = build_meta(A, cfg)
    n = meta.ndim
    coords = all_coords(L, meta)
    caps = chunk_capacities(meta, coords)
    offs, tot = slab_layout(caps)
    buf, cap = slab if slab else (None, 0)
    if cap < tot:
        if buf:
            dev.free(buf)
        buf, cap = dev.malloc(tot), tot
    sizes = dev.array_write(meta, out, [0] * n, shape, [(buf + o, c) for o, c in zip(offs, caps)])
    plan = dev.plan(meta, [(buf + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                    A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    st = plan.stats()
    dev.memset(out, 0, st["out_bytes"])
    for _ in range(2):
        plan.execute(out)
    plan.wait()
    bad = dev.synth_verify(out, shape, [0] * n, shape, 4, SEED)
    if bad:
        raise SystemExit(f"{cfg} decode verification FAILED: {bad}")
    plan.set_timing(True)
    dev.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        plan.execute(out)
    plan.wait()
    el = time.perf_counter() - t0
    roof = roofline_of(plan, st, cfg)
    plan.set_timing(False)
    mn, med = time_steps(dev, plan, out, 5)
    plan.close()
    res = {"description": CONFIGS[cfg][0], "value": round(steps * st["out_bytes"] / el / GiB, 2),
           "unit": "GiB/s", "ms_per_step": round(el * 1e3 / steps, 3), "steps": steps,
           "step_ms_min": round(mn, 3), "step_ms_median": round(med, 3),
           "allocations_sampled": {"output": 1, "input_slab": 1},
           "verified_elements": st["out_bytes"] // 4, "roofline": roof}
    return res, (buf, cap)


def store_inclusive(dev, A, shard_slab, offs, sizes, coords, scratch):
    """core.Array.read from a FilesystemStore on tmpfs through the Python mirror of the
    reference's Array (zarrhip.Array.read: store reads of the shard files — whole shards, or
    the index + the referenced inner-chunk ranges of a partly covered shard
    (StoreHandleDataProvider) — then one zh_array_read: pageable H2D, decode, D2H into a
    numpy array).  Region 1: shards (0,0,0,0) and (0,0,0,1), [1,1024,1024,1536] (6 GiB out);
    region 2: BASELINE.md §3's sub-shard read [1,1024,1024,512] (the CPU baseline's
    workload).  Every element of region 1 is verified against the generator."""
    import shutil
    import numpy as np
    import zarrhip as z
    want = [(0, 0, 0, 0), (0, 0, 0, 1)]
    pos = {c: i for i, c in enumerate(coords)}
    need = sum(sizes[pos[c]] for c in want)
    d = _store_dir(need + (8 << 30))
    if d is None:
        return {"skipped": "no tmpfs room for the two shard files"}
    base = os.path.join(d, f"zh_store_{os.getpid()}")
    res = {}
    try:
        m = (z.ArrayMetadataBuilder().withShape(1, 4096, 4096, 1536)
             .withDataType(z.DataType.UINT32).withChunkShape(1, 1024, 1024, 1024).withFillValue(0)
             .withCodecs(lambda c: c.withSharding(
                 [1, 32, 32, 32], lambda c1: c1.withTranspose([0, 3, 2, 1]).withBytes("BIG")))
             .build())
        z.Array.create(z.FilesystemStore(base).resolve("c4"), m)
        pin = dev.malloc_pinned(max(sizes[pos[c]] for c in want))
        for c in want:
            i = pos[c]
            path = os.path.join(base, "c4", "c", *map(str, c))
            os.makedirs(os.path.dirname(path), exist_ok=True)
            dev.memcpy(pin, shard_slab + offs[i], sizes[i], 1, None, True)
            with open(path, "wb") as f:
                f.write((C.c_char * sizes[i]).from_address(pin))
        dev.free_pinned(pin)
        arr = z.Array.open(z.FilesystemStore(base).resolve("c4"))
        shape = [1, 4096, 4096, 1536]
        def timed(off, shp, reps):
            ts, parts = [], []
            got = None
            for _ in range(reps):
                del got  # the previous result's pages go back outside the timed call
                arr.staged_bytes = 0
                t0 = time.perf_counter()
                got = arr.read(off, shp)
                ts.append(time.perf_counter() - t0)
                parts.append(arr.last_read_timing)
            return got, ts, parts[ts.index(min(ts))]

        for name, off, shp, reps in (("two_shards", [0, 0, 0, 0], [1, 1024, 1024, 1536], 2),
                                     ("sub_shard", [0, 0, 0, 512], [1, 1024, 1024, 512], 3)):
            # the mirror's own store reads into staging buffers, then one library read
            # (ZH_FILES=0; the default before zh_array_read_files)
            os.environ["ZH_FILES"] = "0"
            try:
                got, ts0, p0 = timed(off, shp, reps)
                staged = arr.staged_bytes
            finally:
                os.environ.pop("ZH_FILES", None)
            del got
            got, ts, p = timed(off, shp, reps)  # the default: the library reads the files
            nb = got.nbytes
            r = {"region_offset": off, "region_shape": shp, "ms_min": round(min(ts) * 1e3, 1),
                 "value": round(nb / min(ts) / GiB, 2), "unit": "GiB/s",
                 "call": "zh_array_read_files (pread into the pipelined read's page-locked "
                         "ring)" if p.get("files") else "store reads + zh_array_read_pieces",
                 "store_reads": {"ms_min": round(min(ts0) * 1e3, 1),
                                 "value": round(nb / min(ts0) / GiB, 2),
                                 "store_stage_ms": round(p0["stage_s"] * 1e3, 1),
                                 "zh_array_read_ms": round(p0["device_s"] * 1e3, 1),
                                 "staged_bytes": staged}}
            dev.memcpy(scratch, got.ctypes.data, nb, 0, None, True)
            r["verify_mismatches"] = int(dev.synth_verify(scratch, shape, off, shp, 4, SEED))
            res[name] = r
            del got
        # BASELINE configs[0]'s call shape from the store: Array.read of the unaligned 64^3 region
        # {0,3,517,501} (27 inner chunks, most clipped) from the shard file, median of 200
        sro, srs = [0, 3, 517, 501], [1, 64, 64, 64]
        small = {"region_offset": sro, "region_shape": srs, "reps": 200}
        for mode in ("store_reads", "files"):
            if mode == "store_reads":
                os.environ["ZH_FILES"] = "0"
            try:
                ts = []
                for k in range(220):
                    t0 = time.perf_counter()
                    got = arr.read(sro, srs)
                    if k >= 20:
                        ts.append(time.perf_counter() - t0)
            finally:
                os.environ.pop("ZH_FILES", None)
            ts.sort()
            small[("us_median" if mode == "files" else "store_reads_us_median")] = \
                round(ts[len(ts) // 2] * 1e6, 1)
        dev.memcpy(scratch, got.ctypes.data, got.nbytes, 0, None, True)
        small["verify_mismatches"] = int(dev.synth_verify(scratch, shape, sro, srs, 4, SEED))
        small["call"] = ("zarrhip.Array.read → zh_array_read_files (index + 27 ranges pread, one "
                         "plan) into a fresh numpy array; store_reads: the mirror's store reads "
                         "+ zh_array_read_pieces")
        res["small_read"] = small
        # the write side: Array.write of shard (0,0,0,0)'s region from host memory into a fresh
        # FilesystemStore — the library encodes and writes the file (zh_array_write_files) vs
        # the mirror's own store writes (ZH_FILES=0); the file must equal the stored shard
        wshp = [1, 1024, 1024, 1024]
        wdata = arr.read([0, 0, 0, 0], wshp)
        src_path = os.path.join(base, "c4", "c", "0", "0", "0", "0")
        wres = {"region_offset": [0, 0, 0, 0], "region_shape": wshp,
                "bytes_in": int(wdata.nbytes)}
        for mode in ("store_writes", "files"):
            tgt = os.path.join(base, "w_" + mode)
            wa = z.Array.create(z.FilesystemStore(tgt).resolve("c4"), m)
            if mode == "store_writes":
                os.environ["ZH_FILES"] = "0"
            try:
                t0 = time.perf_counter()
                wa.write([0, 0, 0, 0], wdata)
                tw = time.perf_counter() - t0
            finally:
                os.environ.pop("ZH_FILES", None)
            out_path = os.path.join(tgt, "c4", "c", "0", "0", "0", "0")
            same = os.path.getsize(out_path) == os.path.getsize(src_path)
            if same:
                a_ = np.memmap(out_path, np.uint8, "r")
                b_ = np.memmap(src_path, np.uint8, "r")
                for o in range(0, a_.size, 256 << 20):
                    if not np.array_equal(a_[o:o + (256 << 20)], b_[o:o + (256 << 20)]):
                        same = False
                        break
                del a_, b_
            r = {"ms": round(tw * 1e3, 1), "value": round(wdata.nbytes / tw / GiB, 2),
                 "unit": "GiB/s", "file_equals_stored_shard": bool(same)}
            if mode == "files":
                wres.update(r)
            else:
                wres["store_writes"] = r
            shutil.rmtree(tgt, ignore_errors=True)
        wres["call"] = ("zarrhip.Array.write → zh_array_write_files (H2D, device encode, D2H "
                        "through the page-locked ring, pwrite by the copy lanes); store_writes: "
                        "the mirror's encode + per-chunk store writes (ZH_FILES=0)")
        res["write"] = wres
        del wdata
        res["path"] = ("zarrhip.Array.read (Python mirror of core.Array.read) from a "
                       f"FilesystemStore on {d}: one zh_array_read_files call — the library "
                       "reads each shard's stored index and the ranges the region references "
                       "(whole shards: all of them) with pread straight into the pipelined "
                       "read's page-locked ring, overlapped with the H2D, the index crc32c and "
                       "decode on the device and the D2H into a fresh numpy array; "
                       "store_reads: the same read with the store reads done by the mirror "
                       "into staging buffers first (ZH_FILES=0)")
    finally:
        shutil.rmtree(base, ignore_errors=True)
    return res


def shuffled_variant(dev, A, L, meta, out, shape, slab, offs, sizes, steps, classes=5):
    """SURVEY §8(d)'s second variant: the same c4 shards with their inner chunks stored out of
    C order (Q7: the reference appends them in a nondeterministic order), so only the index
    says where each chunk is.  Chunk rank k moves to class k mod `classes`, each class packed
    in rank order (one block-gather kernel per shard), then the index entries are rewritten
    and re-checksummed.  Decoded, verified against the generator, timed like the headline."""
    import struct
    import numpy as np
    n = meta.ndim
    cb = 4 * 32 * 32 * 32                       # stored inner chunk bytes (c4: 128 KiB)
    isz = int(L.zh_shard_index_size(C.byref(meta)))
    tmp = dev.malloc(max(sizes))
    for o, sz in zip(offs, sizes):
        nchunk = (sz - isz) // cb
        base = slab + o
        starts, pos, src_of = [], 0, []
        for r in range(classes):
            cnt = (nchunk - r + classes - 1) // classes if nchunk > r else 0
            starts.append(pos)
            src_of.extend(range(r, nchunk, classes))
            pos += cnt
        dev.gather_blocks(tmp, base, cb, src_of)      # new position p <- old rank src_of[p]
        dev.memcpy(base, tmp, nchunk * cb, 2, None, True)
        ib = bytearray(dev.d2h(base + sz - isz, isz))
        ent = np.frombuffer(ib, "<u8", count=(isz - 4) // 8).reshape(-1, 2).copy()
        live = ent[:, 0] != np.uint64(2 ** 64 - 1)
        rank = (ent[live, 0] // np.uint64(cb)).astype(np.int64)
        newpos = np.asarray(starts, np.int64)[rank % classes] + rank // classes
        ent[live, 0] = (newpos * cb).astype(np.uint64)
        body = ent.tobytes()
        crc = L.zh_crc32c(0, body, len(body))
        dev.h2d(base + sz - isz, body + struct.pack("<I", crc))
    dev.free(tmp)
    plan = dev.plan(meta, [(slab + o, sz) for o, sz in zip(offs, sizes)], [0] * n, shape,
                    A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    st = plan.stats()
    dev.memset(out, 0, st["out_bytes"])
    plan.execute(out)
    plan.wait()
    bad = dev.synth_verify(out, shape, [0] * n, shape, 4, SEED)
    if bad:
        raise SystemExit(f"shuffled-order decode verification FAILED: {bad}")
    plan.set_timing(True)
    dev.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        plan.execute(out)
    plan.wait()
    el = time.perf_counter() - t0
    roof = roofline_of(plan, st)
    plan.close()
    return {"description": f"c4 with each shard's inner chunks stored in {classes} interleaved "
                           "classes (rank k → class k mod 5), index rewritten: decoding follows "
                           "the index (Q7)",
            "value": round(steps * st["out_bytes"] / el / GiB, 2), "unit": "GiB/s",
            "ms_per_step": round(el * 1e3 / steps, 3), "verified_elements": st["out_bytes"] // 4,
            "roofline": roof}


def oneshot_read(dev, A, meta, sources, shape, out, reps=3):
    """zh_array_read of the whole array, device in and out: plan + tables upload + execute +
    status read-back + teardown in one call, as core.Array.read does every call."""
    n = meta.ndim
    ts = []
    for _ in range(reps):
        dev.sync()
        t0 = time.perf_counter()
        dev.array_read(meta, sources, [0] * n, shape, out, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
        ts.append(time.perf_counter() - t0)
    bad = dev.synth_verify(out, shape, [0] * n, shape, 4, SEED)
    if bad:
        raise SystemExit(f"one-shot read verification FAILED: {bad}")
    nb = 4
    for s in shape:
        nb *= s
    ts.sort()
    return {"ms_min": round(ts[0] * 1e3, 3), "ms_median": round(ts[len(ts) // 2] * 1e3, 3),
            "value": round(nb / ts[len(ts) // 2] / GiB, 2), "unit": "GiB/s", "reps": reps,
            "call": "zh_array_read (plan + execute + wait + teardown), device in/out"}


def small_read(dev, A, meta, sources, coords, shape, reps=200):
    """BASELINE configs[0]'s call shape (the reference's l4_sample read of a 1x64x64x64
    region, ZarrV3Test.java:283-307) on this array's device-resident c4 shards: one-shot
    zh_array_read (plan + execute + status + teardown, as core.Array.read does per call) of an
    unaligned 64³ region (offset {0,3,517,501}: 27 inner chunks, most clipped, one shard and
    its 512 KiB index crc32c), into device memory and into pageable host memory (a Java
    array).  Median of `reps` after 20 warmups; both results verified against the generator."""
    import statistics
    off, shp = [0, 3, 517, 501], [1, 64, 64, 64]
    pos = {c: i for i, c in enumerate(coords)}
    src = [sources[pos[(0, 0, 0, 0)]]]
    nb = 4 * 64 ** 3
    host = (C.c_char * nb)()
    out = dev.malloc(nb)  # its own buffer: the caller's `out` holds the decoded array, reused
    res = {"region_offset": off, "region_shape": shp, "reps": reps}
    for tag, dst, flags in (("device_out_us", out, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE),
                            ("pageable_host_out_us", C.addressof(host), A.ZH_SRC_DEVICE)):
        ts = []
        for i in range(reps + 20):
            t0 = time.perf_counter()
            dev.array_read(meta, src, off, shp, dst, flags)
            if i >= 20:
                ts.append(time.perf_counter() - t0)
        res[tag] = round(statistics.median(ts) * 1e6, 1)
        if dst != out:
            dev.memcpy(out, dst, nb, 0, None, True)
        bad = int(dev.synth_verify(out, shape, off, shp, 4, SEED))
        if bad:
            raise SystemExit(f"small read verification FAILED ({tag}): {bad}")
    dev.free(out)
    res["call"] = "zh_array_read one shot (plan + execute + status + teardown), device shard in"
    return res


# ------------------------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="N=1: skip extra_configs (c3, c2, c4le) and the one-shot read")
    ap.add_argument("--op", default="read", choices=["read", "write"],
                    help="read: the decode path (the metric); write: zh_array_write, the "
                         "encode path (SURVEY §8(f) rank 1)")
    ap.add_argument("--sparse", action="store_true",
                    help="--op write: elide 1/128 of the inner chunks (all fill_value), so the "
                         "write takes its second pass")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--allocations", type=int, default=3,
                    help="N=1 read: time the K steps on this many fresh output allocations "
                         "(value = the median one; min and max alongside)")
    ap.add_argument("--mode", default=None, choices=["weak", "strong"],
                    help="default: weak at N=1 (one full array), strong at N>1 (one array "
                         "split into per-GPU slabs + gather + host-terminated copy)")
    ap.add_argument("--gather-backend", default="nccl", choices=["nccl", "gloo", "none"])
    ap.add_argument("--gather-piece-mb", type=int, default=1024,
                    help="strong mode: largest RCCL message of the overlapped gather (MiB)")
    ap.add_argument("--no-host-out", action="store_true",
                    help="strong mode: skip the host-terminated copy")
    ap.add_argument("--ydiv", type=int, default=1,
                    help="rehearsal only: divide the array's y extent (not a bench config)")
    ap.add_argument("--no-host-inclusive", action="store_true",
                    help="N=1 c4: skip the host-terminated read (pinned and pageable host "
                         "shards in, host array out: 'host_inclusive')")
    ap.add_argument("--dry-run", action="store_true",
                    help="N>1 harness without a GPU (launch, partition, barrier, JSON line)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus))
    ws, rank, local = dist_env()
    if args.gpus != ws:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {ws}: measuring {ws} rank(s)")
    mode = args.mode or ("strong" if ws > 1 else "weak")
    if args.gather_backend == "none":
        args.gather_backend = None
    dist = Dist(ws, need_torch=mode == "strong")
    if args.dry_run:
        dry_run(args, dist, rank, ws)
        dist.close()
        return

    from zarrhip import _abi as A
    meta = build_meta(A, args.config, args.ydiv)
    if mode == "strong":
        res = run_strong(args, dist, A, meta, rank, ws, local)
        log(f"[rank {rank}] strong: {json.dumps(res)}")
        if rank == 0:
            n = meta.ndim
            g = res["gather"]
            print(json.dumps({
                "metric": METRIC, "value": res["value"], "unit": "GiB/s",
                "n_gpus": g["world_size"] if g else ws, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": res["decode_ms_per_step"],
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
                "dtype": "u32", "data": "synthetic",
                "config": {"workload": f"{args.config}: one Array.read of the full "
                                       f"{'x'.join(str(meta.shape[d]) for d in range(n))} "
                                       f"uint32 array ({CONFIGS[args.config][0]}) split into "
                                       f"{ws} contiguous y-slabs of {res['slab_shape'][1]} rows, "
                                       f"one per GPU; value = decode-only aggregate",
                           "parallelism": f"slab-parallel x{ws}",
                           "ranks_share_one_gpu": res["shared_gpu"],
                           "output_allocation": "hipMalloc per rank; RCCL buffers: torch"},
                "roofline": res["roofline"],
                "kernel_ms_max_over_ranks": res["kernel_ms_max_over_ranks"],
                "gather": g, "host_terminated": res["host_terminated"],
                "cpu_baseline": None}), flush=True)
        dist.close()
        return

    from zarrhip._lib import DeviceContext, lib
    # one GPU per rank; ranks beyond the visible GPUs share them (a rehearsal on fewer cards)
    dev = DeviceContext(int(os.environ.get(
        "ZH_DEVICE", local % max(1, visible_devices()) if local else 0)))
    info = dev.info()
    n = meta.ndim
    shape = [meta.shape[d] for d in range(n)]
    L = lib()
    coords = all_coords(L, meta)
    caps = chunk_capacities(meta, coords)
    nel = 1
    for s in shape:
        nel *= s
    out_bytes = nel * 4

    # device buffers: decoded region (also the encode source) + one slab for all shards, the
    # library's default kind (zh_device_malloc: 1 GiB physical chunks at this size, the highest
    # floor of the round-6 allocation A/B, DESIGN §4 "Placement"; ZH_MALLOC picks another kind)
    t0 = time.perf_counter()
    offs, tot = slab_layout(caps)
    out = dev.malloc(max(out_bytes, tot))
    shard_slab = dev.malloc(max(out_bytes, tot))
    alloc_kind = ("zh_device_malloc's default: 1 GiB physical chunks (ZH_MALLOC_SCATTER) for "
                  "buffers of 1 GiB or more" if int(os.environ.get("ZH_MALLOC", "0"), 0) == 0
                  else f"zh_device_malloc_ex flags {os.environ['ZH_MALLOC']}")
    dev.synth_fill(out, nel, 4, 0, SEED)
    dev.sync()
    t1 = time.perf_counter()
    sizes = dev.array_write(meta, out, [0] * n, shape,
                            [(shard_slab + o, c) for o, c in zip(offs, caps)])
    t2 = time.perf_counter()
    assert all(s == c for s, c in zip(sizes, caps)), (sizes[:4], caps[:4])
    log(f"[rank {rank}] {info['name']} {info['arch']} cus={info['cu_count']}: synth "
        f"{t1 - t0:.2f}s, device encode {t2 - t1:.2f}s ({sum(sizes) / GiB:.2f} GiB in "
        f"{len(sizes)} shards)")

    if args.op == "write":
        run_write(args, dist, dev, A, meta, shape, out, out_bytes, shard_slab, offs, caps, rank,
                  ws)
        dev.free(shard_slab)
        dev.free(out)
        dist.close()
        return
    flags = A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE
    sources = [(shard_slab + o, s) for o, s in zip(offs, sizes)]
    plan = dev.plan(meta, sources, [0] * n, shape, flags)
    st = plan.stats()
    state0 = gpu_state(dev.device, static=True) if rank == 0 else None
    # the headline over several fresh output allocations (which physical
    # memory a 96 GiB buffer gets moves the rate; DESIGN §4 "Placement"): W warmup steps, the
    # verify, then exactly K timed steps on each; value = the median allocation's rate
    runs = []
    for a in range(max(1, args.allocations)):
        if a:
            out = reallocate(dev, out, max(out_bytes, tot), a)
        ev = ceiling_probe(dev, out, shard_slab, out_bytes)
        dev.memset(out, 0, out_bytes)
        for _ in range(max(1, args.warmup)):
            plan.execute(out)
        plan.wait()
        bad = dev.synth_verify(out, shape, [0] * n, shape, 4, SEED)
        if bad:
            raise SystemExit(f"decode verification FAILED: {bad} mismatching elements")
        plan.set_timing(True)
        dist.barrier()
        dev.sync()
        t_start = time.perf_counter()
        for _ in range(args.steps):
            plan.execute(out)
        plan.wait()
        t_end = time.perf_counter()
        dist.barrier()
        elapsed = dist.max(t_end - t_start)
        roof = roofline_of(plan, st, args.config if args.ydiv == 1 else None)
        plan.set_timing(False)
        ev["frac_of_copy_ceiling"] = round(roof["achieved"] / ev["copy_ceiling_GBps"], 4)
        runs.append({"elapsed": elapsed, "roofline": roof, "evidence": ev,
                     "verified_elements": nel})
        log(f"[rank {rank}] allocation {a}: {args.steps * out_bytes / elapsed / GiB:.1f} GiB/s, "
            f"kernel {roof['kernel_ms']} ms, {json.dumps(ev)} (verified {nel} elements)")
    order = sorted(range(len(runs)), key=lambda i: runs[i]["elapsed"])
    med = runs[order[len(runs) // 2]]  # the median (of an even count, the slower middle one)
    elapsed = med["elapsed"]
    ms_per_step = elapsed * 1000.0 / args.steps
    value = ws * args.steps * out_bytes / elapsed / GiB
    roofline = dict(med["roofline"])
    roofline.update(med["evidence"])
    allocs = {"count": len(runs), "kind": alloc_kind, "value": "median allocation",
              "GiBps": [round(ws * args.steps * out_bytes / r["elapsed"] / GiB, 2)
                        for r in runs],
              "kernel_ms": [r["roofline"]["kernel_ms"] for r in runs],
              "frac": [r["roofline"]["frac"] for r in runs],
              "copy_ceiling_GBps": [r["evidence"]["copy_ceiling_GBps"] for r in runs],
              "store_probe_GBps": [r["evidence"]["store_probe_GBps"] for r in runs],
              "frac_of_copy_ceiling": [r["evidence"]["frac_of_copy_ceiling"] for r in runs]}
    allocs["GiBps_min"], allocs["GiBps_max"] = min(allocs["GiBps"]), max(allocs["GiBps"])
    hinc = None
    if (not args.no_host_inclusive and ws == 1 and args.ydiv == 1 and args.config == "c4"
            and meta.chain.sharded):
        hinc = host_inclusive(dev, A, meta, coords, offs, sizes, shard_slab, out)
        log(f"[rank {rank}] host-inclusive: {hinc}")
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and meta.chain.sharded:
        cpu = cpu_baseline(dev, A, L, meta, shard_slab + offs[0], sizes[0], args.cpu_budget)
        log(f"[rank {rank}] cpu baseline: {json.dumps(cpu)}")

    line = {
        "metric": METRIC,
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": ws, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": f"{args.config}: Array.read of the full {'x'.join(map(str, shape))} uint32 "
                               f"array, {CONFIGS[args.config][0]}",
                   "array_shape": shape, "chunk_shape": [1, 1024, 1024, 1024],
                   "inner_chunk_shape": [1, 32, 32, 32] if meta.chain.sharded else None,
                   "shards": st["shards"], "inner_chunks": st["items"],
                   "decoded_bytes_per_gpu": out_bytes, "parallelism": f"shard-parallel x{ws}",
                   "output_allocation": f"{alloc_kind} (the output and the shard slab)"},
        "roofline": roofline,
        "allocations": allocs,
        "gpu_state": {"start": state0, "end": gpu_state(dev.device) if rank == 0 else None},
        "cpu_baseline": cpu,
    }
    if hinc is not None:
        line["host_inclusive"] = hinc
    if not args.no_extras and ws == 1 and args.ydiv == 1 and args.config == "c4":
        line["oneshot_read"] = oneshot_read(dev, A, meta, sources, shape, out)
        line["small_read"] = small_read(dev, A, meta, sources, coords, shape)
        log(f"[rank {rank}] small read: {json.dumps(line['small_read'])}")
        plan.close()
        plan = None
        extras = {}
        slab = (shard_slab, tot)
        for cfg in ("c4le", "c3", "c2"):
            extras[cfg], slab = extra_config(dev, A, L, cfg, out, shape, min(args.steps, 10),
                                             slab)
            log(f"[rank {rank}] {cfg}: {json.dumps(extras[cfg])}")
        shard_slab = slab[0]
        line["extra_configs"] = extras
        # the store-inclusive read needs the c4 shards again: re-encode them into the slab
        sizes = dev.array_write(meta, out, [0] * n, shape,
                                [(shard_slab + o, c) for o, c in zip(offs, caps)])
        line["store_inclusive"] = store_inclusive(dev, A, shard_slab, offs, sizes, coords,
                                                  out + (8 << 30))
        log(f"[rank {rank}] store-inclusive: {json.dumps(line['store_inclusive'])}")
        extras["c4shuf"] = shuffled_variant(dev, A, L, meta, out, shape, shard_slab, offs,
                                            sizes, min(args.steps, 10))
        log(f"[rank {rank}] c4shuf: {json.dumps(extras['c4shuf'])}")
    if plan is not None:
        plan.close()
    dev.free(shard_slab)
    if out is not None:
        dev.free(out)
    if rank == 0:
        print(json.dumps(line), flush=True)
    dist.close()


if __name__ == "__main__":
    main()
