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
(+ transpose) + scatter, inputs already resident in HBM.  Synthetic data v(g) = lo32(splitmix64(g ^ 0x5A5A2026)) is written
on the device and encoded by the product's own write path (zh_array_write); after warmup
the decoded array is verified element-by-element on the device against the generator.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c3|c2|c3crc|c4crc|c3nest]

N>1 (launched by torch.distributed.run): every rank decodes its own full-size array on its
own GPU (weak scaling, no data-path collective: shards are independent objects); the
barrier and max-over-ranks timing use torch.distributed (gloo, CPU tensors).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zarr-java_amd"))

SEED = 0x5A5A2026
GiB = 1 << 30
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

CONFIGS = {
    # name: (description, sharded, transpose order[, extra make_meta keywords])
    "c2": ("bytes(big) only, chunk 1x1024x1024x1024", False, None),
    "c3": ("sharding 1x32x32x32 + bytes(big), index [bytes(little), crc32c] at end", True, None),
    "c4": ("c3 + transpose [0,3,2,1] inside the shard", True, [0, 3, 2, 1]),
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
    return A.make_meta([1, 4096 // ydiv, 4096, 1536], [1, 1024, 1024, 1024], 4,
                       endian=A.ZH_ENDIAN_BIG, sharded=sharded, **extra,
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


def pmc_traffic(config):
    """HBM bytes per launch of the scatter kernel from the newest committed PMC summary for
    this config (profiles/rNN/<config>_summary.json, made by profiles/pmc_summary.py from
    separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes, FETCH_SIZE x2 per the gfx950 note)."""
    import glob
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"{config}_summary.json")))
    if not cands:
        return None, None
    d = json.load(open(cands[-1]))
    return int(d["pmc"]["traffic_bytes_per_launch"]), os.path.relpath(cands[-1], ROOT)


def host_inclusive(dev, A, meta, coords, offs, sizes, shard_slab, n_shards=4, reps=2, slabs=8,
                   nslots=3):
    """Host-resident bytes in, host-resident decoded array out: the readChunk /
    ShardingIndexedCodec.decode(ByteBuffer) of `n_shards` interior shards (4 GiB each way)
    from pinned host memory, pipelined over three streams (H2D | decode | D2H) so PCIe traffic
    in both directions overlaps the decode.  Each shard moves as `slabs` y-slabs: a slab's
    inner chunks are one contiguous byte range of the C-order payload, so a unit is that
    range + the index, copied into a device slot that mirrors the shard's address range (the
    decode touches only the index and the referenced chunks), and its decoded rows are one
    contiguous part of the shard's output.  32 units of 512 MiB instead of 4 of 4 GiB cut
    the pipeline's fill and drain from a quarter of the run to 1/32."""
    n = meta.ndim
    cs = [meta.chunk_shape[d] for d in range(n)]
    sel = [i for i, c in enumerate(coords)
           if all((c[d] + 1) * cs[d] <= meta.shape[d] for d in range(n))][:n_shards]
    in_sz = [sizes[i] for i in sel]
    out_sz = 4
    for c in cs:
        out_sz *= c
    ch = meta.chain
    inner = [ch.inner_chunk_shape[d] for d in range(n)]
    cps = 1
    for d in range(n):
        cps *= cs[d] // inner[d]
    isz = 16 * cps + 4
    cn = 4
    for d in range(n):
        cn *= inner[d]
    ys = cs[1] // slabs                    # decoded rows per slab (dim 0 is 1)
    slab_chunks = cps // slabs             # inner chunks per slab: contiguous in C order
    slab_in, slab_out = slab_chunks * cn, out_sz // slabs
    assert cs[0] == 1 and ys % inner[1] == 0 and all(s == in_sz[0] for s in in_sz)
    hin = dev.malloc_pinned(sum(in_sz))
    hout = dev.malloc_pinned(out_sz * len(sel))
    pos, p = [], 0
    for k, i in enumerate(sel):  # stage the encoded shards into pinned host memory
        pos.append(p)
        dev.memcpy(hin + p, shard_slab + offs[i], in_sz[k], 1, None, True)
        p += in_sz[k]
    smeta = A.zh_array_meta.from_buffer_copy(meta)
    for d in range(n):
        smeta.shape[d] = cs[d]
    din = [dev.malloc(in_sz[0]) for _ in range(nslots)]
    dout = [dev.malloc(slab_out) for _ in range(nslots)]
    flags = A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE
    plans = [[dev.plan(smeta, [(din[j], in_sz[0])], [0, ys * q] + [0] * (n - 2),
                       [1, ys] + cs[2:], flags) for q in range(slabs)] for j in range(nslots)]
    s_in, s_dec, s_out = dev.stream(), dev.stream(), dev.stream()
    units = [(k, q) for k in range(len(sel)) for q in range(slabs)]
    times = []
    for _ in range(reps):
        ev = [[dev.event() for _ in range(3)] for _ in units]
        dev.sync()
        t0 = time.perf_counter()
        for u, (k, q) in enumerate(units):
            j = u % nslots
            if u >= nslots:
                dev.wait_event(s_in, ev[u - nslots][1])       # slot j's input consumed
            ioff = in_sz[k] - isz                             # index at the end
            dev.memcpy(din[j] + q * slab_in, hin + pos[k] + q * slab_in, slab_in, 0, s_in, False)
            dev.memcpy(din[j] + ioff, hin + pos[k] + ioff, isz, 0, s_in, False)
            dev.record(ev[u][0], s_in)
            dev.wait_event(s_dec, ev[u][0])
            if u >= nslots:
                dev.wait_event(s_dec, ev[u - nslots][2])      # slot j's output drained
            plans[j][q].execute(dout[j], s_dec)
            dev.record(ev[u][1], s_dec)
            dev.wait_event(s_out, ev[u][1])
            dev.memcpy(hout + k * out_sz + q * slab_out, dout[j], slab_out, 1, s_out, False)
            dev.record(ev[u][2], s_out)
        for s in (s_in, s_dec, s_out):
            dev.sync(s)
        times.append(time.perf_counter() - t0)
        for row in plans:
            for pl in row:
                pl.wait()
    t = min(times)
    res = {"value": round(len(sel) * out_sz / t / GiB, 2), "unit": "GiB/s",
           "h2d_bytes": len(units) * (slab_in + isz), "d2h_bytes": out_sz * len(sel),
           "seconds": round(t, 4),
           "workload": f"readChunk of {len(sel)} interior shards (4 GiB in + 4 GiB out each) "
                       f"from pinned host memory as {len(units)} y-slab units (chunk range + "
                       f"index in, slab out), H2D | decode | D2H pipelined on 3 streams, "
                       f"{nslots} device slots"}
    # every decoded shard must equal the generator's values of its region
    chk = dev.malloc(out_sz)
    bad = 0
    for k, i in enumerate(sel):
        dev.memcpy(chk, hout + k * out_sz, out_sz, 0, None, True)
        c = coords[i]
        bad += dev.synth_verify(chk, [meta.shape[d] for d in range(n)],
                                [c[d] * cs[d] for d in range(n)], cs, 4, SEED)
    res["verify_mismatches"] = bad
    for row in plans:
        for pl in row:
            pl.close()
    for x in din + dout + [chk]:
        dev.free(x)
    dev.free_pinned(hin)
    dev.free_pinned(hout)
    for s in (s_in, s_dec, s_out):
        dev.stream_destroy(s)
    return res


def cpu_baseline(dev, A, meta, shard_ptr, shard_nbytes, budget_s=12.0):
    """The C oracle (restated reference path, oracle/zh_oracle.c) on this host's cores over a
    bounded sample of the same workload: region reads [1,1024,1024,64] inside shard (0,0,0,0)
    (copied D2H), repeated until ~budget_s of CPU work."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    try:
        cores = min(16, len(os.sched_getaffinity(0)))
    except AttributeError:
        cores = min(16, os.cpu_count() or 1)
    host = (C.c_char * shard_nbytes)()
    dev.memcpy(C.addressof(host), shard_ptr, shard_nbytes, 1, None, True)
    srcs = (A.zh_chunk_src * 1)()
    srcs[0].data = C.addressof(host)
    srcs[0].nbytes = shard_nbytes
    shape = [1, 1024, 1024, 64]
    nbytes_out = 1024 * 1024 * 64 * 4
    out = (C.c_char * nbytes_out)()
    total_bytes, total_t, reps = 0, 0.0, 0
    z = 0
    while total_t < budget_s and reps < 64:
        off = [0, 0, 0, z]
        t0 = time.perf_counter()
        O.array_read_into(meta, srcs, 1, off, shape, C.addressof(out), nthreads=cores)
        total_t += time.perf_counter() - t0
        total_bytes += nbytes_out
        reps += 1
        z = (z + 64) % 1024
    # the same oracle on ONE core (BASELINE.md §3 asks for 1 thread and all cores), over
    # smaller [1,256,256,64] reads (16 MiB each) for about a sixth of the budget
    small = [1, 256, 256, 64]
    b1, t1, r1 = 0, 0.0, 0
    while t1 < budget_s / 6 and r1 < 64:
        off = [0, 256 * (r1 % 4), 256 * ((r1 // 4) % 4), 64 * (r1 % 16)]
        t0 = time.perf_counter()
        O.array_read_into(meta, srcs, 1, off, small, C.addressof(out), nthreads=1)
        t1 += time.perf_counter() - t0
        b1 += 256 * 256 * 64 * 4
        r1 += 1
    return {"value": round(total_bytes / total_t / GiB, 4), "unit": "GiB/s",
            "cores": cores, "kind": "port",
            "single_core": {"value": round(b1 / t1 / GiB, 4), "unit": "GiB/s", "cores": 1,
                            "sample": f"{r1} x Array.read [1,256,256,64] (16 MiB each), "
                                      f"{t1:.1f} s"},
            "sample": f"{reps} x Array.read [1,1024,1024,64] (256 MiB each) from one "
                      f"device-encoded shard, C oracle (oracle/zh_oracle.c, OpenMP over inner "
                      f"chunks), {total_t:.1f} s"}


def host_terminated(args, dist, dev, plan, out, out_bytes, shape, so, ss, rank, ws):
    """Host-terminated multi-GPU read (no gather): each rank decodes its slab and
    copies it D2H into ITS slice of one host buffer that holds the whole region (POSIX shared
    memory mapped by every rank; the slabs are contiguous in C order), so N GPUs drive N PCIe
    links at once.  Each rank page-locks only its own slice (zh_host_register).  Falls back
    to a private pinned slab per rank when /dev/shm cannot hold the region.  Timed: barrier,
    K x (decode + D2H) on the plan's stream, sync, max over ranks; D2H alone timed likewise."""
    import mmap
    from zarrhip.parallel import slab_byte_offset
    full = 4
    for s in shape:
        full *= s
    off = slab_byte_offset(shape, so, 4)
    name = f"/dev/shm/zh_region_{os.environ.get('MASTER_PORT', 'solo')}_{os.getuid()}"
    try:
        vfs = os.statvfs("/dev/shm")
        shared = vfs.f_bavail * vfs.f_frsize >= full + (1 << 30)
    except OSError:
        shared = False
    mm = cbuf = None
    reg = 0
    if shared:
        if rank == 0:
            fd = os.open(name, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o600)
            os.ftruncate(fd, full)
            os.close(fd)
        dist.barrier()
        fd = os.open(name, os.O_RDWR)
        mm = mmap.mmap(fd, full, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        os.close(fd)
        cbuf = C.c_char.from_buffer(mm)
        base = C.addressof(cbuf)
        dst = base + off
        reg = dst & ~4095
        dev.host_register(reg, ((dst + out_bytes + 4095) & ~4095) - reg)
        kind = "one region buffer in /dev/shm shared by the ranks; each pins its slice"
    else:
        dst = dev.malloc_pinned(out_bytes)
        kind = "private pinned slab per rank (/dev/shm too small for the region)"
    for _ in range(max(1, args.warmup)):
        plan.execute(out)
        dev.memcpy(dst, out, out_bytes, 1, None, False)
    plan.wait()
    dist.barrier()
    dev.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.execute(out)
        dev.memcpy(dst, out, out_bytes, 1, None, False)
    plan.wait()
    dev.sync()
    t = dist.max(time.perf_counter() - t0)
    dist.barrier()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        dev.memcpy(dst, out, out_bytes, 1, None, False)
    dev.sync()
    t_copy = dist.max(time.perf_counter() - t1)
    # the host slice must hold this rank's slab of the generator's array
    dev.memset(out, 0, out_bytes)
    dev.memcpy(out, dst, out_bytes, 0, None, True)
    bad = dist.max(dev.synth_verify(out, shape, so, ss, 4, SEED))
    if shared:
        dev.host_unregister(reg)
        del cbuf
        mm.close()
        dist.barrier()
        if rank == 0:
            os.unlink(name)
    else:
        dev.free_pinned(dst)
    if bad:
        raise SystemExit(f"[rank {rank}] host-terminated slab verification FAILED: {bad}")
    return {"buffer": kind, "ms_per_step": round(t * 1e3 / args.steps, 3),
            "value": round(full * args.steps / t / GiB, 2), "unit": "GiB/s",
            "d2h_only_ms_per_step": round(t_copy * 1e3 / args.steps, 3),
            "d2h_GBps_per_rank": round(out_bytes * args.steps / t_copy / 1e9, 2),
            "region_bytes": full, "verify_mismatches": int(bad)}


def run_strong(args, dist, dev, A, L, meta, rank, ws, local):
    """Strong scaling: ONE full array split into per-rank y-slabs (512 rows at
    N=8, aligned to inner chunks); each rank holds only the shards its slab touches
    (encoded on its own GPU), decodes its slab, and optionally gathers the assembled region
    to rank 0 (RCCL over xGMI via torch.distributed 'nccl', or 'gloo' through the host)."""
    import ctypes as C
    sys.path.insert(0, os.path.join(ROOT, "zarr-java_amd"))
    from zarrhip.parallel import slab_partition
    from zarrhip._lib import i32arr, i64arr
    n = meta.ndim
    shape = [meta.shape[d] for d in range(n)]
    cs = [meta.chunk_shape[d] for d in range(n)]
    inner_y = meta.chain.inner_chunk_shape[1] if meta.chain.sharded else 1
    so, ss = slab_partition([0] * n, shape, ws, align=inner_y)[rank]
    lo = [(so[d] // cs[d]) * cs[d] for d in range(n)]
    hi = [min(-(-(so[d] + ss[d]) // cs[d]) * cs[d], shape[d]) for d in range(n)]
    ext = [h - l for l, h in zip(lo, hi)]
    for d in range(2, n):
        assert lo[d] == 0 and ext[d] == shape[d]

    def coords_of(off, shp):
        num = L.zh_compute_chunk_coords(n, i64arr(shape), i32arr(cs), i64arr(off), i64arr(shp),
                                        None, 0)
        buf = (C.c_int64 * (num * n))()
        L.zh_compute_chunk_coords(n, i64arr(shape), i32arr(cs), i64arr(off), i64arr(shp), buf, num)
        return [tuple(buf[i * n + d] for d in range(n)) for i in range(num)]
    cover = coords_of(lo, ext)
    caps = chunk_capacities(meta, cover)
    nel_cover = 1
    for e in ext:
        nel_cover *= e
    first = lo[1] * shape[2] * shape[3] if n == 4 else 0
    src = dev.malloc(nel_cover * 4)
    dev.synth_fill(src, nel_cover, 4, first, SEED)
    offs, tot = [], 0
    for c in caps:
        offs.append(tot)
        tot += (c + 255) // 256 * 256
    slab_buf = dev.malloc(tot)
    sizes = dev.array_write(meta, src, lo, ext, [(slab_buf + o, c) for o, c in zip(offs, caps)])
    dev.free(src)
    where = {c: (slab_buf + o, s) for c, o, s in zip(cover, offs, sizes)}
    mine = coords_of(so, ss)
    nel = 1
    for s in ss:
        nel *= s
    out_bytes = nel * 4
    backend = args.gather_backend if ws > 1 else None
    if backend == "nccl":
        import torch
        out_t = torch.empty(out_bytes, dtype=torch.uint8, device=f"cuda:{local}")
        out = out_t.data_ptr()
    else:
        out = dev.malloc(out_bytes)
    plan = dev.plan(meta, [where[c] for c in mine], so, ss, A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    for _ in range(max(1, args.warmup)):
        plan.execute(out)
    plan.wait()
    bad = dev.synth_verify(out, shape, so, ss, 4, SEED)
    if bad:
        raise SystemExit(f"[rank {rank}] slab verification FAILED: {bad} mismatches")
    plan.set_timing(True)
    dist.barrier()
    dev.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.execute(out)
    plan.wait()
    t_dec = dist.max(time.perf_counter() - t0)
    kt = plan.kernel_time()
    host_out = None
    if args.host_out:
        host_out = host_terminated(args, dist, dev, plan, out, out_bytes, shape, so, ss, rank, ws)
    gather = None
    if backend is not None:
        import torch
        import torch.distributed as tdist
        grp = tdist.new_group(backend=backend)
        if backend == "nccl":
            send = out_t
            recv = [torch.empty_like(out_t) for _ in range(ws)] if rank == 0 else None
        else:
            host = (C.c_char * out_bytes)()
            dev.memcpy(C.addressof(host), out, out_bytes, 1, None, True)
            send = torch.frombuffer(host, dtype=torch.uint8)
            recv = [torch.empty(out_bytes, dtype=torch.uint8) for _ in range(ws)] if rank == 0 \
                else None
        dist.barrier()
        t1 = time.perf_counter()
        tdist.gather(send, recv, dst=0, group=grp)
        if backend == "nccl":
            torch.cuda.synchronize(local)
        t_g = dist.max(time.perf_counter() - t1)
        if rank == 0 and backend == "nccl":  # every gathered slab must be the generator's
            tot_bad = 0
            parts = slab_partition([0] * n, shape, ws, align=inner_y)
            for r in range(ws):
                tot_bad += dev.synth_verify(recv[r].data_ptr(), shape, parts[r][0], parts[r][1],
                                            4, SEED)
            if tot_bad:
                raise SystemExit(f"gathered region verification FAILED: {tot_bad}")
        full = 1
        for s in shape:
            full *= s
        gather = {"backend": backend, "gather_ms": round(t_g * 1e3, 3),
                  "value_incl_one_decode": round(full * 4 / (t_dec / args.steps + t_g) / GiB, 2),
                  "unit": "GiB/s"}
    full = 1
    for s in shape:
        full *= s
    res = {"mode": "strong", "slab_offset": so, "slab_shape": ss,
           "decode_ms_per_step": round(t_dec * 1e3 / args.steps, 3),
           "value": round(full * 4 * args.steps / t_dec / GiB, 2),
           "scatter_ms": round(kt["scatter_ms"] / max(1, kt["launches"]), 3), "gather": gather,
           "host_out": host_out}
    plan.close()
    if backend != "nccl":
        dev.free(out)
    dev.free(slab_buf)
    return res


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--op", default="read", choices=["read", "write"],
                    help="read: the decode path (the metric); write: zh_array_write, the "
                         "encode path (SURVEY §8(f) rank 1)")
    ap.add_argument("--sparse", action="store_true",
                    help="--op write: elide 1/128 of the inner chunks (all fill_value), so the "
                         "write takes its second pass")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--mode", default="weak", choices=["weak", "strong"],
                    help="weak: one full array per GPU (the metric); strong: one array split "
                         "into per-GPU slabs, plus a gather to rank 0")
    ap.add_argument("--gather-backend", default="nccl", choices=["nccl", "gloo", "none"])
    ap.add_argument("--host-out", action="store_true",
                    help="strong mode: also time decode + D2H of each slab into its slice of "
                         "one host buffer (the host-terminated read, no gather)")
    ap.add_argument("--ydiv", type=int, default=1,
                    help="rehearsal only: divide the array's y extent (not a bench config)")
    ap.add_argument("--host-inclusive", action="store_true",
                    help="also measure pinned H2D + decode + D2H (adds 'host_inclusive')")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    if args.gpus != ws and ws > 1:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {ws}")
    dist = Dist(ws, need_torch=args.mode == "strong")

    from zarrhip import _abi as A
    from zarrhip._lib import DeviceContext, lib

    dev = DeviceContext(int(os.environ.get("ZH_DEVICE", local)))
    info = dev.info()
    meta = build_meta(A, args.config, args.ydiv)
    if args.mode == "strong":
        if args.gather_backend == "none":
            args.gather_backend = None
        res = run_strong(args, dist, dev, A, lib(), meta, rank, ws, local)
        log(f"[rank {rank}] strong: {res}")
        if rank == 0:
            n = meta.ndim
            print(json.dumps({
                "metric": "GiB/s device-resident chunk decode (sharding+bytes+transpose), "
                          "uint32 1024³ — strong scaling (one array split over GPUs)",
                "value": res["value"], "unit": "GiB/s", "n_gpus": ws, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": res["decode_ms_per_step"],
                "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
                "dtype": "u32", "data": "synthetic",
                "config": {"workload": f"{args.config}: Array.read of "
                                       f"{'x'.join(str(meta.shape[d]) for d in range(n))} "
                                       f"uint32 split into {ws} y-slabs",
                           "parallelism": f"slab-parallel x{ws}"},
                "strong": res}), flush=True)
        dist.close()
        return
    n = meta.ndim
    shape = [meta.shape[d] for d in range(n)]
    L = lib()
    ncoords = L.zh_compute_chunk_coords(n, (C.c_int64 * 8)(*shape),
                                        (C.c_int32 * 8)(*[meta.chunk_shape[d] for d in range(n)]),
                                        (C.c_int64 * 8)(*([0] * n)), (C.c_int64 * 8)(*shape),
                                        None, 0)
    cbuf = (C.c_int64 * (ncoords * n))()
    L.zh_compute_chunk_coords(n, (C.c_int64 * 8)(*shape),
                              (C.c_int32 * 8)(*[meta.chunk_shape[d] for d in range(n)]),
                              (C.c_int64 * 8)(*([0] * n)), (C.c_int64 * 8)(*shape), cbuf, ncoords)
    coords = [tuple(cbuf[i * n + d] for d in range(n)) for i in range(ncoords)]
    caps = chunk_capacities(meta, coords)
    nel = 1
    for s in shape:
        nel *= s
    out_bytes = nel * 4

    # device buffers: decoded region (also the encode source) + one slab for all shards
    t0 = time.perf_counter()
    out = dev.malloc(out_bytes)
    offs, tot = [], 0
    for cap in caps:
        offs.append(tot)
        tot += (cap + 255) // 256 * 256
    shard_slab = dev.malloc(tot)
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
    plan = dev.plan(meta, [(shard_slab + o, s) for o, s in zip(offs, sizes)], [0] * n, shape,
                    flags)
    st = plan.stats()
    dev.memset(out, 0, out_bytes)
    for _ in range(max(1, args.warmup)):
        plan.execute(out)
    plan.wait()
    bad = dev.synth_verify(out, shape, [0] * n, shape, 4, SEED)
    if bad:
        raise SystemExit(f"decode verification FAILED: {bad} mismatching elements")
    log(f"[rank {rank}] verified {nel} decoded elements bit-exact vs generator")

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
    kt = plan.kernel_time()
    scatter_ms = kt["scatter_ms"] / max(1, kt["launches"])
    index_ms = kt["index_ms"] / max(1, kt["launches"])

    ms_per_step = elapsed * 1000.0 / args.steps
    value = ws * args.steps * out_bytes / elapsed / GiB
    traffic_alg = st["in_bytes"] + st["out_bytes"]
    achieved = traffic_alg / (scatter_ms / 1000.0) / 1e9
    traffic, traffic_src = pmc_traffic(args.config) if args.ydiv == 1 else (None, None)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": ("decode_tiles_kernel" if meta.chain.has_transpose
                           else "decode_rows_kernel<4,4>"),
                "kernel_ms": round(scatter_ms, 3), "index_kernels_ms": round(index_ms, 4),
                "alg_bytes_per_launch": traffic_alg}
    hinc = None
    if args.host_inclusive and meta.chain.sharded:
        hinc = host_inclusive(dev, A, meta, coords, offs, sizes, shard_slab)
        log(f"[rank {rank}] host-inclusive: {hinc}")
    cpu = None
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and meta.chain.sharded:
        cpu = cpu_baseline(dev, A, meta, shard_slab + offs[0], sizes[0], args.cpu_budget)

    line = {
        "metric": "GiB/s device-resident chunk decode (sharding+bytes+transpose), uint32 1024³",
        "value": round(value, 2), "unit": "GiB/s", "n_gpus": ws, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": f"{args.config}: Array.read of the full {'x'.join(map(str, shape))} uint32 "
                               f"array, {CONFIGS[args.config][0]}",
                   "array_shape": shape, "chunk_shape": [1, 1024, 1024, 1024],
                   "inner_chunk_shape": [1, 32, 32, 32] if meta.chain.sharded else None,
                   "shards": st["shards"], "inner_chunks": st["items"],
                   "decoded_bytes_per_gpu": out_bytes, "parallelism": f"shard-parallel x{ws}"},
        "roofline": roofline,
        "cpu_baseline": cpu,
    }
    if hinc is not None:
        line["host_inclusive"] = hinc
    plan.close()
    dev.free(shard_slab)
    dev.free(out)
    if rank == 0:
        print(json.dumps(line), flush=True)
    dist.close()


if __name__ == "__main__":
    main()
