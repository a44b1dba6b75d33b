"""Multi-GPU partitioning of one region read.

Shards and inner chunks are independent, so a read splits into per-rank slabs with no
data-path exchange; ranks own one GPU each (one process per GPU).  A slab along the first
axis that is wider than 1 is contiguous in the region's C order, so a root can assemble
the full region by concatenating the ranks' slabs (RCCL gather over xGMI when the slabs
are device tensors, gloo on host tensors).
"""
import numpy as np


def slab_axis(shape, world):
    """First axis long enough to give every rank a slab (slabs along it are contiguous
    in C order because all earlier axes have extent 1 or are the axis itself)."""
    for d, s in enumerate(shape):
        if s >= world:
            return d
        if s != 1:
            break
    raise ValueError(f"region {list(shape)} cannot be split into {world} contiguous slabs")


def slab_partition(offset, shape, world, align=1):
    """Split [offset, offset+shape) into `world` contiguous slabs along slab_axis.
    Boundaries snap to multiples of `align` (e.g. the inner-chunk extent, so that no inner
    chunk is split between ranks) whenever every rank still gets at least one unit.
    Returns [(slab_offset, slab_shape)] per rank (a rank may get an empty slab)."""
    offset = [int(o) for o in offset]
    shape = [int(s) for s in shape]
    ax = slab_axis(shape, world)
    lo, ext = offset[ax], shape[ax]
    units = ext // align if align > 1 and ext % align == 0 and ext // align >= world else None
    bounds = []
    for r in range(world + 1):
        if units is not None:
            b = lo + (units * r // world) * align
        else:
            b = lo + ext * r // world
        bounds.append(b)
    out = []
    for r in range(world):
        o = list(offset)
        s = list(shape)
        o[ax] = bounds[r]
        s[ax] = bounds[r + 1] - bounds[r]
        out.append((o, s))
    return out


def slab_byte_offset(shape, slab_offset, itemsize):
    """Byte offset of a slab's first element in the C-order region buffer of `shape`: where
    a rank's slice starts in a host-terminated read's shared region buffer."""
    off, st = 0, 1
    for d in range(len(shape) - 1, -1, -1):
        off += int(slab_offset[d]) * st
        st *= int(shape[d])
    return off * itemsize


def gather_pieces(shape, parts, itemsize, cap_bytes, align=1):
    """The bounded, overlapped gather's schedule (bench.py strong mode): every
    rank's slab cut, in order, into pieces of at most `cap_bytes` along the slab's first axis
    of extent >= 2 (all earlier axes have extent 1, so each piece is one contiguous C-order
    part of the region, sent into its place in the root's buffer as its decode finishes).
    Piece boundaries fall on multiples of `align` rows (the inner-chunk extent: no inner chunk
    is decoded twice) whenever `align` rows fit the cap; a single row larger than the cap is
    one piece.  Returns, per rank, [(piece_offset, piece_shape, region_byte_offset, nbytes)]."""
    out = []
    for so, ss in parts:
        so, ss = [int(v) for v in so], [int(v) for v in ss]
        pieces = []
        if all(v > 0 for v in ss):
            ax = next((d for d, v in enumerate(ss) if v >= 2), len(ss) - 1)
            if any(ss[d] != 1 for d in range(ax)):
                raise ValueError(f"slab {ss} is not one contiguous C-order part of {shape}")
            row = int(itemsize)
            for d in range(ax + 1, len(ss)):
                row *= ss[d]
            per = max(1, int(cap_bytes) // row)
            if align > 1 and per >= align:
                per = per // align * align
            lo, end = so[ax], so[ax] + ss[ax]
            while lo < end:
                hi = min(end, lo + per)
                if align > 1 and hi < end and hi % align:  # snap to the unit grid
                    snapped = hi // align * align
                    hi = snapped if snapped > lo else hi
                po, ps = list(so), list(ss)
                po[ax], ps[ax] = lo, hi - lo
                nb = (hi - lo) * row
                pieces.append((po, ps, slab_byte_offset(shape, po, itemsize), nb))
                lo = hi
        out.append(pieces)
    return out


def gather_pieces_p2p(tdist, grp, rank, world, sched, send_buf, region, decode=None):
    """The point-to-point part of the pieced gather into rank 0's region buffer (bench.py strong
    mode; gloo on CPU tensors in tests/test_distributed.py).  `sched` = gather_pieces(...);
    `send_buf` holds this rank's slab (byte tensor, piece k at its offset within the slab),
    `region` the root's whole region (byte tensor).  Rank 0 posts round k of every peer as one
    batch (the peers' links in parallel); a peer sends piece k as a batch of one, after calling
    decode(k) when given (the send then waits only for that piece's decode).  Every op, batched
    on both sides, runs on the group's communicator.  Returns the works to wait on."""
    works = []
    if rank == 0:
        for k in range(max((len(p) for p in sched), default=0)):
            ops = [tdist.P2POp(tdist.irecv, region[sched[r][k][2]:sched[r][k][2] + sched[r][k][3]],
                               r, grp)
                   for r in range(1, world) if k < len(sched[r])]
            if ops:
                works += tdist.batch_isend_irecv(ops)
        return works
    mine = sched[rank]
    base = mine[0][2] if mine else 0
    for k, (_, _, b, nb) in enumerate(mine):
        if decode is not None:
            decode(k)
        works += tdist.batch_isend_irecv(
            [tdist.P2POp(tdist.isend, send_buf[b - base:b - base + nb], 0, grp)])
    return works


def error_record(exc):
    """What the other ranks of a group need to raise `exc` again: its class, message, C-ABI
    status and, for a data error, where the failing chunk sits in a sequential read
    (ZarrException.position / ZhError.position: (chunk grid coords, key), zh_last_data_error)."""
    pos = getattr(exc, "position", None)
    return {"cls": type(exc).__name__, "module": type(exc).__module__, "msg": str(exc),
            "status": getattr(exc, "status", None),
            "pos": (tuple(int(c) for c in pos[0]), int(pos[1])) if pos else None}


def pick_error(records):
    """The error one sequential core.Array.read would have thrown, out of every rank's errors
    (`records[r]`: rank r's error_records, in its own order).  When every error is a placed data
    error, the first in the reference's sequential order — chunk grid coords in C order, then
    the larger key (the index crc32c before the inner chunks, lower C-order rank first: DESIGN
    §3 Q17, the rule zh_array_read_multi applies to its slabs); otherwise the first error of the
    first failing rank (the slabs are contiguous in C order).  Returns (rank, index) or None."""
    failing = [(r, i, e) for r, errs in enumerate(records) for i, e in enumerate(errs or [])]
    if not failing:
        return None
    if all(e["pos"] is not None for _, _, e in failing):
        r, i, _ = min(failing, key=lambda t: (tuple(t[2]["pos"][0]), -t[2]["pos"][1], t[0], t[1]))
        return r, i
    return min(failing, key=lambda t: (t[0], t[1]))[:2]


def rebuild_error(rec):
    """An exception equal in class and message to the one error_record described."""
    import builtins
    from . import _lib, errors
    from .store import StoreException
    known = {("zarrhip.errors", "ZarrException"): errors.ZarrException,
             ("zarrhip.errors", "UnsupportedChainError"): errors.UnsupportedChainError,
             ("zarrhip.store", "StoreException"): StoreException}
    if (rec["module"], rec["cls"]) == ("zarrhip._lib", "ZhError"):
        e = _lib.ZhError(rec["status"], rec["msg"], rec["pos"])
    else:
        cls = known.get((rec["module"], rec["cls"]))
        if cls is None and rec["module"] == "builtins":
            b = getattr(builtins, rec["cls"], None)
            cls = b if isinstance(b, type) and issubclass(b, Exception) else None
        try:
            e = (cls or RuntimeError)(rec["msg"])
        except Exception:
            e = RuntimeError(rec["msg"])
    if rec["pos"] is not None:
        e.position = rec["pos"]
    return e


def raise_group_error(tdist, group, rank, world, errs):
    """Collective over `group` (every rank calls it, also as the read's closing barrier): each
    rank contributes the errors its part of a read met, and if any rank met one, EVERY rank
    raises the same pick_error choice — the rank that met it its own exception object, the others
    an equal one (rebuild_error).  The reference throws out of read() when any chunk fails
    (M/core/Array.java:403-407, 436-438); no rank may return a region with a failed slab, and no
    rank waits for a peer that gave up."""
    mine = [error_record(e) for e in errs]
    every = [None] * world
    tdist.all_gather_object(every, mine, group=group)
    pick = pick_error(every)
    if pick is None:
        return
    r, i = pick
    if r == rank:
        raise errs[i]
    raise rebuild_error(every[r][i])


def deferred_errors(decode):
    """The errors a decoder reports only when waited on: decode.wait_errors() (PlanDecoder: one
    per failed plan), else whatever decode.wait() raises."""
    if decode is None:
        return []
    if hasattr(decode, "wait_errors"):
        return list(decode.wait_errors())
    if hasattr(decode, "wait"):
        try:
            decode.wait()
        except Exception as e:  # reported through raise_group_error
            return [e]
    return []


class PlanDecoder:
    """decode(piece_offset, piece_shape, dst) for RegionGather over device-resident chunk
    sources: one zh plan per piece (created on its first use and kept, so a repeated read plans
    nothing), executed asynchronously on torch's current stream into `dst` (a CUDA byte
    tensor): a send that follows on that stream waits for exactly this piece's decode.
    `sources(piece_offset, piece_shape)` gives the piece's chunk sources in computeChunkCoords
    order ((device pointer, nbytes) or (None, 0)).  wait() reports the plans' deferred device
    errors (the reference's messages); close() frees them."""

    def __init__(self, dev, meta, sources, flags=None):
        from . import _abi as A
        self.dev, self.meta, self.sources = dev, meta, sources
        self.flags = (A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE) if flags is None else flags
        self.plans = {}

    def plan(self, po, ps):
        key = (tuple(po), tuple(ps))
        p = self.plans.get(key)
        if p is None:
            p = self.dev.plan(self.meta, self.sources(po, ps), list(po), list(ps), self.flags)
            self.plans[key] = p
        return p

    def __call__(self, po, ps, dst):
        import torch
        self.plan(po, ps).execute(dst.data_ptr(), torch.cuda.current_stream(dst.device).cuda_stream)

    def wait_errors(self):
        """Wait for every plan; the deferred device errors, one per failed plan (ZhError with
        the reference's message and the failing chunk's position)."""
        errs = []
        for p in self.plans.values():
            try:
                p.wait()
            except Exception as e:  # every plan is waited on; the caller picks
                errs.append(e)
        return errs

    def wait(self):
        """Wait for every plan; raise the error a sequential read would have met first."""
        errs = self.wait_errors()
        pick = pick_error([[error_record(e) for e in errs]])
        if pick is not None:
            raise errs[pick[1]]

    def close(self):
        for p in self.plans.values():
            p.close()
        self.plans.clear()


def array_decoder(array, dev=None):
    """decode(piece_offset, piece_shape, dst) for RegionGather over a zarrhip.Array: the piece
    is core.Array.read from the array's store (for a FilesystemStore the library's own file
    reads) straight into `dst` — device memory (Array.read_device, ZH_OUT_DEVICE) for a CUDA
    tensor, host memory for a CPU tensor (the gloo form).  Synchronous: the call returns after
    the piece is in `dst`."""
    import numpy as _np

    def decode(po, ps, dst):
        if dst.is_cuda:
            array.read_device(po, ps, dst.data_ptr(), dev)
        else:
            got = array.read(po, ps)
            dst.numpy()[:] = _np.ascontiguousarray(got).view(_np.uint8).ravel()
    return decode


class RegionGather:
    """One region read spread over the ranks of a process group and assembled on the root
    (the reference's ForkJoin loop over chunks, M/core/Array.java:403-407, becomes
    one slab per rank).  The region splits into contiguous C-order slabs (slab_partition, on the
    inner-chunk grid `align`); every slab is cut into pieces of at most `piece_bytes`
    (gather_pieces).  run(decode) decodes each piece and sends it point-to-point into its place
    in the root's region buffer as soon as its own decode is done, so the decode of piece k+1
    overlaps the transfer of piece k, and the root receives round k of every peer as one batch
    (the peers' links in parallel).  The root decodes its own slab straight into the region, on
    a side stream (device) so that its receives never wait for it.

    Backends: an NCCL (= RCCL on ROCm) group moves CUDA byte tensors over xGMI (device-resident
    read: no host memory on the data path); a gloo group moves CPU tensors (the host form, and
    the form the CPU tests drive).  `decode(piece_offset, piece_shape, dst)` writes the piece's
    C-order bytes into `dst` (a byte tensor on the group's side: enqueued on torch's current
    stream for CUDA, or synchronously); PlanDecoder and array_decoder are the two product ones.
    With decode=None the buffers already hold the slabs (send() only).  The buffers (the send
    slab on peers, the region on the root) are allocated once and reused by every run()."""

    def __init__(self, offset, shape, itemsize, group=None, root=0, align=1,
                 piece_bytes=1 << 30, device=None, region=None, send=None):
        import torch
        import torch.distributed as tdist
        self.torch, self.tdist = torch, tdist
        self.group = group if group is not None else tdist.group.WORLD
        self.rank = tdist.get_rank(self.group)
        self.world = tdist.get_world_size(self.group)
        if root != 0:
            raise ValueError("RegionGather assembles on rank 0 of the group")
        self.root = root
        self.offset = [int(o) for o in offset]
        self.shape = [int(s) for s in shape]
        self.itemsize = int(itemsize)
        self.on_device = tdist.get_backend(self.group) == "nccl"
        from . import _lib
        if self.on_device and _lib._lib is not None and not _lib.LOADED_AFTER_TORCH:
            raise RuntimeError(
                "zarrhip's library was loaded before torch: import torch (and initialise "
                "torch.cuda) before the first zarrhip call, so that both use torch's HIP "
                "runtime (INTEGRATION.md §4)")
        if self.on_device:
            self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                       else int(device))
        else:
            self.device = torch.device("cpu")
        self.parts = slab_partition(self.offset, self.shape, self.world, align)
        rel = [([o - b for o, b in zip(po, self.offset)], ps) for po, ps in self.parts]
        self.sched = gather_pieces(self.shape, rel, self.itemsize, piece_bytes, align)
        nel = 1
        for s in self.shape:
            nel *= s
        self.nbytes = nel * self.itemsize
        so, ss = rel[self.rank]
        self.base = slab_byte_offset(self.shape, so, self.itemsize)
        n = 1
        for s in ss:
            n *= s
        self.slab_bytes = n * self.itemsize
        if self.rank == self.root:
            self.region = region if region is not None else torch.empty(
                self.nbytes, dtype=torch.uint8, device=self.device)
            self.send_buf = self.region[self.base:self.base + self.slab_bytes]
        else:
            self.region = None
            self.send_buf = send if send is not None else torch.empty(
                max(1, self.slab_bytes), dtype=torch.uint8, device=self.device)
        self._side = torch.cuda.Stream(self.device) if self.on_device else None
        if self.on_device:  # every rank creates the communicator together, before any P2P op
            tdist.all_reduce(torch.zeros(1, device=self.device), group=self.group)
            torch.cuda.synchronize(self.device)

    def pieces(self, rank=None):
        """This rank's (or `rank`'s) pieces: [(absolute piece_offset, piece_shape,
        region byte offset, nbytes)]."""
        r = self.rank if rank is None else rank
        return [([o + b for o, b in zip(po, self.offset)], ps, b, nb)
                for po, ps, b, nb in self.sched[r]]

    def _dst(self, b, nb):
        return self.send_buf[b - self.base:b - self.base + nb]

    def run(self, decode=None):
        """Decode (unless None) and gather; returns the region byte tensor on the root and this
        rank's slab byte tensor elsewhere, complete (device work synchronised).

        Errors: a piece whose decode raises is still sent (its bytes are never handed out), so
        no peer or root waits for a send that never comes; after the gather, deferred device
        errors (decode.wait_errors / wait) are collected and raise_group_error makes EVERY rank
        raise the error a sequential read would have met first (the reference's message)."""
        torch = self.torch
        mine = self.pieces()
        errs = []

        def safe(po, ps, dst):
            try:
                decode(po, ps, dst)
            except Exception as e:  # raised on every rank by raise_group_error below
                errs.append(e)

        if self.rank == self.root:
            works = gather_pieces_p2p(self.tdist, self.group, self.rank, self.world, self.sched,
                                      None, self.region)
            if decode is not None:
                if self.on_device:
                    with torch.cuda.stream(self._side):
                        for po, ps, b, nb in mine:
                            safe(po, ps, self._dst(b, nb))
                else:
                    for po, ps, b, nb in mine:
                        safe(po, ps, self._dst(b, nb))
            for w in works:
                w.wait()
        else:
            def dec(k):
                po, ps, b, nb = mine[k]
                safe(po, ps, self._dst(b, nb))
            for w in gather_pieces_p2p(self.tdist, self.group, self.rank, self.world, self.sched,
                                       self.send_buf[:self.slab_bytes] if self.slab_bytes
                                       else self.send_buf[:0], None,
                                       dec if decode is not None else None):
                w.wait()
        if self.on_device:
            torch.cuda.current_stream(self.device).wait_stream(self._side)
            torch.cuda.synchronize(self.device)
        errs += deferred_errors(decode)
        raise_group_error(self.tdist, self.group, self.rank, self.world, errs)
        return self.region if self.rank == self.root else self.send_buf[:self.slab_bytes]


_REGION_SEQ = 0  # SharedHostRegion names: regions created by this process


class SharedHostRegion:
    """One region read over the ranks of a group, delivered to HOST memory with no gather
    (SURVEY §8(e)'s host-terminated form; the reference's read ends in a host array): the
    region's buffer lives in POSIX shared memory (/dev/shm), mapped by every rank; each rank
    page-locks only its own slab's slice (`dev.host_register`) and decodes its slab straight
    into it, so N GPUs drive N PCIe links at once and every rank sees the whole region when
    read() returns.  The slabs are slab_partition's (contiguous in C order, on the inner-chunk
    grid `align`).  `decode(slab_offset, slab_shape, dst_addr)` writes the slab's C-order bytes
    to host address dst_addr: `array_host_decoder(array)` (a zarrhip.Array read, the library's
    pipelined read DMA-ing into the page-locked slice), or a caller's own (a device plan plus a
    D2H copy, as bench.py does).  The buffer needs room in /dev/shm (MemoryError otherwise:
    the caller streams its slab through a smaller buffer instead).  close() unpins, unmaps, and
    rank 0 removes the file; the numpy view (array()) is invalid after it."""

    def __init__(self, offset, shape, itemsize, dev=None, group=None, align=1, name=None):
        import mmap
        import os
        import torch.distributed as tdist
        self.tdist = tdist
        self.group = group if group is not None else tdist.group.WORLD
        self.rank = tdist.get_rank(self.group)
        self.world = tdist.get_world_size(self.group)
        self.offset = [int(o) for o in offset]
        self.shape = [int(s) for s in shape]
        self.itemsize = int(itemsize)
        self.dev = dev
        self.parts = slab_partition(self.offset, self.shape, self.world, align)
        n = self.itemsize
        for v in self.shape:
            n *= v
        self.nbytes = n
        so, ss = self.parts[self.rank]
        self.slab_offset, self.slab_shape = so, ss
        self.base = slab_byte_offset(self.shape, [o - b for o, b in zip(so, self.offset)],
                                     self.itemsize)
        sb = self.itemsize
        for v in ss:
            sb *= v
        self.slab_bytes = sb
        # one file per region: rank 0 picks a fresh name (pid, uid, a per-process counter and
        # random bits, unless the caller names it), creates it exclusively (never another live
        # region's file) and broadcasts the name with the outcome, so every rank raises together
        res = [None, None]
        if self.rank == 0:
            import uuid
            global _REGION_SEQ
            _REGION_SEQ += 1
            path = name or (f"/dev/shm/zh_region_{os.getpid()}_{os.getuid()}_{_REGION_SEQ}_"
                            f"{uuid.uuid4().hex[:12]}")
            res[0] = path
            try:
                vfs = os.statvfs(os.path.dirname(path))
                if vfs.f_bavail * vfs.f_frsize < n + (1 << 30):
                    res[1] = ("MemoryError",
                              f"{os.path.dirname(path)} cannot hold the {n}-byte region")
                else:
                    fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_EXCL, 0o600)
                    try:
                        os.ftruncate(fd, max(1, n))
                    finally:
                        os.close(fd)
            except FileExistsError:
                res[1] = ("FileExistsError", f"shared region file {path} already exists")
            except OSError as e:
                res[1] = ("OSError", f"shared region file {path}: {e}")
        tdist.broadcast_object_list(res, src=0, group=self.group)
        self.name = res[0]
        if res[1] is not None:
            import builtins
            raise getattr(builtins, res[1][0])(res[1][1])
        fd = os.open(self.name, os.O_RDWR)
        self._mm = mmap.mmap(fd, max(1, n), mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        os.close(fd)
        import ctypes
        self._cbuf = ctypes.c_char.from_buffer(self._mm)
        self.addr = ctypes.addressof(self._cbuf)
        self._reg = None
        if dev is not None and self.slab_bytes > 0:  # page-lock this rank's slice only
            dst = self.addr + self.base
            lo = dst & ~4095
            hi = (dst + self.slab_bytes + 4095) & ~4095
            dev.host_register(lo, hi - lo)
            self._reg = lo

    def slice_addr(self):
        """Host address of this rank's slice (its slab's bytes in the region)."""
        return self.addr + self.base

    def read(self, decode):
        """Every rank decodes its slab into its slice; returns after all ranks are done.  If any
        rank's decode failed, every rank raises the same error (raise_group_error, which is also
        the closing barrier), so none returns a region holding a failed slab and none hangs."""
        errs = []
        if self.slab_bytes > 0:
            try:
                decode(self.slab_offset, self.slab_shape, self.slice_addr())
            except Exception as e:  # raised on every rank below
                errs.append(e)
        errs += deferred_errors(decode)
        raise_group_error(self.tdist, self.group, self.rank, self.world, errs)

    def array(self, dtype):
        """The whole region as a numpy array over the shared buffer (valid until close())."""
        import numpy as _np
        return _np.frombuffer(self._mm, dtype=_np.dtype(dtype), count=self.nbytes //
                              _np.dtype(dtype).itemsize).reshape(self.shape)

    def close(self):
        """Unpin and unmap this rank's view, then (every rank, even when unmapping failed — a
        caller still holding array()'s view makes mmap.close raise BufferError) the barrier;
        rank 0 removes the file; a local failure is raised after the barrier."""
        import os
        try:
            if self._reg is not None:
                self._reg, reg = None, self._reg
                self.dev.host_unregister(reg)
            if getattr(self, "_cbuf", None) is not None:
                del self._cbuf
                self._cbuf = None
            self._mm.close()
        finally:
            self.tdist.barrier(group=self.group)
            if self.rank == 0:
                try:
                    os.unlink(self.name)
                except FileNotFoundError:
                    pass


def array_host_decoder(array, dev=None):
    """decode(slab_offset, slab_shape, dst_addr) for SharedHostRegion over a zarrhip.Array:
    core.Array.read of the slab straight into host memory at dst_addr (the library's pipelined
    read DMAs into page-locked memory directly)."""
    def decode(po, ps, addr):
        array.read_into(po, ps, addr, dev)
    return decode


def distributed_read(decode, offset, shape, dtype, group=None, root=0, align=1,
                     piece_bytes=1 << 30, device=None):
    """One region read over the ranks of `group` (RegionGather): on the root the assembled
    region, elsewhere this rank's slab.  NCCL groups return CUDA byte tensors (view them as the
    dtype), gloo groups numpy arrays of `dtype` in the region's / slab's shape."""
    import numpy as _np
    dt = _np.dtype(dtype)
    g = RegionGather(offset, shape, dt.itemsize, group=group, root=root, align=align,
                     piece_bytes=piece_bytes, device=device)
    out = g.run(decode)
    if g.on_device:
        return out
    shp = g.shape if g.rank == root else g.parts[g.rank][1]
    return out.numpy().view(dt).reshape(shp)
