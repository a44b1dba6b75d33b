"""v3 Array — the read/write surface of dev.zarr.zarrjava.v3.Array / core.Array, with the
chunk codec work done by the HIP path through the C-ABI (libzarrhip.so).

  Array.open / create        M/v3/Array.java:41-50, 142-154
  read(offset, shape)        M/core/Array.java:378-441   → zh_array_read (one call, all chunks;
                                                          zh_array_read_multi over ZH_DEVICES)
  readChunk(coords)          M/core/Array.java:167-182
  write(offset, data)        M/core/Array.java:83-133    → zh_array_write (whole chunks)
  access()                   M/core/Array.java:483-536   (ArrayAccessor)

Byte-to-byte compressors stay on the host (north star): their frames are decoded here and
the raw chunk bytes are handed to the device.
"""
import atexit
import ctypes as C
import json
import os
import struct
import time
import threading

import numpy as np

from . import _abi as A
from . import _lib
from .codecs import device_chain, host_bb_decode, host_bb_encode
from .errors import ZarrException, raise_for
from .metadata import ZARR_JSON, ArrayMetadata

_ctx = None
_ctx_lock = threading.Lock()


def device():
    """The process-wide DeviceContext (GPU ZH_DEVICE, default LOCAL_RANK or 0)."""
    global _ctx
    with _ctx_lock:
        if _ctx is None:
            dev = int(os.environ.get("ZH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
            _ctx = _lib.DeviceContext(dev)
        return _ctx


_multi = {}


def devices():
    """DeviceContexts of ZH_DEVICES="0,1,..." (one per listed GPU, a GPU may repeat), or
    [device()]: Array.read spreads a region over them (zh_array_read_multi)."""
    spec = os.environ.get("ZH_DEVICES", "")
    ids = [int(x) for x in spec.split(",") if x.strip()]
    if len(ids) <= 1:
        return [device()]
    with _ctx_lock:
        if spec not in _multi:
            _multi[spec] = [_lib.DeviceContext(i) for i in ids]
        return _multi[spec]


def _parallel(fn, jobs, width=8):
    """Run fn over jobs on up to `width` threads (store reads release the GIL)."""
    if len(jobs) <= 1:
        for j in jobs:
            fn(j)
        return
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=min(width, len(jobs))) as ex:
        for _ in ex.map(fn, jobs):
            pass


class StagingPool:
    """Host staging buffers (store bytes on their way to the device), reused across reads.
    A fresh multi-GiB numpy buffer per read pays twice: its pages fault in while the store
    read fills it, and they are unmapped when it is dropped at the end of the read (a 2 GiB
    sub-shard read: 194 ms inside Array.read, 283 ms around it).  The reference's JVM heap
    keeps such memory; this pool does the same for the mirror.  Buffers are kept up to `cap`
    bytes; `release()` returns them.

    Buffers of at least `pin_min` bytes are page-aligned, and page-locked (zh_host_register
    through the process's DeviceContext, `pin`) when the pool hands one out a second time, so
    repeated reads' H2D copies run as direct DMA instead of through the runtime's pageable
    staging, while a one-off buffer (or one the cap keeps evicting) never pays for pinning
    (≈40 ms per GiB).  Pinned buffers are unregistered before the pool lets go of them.
    Without a usable device (CPU-only use, or a failing registration) they stay pageable."""
    ROUND = 64 << 20
    PAGE = 4096

    def __init__(self, cap=8 << 30, pin=None, pin_min=64 << 20):
        self.cap = cap
        self.pin = pin  # callable returning a DeviceContext, or None: pageable buffers
        self.pin_min = pin_min
        self._free = []
        self._pinned = {}  # id(buffer) -> (context, address)
        self._lock = threading.Lock()

    def _alloc(self, size):
        if self.pin is None or size < self.pin_min:
            return np.empty(size, np.uint8)
        raw = np.empty(size + self.PAGE, np.uint8)
        a = (-raw.ctypes.data) % self.PAGE
        return raw[a:a + size]  # page-aligned; keeps `raw` alive through .base

    def _register(self, b):  # caller holds the lock
        if self.pin is None or b.nbytes < self.pin_min or id(b) in self._pinned:
            return
        try:
            ctx = self.pin()
            ctx.host_register(b.ctypes.data, b.nbytes)
            self._pinned[id(b)] = (ctx, b.ctypes.data)
        except Exception:  # no device or registration refused: stays pageable
            pass

    def _drop(self, b):
        rec = self._pinned.pop(id(b), None)
        if rec is not None:
            rec[0].host_unregister(rec[1])

    def take(self, n, lease):
        """A uint8 view of at least n bytes; its buffer is appended to `lease` (give back
        with give(lease) once the device has consumed it)."""
        with self._lock:
            fit = [i for i, x in enumerate(self._free) if x.nbytes >= n]
            b = self._free.pop(min(fit, key=lambda i: self._free[i].nbytes)) if fit else None
            if b is not None:
                self._register(b)  # second use: worth page-locking
        if b is None:
            b = self._alloc(max(1, -(-n // self.ROUND) * self.ROUND) if n > self.ROUND else
                            max(n, 1))
        lease.append(b)
        return b[:n]

    def give(self, lease):
        with self._lock:
            self._free.extend(lease)
            tot = sum(b.nbytes for b in self._free)
            while tot > self.cap and self._free:  # drop the oldest first
                b = self._free.pop(0)
                tot -= b.nbytes
                self._drop(b)
        lease.clear()

    def pinned_bytes(self):
        with self._lock:
            return sum(b.nbytes for b in self._free if id(b) in self._pinned)

    def release(self):
        with self._lock:
            for b in self._free:
                self._drop(b)
            self._free.clear()


staging_pool = StagingPool(pin=lambda: devices()[0])
atexit.register(staging_pool.release)  # unregister before the buffers' memory goes


def _new_buf(n, lease=None):
    return np.empty(n, np.uint8) if lease is None else staging_pool.take(n, lease)


def _read_whole(h, piece=64 << 20, lease=None):
    """StoreHandle.read() of a whole chunk; stores that report sizes are read in parallel
    pieces straight into one buffer (a 4 GiB shard is one bytes copy otherwise)."""
    n = h.size() if hasattr(h, "size") else None
    if n is None or n <= piece:
        return h.read()
    out = _new_buf(n, lease)
    mv = memoryview(out)

    def fetch(o):
        ln = min(piece, n - o)
        got = h.read_into(mv[o:o + ln], o, o + ln)
        if got is None or got < ln:
            raise ZarrException(f"Could not load byte data of {h!r}")
    _parallel(fetch, list(range(0, n, piece)))
    return out


def _host_buf(b):
    return (C.c_char * max(1, len(b))).from_buffer_copy(bytes(b) if len(b) else b"\0")


class Array:
    def __init__(self, store_handle, metadata):
        self.storeHandle = store_handle
        self.metadata = metadata
        self.staged_bytes = 0  # encoded bytes read from the store and handed to the device
        self._stage_lock = threading.Lock()  # chunk loads run on several threads
        self.chain = device_chain(metadata.codecs, metadata.ndim,
                                  metadata.data_type.getByteCount(), metadata.chunk_shape)
        self.zmeta = metadata.to_zh_meta(self.chain)
        err = C.create_string_buffer(512)
        st = _lib.lib().zh_validate_meta(C.byref(self.zmeta), err, 512)
        if st != A.ZH_OK:
            raise_for(_lib.ZhError(st, err.value.decode()))

    # ---------------------------------------------------------------- open / create
    META_FILE = ZARR_JSON          # v2.Array: ".zarray"
    METADATA = ArrayMetadata

    @classmethod
    def open(cls, store_handle):
        raw = store_handle.resolve(cls.META_FILE).read()
        if raw is None:
            raise ZarrException(f"No Zarr array found at {store_handle!r}")
        return cls(store_handle, cls.METADATA.from_json(json.loads(raw)))

    @classmethod
    def create(cls, store_handle, metadata, exist_ok=False):
        h = store_handle.resolve(cls.META_FILE)
        if not exist_ok and h.exists():
            raise ZarrException(f"Trying to create a new array in {store_handle!r}. But "
                                f"{cls.META_FILE} already exists.")
        h.set(metadata.dumps().encode())
        return cls(store_handle, metadata)

    # ---------------------------------------------------------------- helpers
    @property
    def ndim(self):
        return self.metadata.ndim

    def _chunk_coords(self, offset, shape):
        n = self.ndim
        L = _lib.lib()
        args = (n, _lib.i64arr(self.metadata.shape), _lib.i32arr(self.metadata.chunk_shape),
                _lib.i64arr(offset), _lib.i64arr(shape))
        num = L.zh_compute_chunk_coords(*args, None, 0)
        if num < 0:
            raise ArithmeticError("Number of chunks exceeds Integer.MAX_VALUE")
        out = (C.c_int64 * max(1, num * n))()
        L.zh_compute_chunk_coords(*args, out, num)
        return [tuple(out[i * n:(i + 1) * n]) for i in range(num)]

    def _handle(self, coords):
        return self.storeHandle.resolve(*self.metadata.chunk_key_encoding.encode_chunk_key(coords))

    def _check_region(self, offset, shape):
        n = self.ndim
        if len(offset) != n:
            raise ValueError(f"'offset' needs to have rank '{n}'.")
        if len(shape) != n:
            raise ValueError(f"'shape' needs to have rank '{n}'.")
        for d in range(n):  # M/core/Array.java:386-390
            if offset[d] < 0 or offset[d] + shape[d] > self.metadata.shape[d]:
                raise ZarrException("Requested data is outside of the array's domain.")

    def _count_staged(self, n):
        with self._stage_lock:
            self.staged_bytes += n

    def _n_inner(self):
        inner = self.chain.chain["inner_chunk_shape"]
        n = 1
        for c, i in zip(self.metadata.chunk_shape, inner):
            n *= c // i
        return n

    def _wrap_inner(self, shard):
        """Inverse of _unwrap_inner for the write path."""
        ch = self.chain.chain
        n_in = self._n_inner()
        crc = ch["index_crc32c"]
        isz = 16 * n_in + (4 if crc else 0)
        start = ch["index_location"] == A.ZH_INDEX_START
        idx = shard[:isz] if start else shard[len(shard) - isz:]
        body = idx[:16 * n_in]
        fmt = ">QQ" if ch["index_endian"] == A.ZH_ENDIAN_BIG else "<QQ"
        pos = isz if start else 0
        payload, new = [], []
        for k in range(n_in):
            off, nb = struct.unpack(fmt, body[16 * k:16 * k + 16])
            if off == 2 ** 64 - 1:
                new.append((off, nb))
                continue
            enc = host_bb_encode(self.chain.inner_host_bb, shard[off:off + nb])
            new.append((pos, len(enc)))
            payload.append(enc)
            pos += len(enc)
        ib = b"".join(struct.pack(fmt, *e) for e in new)
        if crc:
            ib = self.chain.index_codecs[1].encode(ib)
        pb = b"".join(payload)
        return ib + pb if start else pb + ib

    def _stage_shard(self, h, part_lo, part_hi, lease, full=False):
        """StoreHandleDataProvider semantics (ShardingIndexedCodec.java:190-230, 333-357): one
        range read for the index, zh_shard_ranges for the inner chunks the part references,
        one store read per range (in parallel, straight into one pooled buffer).  The stored
        index goes to the device unchanged — its crc32c and entries are checked there, never
        here — so a corrupt entry cannot size a host allocation.  Inner host byte-to-byte
        stages (zstd, gzip, blosc) are undone per inner chunk: those pieces hold the raw
        payload.  A range the store cannot deliver is left out (the device then reports the
        reference's "Could not load byte data for chunk").  `full`: the part is the whole shard
        (decodePartial → chunkHandle.read() → ByteBufferDataProvider, :246-251, 301-331), so
        the shard is the file as it is — an entry beyond its bytes is an error (Q14), not a
        zero-padded range.  Returns a ShardSource plus the buffers it points into, or None for
        a missing shard."""
        if not h.exists():
            return None
        isz = _lib.lib().zh_shard_index_size(C.byref(self.zmeta))
        start = self.chain.chain["index_location"] == A.ZH_INDEX_START
        try:
            idx = h.read(0, isz) if start else h.read(-isz)
        except ValueError:  # a suffix longer than the file (the reference's position(< 0))
            idx = h.read()  # what it holds: the device reports "Shard [...] smaller than its index"
        if idx is None:
            return None
        idx = bytes(idx)
        from .store import FilesystemStore
        size = h.size() if hasattr(h, "size") else None
        # a FilesystemStore range read past the end of the file returns zeros
        # (FilesystemStore.get(keys, start, end), FilesystemStore.java:84-102): no entry is out
        # of reach by its offset, so the shard size bounds nothing
        if full and size is not None:
            size = int(size)  # the whole object: sliced, never padded (zh_files.cpp file_sources)
        else:
            size = -1 if size is None or isinstance(h.store, FilesystemStore) else int(size)
        ibuf = np.frombuffer(idx if idx else b"\0", np.uint8)
        keep = [ibuf]
        self._count_staged(len(idx))
        if len(idx) < isz:  # the device reports "Shard [..] is smaller than its index"
            return _lib.ShardSource(ibuf.ctypes.data, len(idx), size, []), keep
        host = self.chain.inner_host_bb
        if host or size < 0:
            # the index decides host work before the device sees it (host decodes of every
            # referenced range; range reads bounded by nothing but the entries): check its
            # crc32c first, as the reference does (ShardingIndexedCodec.java:205)
            try:
                _lib.shard_index_check(self.zmeta, idx)
            except _lib.ZhError as e:
                raise_for(e)
        rs = _lib.shard_ranges(self.zmeta, idx, size, part_lo, part_hi,
                               0 if host else 64 << 20)
        pieces = []
        if host:  # per inner chunk: undo the host codecs
            for o, nb in rs:
                if full and o + nb > size:  # beyond the object: left out, the device reports it
                    continue
                blob = h.read(o, o + nb)
                if blob is None or len(blob) < nb:
                    continue
                self._count_staged(nb)
                raw = np.frombuffer(host_bb_decode(host, blob) or b"\0", np.uint8)
                keep.append(raw)
                pieces.append((o, nb, raw.ctypes.data, len(raw)))
            return _lib.ShardSource(ibuf.ctypes.data, len(idx), size, pieces), keep
        buf = _new_buf(max(1, sum(nb for _, nb in rs)), lease)
        keep.append(buf)
        mv = memoryview(buf)
        jobs, pos = [], 0
        for o, nb in rs:
            jobs.append((pos, o, nb))
            pos += nb
        got = [0] * len(jobs)

        def fetch(k):
            p0, o, nb = jobs[k]
            g = h.read_into(mv[p0:p0 + nb], o, o + nb)
            got[k] = g or 0
        _parallel(fetch, list(range(len(jobs))))
        for k, (p0, o, nb) in enumerate(jobs):
            if got[k] >= nb:
                self._count_staged(nb)
                pieces.append((o, nb, buf.ctypes.data + p0, nb))
        return _lib.ShardSource(ibuf.ctypes.data, len(idx), size, pieces), keep

    def _load_source(self, coords, part_lo=None, part_hi=None, lease=None):
        """One stored chunk / shard of a read: None (missing key), ("whole", bytes-like), or
        ("pieces", ShardSource, keepalive) for a sharded part."""
        h = self._handle(coords)
        ch = self.chain.chain
        if ch["sharded"]:
            n = self.ndim
            if part_lo is None:
                part_lo, part_hi = [0] * n, list(self.metadata.chunk_shape)
            full = all(lo == 0 and hi == c for lo, hi, c in
                       zip(part_lo, part_hi, self.metadata.chunk_shape))
            if not full or self.chain.inner_host_bb:  # the index + the referenced ranges
                st = self._stage_shard(h, part_lo, part_hi, lease, full)
                return None if st is None else ("pieces",) + st
        # raw payloads go to the device as they are: parallel reads into one buffer; host
        # byte-to-byte stages take the store's bytes
        b = h.read() if self.chain.host_bb else _read_whole(h, lease=lease)
        if b is None:
            return None
        self._count_staged(len(b))
        if self.chain.host_bb:
            b = host_bb_decode(self.chain.host_bb, b)
        return ("whole", b)

    def _file_paths(self, coords, devs):
        """The chunk files of a read that zh_array_read_files(_multi) can do (FilesystemStore,
        a chain without host byte-to-byte stages; ZH_FILES=0 keeps the store reads here), in
        computeChunkCoords order, else None.  The reads themselves follow
        FilesystemStore.exists / get (M/store/FilesystemStore.java:43-102) in the library."""
        from .store import FilesystemStore
        st = self.storeHandle.store
        if (not isinstance(st, FilesystemStore) or self.chain.host_bb or
                self.chain.inner_host_bb or os.environ.get("ZH_FILES", "1") == "0"):
            return None
        return [st._p(self._handle(c).keys) for c in coords]

    def _file_store(self):
        """The FilesystemStore the chunk files belong to, as (root, FilesystemStore.toString())
        for StoreException's text."""
        st = self.storeHandle.store
        return (st.path, repr(st))

    # ---------------------------------------------------------------- read
    def read(self, offset=None, shape=None, parallel=True):
        """core.Array.read → numpy array (C order, the array's dtype)."""
        t_enter = time.perf_counter()
        n = self.ndim
        offset = [0] * n if offset is None else [int(o) for o in offset]
        shape = list(self.metadata.shape) if shape is None else [int(s) for s in shape]
        self._check_region(offset, shape)
        dt = self.metadata.data_type.numpy
        if any(s == 0 for s in shape):
            return np.zeros(shape, dtype=dt)
        out = np.empty(shape, dtype=dt)
        self._read_into(offset, shape, out.ctypes.data, 0, devices(), parallel, t_enter)
        return out

    def read_into(self, offset, shape, out_addr, dev=None, parallel=True):
        """core.Array.read into caller-owned HOST memory at out_addr (C order, the array's
        dtype; page-locked memory is DMA'd straight into): the per-rank decode of
        zarrhip.parallel.SharedHostRegion.  `dev`: the DeviceContext to read with (default: the
        process's contexts, as read())."""
        t_enter = time.perf_counter()
        offset = [int(o) for o in offset]
        shape = [int(s) for s in shape]
        self._check_region(offset, shape)
        if any(s == 0 for s in shape):
            return
        self._read_into(offset, shape, int(out_addr), 0,
                        [dev] if dev is not None else devices(), parallel, t_enter)

    def read_device(self, offset, shape, out_ptr, dev=None, parallel=True):
        """core.Array.read delivered to device memory: the C-order region is written to
        `out_ptr` on `dev`'s device (a DeviceContext; default the first context) and nothing
        is copied back to the host (ZH_OUT_DEVICE).  The store I/O is the same as read()'s
        (for a FilesystemStore the library's own file reads).  The per-rank decode of
        zarrhip.parallel.array_decoder."""
        t_enter = time.perf_counter()
        offset = [int(o) for o in offset]
        shape = [int(s) for s in shape]
        self._check_region(offset, shape)
        if any(s == 0 for s in shape):
            return
        self._read_into(offset, shape, int(out_ptr), A.ZH_OUT_DEVICE,
                        [dev if dev is not None else device()], parallel, t_enter)

    def _read_into(self, offset, shape, out_addr, flags, devs, parallel, t_enter):
        """The device read of a checked, non-empty region into out_addr (host memory, or
        device memory with flags ZH_OUT_DEVICE and one context)."""
        coords = self._chunk_coords(offset, shape)
        t0 = time.perf_counter()
        paths = self._file_paths(coords, devs)
        if paths is not None:  # the library reads the store's files itself
            t1 = time.perf_counter()
            try:
                if len(devs) > 1:  # one slab per device, each over its own PCIe link
                    _lib.array_read_files_multi(devs, self.zmeta, paths, offset, shape,
                                                out_addr, flags, store=self._file_store())
                else:
                    devs[0].array_read_files(self.zmeta, paths, offset, shape, out_addr,
                                             flags, store=self._file_store())
            except _lib.ZhError as e:
                raise_for(e)
            self.last_read_timing = {"prep_s": t0 - t_enter, "stage_s": t1 - t0,
                                     "device_s": time.perf_counter() - t1, "files": True}
            return
        lease = []  # staging buffers of this read, back to the pool after the device read
        sharded = self.chain.chain["sharded"]
        try:
            def load(c):
                lo = [max(o, ci * cs) - ci * cs
                      for o, ci, cs in zip(offset, c, self.metadata.chunk_shape)]
                hi = [min(o + s, (ci + 1) * cs) - ci * cs
                      for o, s, ci, cs in zip(offset, shape, c, self.metadata.chunk_shape)]
                return self._load_source(c, lo, hi, lease)
            if parallel and len(coords) > 1:  # the store reads of the chunks, concurrently
                # (core.Array.read's parallel stream over chunks, M/core/Array.java:403-407)
                from concurrent.futures import ThreadPoolExecutor
                with ThreadPoolExecutor(max_workers=min(8, len(coords))) as ex:
                    sources = list(ex.map(load, coords))
            else:
                sources = [load(c) for c in coords]
            t1 = time.perf_counter()
            keep = []
            try:
                if sharded:  # index + pieces (or whole objects as one piece at 0)
                    shards = []
                    for s in sources:
                        if s is None:
                            shards.append(None)
                        elif s[0] == "pieces":
                            shards.append(s[1])
                            keep.append(s[2])
                        else:
                            v = np.frombuffer(s[1], np.uint8) if len(s[1]) else \
                                np.zeros(1, np.uint8)
                            keep.append(v)
                            shards.append(_lib.ShardSource(None, 0, len(s[1]),
                                                           [(0, len(s[1]), v.ctypes.data,
                                                             len(s[1]))]))
                    if len(devs) > 1:
                        _lib.array_read_pieces_multi(devs, self.zmeta, shards, offset, shape,
                                                     out_addr, flags)
                    else:
                        devs[0].array_read_pieces(self.zmeta, shards, offset, shape,
                                                  out_addr, flags)
                else:
                    # views of the staged bytes (the library only reads them); an empty but
                    # present chunk keeps a non-null pointer (null = missing key → fill)
                    bufs = [None if s is None else
                            np.frombuffer(s[1] if len(s[1]) else b"\0", np.uint8)
                            for s in sources]
                    keep.append(bufs)
                    srcs = [((int(b.ctypes.data), len(s[1])) if s is not None else (None, 0))
                            for b, s in zip(bufs, sources)]
                    if len(devs) > 1:  # one slab per device, each D2H'd into its slice of `out`
                        _lib.array_read_multi(devs, self.zmeta, srcs, offset, shape,
                                              out_addr, flags)
                    else:
                        devs[0].array_read(self.zmeta, srcs, offset, shape, out_addr, flags)
            except _lib.ZhError as e:
                raise_for(e)
            finally:  # the call has consumed the staged bytes (it returns after its copies)
                del keep, sources
        finally:  # also when a store read or a host codec raised: the lease goes back
            staging_pool.give(lease)
        self.last_read_timing = {"prep_s": t0 - t_enter, "stage_s": t1 - t0,
                                 "device_s": time.perf_counter() - t1}

    def readChunk(self, coords):
        """core.Array.readChunk (M/core/Array.java:167-182)."""
        cs = self.metadata.chunk_shape
        for d, c in enumerate(coords):
            if c < 0 or c * cs[d] >= self.metadata.shape[d]:
                raise ZarrException("Attempting to read data outside of the array's domain.")
        out = np.empty(cs, dtype=self.metadata.data_type.numpy)
        paths = self._file_paths([tuple(coords)], [device()])
        if paths is not None:  # the chunk file, read by the library (one-chunk view)
            m = A.zh_array_meta.from_buffer_copy(self.zmeta)
            for d in range(self.ndim):
                m.shape[d] = cs[d]
            try:
                device().array_read_files(m, paths, [0] * self.ndim, cs, out.ctypes.data, 0,
                                          store=self._file_store())
            except _lib.ZhError as e:
                raise_for(e)
            return out
        src = self._load_source(tuple(coords))
        if src is None:
            out.view(np.uint8).reshape(-1)[:] = np.frombuffer(
                self.metadata.fill_bytes * int(np.prod(cs)), np.uint8)
            return out
        # one chunk viewed as a one-chunk array: ShardingIndexedCodec.decode / bytes decode
        m = A.zh_array_meta.from_buffer_copy(self.zmeta)
        for d in range(self.ndim):
            m.shape[d] = cs[d]
        try:
            if src[0] == "pieces":
                device().array_read_pieces(m, [src[1]], [0] * self.ndim, cs, out.ctypes.data,
                                           0)
            else:
                b = _host_buf(src[1])
                device().array_read(m, [(C.addressof(b), len(src[1]))], [0] * self.ndim, cs,
                                    out.ctypes.data, 0)
        except _lib.ZhError as e:
            raise_for(e)
        return out

    # ---------------------------------------------------------------- write
    def write(self, offset, data, parallel=True):
        """core.Array.write(offset, array, parallel) (M/core/Array.java:83-156): whole-chunk
        regions are encoded on the device in one call; partial chunks are read-modify-written
        (decode → patch → encode).  `parallel` is the reference's switch between a serial and a
        parallel chunk stream; the device encodes every chunk of a call in one launch either
        way, so it only reaches the read of a read-modify-write."""
        data = np.ascontiguousarray(data, dtype=self.metadata.data_type.numpy)
        n = self.ndim
        offset = [0] * n if offset is None else [int(o) for o in offset]
        shape = list(data.shape)
        self._check_region(offset, shape)
        cs, ash = self.metadata.chunk_shape, self.metadata.shape
        lo = [(o // c) * c for o, c in zip(offset, cs)]
        hi = [min(-(-(o + s) // c) * c, a) for o, s, c, a in zip(offset, shape, cs, ash)]
        if lo != offset or hi != [o + s for o, s in zip(offset, shape)]:
            ext = [h - l for l, h in zip(lo, hi)]
            region = self.read(lo, ext, parallel)
            sl = tuple(slice(o - l, o - l + s) for o, l, s in zip(offset, lo, shape))
            region[sl] = data
            data, offset, shape = region, lo, ext
        coords = self._chunk_coords(offset, shape)
        dev = device()
        keep_fill = getattr(self.metadata, "fill_value", 0) is None and \
            not self.chain.chain["sharded"]
        paths = None if keep_fill else self._file_paths(coords, [dev])
        if paths is not None:  # the library writes (and deletes) the chunk files itself
            try:
                dev.array_write_files(self.zmeta, data.ctypes.data, offset, shape, paths,
                                      store=self._file_store())
            except _lib.ZhError as e:
                raise_for(e)
            return
        L = _lib.lib()
        cap = L.zh_array_encoded_bound(C.byref(self.zmeta))
        src = dev.malloc(max(1, data.nbytes))
        bufs = []
        try:
            dev.memcpy(src, data.ctypes.data, data.nbytes, 0)
            bufs = [dev.malloc(cap) for _ in coords]
            try:
                sizes = dev.array_write(self.zmeta, src, offset, shape, [(b, cap) for b in bufs])
            except _lib.ZhError as e:
                raise_for(e)
            for c, b, sz in zip(coords, bufs, sizes):
                h = self._handle(c)
                if sz == 0 and not keep_fill:
                    h.delete()  # all fill → writeChunk deletes the key (Array.java:150-151)
                    continue
                if sz == 0:
                    # no fill value (v2 "fill_value": null): writeChunk never deletes
                    # (Array.java:150 tests parsedFillValue != null) — store the zero chunk
                    enc = bytes(int(np.prod(cs)) * self.metadata.data_type.getByteCount())
                    if self.chain.chain.get("inner_crc32c"):
                        enc += struct.pack("<I", L.zh_crc32c(0, enc, len(enc)))
                else:
                    enc = dev.d2h(b, sz)
                if self.chain.host_bb:
                    enc = host_bb_encode(self.chain.host_bb, enc)
                elif self.chain.inner_host_bb:
                    enc = self._wrap_inner(enc)
                h.set(enc)
        finally:
            for b in bufs:
                dev.free(b)
            dev.free(src)

    def access(self):
        return ArrayAccessor(self)


class ArrayAccessor:
    """core.Array.ArrayAccessor (M/core/Array.java:483-536)."""

    def __init__(self, array):
        self.array = array
        self.offset = None
        self.shape = None

    def withOffset(self, *offset):
        self.offset = list(offset)
        return self

    def withShape(self, *shape):
        self.shape = list(shape)
        return self

    def read(self):
        return self.array.read(self.offset, self.shape)

    def write(self, data):
        self.array.write(self.offset, data)
