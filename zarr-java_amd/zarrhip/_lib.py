"""Loader for libzarrhip.so (the HIP path).  There is no CPU fallback: if the library or
the GPU is missing, the product raises instead of silently computing on the host."""
import ctypes as C
import os

from . import _abi as A

_HERE = os.path.dirname(os.path.abspath(__file__))
# ZH_LIB_PATH: another build of the same library (the host-sanitizer build, make asan)
LIB_PATH = os.environ.get("ZH_LIB_PATH") or os.path.join(_HERE, "libzarrhip.so")

_lib = None
# Whether torch was imported before the library was loaded.  torch's ROCm wheel bundles its own
# HIP runtime with the same SONAME (libamdhip64.so.7) as the system's: loaded first, torch's
# runtime is the one libzarrhip.so binds to and both share it; loaded after ours, torch gets a
# second copy and its CUDA init fails ("No HIP GPUs are available").  zarrhip.parallel, which
# moves torch tensors, checks this.
LOADED_AFTER_TORCH = None

P = C.c_void_p
I32 = C.c_int32
I64 = C.c_int64
U32 = C.c_uint32
U64 = C.c_uint64
SZ = C.c_size_t
CH = C.c_char_p
PI64 = C.POINTER(C.c_int64)
PI32 = C.POINTER(C.c_int32)
PMETA = C.POINTER(A.zh_array_meta)
PSTORE = C.POINTER(A.zh_file_store)

_SIGS = {
    "zh_version": (CH, []),
    "zh_ctx_create": (C.c_int, [C.c_int, C.POINTER(P)]),
    "zh_ctx_destroy": (None, [P]),
    "zh_ctx_device": (C.c_int, [P]),
    "zh_ctx_stream": (P, [P]),
    "zh_ctx_release_cache": (I64, [P]),
    "zh_validate_meta": (C.c_int, [PMETA, CH, SZ]),
    "zh_shard_index_size": (I64, [PMETA]),
    "zh_crc32c": (U32, [U32, P, SZ]),
    "zh_compute_chunk_coords": (I64, [C.c_int, PI64, PI32, PI64, PI64, PI64, I64]),
    "zh_compute_projection": (C.c_int, [C.c_int, PI64, PI64, PI32, PI64, PI64, PI32, PI32, PI32]),
    "zh_is_permutation": (C.c_int, [C.c_int, PI32]),
    "zh_inverse_permutation": (C.c_int, [C.c_int, PI32, PI32]),
    "zh_plan_create": (C.c_int, [P, PMETA, C.POINTER(A.zh_chunk_src), I64, PI64, PI64, U32,
                                 C.POINTER(P), CH, SZ]),
    "zh_plan_execute": (C.c_int, [P, P, P]),
    "zh_plan_wait": (C.c_int, [P, CH, SZ]),
    "zh_last_data_error": (C.c_int, [PI64, C.c_int, C.POINTER(U64)]),
    "zh_plan_destroy": (None, [P]),
    "zh_plan_stats": (C.c_int, [P, PI64, PI64, PI64, PI64]),
    "zh_plan_set_timing": (C.c_int, [P, C.c_int]),
    "zh_plan_set_graph": (C.c_int, [P, C.c_int]),
    "zh_plan_kernel_time": (C.c_int, [P, C.POINTER(C.c_double), PI64, C.POINTER(C.c_double)]),
    "zh_array_read": (C.c_int, [P, PMETA, C.POINTER(A.zh_chunk_src), I64, PI64, PI64, P, U32, P,
                                CH, SZ]),
    "zh_array_read_multi": (C.c_int, [C.POINTER(P), C.c_int, C.c_int, PMETA,
                                      C.POINTER(A.zh_chunk_src), I64, PI64, PI64, P, U32, CH,
                                      SZ]),
    "zh_array_read_multi_routed": (C.c_int, [C.POINTER(P), C.c_int, C.c_int, PMETA,
                                             C.POINTER(A.zh_chunk_src), I64, PI64, PI64, P, U32,
                                             PI32, CH, SZ]),
    "zh_device_count": (C.c_int, []),
    "zh_slab_partition": (C.c_int, [C.c_int, PI64, PI64, C.c_int, I64, PI64, PI64]),
    "zh_sharding_decode": (C.c_int, [P, PMETA, P, I64, P, U32, P, CH, SZ]),
    "zh_sharding_decode_partial": (C.c_int, [P, PMETA, P, I64, PI64, PI32, P, U32, P, CH, SZ]),
    "zh_shard_ranges": (I64, [PMETA, P, I64, I64, PI64, PI64, I64, PI64, I64]),
    "zh_shard_index_check": (C.c_int, [PMETA, P, I64, C.c_char_p, SZ]),
    "zh_array_read_pieces": (C.c_int, [P, PMETA, C.POINTER(A.zh_shard_src), I64, PI64, PI64, P,
                                       U32, P, CH, SZ]),
    "zh_array_read_pieces_multi": (C.c_int, [C.POINTER(P), C.c_int, C.c_int, PMETA,
                                             C.POINTER(A.zh_shard_src), I64, PI64, PI64, P, U32,
                                             PI32, CH, SZ]),
    "zh_sharding_decode_pieces": (C.c_int, [P, PMETA, C.POINTER(A.zh_shard_src), PI64, PI32, P,
                                            U32, P, CH, SZ]),
    "zh_host_staging": (C.c_int, [P, SZ, C.POINTER(P)]),
    "zh_array_read_files": (C.c_int, [P, PMETA, PSTORE, C.POINTER(C.c_char_p), I64, PI64, PI64,
                                      P, U32, CH, SZ]),
    "zh_debug_file_reads": (I64, [PMETA, PSTORE, C.POINTER(C.c_char_p), I64, PI64, PI64, PI64,
                                  I64, CH, SZ]),
    "zh_debug_file_table": (C.c_int, [PI64]),
    "zh_array_write_files": (C.c_int, [P, PMETA, P, PI64, PI64, PSTORE, C.POINTER(C.c_char_p),
                                       I64, U32, PI64, CH, SZ]),
    "zh_array_read_files_multi": (C.c_int, [C.POINTER(P), C.c_int, C.c_int, PMETA, PSTORE,
                                            C.POINTER(C.c_char_p), I64, PI64, PI64, P, U32, PI32,
                                            CH, SZ]),
    "zh_array_encoded_bound": (I64, [PMETA]),
    "zh_array_write": (C.c_int, [P, PMETA, P, PI64, PI64, C.POINTER(A.zh_chunk_dst), I64, P, CH,
                                 SZ]),
    "zh_array_write_host": (C.c_int, [P, PMETA, P, PI64, PI64, C.POINTER(P), PI64, PI64, I64, CH,
                                      SZ]),
    "zh_abi_sizes": (C.c_int, [C.POINTER(C.c_int64), C.c_int]),
    "zh_plan_staged_bytes": (C.c_int64, [P]),
    "zh_blosc_decompress": (C.c_int, [P, SZ, P, SZ, C.POINTER(SZ), C.c_char_p, SZ]),
    "zh_zstd_decompress": (C.c_int, [P, SZ, P, SZ, C.POINTER(SZ), C.c_char_p, SZ]),
    "zh_zstd_compress_raw": (C.c_int, [P, SZ, C.c_int, P, SZ, C.POINTER(SZ)]),
    "zh_xxh64": (U64, [P, SZ, U64]),
    "zh_device_malloc": (C.c_int, [P, SZ, C.POINTER(P)]),
    "zh_device_malloc_ex": (C.c_int, [P, SZ, C.c_uint, C.POINTER(P)]),
    "zh_device_free": (C.c_int, [P, P]),
    "zh_device_scatter_view": (C.c_int, [P, P, U64, C.POINTER(P)]),
    "zh_device_alloc_probes": (C.c_int, [P, P, C.POINTER(C.c_double), C.c_int,
                                         C.POINTER(C.c_int)]),
    "zh_device_write_rate": (C.c_int, [P, P, SZ, C.c_int, C.c_int, C.POINTER(C.c_double)]),
    "zh_device_copy_rate": (C.c_int, [P, P, P, SZ, C.c_int, C.POINTER(C.c_double)]),
    "zh_host_malloc_pinned": (C.c_int, [P, SZ, C.POINTER(P)]),
    "zh_host_free_pinned": (C.c_int, [P, P]),
    "zh_host_register": (C.c_int, [P, P, SZ]),
    "zh_host_unregister": (C.c_int, [P, P]),
    "zh_memcpy_async": (C.c_int, [P, P, P, SZ, C.c_int, P]),
    "zh_memset_async": (C.c_int, [P, P, C.c_int, SZ, P]),
    "zh_stream_synchronize": (C.c_int, [P, P]),
    "zh_stream_create": (C.c_int, [P, C.POINTER(P)]),
    "zh_stream_destroy": (C.c_int, [P, P]),
    "zh_stream_wait_event": (C.c_int, [P, P, P]),
    "zh_memcpy2d_async": (C.c_int, [P, P, SZ, P, SZ, SZ, SZ, C.c_int, P]),
    "zh_event_create": (C.c_int, [P, C.POINTER(P)]),
    "zh_event_destroy": (C.c_int, [P, P]),
    "zh_event_record": (C.c_int, [P, P, P]),
    "zh_event_elapsed_ms": (C.c_int, [P, P, P, C.POINTER(C.c_float)]),
    "zh_device_info": (C.c_int, [P, CH, SZ, PI64, C.POINTER(C.c_int), CH, SZ]),
    "zh_gather_blocks": (C.c_int, [P, P, P, I64, PI64, I64]),
    "zh_debug_last_fast_path": (I64, [C.c_int]),
    "zh_synth_fill": (C.c_int, [P, P, I64, C.c_int, I64, U64, P]),
    "zh_synth_verify": (C.c_int, [P, P, C.c_int, PI64, PI64, PI64, C.c_int, U64,
                                  C.POINTER(U64), P]),
}


def lib():
    """The loaded libzarrhip.so (raises ImportError when it has not been built)."""
    global _lib, LOADED_AFTER_TORCH
    if _lib is None:
        import sys
        LOADED_AFTER_TORCH = "torch" in sys.modules
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libzarrhip.so not found at {LIB_PATH}: build it with "
                "`make -C zarr-java_amd` (the HIP path has no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name, None)
            if f is None:  # an older build via ZH_LIB_PATH (A/B labs); test_abi checks ours
                continue
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def declared_symbols():
    return list(_SIGS)


def i64arr(vals):
    return (C.c_int64 * max(1, len(vals)))(*[int(v) for v in vals])


def i32arr(vals):
    return (C.c_int32 * max(1, len(vals)))(*[int(v) for v in vals])


class ZhError(RuntimeError):
    def __init__(self, status, message, position=None):
        super().__init__(message)
        self.status = status
        # ZH_EDATA: (chunk grid coords, key) of the failing chunk in a sequential read's order
        # (zh_last_data_error), or None
        self.position = position


def last_data_error():
    """zh_last_data_error for this thread's last read call: (coords tuple, key) or None."""
    cc = (C.c_int64 * 32)()
    key = C.c_uint64()
    n = lib().zh_last_data_error(cc, 32, C.byref(key))
    return (tuple(cc[i] for i in range(n)), key.value) if n > 0 else None


def check(status, err=None):
    if status != A.ZH_OK:
        msg = err.value.decode(errors="replace") if err is not None else ""
        pos = last_data_error() if status == A.ZH_EDATA else None
        raise ZhError(status, msg or f"zarrhip status {status}", pos)


class DeviceContext:
    """One GPU (a zh_ctx): device memory, streams and the decode/encode entry points."""

    def __init__(self, device=0):
        self.L = lib()
        h = P()
        st = self.L.zh_ctx_create(int(device), C.byref(h))
        if st != A.ZH_OK:
            raise ZhError(st, f"zh_ctx_create(device={device}) failed (status {st}); "
                              "is a GPU visible?")
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            self.L.zh_ctx_destroy(self.h)
            self.h = None

    def release_cache(self):
        """zh_ctx_release_cache: hand the finished plans' cached device blocks back."""
        return self.L.zh_ctx_release_cache(self.h)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- memory ---------------------------------------------------------------------
    def malloc(self, nbytes, flags=None):
        """Device allocation; `flags` (A.ZH_MALLOC_*) defaults to ZH_MALLOC env (else 0)."""
        p = P()
        if flags is None:
            flags = int(os.environ.get("ZH_MALLOC", "0"), 0)
        st = self.L.zh_device_malloc_ex(self.h, int(nbytes), int(flags), C.byref(p))
        if st != A.ZH_OK:
            raise ZhError(st, f"device malloc of {nbytes} bytes failed")
        return p.value

    def free(self, ptr):
        if ptr:
            self.L.zh_device_free(self.h, P(ptr))

    def scatter_view(self, ptr, order=0):
        """Map a ZH_MALLOC_SCATTER allocation's chunks again at a fresh virtual range, in
        chunk order `order`; free the view (self.free) before the allocation."""
        p = P()
        check(self.L.zh_device_scatter_view(self.h, P(ptr), int(order), C.byref(p)))
        return p.value

    def alloc_probes(self, ptr):
        """ZH_MALLOC_CALIBRATE record of `ptr`: (probe GB/s of every candidate, chosen index),
        ([], -1) for an allocation that was not calibrated."""
        buf = (C.c_double * 16)()
        ch = C.c_int(-1)
        k = self.L.zh_device_alloc_probes(self.h, P(ptr), buf, 16, C.byref(ch))
        if k < 0:
            check(-k)
        return [round(buf[i], 1) for i in range(min(k, 16))], ch.value

    def write_rate(self, ptr, nbytes, pattern=1, reps=3):
        """Write bandwidth of a device range by a store-only probe, GB/s (overwrites it)."""
        g = C.c_double()
        check(self.L.zh_device_write_rate(self.h, P(ptr), int(nbytes), int(pattern), int(reps),
                                          C.byref(g)))
        return g.value

    def copy_rate(self, dst, src, nbytes, reps=3):
        """Copy ceiling of a buffer pair by a streaming byte-swapping copy src -> dst,
        GB/s of bytes read + written (overwrites dst)."""
        g = C.c_double()
        check(self.L.zh_device_copy_rate(self.h, P(dst), P(src), int(nbytes), int(reps),
                                         C.byref(g)))
        return g.value

    def malloc_pinned(self, nbytes):
        p = P()
        check(self.L.zh_host_malloc_pinned(self.h, int(nbytes), C.byref(p)))
        return p.value

    def free_pinned(self, ptr):
        if ptr:
            self.L.zh_host_free_pinned(self.h, P(ptr))

    def host_register(self, ptr, nbytes):
        check(self.L.zh_host_register(self.h, P(ptr), int(nbytes)))

    def host_unregister(self, ptr):
        if ptr:
            self.L.zh_host_unregister(self.h, P(ptr))

    def memcpy(self, dst, src, nbytes, kind, stream=None, sync=True):
        check(self.L.zh_memcpy_async(self.h, P(dst), P(src), int(nbytes), int(kind), P(stream)))
        if sync:
            self.sync(stream)

    def h2d(self, dst, host_bytes, stream=None):
        buf = (C.c_char * len(host_bytes)).from_buffer_copy(host_bytes) \
            if not isinstance(host_bytes, C.Array) else host_bytes
        self.memcpy(dst, C.addressof(buf), len(host_bytes), 0, stream, True)

    def d2h(self, src, nbytes, stream=None):
        buf = (C.c_char * int(nbytes))()
        self.memcpy(C.addressof(buf), src, nbytes, 1, stream, True)
        return bytes(buf)

    def memset(self, dst, value, nbytes, stream=None):
        check(self.L.zh_memset_async(self.h, P(dst), int(value), int(nbytes), P(stream)))

    def sync(self, stream=None):
        check(self.L.zh_stream_synchronize(self.h, P(stream)))

    def info(self):
        name = C.create_string_buffer(256)
        arch = C.create_string_buffer(64)
        mem = C.c_int64()
        cus = C.c_int()
        check(self.L.zh_device_info(self.h, name, 256, C.byref(mem), C.byref(cus), arch, 64))
        return {"name": name.value.decode(), "arch": arch.value.decode(),
                "total_mem": mem.value, "cu_count": cus.value}

    def stream(self):
        s = P()
        check(self.L.zh_stream_create(self.h, C.byref(s)))
        return s.value

    def stream_destroy(self, s):
        if s:
            self.L.zh_stream_destroy(self.h, P(s))

    def wait_event(self, stream, ev):
        check(self.L.zh_stream_wait_event(self.h, P(stream), P(ev)))

    def memcpy2d(self, dst, dpitch, src, spitch, width, height, kind, stream=None):
        check(self.L.zh_memcpy2d_async(self.h, P(dst), int(dpitch), P(src), int(spitch),
                                       int(width), int(height), int(kind), P(stream)))

    # -- events ---------------------------------------------------------------------
    def event(self):
        e = P()
        check(self.L.zh_event_create(self.h, C.byref(e)))
        return e.value

    def record(self, ev, stream=None):
        check(self.L.zh_event_record(self.h, P(ev), P(stream)))

    def elapsed_ms(self, a, b):
        ms = C.c_float()
        check(self.L.zh_event_elapsed_ms(self.h, P(a), P(b), C.byref(ms)))
        return ms.value

    def gather_blocks(self, dst, src, block_bytes, src_blocks):
        """zh_gather_blocks: dst block b <- src block src_blocks[b] (synchronous)."""
        idx = (C.c_int64 * max(1, len(src_blocks)))(*[int(x) for x in src_blocks])
        check(self.L.zh_gather_blocks(self.h, P(dst), P(src), int(block_bytes), idx,
                                      len(src_blocks)))

    # -- synthetic data ---------------------------------------------------------------
    def synth_fill(self, dst, n, dtype_size, first=0, seed=0x5A5A2026, stream=None):
        check(self.L.zh_synth_fill(self.h, P(dst), int(n), int(dtype_size), int(first),
                                   int(seed), P(stream)))

    def synth_verify(self, region, array_shape, offset, shape, dtype_size, seed=0x5A5A2026,
                     stream=None):
        mm = C.c_uint64()
        n = len(array_shape)
        check(self.L.zh_synth_verify(self.h, P(region), n, i64arr(array_shape), i64arr(offset),
                                     i64arr(shape), int(dtype_size), int(seed), C.byref(mm),
                                     P(stream)))
        return mm.value

    # -- codec path -------------------------------------------------------------------
    def array_read(self, meta, sources, offset, shape, out, flags, stream=None):
        """zh_array_read.  sources: list of (pointer or None, nbytes)."""
        srcs = (A.zh_chunk_src * max(1, len(sources)))()
        for i, (ptr, nb) in enumerate(sources):
            srcs[i].data = ptr
            srcs[i].nbytes = int(nb)
        err = C.create_string_buffer(1024)
        st = self.L.zh_array_read(self.h, C.byref(meta), srcs, len(sources), i64arr(offset),
                                  i64arr(shape), P(out), int(flags), P(stream), err, 1024)
        check(st, err)

    def array_read_pieces(self, meta, shards, offset, shape, out, flags, stream=None):
        """zh_array_read_pieces.  shards: list of ShardSource (or None = missing key)."""
        arr, keep = shard_src_array(shards)
        err = C.create_string_buffer(1024)
        st = self.L.zh_array_read_pieces(self.h, C.byref(meta), arr, len(shards), i64arr(offset),
                                         i64arr(shape), P(out), int(flags), P(stream), err, 1024)
        del keep
        check(st, err)

    def sharding_decode_pieces(self, meta, shard, offset, shape, out, flags=0, stream=None):
        """zh_sharding_decode_pieces: decodePartial of one shard given as index + pieces."""
        arr, keep = shard_src_array([shard])
        err = C.create_string_buffer(1024)
        st = self.L.zh_sharding_decode_pieces(self.h, C.byref(meta), arr, i64arr(offset),
                                              i32arr(shape), P(out), int(flags), P(stream), err,
                                              1024)
        del keep
        check(st, err)

    def array_read_files(self, meta, paths, offset, shape, out, flags=0, store=None):
        """zh_array_read_files: the chunks as files of a FilesystemStore (None or a path that
        is not a regular file = missing key); the library does the store reads.  `store`: the
        store the paths belong to (file_store), for StoreException's text."""
        arr = path_array(paths)
        err = C.create_string_buffer(1024)
        fs = file_store(store)
        st = self.L.zh_array_read_files(self.h, C.byref(meta), fs, arr, len(paths),
                                        i64arr(offset), i64arr(shape), P(out), int(flags), err,
                                        1024)
        check(st, err)

    def array_write_files(self, meta, src, offset, shape, paths, flags=0, store=None):
        """zh_array_write_files: encode the region (host pointer, or device with ZH_SRC_DEVICE)
        and write / delete the chunk files; returns the bytes written per chunk (0: deleted)."""
        n = len(paths)
        sizes = (C.c_int64 * max(1, n))()
        err = C.create_string_buffer(1024)
        fs = file_store(store)
        st = self.L.zh_array_write_files(self.h, C.byref(meta), P(src), i64arr(offset),
                                         i64arr(shape), fs, path_array(paths), n, int(flags),
                                         sizes, err, 1024)
        check(st, err)
        return [int(sizes[i]) for i in range(n)]

    def host_staging(self, nbytes):
        """zh_host_staging: the context's page-locked staging (valid until the next call)."""
        p = P()
        check(self.L.zh_host_staging(self.h, int(nbytes), C.byref(p)))
        return p.value

    def plan(self, meta, sources, offset, shape, flags):
        return Plan(self, meta, sources, offset, shape, flags)

    def array_write_host(self, meta, data, offset, shape, nchunks):
        """zh_array_write_host: region bytes (host) → list of encoded chunk bytes (None =
        all fill, delete the key), staged through the device inside the call."""
        bound = self.L.zh_array_encoded_bound(C.byref(meta))
        bufs = [(C.c_char * max(1, bound))() for _ in range(nchunks)]
        outs = (P * max(1, nchunks))(*[C.addressof(b) for b in bufs])
        caps = (C.c_int64 * max(1, nchunks))(*([bound] * nchunks))
        sizes = (C.c_int64 * max(1, nchunks))()
        src = (C.c_char * max(1, len(data))).from_buffer_copy(data if len(data) else b"\0")
        err = C.create_string_buffer(1024)
        st = self.L.zh_array_write_host(self.h, C.byref(meta), src, i64arr(offset), i64arr(shape),
                                        outs, caps, sizes, nchunks, err, 1024)
        check(st, err)
        return [bytes(b)[:sizes[i]] if sizes[i] else None for i, b in enumerate(bufs)]

    def array_write(self, meta, src, offset, shape, dsts, stream=None):
        """zh_array_write.  dsts: list of (device pointer, capacity) → list of nbytes."""
        arr = (A.zh_chunk_dst * max(1, len(dsts)))()
        for i, (ptr, cap) in enumerate(dsts):
            arr[i].data = ptr
            arr[i].capacity = int(cap)
            arr[i].nbytes = 0
        err = C.create_string_buffer(1024)
        st = self.L.zh_array_write(self.h, C.byref(meta), P(src), i64arr(offset), i64arr(shape),
                                   arr, len(dsts), P(stream), err, 1024)
        check(st, err)
        return [arr[i].nbytes for i in range(len(dsts))]


def array_read_multi(ctxs, meta, sources, offset, shape, out, flags, root=0):
    """zh_array_read_multi_routed: one region read split into per-device slabs (one
    DeviceContext per slab), delivered to a host buffer or to a buffer on ctxs[root]'s
    device.  Returns the per-slab routes (A.ZH_ROUTE_*)."""
    L = lib()
    hs = (P * len(ctxs))(*[c.h for c in ctxs])
    srcs = (A.zh_chunk_src * max(1, len(sources)))()
    for i, (ptr, nb) in enumerate(sources):
        srcs[i].data = ptr
        srcs[i].nbytes = int(nb)
    routes = (C.c_int32 * len(ctxs))()
    err = C.create_string_buffer(1024)
    st = L.zh_array_read_multi_routed(hs, len(ctxs), int(root), C.byref(meta), srcs,
                                      len(sources), i64arr(offset), i64arr(shape), P(out),
                                      int(flags), routes, err, 1024)
    check(st, err)
    return list(routes)


class ShardSource:
    """One stored shard of a pieces read (zh_shard_src): the stored index bytes as the
    prefix/suffix read returned them (None: a whole shard in one piece at offset 0), the
    shard size (StoreHandle.getSize(), -1 unknown) and its pieces as (offset, stored nbytes,
    pointer, held nbytes) tuples."""

    def __init__(self, index_ptr, index_nbytes, shard_nbytes, pieces):
        self.index_ptr = index_ptr
        self.index_nbytes = int(index_nbytes)
        self.shard_nbytes = int(shard_nbytes)
        self.pieces = list(pieces)


def shard_src_array(shards):
    """ctypes zh_shard_src[] for a list of ShardSource / None; returns (array, keepalive)."""
    arr = (A.zh_shard_src * max(1, len(shards)))()
    keep = []
    for i, s in enumerate(shards):
        if s is None:
            continue
        ps = (A.zh_shard_piece * max(1, len(s.pieces)))()
        for k, (off, nb, ptr, held) in enumerate(s.pieces):
            ps[k].offset, ps[k].nbytes, ps[k].data, ps[k].data_nbytes = int(off), int(nb), ptr, \
                int(held)
        keep.append(ps)
        arr[i].index = s.index_ptr
        arr[i].index_nbytes = s.index_nbytes
        arr[i].shard_nbytes = s.shard_nbytes
        arr[i].pieces = ps
        arr[i].npieces = len(s.pieces)
    return arr, keep


def shard_ranges(meta, index, shard_nbytes, part_lo, part_hi, max_run=64 << 20):
    """zh_shard_ranges over index bytes (bytes-like) → [(offset, nbytes)] to read."""
    L = lib()
    buf = (C.c_char * max(1, len(index))).from_buffer_copy(bytes(index) or b"\0")
    n = L.zh_shard_ranges(C.byref(meta), buf, len(index), int(shard_nbytes), i64arr(part_lo),
                          i64arr(part_hi), int(max_run), None, 0)
    if n < 0:
        check(-n)
    out = (C.c_int64 * max(2, 2 * n))()
    n2 = L.zh_shard_ranges(C.byref(meta), buf, len(index), int(shard_nbytes), i64arr(part_lo),
                           i64arr(part_hi), int(max_run), out, n)
    assert n2 == n
    return [(out[2 * k], out[2 * k + 1]) for k in range(n)]


def shard_index_check(meta, index):
    """zh_shard_index_check: Crc32cCodec.decode of a stored shard index on the host; raises
    ZhError(ZH_EDATA) with the reference's message when its crc32c does not match."""
    L = lib()
    buf = (C.c_char * max(1, len(index))).from_buffer_copy(bytes(index) or b"\0")
    err = C.create_string_buffer(1024)
    check(L.zh_shard_index_check(C.byref(meta), buf, len(index), err, 1024), err)


def array_read_pieces_multi(ctxs, meta, shards, offset, shape, out, flags, root=0):
    """zh_array_read_pieces_multi: the pieces form of array_read_multi; returns the routes."""
    L = lib()
    hs = (P * len(ctxs))(*[c.h for c in ctxs])
    arr, keep = shard_src_array(shards)
    routes = (C.c_int32 * len(ctxs))()
    err = C.create_string_buffer(1024)
    st = L.zh_array_read_pieces_multi(hs, len(ctxs), int(root), C.byref(meta), arr, len(shards),
                                      i64arr(offset), i64arr(shape), P(out), int(flags), routes,
                                      err, 1024)
    del keep
    check(st, err)
    return list(routes)


def path_array(paths):
    """char*[] of chunk file paths (None → NULL: a missing key)."""
    return (C.c_char_p * max(1, len(paths)))(
        *[None if p is None else os.fsencode(p) for p in paths])


def file_store(store):
    """zh_file_store* for a store argument: None (the filesystem root), a directory (str or
    path-like: name "file://<dir>") or a (root, name) pair; the struct keeps its strings."""
    if store is None:
        return None
    if isinstance(store, tuple):
        root, name = store
    else:
        root, name = os.fspath(store), None
    fs = A.zh_file_store(os.fsencode(root), None if name is None else name.encode())
    return C.pointer(fs)


def file_reads(meta, paths, offset, shape, store=None):
    """zh_debug_file_reads: [(chunk index, file offset, bytes)] the files read would make
    (raises ZhError with the read's status and message)."""
    L = lib()
    arr = path_array(paths)
    err = C.create_string_buffer(1024)
    fs = file_store(store)
    n = L.zh_debug_file_reads(C.byref(meta), fs, arr, len(paths), i64arr(offset),
                              i64arr(shape), None, 0, err, 1024)
    if n < 0:
        check(-n, err)
    buf = (C.c_int64 * max(1, 3 * n))()
    L.zh_debug_file_reads(C.byref(meta), fs, arr, len(paths), i64arr(offset), i64arr(shape),
                          buf, n, err, 1024)
    return [tuple(buf[3 * k:3 * k + 3]) for k in range(n)]


def array_read_files_multi(ctxs, meta, paths, offset, shape, out, flags=0, root=0,
                           store=None):
    """zh_array_read_files_multi: the files form of array_read_multi; returns the routes."""
    L = lib()
    hs = (P * len(ctxs))(*[c.h for c in ctxs])
    routes = (C.c_int32 * len(ctxs))()
    err = C.create_string_buffer(1024)
    fs = file_store(store)
    st = L.zh_array_read_files_multi(hs, len(ctxs), int(root), C.byref(meta), fs,
                                     path_array(paths), len(paths), i64arr(offset),
                                     i64arr(shape), P(out), int(flags), routes, err, 1024)
    check(st, err)
    return list(routes)


def device_count():
    """Visible HIP devices (zh_device_count)."""
    return int(lib().zh_device_count())


def slab_partition(offset, shape, nslabs, align=1):
    """zh_slab_partition → [(slab_offset, slab_shape)] (the C twin of parallel.slab_partition)."""
    n = len(shape)
    so = (C.c_int64 * (n * nslabs))()
    ss = (C.c_int64 * (n * nslabs))()
    check(lib().zh_slab_partition(n, i64arr(offset), i64arr(shape), int(nslabs), int(align),
                                  so, ss))
    return [(list(so[r * n:(r + 1) * n]), list(ss[r * n:(r + 1) * n])) for r in range(nslabs)]


class Plan:
    """A prepared region read (zh_plan): plan once, execute many times."""

    def __init__(self, ctx, meta, sources, offset, shape, flags):
        self.ctx = ctx
        self.L = ctx.L
        self._meta = meta
        srcs = (A.zh_chunk_src * max(1, len(sources)))()
        for i, (ptr, nb) in enumerate(sources):
            srcs[i].data = ptr
            srcs[i].nbytes = int(nb)
        self._srcs = srcs
        h = P()
        err = C.create_string_buffer(1024)
        st = self.L.zh_plan_create(ctx.h, C.byref(meta), srcs, len(sources), i64arr(offset),
                                   i64arr(shape), int(flags), C.byref(h), err, 1024)
        check(st, err)
        self.h = h

    def execute(self, out, stream=None):
        check(self.L.zh_plan_execute(self.h, P(out), P(stream)))

    def wait(self):
        err = C.create_string_buffer(1024)
        check(self.L.zh_plan_wait(self.h, err, 1024), err)

    def stats(self):
        a, b, c, d = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        check(self.L.zh_plan_stats(self.h, C.byref(a), C.byref(b), C.byref(c), C.byref(d)))
        return {"in_bytes": a.value, "out_bytes": b.value, "items": c.value, "shards": d.value}

    def set_timing(self, on=True):
        check(self.L.zh_plan_set_timing(self.h, 1 if on else 0))

    def set_graph(self, on=True):
        check(self.L.zh_plan_set_graph(self.h, 1 if on else 0))

    def staged_bytes(self):
        return int(self.L.zh_plan_staged_bytes(self.h))

    def kernel_time(self):
        sc, ix, n = C.c_double(), C.c_double(), C.c_int64()
        check(self.L.zh_plan_kernel_time(self.h, C.byref(sc), C.byref(n), C.byref(ix)))
        return {"scatter_ms": sc.value, "index_ms": ix.value, "launches": n.value}

    def close(self):
        if self.h:
            self.L.zh_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
