"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the C oracle (oracle/zh_oracle.c).

The oracle is the CPU restatement of zarr-java's codec path used to check the HIP path.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it; the
product (zarr-java_amd/zarrhip) never imports this module.
"""
import ctypes as C
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "zarr-java_amd"))

from zarrhip import _abi as A  # noqa: E402  (ABI struct definitions only)

LIB = os.path.join(HERE, "_build", "libzh_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P, I64 = C.c_void_p, C.c_int64
        PI64, PI32 = C.POINTER(C.c_int64), C.POINTER(C.c_int32)
        PM = C.POINTER(A.zh_array_meta)
        L.zo_crc32c.restype = C.c_uint32
        L.zo_crc32c.argtypes = [C.c_uint32, P, C.c_size_t]
        L.zo_compute_chunk_coords.restype = I64
        L.zo_compute_chunk_coords.argtypes = [C.c_int, PI64, PI32, PI64, PI64, PI64, I64]
        L.zo_compute_projection.restype = C.c_int
        L.zo_compute_projection.argtypes = [C.c_int, PI64, PI64, PI32, PI64, PI64, PI32, PI32,
                                            PI32]
        L.zo_is_permutation.restype = C.c_int
        L.zo_is_permutation.argtypes = [C.c_int, PI32]
        L.zo_inverse_permutation.restype = C.c_int
        L.zo_inverse_permutation.argtypes = [C.c_int, PI32, PI32]
        L.zo_array_read.restype = C.c_int
        L.zo_array_read.argtypes = [PM, C.POINTER(A.zh_chunk_src), I64, PI64, PI64, P, C.c_int,
                                    C.c_char_p, C.c_size_t]
        L.zo_array_read_store.restype = C.c_int
        L.zo_array_read_store.argtypes = [PM, C.POINTER(C.c_char_p), I64, PI64, PI64, P, C.c_int,
                                          C.c_char_p, C.c_size_t]
        L.zo_sharding_decode_partial.restype = C.c_int
        L.zo_sharding_decode_partial.argtypes = [PM, P, I64, PI64, PI32, P, C.c_int, C.c_char_p,
                                                 C.c_size_t]
        L.zo_array_write.restype = C.c_int
        L.zo_array_write.argtypes = [PM, P, PI64, PI64, C.POINTER(P), PI64, I64, C.c_char_p,
                                     C.c_size_t]
        L.zo_free.argtypes = [P]
        _lib = L
    return _lib


def _i64(v):
    return (C.c_int64 * max(1, len(v)))(*[int(x) for x in v])


def _i32(v):
    return (C.c_int32 * max(1, len(v)))(*[int(x) for x in v])


class OracleError(Exception):
    def __init__(self, status, msg):
        super().__init__(msg)
        self.status = status


def crc32c(data, crc=0):
    b = bytes(data)
    return lib().zo_crc32c(crc, b, len(b))


def compute_chunk_coords(array_shape, chunk_shape, sel_offset, sel_shape):
    n = len(array_shape)
    L = lib()
    num = L.zo_compute_chunk_coords(n, _i64(array_shape), _i32(chunk_shape), _i64(sel_offset),
                                    _i64(sel_shape), None, 0)
    if num < 0:
        raise ArithmeticError("Number of chunks exceeds Integer.MAX_VALUE")
    out = (C.c_int64 * max(1, num * n))()
    L.zo_compute_chunk_coords(n, _i64(array_shape), _i32(chunk_shape), _i64(sel_offset),
                              _i64(sel_shape), out, num)
    return [tuple(out[i * n + d] for d in range(n)) for i in range(num)]


def compute_projection(chunk_coords, array_shape, chunk_shape, sel_offset, sel_shape):
    n = len(chunk_coords)
    co, oo, ps = _i32([0] * n), _i32([0] * n), _i32([0] * n)
    st = lib().zo_compute_projection(n, _i64(chunk_coords), _i64(array_shape), _i32(chunk_shape),
                                     _i64(sel_offset), _i64(sel_shape), co, oo, ps)
    if st != 0:
        raise ArithmeticError("projection overflow")
    return list(co[:n]), list(oo[:n]), list(ps[:n])


def array_read(meta, sources, offset, shape, nthreads=1):
    """core.Array.read.  sources: list of bytes-like or None, in computeChunkCoords order."""
    n = meta.ndim
    nel = 1
    for d in range(n):
        nel *= int(shape[d])
    out = (C.c_char * max(1, nel * meta.dtype_size))()
    keep = []
    srcs = (A.zh_chunk_src * max(1, len(sources)))()
    for i, s in enumerate(sources):
        if s is None:
            srcs[i].data = None
            srcs[i].nbytes = 0
        else:
            b = (C.c_char * len(s)).from_buffer_copy(bytes(s)) if len(s) else (C.c_char * 1)()
            keep.append(b)
            srcs[i].data = C.addressof(b)
            srcs[i].nbytes = len(s)
    err = C.create_string_buffer(1024)
    st = lib().zo_array_read(C.byref(meta), srcs, len(sources), _i64(offset), _i64(shape), out,
                             nthreads, err, 1024)
    if st != 0:
        raise OracleError(st, err.value.decode())
    return bytes(out)[: nel * meta.dtype_size]


def array_read_into(meta, srcs_struct, nsrc, offset, shape, out_addr, nthreads=1):
    """Low-level form for timing: sources already a zh_chunk_src array of host pointers."""
    err = C.create_string_buffer(1024)
    st = lib().zo_array_read(C.byref(meta), srcs_struct, nsrc, _i64(offset), _i64(shape),
                             C.c_void_p(out_addr), nthreads, err, 1024)
    if st != 0:
        raise OracleError(st, err.value.decode())


def array_read_store(meta, paths, offset, shape, out_addr=None, nthreads=1):
    """core.Array.read from a FilesystemStore: `paths` = one file path (str) or None per chunk
    key, in computeChunkCoords order.  Sub-shard regions go through the partial path's
    per-inner-chunk range reads.  Returns bytes, or fills `out_addr` when given."""
    n = meta.ndim
    nel = 1
    for d in range(n):
        nel *= int(shape[d])
    buf = None
    if out_addr is None:
        buf = (C.c_char * max(1, nel * meta.dtype_size))()
        out_addr = C.addressof(buf)
    arr = (C.c_char_p * max(1, len(paths)))(*[None if p is None else os.fsencode(p)
                                               for p in paths])
    err = C.create_string_buffer(1024)
    st = lib().zo_array_read_store(C.byref(meta), arr, len(paths), _i64(offset), _i64(shape),
                                   C.c_void_p(out_addr), nthreads, err, 1024)
    if st != 0:
        raise OracleError(st, err.value.decode())
    return None if buf is None else bytes(buf)[: nel * meta.dtype_size]


def array_write(meta, src, offset, shape):
    """core.Array.write over whole chunks → list (computeChunkCoords order) of bytes|None."""
    n = meta.ndim
    coords = compute_chunk_coords([meta.shape[d] for d in range(n)],
                                  [meta.chunk_shape[d] for d in range(n)], offset, shape)
    k = len(coords)
    bufs = (C.c_void_p * max(1, k))()
    sizes = (C.c_int64 * max(1, k))()
    b = bytes(src)
    sb = (C.c_char * max(1, len(b))).from_buffer_copy(b if b else b"\0")
    err = C.create_string_buffer(1024)
    L = lib()
    st = L.zo_array_write(C.byref(meta), sb, _i64(offset), _i64(shape), bufs, sizes, k, err,
                          1024)
    if st != 0:
        raise OracleError(st, err.value.decode())
    out = []
    for i in range(k):
        if bufs[i]:
            out.append(C.string_at(bufs[i], sizes[i]))
            L.zo_free(bufs[i])
        else:
            out.append(None)
    return out
