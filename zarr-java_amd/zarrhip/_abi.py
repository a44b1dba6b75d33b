"""ctypes mirror of include/zarrhip.h (types and constants only; no library load)."""
import ctypes as C

ZH_MAX_DIMS = 8

ZH_OK = 0
ZH_EINVAL = 1
ZH_EDATA = 2
ZH_EUNSUPPORTED = 3
ZH_EHIP = 4
ZH_ENOMEM = 5
ZH_EARITH = 6
ZH_EIO = 7

ZH_ENDIAN_LITTLE = 0
ZH_ENDIAN_BIG = 1
ZH_INDEX_END = 0
ZH_INDEX_START = 1

ZH_SRC_DEVICE = 0x1
ZH_MALLOC_CONTIGUOUS = 0x1
ZH_MALLOC_REQUIRE = 0x2
ZH_MALLOC_SCATTER = 0x4
ZH_MALLOC_CALIBRATE = 0x8
ZH_MALLOC_PLAIN = 0x10
ZH_OUT_DEVICE = 0x2
# zh_array_read_multi_routed per-slab routes (include/zarrhip.h)
ZH_ROUTE_DIRECT = 0
ZH_ROUTE_PEER = 1
ZH_ROUTE_STAGED = 2
ZH_ROUTE_SAME = 3
ZH_ROUTE_SRC_PEER = 4
ZH_ROUTE_SRC_STAGED = 8


class zh_codec_chain(C.Structure):
    _fields_ = [
        ("sharded", C.c_int32),
        ("inner_chunk_shape", C.c_int32 * ZH_MAX_DIMS),
        ("has_transpose", C.c_int32),
        ("transpose_order", C.c_int32 * ZH_MAX_DIMS),
        ("endian", C.c_int32),
        ("index_endian", C.c_int32),
        ("index_has_crc32c", C.c_int32),
        ("index_location", C.c_int32),
        ("nested", C.c_int32),
        ("nested_chunk_shape", C.c_int32 * ZH_MAX_DIMS),
        ("nested_index_endian", C.c_int32),
        ("nested_index_has_crc32c", C.c_int32),
        ("nested_index_location", C.c_int32),
        ("inner_crc32c", C.c_int32),
    ]


class zh_array_meta(C.Structure):
    _fields_ = [
        ("ndim", C.c_int32),
        ("dtype_size", C.c_int32),
        ("dtype_is_bool", C.c_int32),
        ("dtype_is_float", C.c_int32),
        ("shape", C.c_int64 * ZH_MAX_DIMS),
        ("chunk_shape", C.c_int32 * ZH_MAX_DIMS),
        ("fill_value", C.c_uint8 * 8),
        ("chain", zh_codec_chain),
    ]


class zh_chunk_src(C.Structure):
    _fields_ = [("data", C.c_void_p), ("nbytes", C.c_int64)]


class zh_chunk_dst(C.Structure):
    _fields_ = [("data", C.c_void_p), ("capacity", C.c_int64), ("nbytes", C.c_int64)]


class zh_shard_piece(C.Structure):
    """One byte range of a stored shard (zarrhip.h zh_shard_piece)."""
    _fields_ = [("offset", C.c_int64), ("nbytes", C.c_int64), ("data", C.c_void_p),
                ("data_nbytes", C.c_int64)]


class zh_shard_src(C.Structure):
    """One stored shard as its index + the ranges read (zarrhip.h zh_shard_src)."""
    _fields_ = [("index", C.c_void_p), ("index_nbytes", C.c_int64),
                ("shard_nbytes", C.c_int64), ("pieces", C.POINTER(zh_shard_piece)),
                ("npieces", C.c_int64)]


class zh_file_store(C.Structure):
    """A FilesystemStore as the file reads name it (zarrhip.h zh_file_store)."""
    _fields_ = [("root", C.c_char_p), ("name", C.c_char_p)]


def make_meta(shape, chunk_shape, dtype_size, *, fill=b"\0" * 8, is_bool=False, is_float=False,
              sharded=False,
              inner_chunk_shape=None, transpose_order=None, endian=ZH_ENDIAN_LITTLE,
              index_endian=ZH_ENDIAN_LITTLE, index_crc32c=True, index_location=ZH_INDEX_END,
              nested_chunk_shape=None, nested_index_endian=ZH_ENDIAN_LITTLE,
              nested_index_crc32c=True, nested_index_location=ZH_INDEX_END,
              inner_crc32c=False):
    """Build a zh_array_meta from Python values.  `fill` is the element's bytes (LE)."""
    m = zh_array_meta()
    n = len(shape)
    m.ndim = n
    m.dtype_size = dtype_size
    m.dtype_is_bool = 1 if is_bool else 0
    m.dtype_is_float = 1 if is_float else 0
    for d in range(n):
        m.shape[d] = int(shape[d])
        m.chunk_shape[d] = int(chunk_shape[d])
    fb = bytes(fill)[:8].ljust(8, b"\0")
    for i in range(8):
        m.fill_value[i] = fb[i]
    ch = m.chain
    ch.sharded = 1 if sharded else 0
    if sharded:
        for d in range(n):
            ch.inner_chunk_shape[d] = int(inner_chunk_shape[d])
    if transpose_order is not None:
        ch.has_transpose = 1
        for d in range(n):
            ch.transpose_order[d] = int(transpose_order[d])
    ch.endian = endian
    ch.index_endian = index_endian
    ch.index_has_crc32c = 1 if index_crc32c else 0
    ch.index_location = index_location
    ch.inner_crc32c = 1 if inner_crc32c else 0
    if nested_chunk_shape is not None:
        ch.nested = 1
        for d in range(n):
            ch.nested_chunk_shape[d] = int(nested_chunk_shape[d])
        ch.nested_index_endian = nested_index_endian
        ch.nested_index_has_crc32c = 1 if nested_index_crc32c else 0
        ch.nested_index_location = nested_index_location
    return m
