"""Zarr v2 arrays (M/v2/): `.zarray` metadata, the v2 dtypes with their byte order, the
zlib/blosc/zstd compressors and the v2 chunk keys, on the same device chunk path as v3.

The reference builds a v2 array's pipeline as `filters + bytes(dtype endianness) +
compressor` (M/v2/Array.java:34-43): the device runs the `bytes` stage (endian swap +
scatter), the compressor stays on the host.  `order` is metadata only there — the pipeline
never transposes an "F" array — and it is reproduced as such.
"""
import enum
import json
import zlib

from . import array as _array
from .codecs import BloscCodec as _Blosc3, BytesCodec, Codec, ZstdCodec as _Zstd3, validate_pipeline
from .dtypes import DataType as _DT3
from .errors import ZarrException
from .metadata import ChunkKeyEncoding, calculate_default_chunks, fill_value_to_json, \
    parse_fill_value, zh_meta_for

ZARRAY = ".zarray"


class DataType(enum.Enum):
    """M/v2/DataType.java:5-87: dtype code, byte order ("<", ">", "|"), v3 core type."""
    BOOL = ("b1", "|", _DT3.BOOL)
    INT8 = ("i1", "|", _DT3.INT8)
    INT16 = ("i2", "<", _DT3.INT16)
    INT32 = ("i4", "<", _DT3.INT32)
    INT64 = ("i8", "<", _DT3.INT64)
    UINT8 = ("u1", "|", _DT3.UINT8)
    UINT16 = ("u2", "<", _DT3.UINT16)
    UINT32 = ("u4", "<", _DT3.UINT32)
    UINT64 = ("u8", "<", _DT3.UINT64)
    FLOAT32 = ("f4", "<", _DT3.FLOAT32)
    FLOAT64 = ("f8", "<", _DT3.FLOAT64)
    INT16_BE = ("i2", ">", _DT3.INT16)
    INT32_BE = ("i4", ">", _DT3.INT32)
    INT64_BE = ("i8", ">", _DT3.INT64)
    UINT16_BE = ("u2", ">", _DT3.UINT16)
    UINT32_BE = ("u4", ">", _DT3.UINT32)
    UINT64_BE = ("u8", ">", _DT3.UINT64)
    FLOAT32_BE = ("f4", ">", _DT3.FLOAT32)
    FLOAT64_BE = ("f8", ">", _DT3.FLOAT64)

    @property
    def value_name(self):          # getValue(): "<u4", "|b1", ">f8" ...
        return self.value[1] + self.value[0]

    @property
    def core(self):
        return self.value[2]

    @property
    def endian(self):              # Endianness.toEndian: unspecified → little
        return "big" if self.value[1] == ">" else "little"

    def getByteCount(self):
        return int(self.value[0][1:])

    @property
    def numpy(self):               # decoded elements, host order (as ucar holds them)
        return self.core.numpy

    @classmethod
    def of(cls, s):
        # numpy writes "<u1" / ">i1" for 1-byte types; the byte order is immaterial there
        if len(s) == 3 and s[2] == "1" and s[0] in "<>":
            s = "|" + s[1:]
        for d in cls:
            if d.value_name == s:
                return d
        raise ZarrException(f"Unsupported v2 dtype '{s}'.")


class ZlibCodec(Codec):
    """M/v2/codec/core/ZlibCodec.java: level 0..9 (default 1), zlib stream."""
    name, kind = "zlib", "bb"

    def __init__(self, level=1):
        if level < 0 or level > 9:
            raise ZarrException("'level' needs to be between 0 and 9.")
        self.level = int(level)

    def decode(self, b):
        try:
            return zlib.decompress(bytes(b))
        except zlib.error as e:
            raise ZarrException("Error in decoding gzip.") from e

    def encode(self, b):
        return zlib.compress(bytes(b), self.level)

    def to_json(self):
        return {"id": "zlib", "level": self.level}


class BloscCodec(_Blosc3):
    """M/v2/codec/core/BloscCodec.java: clevel 0..9; shuffle serialised as its ordinal;
    typesize 0 → the dtype's byte count (evolveFromCoreArrayMetadata :75-86)."""
    SHUFFLES = ["noshuffle", "shuffle", "bitshuffle"]

    def __init__(self, cname="zstd", clevel=5, shuffle="noshuffle", typesize=0, blocksize=0):
        if clevel < 0 or clevel > 9:
            raise ZarrException("'clevel' needs to be between 0 and 9.")
        if isinstance(shuffle, int):
            shuffle = self.SHUFFLES[shuffle]
        super().__init__(cname, clevel, shuffle, typesize, blocksize)

    def to_json(self):
        c = self.cfg
        return {"id": "blosc", "cname": c["cname"], "clevel": c["clevel"],
                "shuffle": self.SHUFFLES.index(c["shuffle"]), "typesize": c["typesize"] or 0,
                "blocksize": c["blocksize"]}


class ZstdCodec(_Zstd3):
    def to_json(self):
        return {"id": "zstd", "level": self.level, "checksum": self.checksum}


def codec_from_json(j):
    """v2 CodecRegistry (M/v2/codec/CodecRegistry.java:16-18): by "id"."""
    if j is None:
        return None
    cid = j.get("id")
    if cid == "zlib":
        return ZlibCodec(j.get("level", 1))
    if cid == "blosc":
        return BloscCodec(j.get("cname", "zstd"), j.get("clevel", 5), j.get("shuffle", 0),
                          j.get("typesize", 0), j.get("blocksize", 0))
    if cid == "zstd":
        return ZstdCodec(j.get("level", 5), j.get("checksum", False))
    raise ZarrException(f"Unknown v2 codec '{cid}'")


class ArrayMetadata:
    """M/v2/ArrayMetadata.java:50-110."""

    def __init__(self, shape, chunks, dtype, fill_value=None, order="C", filters=None,
                 compressor=None, dimension_separator=".", attributes=None, zarr_format=2):
        if zarr_format != 2:
            raise ZarrException(f"Expected zarr format '2', got '{zarr_format}'.")
        self.shape = [int(s) for s in shape]
        self.chunk_shape = [int(c) for c in chunks]
        if len(self.shape) != len(self.chunk_shape):
            raise ZarrException("Shape and chunks need to have the same number of dimensions.")
        self.data_type = dtype if isinstance(dtype, DataType) else DataType.of(dtype)
        if order not in ("C", "F"):
            raise ZarrException(f"Invalid order '{order}'.")
        self.order = order
        self.fill_value = fill_value
        self.fill_bytes = parse_fill_value(fill_value, self.data_type.core)
        self.filters = list(filters) if filters else None
        self.compressor = compressor
        if isinstance(self.compressor, BloscCodec) and not self.compressor.cfg["typesize"]:
            self.compressor.cfg["typesize"] = self.data_type.getByteCount()
        self.dimension_separator = dimension_separator or "."
        self.chunk_key_encoding = ChunkKeyEncoding("v2", self.dimension_separator)
        self.attributes = dict(attributes or {})

    @property
    def ndim(self):
        return len(self.shape)

    @property
    def codecs(self):
        """The pipeline the reference builds (M/v2/Array.java:34-43)."""
        cs = list(self.filters or []) + [BytesCodec(self.data_type.endian)]
        if self.compressor is not None:
            cs.append(self.compressor)
        validate_pipeline(cs)
        return cs

    def to_zh_meta(self, device_chain):
        return zh_meta_for(self, device_chain, self.data_type == DataType.BOOL)

    def to_json(self):
        fill = None if self.fill_value is None else \
            fill_value_to_json(self.fill_bytes, self.data_type.core)
        return {"zarr_format": 2, "shape": self.shape, "chunks": self.chunk_shape,
                "dtype": self.data_type.value_name, "fill_value": fill, "order": self.order,
                "filters": None if not self.filters else [f.to_json() for f in self.filters],
                "dimension_separator": self.dimension_separator,
                "compressor": None if self.compressor is None else self.compressor.to_json()}

    def dumps(self):
        return json.dumps(self.to_json(), indent=2)

    @classmethod
    def from_json(cls, j):
        return cls(j["shape"], j["chunks"], DataType.of(j["dtype"]), j.get("fill_value"),
                   j.get("order", "C"), [codec_from_json(f) for f in (j.get("filters") or [])],
                   codec_from_json(j.get("compressor")), j.get("dimension_separator", "."),
                   zarr_format=j.get("zarr_format"))


class ArrayMetadataBuilder:
    """M/v2/ArrayMetadataBuilder.java: order C, separator ".", no fill, no compressor."""

    def __init__(self):
        self.shape = self.chunks = self.dtype = None
        self.order, self.sep, self.fill, self.compressor = "C", ".", None, None

    def withShape(self, *shape):
        self.shape = list(shape[0]) if len(shape) == 1 and isinstance(shape[0], (list, tuple)) \
            else list(shape)
        return self

    def withChunks(self, *chunks):
        self.chunks = list(chunks[0]) if len(chunks) == 1 and isinstance(chunks[0], (list, tuple)) \
            else list(chunks)
        return self

    def withDataType(self, dt):
        self.dtype = dt
        return self

    def withOrder(self, order):
        self.order = order
        return self

    def withDimensionSeparator(self, sep):
        self.sep = sep
        return self

    def withFillValue(self, fill):
        self.fill = fill
        return self

    def withCompressor(self, c):
        self.compressor = c
        return self

    def withBloscCompressor(self, cname="zstd", shuffle="noshuffle", clevel=5, blocksize=0):
        self.compressor = BloscCodec(cname, clevel, shuffle, self.dtype.getByteCount(), blocksize)
        return self

    def withZlibCompressor(self, level=5):
        self.compressor = ZlibCodec(level)
        return self

    def withZstdCompressor(self, level=5, checksum=False):
        self.compressor = ZstdCodec(level, checksum)
        return self

    def build(self):
        if self.shape is None:
            raise ValueError("Please call `withShape` first.")
        if self.dtype is None:
            raise ValueError("Please call `withDataType` first.")
        chunks = self.chunks if self.chunks is not None else calculate_default_chunks(self.shape)
        return ArrayMetadata(self.shape, chunks, self.dtype, self.fill, self.order, None,
                             self.compressor, self.sep)


class Array(_array.Array):
    """M/v2/Array.java: open/create at `.zarray`; read/write/readChunk are core.Array's,
    through the same device path as v3 arrays."""
    META_FILE = ZARRAY
    METADATA = ArrayMetadata

    @staticmethod
    def metadataBuilder():
        return ArrayMetadataBuilder()
