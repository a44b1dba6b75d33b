"""v3 array metadata (zarr.json) — host-side, mirrors M/v3/ArrayMetadata.java,
ArrayMetadataBuilder.java, the chunk key encodings and core parseFillValue."""
import json
import math
import struct

from . import _abi as A
from .codecs import BytesCodec, CodecBuilder, CodecRegistry, ShardingIndexedCodec
from .dtypes import DataType
from .errors import ZarrException

ZARR_JSON = "zarr.json"


def parse_fill_value(fill, dtype):
    """core ArrayMetadata.parseFillValue (M/core/ArrayMetadata.java:32-135) → the element's
    bytes, little-endian (as the ucar array holds them).  None → no fill (zeros)."""
    ds = dtype.getByteCount()
    if fill is None:
        return bytes(ds)
    isfloat = dtype in (DataType.FLOAT32, DataType.FLOAT64)
    fmt = {DataType.FLOAT32: "<f", DataType.FLOAT64: "<d"}.get(dtype)
    if isinstance(fill, bool):
        if dtype == DataType.BOOL:
            return bytes([1 if fill else 0])
        raise ZarrException(f"Invalid fill value '{fill}'.")
    if isinstance(fill, (int, float)):
        if dtype == DataType.BOOL:
            return bytes([1 if int(fill) & 0xFF else 0])  # byteValue() != 0
        if isfloat:
            return struct.pack(fmt, float(fill))
        v = int(fill) & ((1 << (8 * ds)) - 1)  # Java narrowing (intValue / longValue ...)
        return v.to_bytes(ds, "little")
    if isinstance(fill, str):
        specials = {"NaN": math.nan, "+Infinity": math.inf, "Infinity": math.inf,
                    "-Infinity": -math.inf}
        if fill in specials:
            if isfloat:
                return struct.pack(fmt, specials[fill])
            raise ZarrException(f"Invalid fill value '{fill}' for data type '{dtype.value_name}'.")
        if fill.startswith("0x") or fill.startswith("0b"):
            base, w = (16, 2) if fill.startswith("0x") else (2, 8)
            # Utils.makeByteBuffer: bytes put in string order into a little-endian buffer
            return bytes(int(fill[2 + i * w:2 + (i + 1) * w], base) for i in range(ds))
    raise ZarrException(f"Invalid fill value '{fill}'.")


def fill_value_to_json(fill_bytes, dtype):
    if dtype == DataType.BOOL:
        return bool(fill_bytes[0])
    if dtype == DataType.FLOAT32:
        v = struct.unpack("<f", fill_bytes[:4])[0]
    elif dtype == DataType.FLOAT64:
        v = struct.unpack("<d", fill_bytes[:8])[0]
    else:
        signed = dtype.value_name.startswith("int")
        return int.from_bytes(fill_bytes[:dtype.getByteCount()], "little", signed=signed)
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Infinity" if v > 0 else "-Infinity"
    return v


class ChunkKeyEncoding:
    """DefaultChunkKeyEncoding (:33-40) / V2ChunkKeyEncoding."""

    def __init__(self, name="default", separator=None):
        self.name = name
        self.separator = separator if separator is not None else ("/" if name == "default" else ".")

    def encode_chunk_key(self, coords):
        parts = ([] if self.name == "v2" else ["c"]) + [str(int(c)) for c in coords]
        if self.name == "v2" and not coords:
            parts = ["0"]
        if self.separator == "/":
            return parts
        return [self.separator.join(parts)]

    def to_json(self):
        return {"name": self.name, "configuration": {"separator": self.separator}}

    @classmethod
    def from_json(cls, j):
        return cls(j.get("name", "default"), (j.get("configuration") or {}).get("separator"))


class ArrayMetadata:
    """v3 ArrayMetadata; the constructor applies the reference's validation
    (M/v3/ArrayMetadata.java:90-125: rank match, sharding divisibility)."""

    def __init__(self, shape, data_type, chunk_shape, chunk_key_encoding=None, fill_value=0,
                 codecs=None, dimension_names=None, attributes=None):
        self.shape = [int(s) for s in shape]
        self.data_type = data_type if isinstance(data_type, DataType) else DataType.of(data_type)
        self.chunk_shape = [int(c) for c in chunk_shape]
        self.chunk_key_encoding = chunk_key_encoding or ChunkKeyEncoding()
        self.fill_value = fill_value
        self.codecs = list(codecs) if codecs else [BytesCodec("little")]
        self.dimension_names = dimension_names
        self.attributes = dict(attributes or {})
        if len(self.shape) != len(self.chunk_shape):
            raise ZarrException(
                f"Shape (ndim={len(self.shape)}) and chunk grid shape (ndim="
                f"{len(self.chunk_shape)}) need to have the same number of dimensions.")
        outer = self.chunk_shape
        sh = next((c for c in self.codecs if isinstance(c, ShardingIndexedCodec)), None)
        while sh is not None:
            inner = sh.chunk_shape
            if len(inner) != len(outer):
                raise ZarrException(f"Sharding dimensions mismatch of outer chunk shape "
                                    f"{_jarr(outer)} and inner chunk shape{_jarr(inner)}")
            for o, i in zip(outer, inner):
                if i <= 0 or o % i != 0:
                    raise ZarrException(f"Sharding inner chunk shape {_jarr(inner)} does not "
                                        f"evenly divide the outer chunk size {_jarr(outer)}")
            outer = inner
            sh = next((c for c in sh.codecs if isinstance(c, ShardingIndexedCodec)), None)
        self.fill_bytes = parse_fill_value(fill_value, self.data_type)

    @property
    def ndim(self):
        return len(self.shape)

    def to_json(self):
        j = {"zarr_format": 3, "node_type": "array", "shape": self.shape,
             "data_type": self.data_type.value_name,
             "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": self.chunk_shape}},
             "chunk_key_encoding": self.chunk_key_encoding.to_json(),
             "fill_value": fill_value_to_json(self.fill_bytes, self.data_type),
             "codecs": [c.to_json() for c in self.codecs], "attributes": self.attributes}
        if self.dimension_names is not None:
            j["dimension_names"] = list(self.dimension_names)
        return j

    def dumps(self):
        return json.dumps(self.to_json(), indent=2)

    @classmethod
    def from_json(cls, j):
        if j.get("zarr_format") != 3 or j.get("node_type", "array") != "array":
            raise ZarrException("not a zarr v3 array")
        grid = j["chunk_grid"]
        if grid.get("name") != "regular":
            raise ZarrException(f"Unsupported chunk grid '{grid.get('name')}'")
        return cls(j["shape"], DataType.of(j["data_type"]), grid["configuration"]["chunk_shape"],
                   ChunkKeyEncoding.from_json(j.get("chunk_key_encoding") or {}),
                   j.get("fill_value"), [CodecRegistry.codec_from_json(c) for c in j["codecs"]],
                   j.get("dimension_names"), j.get("attributes"))

    def to_zh_meta(self, device_chain):
        """zh_array_meta for the C-ABI."""
        return zh_meta_for(self, device_chain, self.data_type == DataType.BOOL)


def zh_meta_for(md, device_chain, is_bool):
    """zh_array_meta of an array's metadata (v3 or v2) and its device chain."""
    ch = device_chain.chain
    core = getattr(md.data_type, "core", md.data_type)  # v2: its v3 core type
    return A.make_meta(md.shape, md.chunk_shape, md.data_type.getByteCount(),
                       fill=md.fill_bytes, is_bool=is_bool,
                       is_float=core in (DataType.FLOAT32, DataType.FLOAT64),
                       sharded=ch["sharded"], inner_chunk_shape=ch.get("inner_chunk_shape"),
                       transpose_order=ch["transpose_order"], endian=ch["endian"],
                       index_endian=ch.get("index_endian", A.ZH_ENDIAN_LITTLE),
                       index_crc32c=ch.get("index_crc32c", False),
                       index_location=ch.get("index_location", A.ZH_INDEX_END),
                       nested_chunk_shape=ch.get("nested_chunk_shape"),
                       nested_index_endian=ch.get("nested_index_endian", A.ZH_ENDIAN_LITTLE),
                       nested_index_crc32c=ch.get("nested_index_crc32c", True),
                       nested_index_location=ch.get("nested_index_location", A.ZH_INDEX_END),
                       inner_crc32c=ch.get("inner_crc32c", False))


def calculate_default_chunks(shape):
    """Utils.calculateDefaultChunks (M/utils/Utils.java:125-143)."""
    chunks = []
    for s in shape:
        n = s // 512
        if n > 0:
            c = s // (n + 1)
            chunks.append(c if s % c == 0 else c + 1)
        else:
            chunks.append(int(s))
    return chunks


def _jarr(v):
    return "[" + ", ".join(str(x) for x in v) + "]"


class ArrayMetadataBuilder:
    """ArrayMetadataBuilder (M/v3/ArrayMetadataBuilder.java:20-200); defaults :26-33."""

    def __init__(self):
        self.shape = None
        self.data_type = None
        self.chunk_shape = None
        self.chunk_key_encoding = ChunkKeyEncoding("default", "/")
        self.fill_value = 0
        self.codecs = [BytesCodec("little")]
        self.dimension_names = None
        self.attributes = {}

    def withShape(self, *shape):
        self.shape = list(shape[0]) if len(shape) == 1 and hasattr(shape[0], "__len__") else list(shape)
        return self

    def withDataType(self, dt):
        self.data_type = dt if isinstance(dt, DataType) else DataType.of(dt)
        return self

    def withChunkShape(self, *cs):
        self.chunk_shape = list(cs[0]) if len(cs) == 1 and hasattr(cs[0], "__len__") else list(cs)
        return self

    def withDefaultChunkKeyEncoding(self, separator="/"):
        self.chunk_key_encoding = ChunkKeyEncoding("default", separator)
        return self

    def withV2ChunkKeyEncoding(self, separator="."):
        self.chunk_key_encoding = ChunkKeyEncoding("v2", separator)
        return self

    def withFillValue(self, fill):
        self.fill_value = fill
        return self

    def withCodecs(self, fn):
        self.codecs = fn(CodecBuilder(self.data_type)).build()
        return self

    def withDimensionNames(self, *names):
        self.dimension_names = list(names)
        return self

    def putAttribute(self, k, v):
        self.attributes[k] = v
        return self

    def build(self):
        if self.shape is None:
            raise ZarrException("Shape needs to be provided. Please call `.withShape`.")
        if self.data_type is None:
            raise ZarrException("Data type needs to be provided. Please call `.withDataType`.")
        chunk = self.chunk_shape or calculate_default_chunks(self.shape)
        return ArrayMetadata(self.shape, self.data_type, chunk, self.chunk_key_encoding,
                             self.fill_value, self.codecs, self.dimension_names, self.attributes)
