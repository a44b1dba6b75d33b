"""Codec model, registry and builder mirroring zarr-java's v3 codec surface.

  Codec JSON polymorphism       M/v3/codec/Codec.java:7-9 (name + configuration)
  CodecRegistry.addType         M/v3/codec/CodecRegistry.java:11-34 (the plug-in point)
  CodecBuilder                  M/v3/codec/CodecBuilder.java:62-176
  CodecPipeline validation      M/core/codec/CodecPipeline.java:18-57

The objects are host-side descriptions; `device_chain` maps a codec list onto the
zh_codec_chain the HIP path executes (bytes/transpose/sharding/crc32c-index).  Byte-to-
byte compressors (gzip, blosc, zstd, inner crc32c) stay on the host (north star): they
are applied by `host_bb_decode` before the bytes reach the device.
"""
import gzip as _gzip
import struct
import zlib

from . import _abi as A
from .errors import UnsupportedChainError, ZarrException


class Codec:
    name = None
    kind = None  # "aa" (array→array), "ab" (array→bytes), "bb" (bytes→bytes)

    def to_json(self):
        raise NotImplementedError

    @classmethod
    def from_json(cls, cfg, registry):
        raise NotImplementedError

    def __eq__(self, other):
        return type(self) is type(other) and self.to_json() == other.to_json()

    def __repr__(self):
        return f"{type(self).__name__}({self.to_json()})"


class BytesCodec(Codec):
    """v3 BytesCodec (M/v3/codec/core/BytesCodec.java): endian None = no configuration."""
    name, kind = "bytes", "ab"

    def __init__(self, endian="little"):
        if endian is not None:
            endian = str(getattr(endian, "value", endian)).lower()
            if endian not in ("little", "big"):
                raise ZarrException(f"Invalid endian '{endian}'")
        self.endian = endian

    def byte_order(self, dtype_size):
        if dtype_size <= 1:  # core BytesCodec.decode :16-18 (Q9)
            return A.ZH_ENDIAN_BIG
        if self.endian is None:  # v3 BytesCodec.getByteOrder :43-48 (Q11)
            raise ZarrException("BytesCodec configuration is required to determine endianess.")
        return A.ZH_ENDIAN_BIG if self.endian == "big" else A.ZH_ENDIAN_LITTLE

    def to_json(self):
        if self.endian is None:
            return {"name": "bytes"}
        return {"name": "bytes", "configuration": {"endian": self.endian}}

    @classmethod
    def from_json(cls, cfg, registry):
        return cls((cfg or {}).get("endian", "little") if cfg is not None else None)


class TransposeCodec(Codec):
    """TransposeCodec (M/v3/codec/core/TransposeCodec.java:18-93)."""
    name, kind = "transpose", "aa"

    def __init__(self, order):
        self.order = [int(o) for o in order]

    def validate(self, ndim):
        o = self.order
        if not o or sorted(o) != list(range(len(o))):  # Utils.isPermutation :91-100
            raise ZarrException("Order is no permutation array")
        if len(o) != ndim:
            raise ZarrException("Array has not the same ndim as transpose codec order")

    def to_json(self):
        return {"name": "transpose", "configuration": {"order": list(self.order)}}

    @classmethod
    def from_json(cls, cfg, registry):
        return cls(cfg["order"])


class Crc32cCodec(Codec):
    """Crc32cCodec (M/v3/codec/core/Crc32cCodec.java:24-60)."""
    name, kind = "crc32c", "bb"

    def decode(self, b):
        from ._lib import lib
        body, stored = b[:-4], struct.unpack("<i", b[-4:])[0]
        computed = struct.unpack("<i", struct.pack("<I", lib().zh_crc32c(0, body, len(body))))[0]
        if computed != stored:
            raise ZarrException("The checksum of the sharding index is invalid. Stored: %d "
                                "Computed: %d" % (stored, computed))
        return body

    def encode(self, b):
        from ._lib import lib
        return bytes(b) + struct.pack("<I", lib().zh_crc32c(0, bytes(b), len(b)))

    def to_json(self):
        return {"name": "crc32c"}

    @classmethod
    def from_json(cls, cfg, registry):
        return cls()


class GzipCodec(Codec):
    """GzipCodec (M/v3/codec/core/GzipCodec.java:35-46) — host only."""
    name, kind = "gzip", "bb"

    def __init__(self, level=5):
        if not 0 <= int(level) <= 9:
            raise ZarrException("'level' needs to be between 0 and 9.")
        self.level = int(level)

    def decode(self, b):
        return zlib.decompress(bytes(b), 31)

    def encode(self, b):
        return _gzip.compress(bytes(b), compresslevel=self.level, mtime=0)

    def to_json(self):
        return {"name": "gzip", "configuration": {"level": self.level}}

    @classmethod
    def from_json(cls, cfg, registry):
        return cls((cfg or {}).get("level", 5))


class BloscCodec(Codec):
    """BloscCodec (M/v3/codec/core/BloscCodec.java) — host only.  Without the blosc
    library only MEMCPYED frames (flags & 0x02: raw bytes after the 16-byte header) can be
    decoded; other frames raise UnsupportedChainError."""
    name, kind = "blosc", "bb"

    def __init__(self, cname="zstd", clevel=5, shuffle="noshuffle", typesize=None, blocksize=0):
        self.cfg = {"typesize": typesize, "cname": cname, "clevel": clevel, "shuffle": shuffle,
                    "blocksize": blocksize}

    def decode(self, b):
        b = bytes(b)
        if len(b) < 16:
            raise ZarrException("blosc frame too short")
        flags = b[2]
        nbytes = struct.unpack("<I", b[4:8])[0]
        if flags & 0x02:
            return b[16:16 + nbytes]
        raise UnsupportedChainError("blosc frames other than MEMCPYED need the host blosc "
                                    "library, which is not available here")

    def encode(self, b):
        b = bytes(b)
        ts = self.cfg.get("typesize") or 1
        hdr = struct.pack("<BBBBIII", 2, 1, 0x02 | 0x01, ts, len(b), len(b), len(b) + 16)
        return hdr + b

    def to_json(self):
        return {"name": "blosc", "configuration": dict(self.cfg)}

    @classmethod
    def from_json(cls, cfg, registry):
        cfg = cfg or {}
        return cls(cfg.get("cname", "zstd"), cfg.get("clevel", 5), cfg.get("shuffle", "noshuffle"),
                   cfg.get("typesize"), cfg.get("blocksize", 0))


class ZstdCodec(Codec):
    """ZstdCodec — host only; no zstd library in this image."""
    name, kind = "zstd", "bb"

    def __init__(self, level=5, checksum=True):
        self.level, self.checksum = level, checksum

    def decode(self, b):
        raise UnsupportedChainError("zstd needs the host zstd library (not available here)")

    encode = decode

    def to_json(self):
        return {"name": "zstd", "configuration": {"level": self.level, "checksum": self.checksum}}

    @classmethod
    def from_json(cls, cfg, registry):
        cfg = cfg or {}
        return cls(cfg.get("level", 5), cfg.get("checksum", True))


class ShardingIndexedCodec(Codec):
    """ShardingIndexedCodec.Configuration (ShardingIndexedCodec.java:267-299)."""
    name, kind = "sharding_indexed", "ab"

    def __init__(self, chunk_shape, codecs=None, index_codecs=None, index_location="end"):
        if index_location is None:
            index_location = "end"
        if index_location not in ("start", "end"):
            raise ZarrException('Only index_location "start" or "end" are supported.')
        self.chunk_shape = [int(c) for c in chunk_shape]
        self.codecs = list(codecs) if codecs is not None else [BytesCodec("little")]
        self.index_codecs = list(index_codecs) if index_codecs is not None else \
            [BytesCodec("little"), Crc32cCodec()]
        self.index_location = index_location

    def to_json(self):
        return {"name": "sharding_indexed", "configuration": {
            "chunk_shape": list(self.chunk_shape),
            "codecs": [c.to_json() for c in self.codecs],
            "index_codecs": [c.to_json() for c in self.index_codecs],
            "index_location": self.index_location}}

    @classmethod
    def from_json(cls, cfg, registry):
        return cls(cfg["chunk_shape"], [registry.codec_from_json(c) for c in cfg["codecs"]],
                   [registry.codec_from_json(c) for c in cfg["index_codecs"]],
                   cfg.get("index_location", "end"))


class CodecRegistry:
    """CodecRegistry (M/v3/codec/CodecRegistry.java:9-35): name → class.  addType replaces
    an existing entry — the hook the device codec uses in the Java integration."""
    map = {}

    @classmethod
    def addType(cls, name, codec_cls):
        cls.map[name] = codec_cls

    @classmethod
    def getNamedTypes(cls):
        return dict(cls.map)

    @classmethod
    def codec_from_json(cls, j):
        name = j.get("name")
        if name not in cls.map:
            raise ZarrException(f"Unknown codec '{name}'")
        return cls.map[name].from_json(j.get("configuration"), cls)


for _c in (TransposeCodec, BytesCodec, BloscCodec, GzipCodec, ZstdCodec, Crc32cCodec,
           ShardingIndexedCodec):
    CodecRegistry.addType(_c.name, _c)


class CodecBuilder:
    """CodecBuilder (M/v3/codec/CodecBuilder.java)."""

    def __init__(self, data_type):
        self.data_type = data_type
        self.codecs = []

    def withTranspose(self, order):
        self.codecs.append(TransposeCodec(order))
        return self

    def withBytes(self, endian="LITTLE"):
        if self.data_type.getByteCount() <= 1:  # :76-82
            self.codecs.append(BytesCodec(None))
        else:
            self.codecs.append(BytesCodec(str(getattr(endian, "value", endian)).lower()))
        return self

    def withGzip(self, level=5):
        self.codecs.append(GzipCodec(level))
        return self

    def withBlosc(self, cname="zstd", shuffle="noshuffle", clevel=5):
        self.codecs.append(BloscCodec(cname, clevel, shuffle, self.data_type.getByteCount(), 0))
        return self

    def withZstd(self, level=5, checksum=True):
        self.codecs.append(ZstdCodec(level, checksum))
        return self

    def withCrc32c(self):
        self.codecs.append(Crc32cCodec())
        return self

    def withSharding(self, chunk_shape, codec_builder=None, index_location="end"):
        """:122-153 — the short form uses inner [bytes LE] and index [bytes LE, crc32c]."""
        if codec_builder is None:
            inner = [BytesCodec("little")]
        else:
            inner = codec_builder(CodecBuilder(self.data_type)).build()
        self.codecs.append(ShardingIndexedCodec(chunk_shape, inner,
                                                [BytesCodec("little"), Crc32cCodec()],
                                                index_location))
        return self

    def build(self):
        """autoInsertBytesCodec (:160-176)."""
        if not any(c.kind == "ab" for c in self.codecs):
            aa = [c for c in self.codecs if c.kind == "aa"]
            bb = [c for c in self.codecs if c.kind == "bb"]
            self.codecs = aa + [BytesCodec("little")] + bb
        return list(self.codecs)


def validate_pipeline(codecs):
    """CodecPipeline constructor checks (M/core/codec/CodecPipeline.java:18-57)."""
    n_ab = sum(1 for c in codecs if c.kind == "ab")
    if n_ab != 1:
        raise ZarrException(f"Exactly 1 ArrayBytesCodec is required. Found {n_ab}.")
    prev = None
    for c in codecs:
        if prev is not None:
            if c.kind == "ab" and prev.kind == "bb":
                raise ZarrException(f"ArrayBytesCodec '{type(c).__name__}' cannot follow after "
                                    f"BytesBytesCodec '{type(prev).__name__}'.")
            if c.kind == "aa" and prev.kind == "ab":
                raise ZarrException(f"ArrayArrayCodec '{type(c).__name__}' cannot follow after "
                                    f"ArrayBytesCodec '{type(prev).__name__}'.")
            if c.kind == "aa" and prev.kind == "bb":
                raise ZarrException(f"ArrayArrayCodec '{type(c).__name__}' cannot follow after "
                                    f"BytesBytesCodec '{type(prev).__name__}'.")
        prev = c


class DeviceChain:
    """How a codec list runs: the zh_codec_chain for the device plus the host byte-to-byte
    stages that wrap it (applied outermost-last on decode, like CodecPipeline.decode)."""

    def __init__(self, chain, host_bb, inner_host_bb, index_codecs=None):
        self.chain = chain                   # zh_codec_chain fields (dict)
        self.host_bb = host_bb               # BB codecs around whole chunks (unsharded)
        self.inner_host_bb = inner_host_bb   # BB codecs around inner chunks (sharded)
        self.index_codecs = index_codecs


def _split_inner(codecs, ndim, dsize):
    validate_pipeline(codecs)
    aa = [c for c in codecs if c.kind == "aa"]
    ab = [c for c in codecs if c.kind == "ab"][0]
    bb = [c for c in codecs if c.kind == "bb"]
    if len(aa) > 1 or any(not isinstance(c, TransposeCodec) for c in aa):
        raise UnsupportedChainError("only a single transpose array→array codec is device-supported")
    if not isinstance(ab, BytesCodec):
        raise UnsupportedChainError("only bytes (or one nested sharding level) is device-supported")
    order = None
    if aa:
        aa[0].validate(ndim)
        order = aa[0].order
    return order, ab.byte_order(dsize), bb


def _take_crc(bb):
    """A trailing-only [crc32c] byte-to-byte chain runs on the device (zh_codec_chain
    .inner_crc32c); anything else stays a host byte-to-byte stage."""
    if len(bb) == 1 and isinstance(bb[0], Crc32cCodec):
        return [], True
    return bb, False


def _index_chain(sh):
    ic = sh.index_codecs
    if not ic or not isinstance(ic[0], BytesCodec) or \
            any(not isinstance(c, Crc32cCodec) for c in ic[1:]) or len(ic) > 2:
        raise UnsupportedChainError("index codecs must be [bytes, crc32c?]")
    return ic


def device_chain(codecs, ndim, dsize):
    """Map a v3 codec list onto the device path (raises UnsupportedChainError otherwise)."""
    validate_pipeline(codecs)
    ab = [c for c in codecs if c.kind == "ab"][0]
    if isinstance(ab, ShardingIndexedCodec):
        if len(codecs) != 1:
            # array-level codecs next to sharding disable partial decode
            # (CodecPipeline.supportsPartialDecode :82-84)
            raise UnsupportedChainError("sharding_indexed must be the only array-level codec")
        ic = _index_chain(ab)
        nested = None
        validate_pipeline(ab.codecs)
        inner_ab = [c for c in ab.codecs if c.kind == "ab"][0]
        if isinstance(inner_ab, ShardingIndexedCodec):
            # nested sharding (ZarrPythonTests.java:177-179): the inner pipeline is exactly
            # [sharding_indexed{...}] whose own inner pipeline is [transpose?, bytes]
            if len(ab.codecs) != 1:
                raise UnsupportedChainError("nested sharding must be the only inner codec")
            nested = inner_ab
            order, endian, inner_bb = _split_inner(nested.codecs, ndim, dsize)
            inner_bb, crc = _take_crc(inner_bb)
            if inner_bb:
                raise UnsupportedChainError("nested sharding with byte-to-byte leaf codecs")
        else:
            order, endian, inner_bb = _split_inner(ab.codecs, ndim, dsize)
            inner_bb, crc = _take_crc(inner_bb)
        chain = dict(sharded=True, inner_chunk_shape=ab.chunk_shape, transpose_order=order,
                     endian=endian, inner_crc32c=crc, index_endian=ic[0].byte_order(8),
                     index_crc32c=len(ic) == 2,
                     index_location=A.ZH_INDEX_START if ab.index_location == "start"
                     else A.ZH_INDEX_END)
        if nested is not None:
            nic = _index_chain(nested)
            chain.update(nested_chunk_shape=nested.chunk_shape,
                         nested_index_endian=nic[0].byte_order(8),
                         nested_index_crc32c=len(nic) == 2,
                         nested_index_location=A.ZH_INDEX_START
                         if nested.index_location == "start" else A.ZH_INDEX_END)
        return DeviceChain(chain, [], inner_bb, ic)
    order, endian, bb = _split_inner(codecs, ndim, dsize)
    bb, crc = _take_crc(bb)
    chain = dict(sharded=False, transpose_order=order, endian=endian, inner_crc32c=crc)
    return DeviceChain(chain, bb, [])


def host_bb_decode(bb_codecs, b):
    for c in reversed(bb_codecs):
        b = c.decode(b)
    return b


def host_bb_encode(bb_codecs, b):
    for c in bb_codecs:
        b = c.encode(b)
    return b
