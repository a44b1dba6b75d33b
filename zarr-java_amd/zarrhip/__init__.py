"""zarrhip — MI355X-native Zarr v3 chunk codec path (sharding + bytes + transpose +
region scatter on the GPU) behind a host mirror of zarr-java's v3 read/write surface.

The device work goes through libzarrhip.so's C-ABI (include/zarrhip.h); there is no CPU
compute fallback in this package.
"""
from .array import Array, ArrayAccessor, device
from .codecs import (BloscCodec, BytesCodec, CodecBuilder, CodecRegistry, Crc32cCodec, GzipCodec,
                     ReshapeCodec,
                     ShardingIndexedCodec, TransposeCodec, ZstdCodec, device_chain)
from .dtypes import DataType
from .errors import UnsupportedChainError, ZarrException
from .metadata import ArrayMetadata, ArrayMetadataBuilder, ChunkKeyEncoding, parse_fill_value
from .store import FilesystemStore, HttpStore, MemoryStore, StoreException, StoreHandle

__all__ = ["Array", "ArrayAccessor", "ArrayMetadata", "ArrayMetadataBuilder", "BloscCodec",
           "ReshapeCodec",
           "BytesCodec", "ChunkKeyEncoding", "CodecBuilder", "CodecRegistry", "Crc32cCodec",
           "DataType", "FilesystemStore", "GzipCodec", "HttpStore", "MemoryStore",
           "ShardingIndexedCodec", "StoreException",
           "StoreHandle", "TransposeCodec", "UnsupportedChainError", "ZarrException",
           "ZstdCodec", "device", "device_chain", "parse_fill_value"]
