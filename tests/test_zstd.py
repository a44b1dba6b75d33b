"""Host zstd decoding (zh_zstd_decompress, zarr-java_amd/csrc/zh_zstd.cpp, RFC 8878 written
from the format specification) behind ZstdCodec.decode (M/core/codec/core/ZstdCodec.java:14-22).

Pinned two ways, with no zstd in the product's dependencies:
- the reference's own zstd fixtures (testdata/ome/v0.5/{0,1}, labels/nuclei/0, v0.5_hcs;
  tests/golden/ome_zstd/, copied as data): frame content size = the chunk's bytes, decoded
  float32/uint values are finite, and the two channel chunks of one image differ;
- libzstd itself (the library zstd-jni wraps, here the copy bundled with pyarrow) as an
  independent encoder: levels -5..22, every block and literal kind, sizes 0..1 MiB.
The XXH64 content checksum is pinned against the xxhash module."""
import ctypes as C
import json
import os
import struct

import numpy as np
import pytest

import zarrhip as z
from helpers import GOLDEN
from zarrhip._lib import lib
from zarrhip.codecs import ZstdCodec

pa = pytest.importorskip("pyarrow")
OME = os.path.join(GOLDEN, "ome_zstd")


def dec(b):
    return ZstdCodec().decode(b)


def libzstd(data, level):
    return pa.Codec("zstd", compression_level=level).compress(bytes(data), asbytes=True)


def _payloads(seed):
    rng = np.random.default_rng(seed)
    yield "empty", b""
    yield "one", b"\x07"
    yield "random", rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    yield "low_entropy", rng.integers(0, 4, 300000, dtype=np.uint8).tobytes()
    yield "ramp", (np.arange(200000) % 251).astype(np.uint8).tobytes()
    yield "float_walk", np.cumsum(rng.normal(size=90000)).astype("<f4").tobytes()
    yield "u32_be", rng.integers(0, 1 << 20, 50000, dtype=np.uint32).astype(">u4").tobytes()
    words = [b"zarr ", b"shard ", b"index ", b"crc32c ", b"transpose ", b"bytes "]
    yield "text", b"".join(words[i] for i in rng.integers(0, len(words), 60000))
    yield "zeros_1MiB", bytes(1 << 20)
    yield "block_edge", rng.integers(0, 3, (128 << 10) + 1, dtype=np.uint8).tobytes()


@pytest.mark.parametrize("level", [-5, -1, 1, 3, 6, 9, 15, 19, 22])
def test_libzstd_frames_roundtrip(level):
    for name, data in _payloads(level + 40):
        assert dec(libzstd(data, level)) == data, (name, level)


def test_concatenated_and_skippable_frames():
    a, b = b"first frame " * 100, bytes(range(256)) * 40
    skip = struct.pack("<II", 0x184D2A53, 5) + b"hello"
    assert dec(libzstd(a, 3) + skip + libzstd(b, 7)) == a + b


def _with_checksum(frame, content):
    """Set the content-checksum flag of a single-frame libzstd output and append XXH64."""
    import xxhash
    f = bytearray(frame)
    assert f[4] & 0x04 == 0
    f[4] |= 0x04
    return bytes(f) + struct.pack("<I", xxhash.xxh64(content).intdigest() & 0xFFFFFFFF)


def test_content_checksum_verified():
    data = np.arange(40000, dtype="<i4").tobytes()
    good = _with_checksum(libzstd(data, 5), data)
    assert dec(good) == data
    bad = bytearray(good)
    bad[-1] ^= 1
    with pytest.raises(z.ZarrException, match="checksum"):
        dec(bytes(bad))


def test_xxh64_matches_reference_hash():
    import xxhash
    rng = np.random.default_rng(3)
    for n in (0, 1, 3, 4, 7, 8, 31, 32, 33, 63, 64, 100, 1000, 4099):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for seed in (0, 1, 0xDEADBEEF):
            assert lib().zh_xxh64(b, n, seed) == xxhash.xxh64(b, seed=seed).intdigest()


@pytest.mark.parametrize("checksum", [True, False])
def test_encoder_frames_readable_by_libzstd(checksum):
    """ZstdCodec.encode writes raw-block frames; libzstd must read them back."""
    rng = np.random.default_rng(5)
    for n in (0, 1, 1000, (128 << 10), (128 << 10) + 5, 300000):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        f = ZstdCodec(5, checksum).encode(data)
        assert pa.Codec("zstd").decompress(f, decompressed_size=n, asbytes=True) == data
        assert dec(f) == data


def test_ome_fixtures_decode():
    """The reference's zstd chunks (OME-Zarr v0.5 samples; codecs [bytes little, zstd])."""
    seen = {}
    for root, _, files in os.walk(OME):
        if "zarr.json" not in files:
            continue
        meta = json.load(open(os.path.join(root, "zarr.json")))
        if meta.get("node_type") != "array":
            continue
        names = [c["name"] for c in meta["codecs"]]
        assert names == ["bytes", "zstd"], names
        dt = {"float32": "<f4", "uint8": "u1", "uint16": "<u2", "int32": "<i4",
              "uint32": "<u4", "int64": "<i8", "float64": "<f8"}[meta["data_type"]]
        cs = meta["chunk_grid"]["configuration"]["chunk_shape"]
        want = int(np.prod(cs)) * np.dtype(dt).itemsize
        for r2, _, fs in os.walk(os.path.join(root, "c")):
            for f in fs:
                raw = open(os.path.join(r2, f), "rb").read()
                assert raw[:4] == b"\x28\xb5\x2f\xfd"
                out = dec(raw)
                assert len(out) == want
                v = np.frombuffer(out, dt)
                if v.dtype.kind == "f":
                    assert np.all(np.isfinite(v))
                seen[os.path.relpath(os.path.join(r2, f), OME)] = v
    assert len(seen) == 7
    c0 = seen[os.path.join("v0.5", "0", "c", "0", "0", "0", "0", "0")]
    c1 = seen[os.path.join("v0.5", "0", "c", "0", "1", "0", "0", "0")]
    assert not np.array_equal(c0, c1) and np.ptp(c0) > 0


def test_corrupt_frames_raise_and_never_crash():
    """Byte flips and truncations of valid frames decode or raise the codec's error (the
    decoder must stay in bounds: run under tools/run_host_asan.sh as well)."""
    rng = np.random.default_rng(11)
    data = b"".join(bytes([i % 7]) * (i % 13 + 1) for i in range(3000))
    good = [libzstd(data, 3), libzstd(data, 19),
            libzstd(np.cumsum(rng.normal(size=5000)).astype("<f4").tobytes(), 9)]
    for g in good:
        for i in range(300):
            b = bytearray(g)
            if i % 2:
                b = b[:int(rng.integers(0, len(b)))]
            else:
                for _ in range(int(rng.integers(1, 4))):
                    b[int(rng.integers(4, len(b)))] ^= int(rng.integers(1, 256))
            try:
                dec(bytes(b))
            except z.ZarrException:
                pass


def test_size_query_and_small_destination():
    data = bytes(range(256)) * 10
    f = libzstd(data, 3)
    L = lib()
    n = C.c_size_t()
    assert L.zh_zstd_decompress(f, len(f), None, 0, C.byref(n), None, 0) == 0
    assert n.value == len(data)
    out = (C.c_char * 100)()
    err = C.create_string_buffer(128)
    assert L.zh_zstd_decompress(f, len(f), out, 100, C.byref(n), err, 128) != 0
    assert b"exceeds" in err.value
