"""Seeded random arrays through the Python mirror's Array API (Array.create / write / read,
M/v3/Array.java, M/core/Array.java:83-156, 378-441): random data types, shapes, chunk
grids and codec chains — transpose, bytes endianness, sharding with the index at either end,
and the host byte-to-byte stages (gzip, zstd, blosc, crc32c: SURVEY §8(f) rank 3) on whole
chunks or on a shard's inner chunks — written to a FilesystemStore and read back, whole and in random regions,
through the library's own file reads (ZH_FILES=1, the default) and through the mirror's
store reads (ZH_FILES=0).  No oracle runs the compressors, so the check is the round trip:
the read equals the written array (fill 0, so an elided inner chunk reads the same, Q1).
ZH_FUZZ_APICASES widens the search (default 24; the round-5 search ran 300 on the GPU)."""
import os

import numpy as np
import pytest

import zarrhip as z

pytestmark = pytest.mark.gpu

DTYPES = [z.DataType.INT8, z.DataType.UINT8, z.DataType.INT16, z.DataType.UINT16,
          z.DataType.INT32, z.DataType.UINT32, z.DataType.INT64, z.DataType.UINT64,
          z.DataType.FLOAT32, z.DataType.FLOAT64, z.DataType.BOOL]


def _divisors(n):
    return [d for d in range(1, n + 1) if n % d == 0]


def _bb(rng):
    """A random host byte-to-byte stage (or none) as a CodecBuilder step."""
    k = int(rng.integers(0, 5))
    if k == 0:
        return lambda c: c
    if k == 1:
        lvl = int(rng.integers(1, 9))
        return lambda c: c.withGzip(lvl)
    if k == 2:
        lvl, ck = int(rng.integers(1, 8)), bool(rng.random() < 0.5)
        return lambda c: c.withZstd(lvl, ck)
    if k == 3:
        return lambda c: c.withBlosc()
    return lambda c: c.withCrc32c()


def random_array(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 4))
    dt = DTYPES[int(rng.integers(len(DTYPES)))]
    chunk = [int(rng.choice([2, 4, 6, 8])) for _ in range(n)]
    shape = [int(rng.integers(1, 3 * c + 2)) for c in chunk]
    sharded = rng.random() < 0.6
    inner = [int(rng.choice(_divisors(c))) for c in chunk]
    order = [int(x) for x in rng.permutation(n)] if rng.random() < 0.4 else None
    endian = "BIG" if rng.random() < 0.5 else "LITTLE"
    bb = _bb(rng)

    def leaf(c):
        if order is not None:
            c = c.withTranspose(order)
        return bb(c.withBytes(endian))
    if sharded:
        loc = "start" if rng.random() < 0.4 else "end"
        codecs = lambda c: c.withSharding(inner, leaf, loc)  # noqa: E731
    else:
        codecs = leaf
    meta = (z.ArrayMetadataBuilder().withShape(*shape).withDataType(dt).withChunkShape(*chunk)
            .withFillValue(0).withCodecs(codecs).build())
    npdt = dt.numpy
    if dt == z.DataType.BOOL:
        a = rng.random(shape) < 0.5
    elif npdt.kind == "f":
        a = rng.standard_normal(shape).astype(npdt)
    else:
        info = np.iinfo(npdt)
        a = rng.integers(info.min, info.max, size=shape, dtype=npdt, endpoint=True)
    blk = inner if sharded else chunk
    for _ in range(int(rng.integers(0, 3))):  # fill blocks: elided chunks / inner chunks
        lo = [int(rng.integers(0, s)) // b * b for s, b in zip(shape, blk)]
        a[tuple(slice(o, o + b) for o, b in zip(lo, blk))] = 0
    return meta, a, rng


CASES = list(range(int(os.environ.get("ZH_FUZZ_APICASES", "24"))))


@pytest.mark.parametrize("seed", CASES)
def test_api_random_arrays_round_trip(tmp_path, monkeypatch, seed):
    meta, a, rng = random_array(seed)
    arr = z.Array.create(z.FilesystemStore(tmp_path).resolve("a"), meta)
    arr.write(None, a)
    regions = [([0] * a.ndim, list(a.shape))]
    for _ in range(3):
        off = [int(rng.integers(0, s)) for s in a.shape]
        regions.append((off, [int(rng.integers(1, s - o + 1)) for s, o in zip(a.shape, off)]))
    for files in ("1", "0"):
        monkeypatch.setenv("ZH_FILES", files)
        b = z.Array.open(z.FilesystemStore(tmp_path).resolve("a"))
        for off, shp in regions:
            want = a[tuple(slice(o, o + s) for o, s in zip(off, shp))]
            np.testing.assert_array_equal(b.read(off, shp), want,
                                          err_msg=f"seed {seed} files {files} {off} {shp}")
