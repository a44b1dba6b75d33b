"""Seeded random codec chains through the write path: the device encode against the oracle's
bytes (ShardingIndexedCodec.encode :105-168, BytesCodec.encode, Crc32cCodec.encode :50-60,
TransposeCodec.encode, Array.writeChunk's all-fill elision :148-151), then the stored chunks
read back (device and oracle) against the array.

Each case draws: rank 1-4, array / chunk / inner / leaf shapes (boundary chunks included),
dtype 1/2/4/8 bytes (bool among the 1-byte ones; float32/float64 with a 0, -0, NaN or ordinary
fill among them), transpose
order, bytes and index endianness, index at start or end, index crc32c, chunk crc32c, nested
sharding; the data holds blocks of fill so that chunks, inner chunks and leaves are elided.
The CPU test holds the oracle to its own round trip; the GPU test compares the device's bytes
with it."""
import os

import numpy as np
import pytest

import oracle as O
from helpers import NP_DT, device_read, device_write, encode_oracle
from test_gpu_files import three_ctxs  # noqa: F401 (fixture)
from zarrhip import _abi as A

FLOATS = {4: "<f4", 8: "<f8"}


def _divisors(n):
    return [d for d in range(1, n + 1) if n % d == 0]


def random_case(seed):
    """(meta, array, numpy dtype) of one random case."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 5))
    sharded = rng.random() < 0.75
    nested = sharded and rng.random() < 0.3
    chunk, inner, leaf, shape = [], [], [], []
    for _ in range(n):
        c = int(rng.choice([2, 4, 6, 8, 12, 16]))
        i = int(rng.choice(_divisors(c))) if sharded else c
        lf = int(rng.choice(_divisors(i))) if nested else i
        chunk.append(c)
        inner.append(i)
        leaf.append(lf)
        shape.append(int(rng.integers(1, 2 * c + 3)))
    # keep the element count small (the oracle is a C loop, the cases many)
    while int(np.prod(shape)) > 6000:
        d = int(np.argmax(shape))
        shape[d] = max(1, shape[d] // 2)
    ds = int(rng.choice([1, 2, 4, 8]))
    is_float = ds in FLOATS and rng.random() < 0.5
    is_bool = ds == 1 and rng.random() < 0.3
    dt = np.dtype(FLOATS[ds]) if is_float else NP_DT[ds]
    if is_float:
        fill = float(rng.choice([0.0, -0.0, np.nan, 1.5]))
    else:
        fill = int(rng.integers(0, 2 if is_bool else 4))
    fill_bytes = np.array([fill], dt).tobytes()
    order = [int(x) for x in rng.permutation(n)] if rng.random() < 0.5 else None
    kw = dict(fill=fill_bytes, is_float=is_float, is_bool=is_bool,
              transpose_order=order,
              endian=A.ZH_ENDIAN_BIG if rng.random() < 0.5 else A.ZH_ENDIAN_LITTLE,
              inner_crc32c=bool(rng.random() < 0.3))
    if sharded:
        kw.update(sharded=True, inner_chunk_shape=inner,
                  index_endian=A.ZH_ENDIAN_BIG if rng.random() < 0.3 else A.ZH_ENDIAN_LITTLE,
                  index_crc32c=bool(rng.random() < 0.6),
                  index_location=A.ZH_INDEX_START if rng.random() < 0.4 else A.ZH_INDEX_END)
        if nested:
            kw.update(nested_chunk_shape=leaf,
                      nested_index_crc32c=bool(rng.random() < 0.6),
                      nested_index_location=(A.ZH_INDEX_START if rng.random() < 0.4
                                             else A.ZH_INDEX_END))
    meta = A.make_meta(shape, chunk, ds, **kw)
    if is_float:
        a = rng.standard_normal(shape).astype(dt)
        a[rng.random(shape) < 0.1] = -0.0
    elif is_bool:
        a = (rng.random(shape) < 0.5).astype(dt)
    else:
        a = rng.integers(0, 2 ** (8 * ds) - 1, size=shape, dtype=np.uint64).astype(dt)
    # blocks of fill (whole chunks, inner chunks or leaves where they line up)
    blk = leaf if nested else inner
    for _ in range(int(rng.integers(0, 4))):
        lo = [int(rng.integers(0, max(1, s))) // b * b for s, b in zip(shape, blk)]
        sl = tuple(slice(lo_, lo_ + b * int(rng.integers(1, 3))) for lo_, b in zip(lo, blk))
        a[sl] = fill
    return meta, a, dt


# ZH_FUZZ_WCASES widens the search (default 40 cases; the round-5 search ran 1000 on the GPU)
CASES = list(range(int(os.environ.get("ZH_FUZZ_WCASES", "40"))))


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint8)


def _decode(meta, chunks, dt, shape):
    return np.frombuffer(O.array_read(meta, chunks, [0] * len(shape), shape), dt).reshape(shape)


@pytest.mark.parametrize("seed", CASES)
def test_oracle_write_read_round_trip(seed):
    """The oracle's write then read: every element equal to the array, except the values the
    reference's elision rewrites (an elided inner chunk reads 0 — Q1 — and an elided chunk the
    fill value; under Java's == a -0.0 chunk with a 0.0 fill reads +0.0)."""
    meta, a, dt = random_case(seed)
    shape = list(a.shape)
    chunks = encode_oracle(meta, a)
    got = _decode(meta, chunks, dt, shape)
    fill = np.frombuffer(bytes(meta.fill_value)[:meta.dtype_size], dt)[0]
    same = _bits(got).reshape(shape + [-1]).tolist() == _bits(a).reshape(shape + [-1]).tolist()
    if not same:  # only elided blocks may differ: they read 0 or the fill, and held fill
        g, x = got.reshape(-1), a.reshape(-1)
        diff = g.view(np.uint8).reshape(len(g), -1) != x.view(np.uint8).reshape(len(x), -1)
        bad = np.nonzero(diff.any(axis=1))[0]
        for i in bad:
            if np.dtype(dt).kind == "f":
                assert x[i] == fill or (np.isnan(fill) and np.isnan(x[i])), (seed, i)
                assert g[i] == 0 or g[i] == fill, (seed, i)
            else:
                assert x[i] == fill and g[i] == 0, (seed, i)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", CASES)
def test_device_write_matches_oracle_bytes(dev, seed):
    meta, a, dt = random_case(seed)
    shape = list(a.shape)
    got = device_write(dev, meta, a)
    want = encode_oracle(meta, a)
    assert len(got) == len(want)
    for k, (g, w) in enumerate(zip(got, want)):
        assert g == w, (seed, k, None if g is None else len(g), None if w is None else len(w))
    np.testing.assert_array_equal(_bits(device_read(dev, meta, got, [0] * len(shape), shape)),
                                  _bits(_decode(meta, want, dt, shape)))


@pytest.mark.gpu
@pytest.mark.parametrize("small_one", ["0", "1"])
@pytest.mark.parametrize("pipelined", [False, True])
@pytest.mark.parametrize("seed", CASES)
def test_device_read_random_regions_match_oracle(dev, three_ctxs, tmp_path, monkeypatch, seed,
                                                 pipelined, small_one):
    """The same random chains read back: three random regions per case (any offset and
    extent inside the array), from memory and from the chunk files through the library's own
    store reads, against the oracle's read of the same stored chunks.  pipelined: thresholds
    shrunk so that the reads run in slabs through the page-locked rings (test_gpu_files).
    small_one: plans of at most 64 inner chunks in one launch (the library's default, conftest)."""
    monkeypatch.setenv("ZH_SMALL_ONE", small_one)
    if pipelined:
        for k, v in (("ZH_PIPE_MIN_KB", "1"), ("ZH_PIPE_SLAB_KB", "4"),
                     ("ZH_PIPE_CHUNK_KB", "64"), ("ZH_PIPE_THREADS", "3")):
            monkeypatch.setenv(k, v)
    from helpers import chunk_coords
    from test_gpu_files import files_read, store_read
    from test_gpu_pieces import region_paths, write_store
    meta, a, dt = random_case(seed)
    shape = list(a.shape)
    chunks = encode_oracle(meta, a)
    rng = np.random.default_rng(10_000 + seed)
    allc = chunk_coords(meta, [0] * len(shape), shape)
    pos = {c: i for i, c in enumerate(allc)}
    paths = write_store(tmp_path, meta, chunks) if seed % 2 == 0 else None
    for _ in range(3):
        off = [int(rng.integers(0, s)) for s in shape]
        shp = [int(rng.integers(1, s - o + 1)) for s, o in zip(shape, off)]
        src = [chunks[pos[c]] for c in chunk_coords(meta, off, shp)]
        want = np.frombuffer(O.array_read(meta, src, off, shp), dt).reshape(shp)
        got = device_read(dev, meta, src, off, shp)
        np.testing.assert_array_equal(_bits(got), _bits(want), err_msg=f"{seed} {off} {shp}")
        if seed % 3 == 0:  # the region in slabs over three contexts (zh_array_read_multi)
            from test_gpu_fuzz_index import _multi_read
            got = _multi_read(three_ctxs, meta, src, off, shp).view(dt)
            np.testing.assert_array_equal(_bits(got), _bits(want),
                                          err_msg=f"multi {seed} {off} {shp}")
        if paths is not None:
            rp = region_paths(meta, paths, off, shp)
            np.testing.assert_array_equal(_bits(files_read(dev, meta, rp, off, shp).view(dt)),
                                          _bits(store_read(meta, rp, off, shp).view(dt)),
                                          err_msg=f"files {seed} {off} {shp}")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", CASES[:max(1, len(CASES) // 2)])
def test_jni_shim_random_chains(dev, seed):
    """The same random chains through the JNI shim under the fake JVM (HipArray.write's
    arrayWrite and HipArray.read's arrayRead: zh_array_meta packed from Java primitives, the
    float flag included): the encoded chunk objects equal the oracle's (null where all fill),
    and a random region reads back as the oracle reads it; the JNI rules hold."""
    from helpers import chunk_coords
    from jni_harness import FakeJVM
    meta, a, dt = random_case(seed)
    shape = list(a.shape)
    want = encode_oracle(meta, a)
    jvm = FakeJVM()
    got = jvm.array_write(dev.h.value, meta, a, [0] * len(shape))
    assert got == want, seed
    rng = np.random.default_rng(20_000 + seed)
    off = [int(rng.integers(0, s)) for s in shape]
    shp = [int(rng.integers(1, s - o + 1)) for s, o in zip(shape, off)]
    allc = chunk_coords(meta, [0] * len(shape), shape)
    pos = {c: i for i, c in enumerate(allc)}
    src = [want[pos[c]] for c in chunk_coords(meta, off, shp)]
    rc, out = jvm.array_read(dev.h.value, meta, src, off, shp)
    assert rc == 0, seed
    ref = np.frombuffer(O.array_read(meta, src, off, shp), dt).reshape(shp)
    np.testing.assert_array_equal(_bits(out), _bits(ref))
    jvm.check_rules()
