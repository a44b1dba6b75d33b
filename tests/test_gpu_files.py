"""Region reads straight from a FilesystemStore's files (zh_array_read_files).

Reference: core.Array.read over a FilesystemStore (M/core/Array.java:378-441) —
`exists` per chunk key (a regular file, FilesystemStore.java:42-45), `get(keys)` for a whole
chunk (:47-57), and for a part of a shard the StoreHandleDataProvider reads
(ShardingIndexedCodec.java:333-357): the index by a prefix / suffix read, one range per
referenced inner chunk, each a get(keys, start, end) that returns end - start bytes, zeros past
the end of the file (:84-102).  Here the library does those reads (pread straight into the
pipelined read's page-locked ring); every case is compared bit-exactly with the oracle
(oracle/zh_oracle.c) on the same stored bytes, read from the same files
(oracle.array_read_store) where the store semantics matter."""
import os
import stat

import numpy as np
import pytest

import oracle as O
import zarrhip as z
from helpers import NP_DT, chunk_coords, encode_oracle, rand_array
from test_gpu_pieces import CHAINS, REGIONS, make_case, oracle_region, region_paths, write_store
from zarrhip import _abi as A
from zarrhip._lib import ZhError

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["one_plan", "pipelined"])
def mode(request, monkeypatch):
    """one_plan: a small read (the file bytes staged in the context's page-locked buffer and
    DMA'd batch by batch, then one plan);
    pipelined: thresholds shrunk so that the same reads run in slabs through the rings, each
    range pread straight into a ring slot."""
    if request.param == "pipelined":
        monkeypatch.setenv("ZH_PIPE_MIN_KB", "1")
        monkeypatch.setenv("ZH_PIPE_SLAB_KB", "4")
        monkeypatch.setenv("ZH_PIPE_CHUNK_KB", "64")
        monkeypatch.setenv("ZH_PIPE_THREADS", "3")
    return request.param


def files_read(dev, meta, paths, off, shp, flags=0, store=None):
    out = np.empty(shp, NP_DT[meta.dtype_size])
    dev.array_read_files(meta, paths, off, shp, out.ctypes.data, flags, store=store)
    return out


def store_read(meta, paths, off, shp):
    """The oracle's core.Array.read over the same files (zo_array_read_store)."""
    return np.frombuffer(O.array_read_store(meta, paths, off, shp),
                         NP_DT[meta.dtype_size]).reshape(shp)


@pytest.mark.parametrize("chain", list(CHAINS))
def test_files_read_matches_oracle(dev, tmp_path, mode, chain):
    meta, arr, shards = make_case(chain, seed=43)
    shards[3] = None  # a missing shard (no file) reads fill_value
    paths = write_store(tmp_path, meta, shards)
    paths[5] = str(tmp_path / "no_such_file")  # a key whose file does not exist: fill too
    shards[5] = None
    for off, shp in REGIONS:
        got = files_read(dev, meta, region_paths(meta, paths, off, shp), off, shp)
        np.testing.assert_array_equal(got, oracle_region(meta, shards, off, shp))


@pytest.mark.parametrize("chain", list(CHAINS))
def test_files_random_regions(dev, tmp_path, mode, chain):
    """Seeded random regions (any offset and extent inside the array) over a store with a
    missing shard: every read equals the oracle's."""
    meta, arr, shards = make_case(chain, seed=131)
    shards[4] = None
    paths = write_store(tmp_path, meta, shards)
    rng = np.random.default_rng(137)
    shape = [meta.shape[d] for d in range(meta.ndim)]
    for _ in range(12):
        off = [int(rng.integers(0, s)) for s in shape]
        shp = [int(rng.integers(1, s - o + 1)) for s, o in zip(shape, off)]
        got = files_read(dev, meta, region_paths(meta, paths, off, shp), off, shp)
        np.testing.assert_array_equal(got, oracle_region(meta, shards, off, shp),
                                      err_msg=f"offset {off} shape {shp}")


@pytest.mark.parametrize("dsize", [1, 2, 8])
def test_files_dtypes_read_and_write(dev, tmp_path, mode, dsize):
    """1-, 2- and 8-byte elements (endian ignored for 1 byte, core BytesCodec.java:16-18)
    through both file entry points: the written files equal the oracle's encoding and read
    back, whole and as an unaligned part, equal to the oracle's reads."""
    shape = [24, 32, 48]
    meta = A.make_meta(shape, [8, 16, 24], dsize, fill=(3).to_bytes(dsize, "little"),
                       **CHAINS["transpose_be"])
    arr = rand_array(shape, dsize, seed=157, fill_frac=0.1, fill=3)
    want = encode_oracle(meta, arr)
    coords = chunk_coords(meta, [0, 0, 0], shape)
    paths = [str(tmp_path / "d" / "c" / "/".join(map(str, c))) for c in coords]
    dev.array_write_files(meta, arr.ctypes.data, [0, 0, 0], shape, paths)
    for p, w in zip(paths, want):
        assert (not os.path.exists(p)) if w is None else open(p, "rb").read() == w
    files = [p if w is not None else None for p, w in zip(paths, want)]
    for off, shp in REGIONS:
        got = files_read(dev, meta, region_paths(meta, files, off, shp), off, shp)
        np.testing.assert_array_equal(got, oracle_region(meta, want, off, shp))
        np.testing.assert_array_equal(got, arr[tuple(slice(o, o + s) for o, s in zip(off, shp))])


@pytest.mark.parametrize("order", [None, [2, 0, 1]])
def test_files_unsharded(dev, tmp_path, mode, order):
    """Unsharded chunks: each file is one whole object (get(keys))."""
    shape = [24, 32, 48]
    meta = A.make_meta(shape, [8, 16, 24], 4, fill=(9).to_bytes(4, "little"),
                       endian=A.ZH_ENDIAN_BIG, transpose_order=order)
    arr = rand_array(shape, 4, seed=47, fill_frac=0.1, fill=9)
    chunks = encode_oracle(meta, arr)
    chunks[2] = None
    paths = write_store(tmp_path, meta, chunks)
    for off, shp in REGIONS:
        got = files_read(dev, meta, region_paths(meta, paths, off, shp), off, shp)
        np.testing.assert_array_equal(got, oracle_region(meta, chunks, off, shp))


@pytest.mark.parametrize("pin", ["1", "0"])
def test_files_one_plan_batches(dev, tmp_path, monkeypatch, pin):
    """A one-plan read whose staged bytes span several 1 MiB batches: each batch is DMA'd from
    the context's page-locked buffer while the next is read (ZH_FILE_PIN=1, the default), or
    the bytes go through buffers of the plan's own (0).  Two shards with index crc32c and a
    transpose, an unaligned region over both; then a second, smaller read on the same context
    reuses the buffer."""
    monkeypatch.setenv("ZH_FILE_PIN", pin)
    shape = [1, 96, 96, 192]
    meta = A.make_meta(shape, [1, 96, 96, 96], 4, sharded=True, inner_chunk_shape=[1, 16, 16, 32],
                       transpose_order=[0, 3, 2, 1], endian=A.ZH_ENDIAN_BIG, index_crc32c=True)
    arr = rand_array(shape, 4, seed=113)
    shards = encode_oracle(meta, arr)
    paths = write_store(tmp_path, meta, shards)
    for off, shp in (([0, 5, 3, 40], [1, 90, 91, 140]), ([0, 17, 33, 90], [1, 9, 40, 12])):
        got = files_read(dev, meta, region_paths(meta, paths, off, shp), off, shp)
        want = arr[tuple(slice(o, o + s) for o, s in zip(off, shp))]
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(got, oracle_region(meta, shards, off, shp))


def test_files_shrinking_file_mid_read(dev, tmp_path, monkeypatch):
    """A whole-shard read whose file is cut short by someone else while the pipelined read is
    under way (the reference would read the file in one readAllBytes): the read either
    completes (the cut came after the last pread), reports what the reference reports for the
    shorter file (the cut came before the file's size was taken), or fails with the store
    error of a pread that hit the end (ZH_EIO, readFailed "unexpected end of file") — never a
    hang, a crash or a silently zero-padded whole shard — and the context reads correctly
    afterwards (the aborted lanes left it clean)."""
    import threading
    import time
    monkeypatch.setenv("ZH_PIPE_MIN_KB", "1")
    monkeypatch.setenv("ZH_PIPE_SLAB_KB", "512")
    monkeypatch.setenv("ZH_PIPE_CHUNK_KB", "64")
    monkeypatch.setenv("ZH_PIPE_THREADS", "2")
    shape = [1, 256, 256, 256]
    meta = A.make_meta(shape, shape, 4, sharded=True, inner_chunk_shape=[1, 32, 32, 32],
                       transpose_order=[0, 3, 2, 1], endian=A.ZH_ENDIAN_BIG, index_crc32c=True)
    arr = rand_array(shape, 4, seed=139)
    shard = encode_oracle(meta, arr)[0]
    p = tmp_path / "s"
    seen = set()
    for delay in (0.0, 0.002, 0.01, 0.05):
        p.write_bytes(shard)
        cut = threading.Timer(delay, lambda: os.truncate(p, len(shard) // 2))
        cut.start()
        try:
            got = files_read(dev, meta, [str(p)], [0] * 4, shape, store=tmp_path)
            np.testing.assert_array_equal(got, arr)
            seen.add("complete")
        except ZhError as e:
            msg = str(e)
            if e.status == A.ZH_EIO:
                assert msg == (f"Failed to read from store 'file://{tmp_path}' at key 's': "
                               "unexpected end of file"), msg
                seen.add("eio")
            else:  # the size was taken after the cut: entries past the end, or the index
                # read from the middle of the old payload
                assert e.status == A.ZH_EDATA, (e.status, msg)
                assert (msg.startswith("Could not load byte data for chunk [")
                        or msg.startswith("The checksum of the sharding index is invalid.")), msg
                seen.add("short")
        finally:
            cut.join()
        time.sleep(0.01)
    p.write_bytes(shard)
    np.testing.assert_array_equal(files_read(dev, meta, [str(p)], [0] * 4, shape), arr)
    print(f"outcomes: {sorted(seen)}")
    assert seen  # which outcomes occurred depends on timing; all of them are correct


def test_files_directory_is_a_missing_key(dev, tmp_path):
    """FilesystemStore.exists is Files.isRegularFile: a directory at a key reads as fill."""
    meta, arr, shards = make_case("sharded", seed=53)
    paths = write_store(tmp_path, meta, shards)
    os.remove(paths[0])
    os.mkdir(paths[0])
    shards[0] = None
    off, shp = [0, 0, 0], [24, 32, 48]
    got = files_read(dev, meta, region_paths(meta, paths, off, shp), off, shp)
    np.testing.assert_array_equal(got, oracle_region(meta, shards, off, shp))


@pytest.mark.parametrize("where", ["entry", "stored_crc"])
def test_files_corrupt_index_reports_device_crc(dev, tmp_path, mode, where):
    """The stored index goes to the device unchanged: the device's crc32c fails with the
    reference's message (Crc32cCodec.java:39-44), the oracle's text, for whole shards and
    parts."""
    meta, arr, shards = make_case("sharded", seed=59, fill_frac=0.0)
    bad = list(shards)
    b = bytearray(bad[1])
    b[-9 if where == "entry" else -2] ^= 0x10
    bad[1] = bytes(b)
    paths = write_store(tmp_path, meta, bad)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, [bad[1]], [0, 0, 24], [8, 16, 24])
    for off, shp in (([0, 0, 24], [8, 16, 24]), ([1, 0, 24], [6, 16, 24])):
        with pytest.raises(ZhError) as ed:
            files_read(dev, meta, region_paths(meta, paths, off, shp), off, shp)
        assert str(ed.value) == str(eo.value)
        assert str(ed.value).startswith("The checksum of the sharding index is invalid.")


def test_files_truncated_whole_shard(dev, tmp_path):
    """A whole shard read from a file cut short: the reference reads the file in one piece and
    slices it (decodePartial → chunkHandle.read(), ShardingIndexedCodec.java:246-251), which
    throws for an entry beyond its bytes (IllegalArgumentException).  Here that is the
    oracle's and the device's "Could not load byte data for chunk [...]", and a file shorter
    than its index "... is smaller than its index" (the error's class and
    text differ from the reference's, that it is an error does not)."""
    meta, arr, shards = make_case("start_beindex", seed=61, fill_frac=0.0)
    paths = write_store(tmp_path, meta, shards)
    full = os.path.getsize(paths[0])
    os.truncate(paths[0], full - 100)  # the last inner chunk's payload loses 100 bytes
    off, shp = [0, 0, 0], [8, 16, 24]
    with pytest.raises(O.OracleError) as eo:
        store_read(meta, region_paths(meta, paths, off, shp), off, shp)
    with pytest.raises(ZhError) as ed:
        files_read(dev, meta, region_paths(meta, paths, off, shp), off, shp)
    assert str(ed.value) == str(eo.value)
    assert str(ed.value).startswith("Could not load byte data for chunk [")
    os.truncate(paths[0], 10)
    with pytest.raises(ZhError) as ed:
        files_read(dev, meta, region_paths(meta, paths, off, shp), off, shp)
    assert "is smaller than its index" in str(ed.value)


@pytest.mark.parametrize("chain", ["sharded", "start_beindex", "transpose_be", "chunk_crc"])
def test_files_truncated_part_reads_zeros(dev, tmp_path, mode, chain):
    """A part of a shard whose file was cut short: each range read is
    FilesystemStore.get(keys, start, end) (FilesystemStore.java:84-102), a buffer of the
    entry's length holding what the file has and zeros after its end, so the part decodes
    (where the chunk codecs accept those bytes) — equal to the oracle reading the same files.
    With a chunk crc32c the zeros fail the chunk's check with the reference's message."""
    meta, arr, shards = make_case(chain, seed=163, fill_frac=0.0)
    paths = write_store(tmp_path, meta, shards)
    p = paths[0]
    whole = open(p, "rb").read()
    isz = 16 * (2 * 2 * 3) + 4
    end_idx = meta.chain.index_location == A.ZH_INDEX_END
    for cut in (100, 3000):
        open(p, "wb").write(whole[:-cut - isz] + whole[-isz:] if end_idx else whole[:-cut])
        for off, shp in (([0, 0, 0], [8, 16, 23]), ([4, 8, 16], [4, 8, 8]), ([1, 3, 5], [6, 9, 17])):
            rp = region_paths(meta, paths, off, shp)
            try:
                want = store_read(meta, rp, off, shp)
            except O.OracleError as eo:
                with pytest.raises(ZhError) as ed:
                    files_read(dev, meta, rp, off, shp)
                if chain == "chunk_crc":  # several chunks fail: the device names any of them
                    pre = "The checksum of the sharding index is invalid. Stored: "
                    assert str(ed.value).startswith(pre) and str(eo).startswith(pre)
                else:
                    assert str(ed.value) == str(eo), (cut, off)
                continue
            np.testing.assert_array_equal(files_read(dev, meta, rp, off, shp), want,
                                          err_msg=f"cut {cut} region {off} {shp}")


def test_files_short_prefix_index_of_a_part(dev, tmp_path):
    """index_location start, a part of a file shorter than its index: the prefix read returns
    the file's bytes zero-padded to the index's length (get(keys, 0, n)), whose crc32c fails
    with the reference's message — the oracle's text, read from the same file."""
    meta, arr, shards = make_case("start_beindex", seed=167, fill_frac=0.0)
    paths = write_store(tmp_path, meta, shards)
    os.truncate(paths[0], 37)
    off, shp = [1, 3, 5], [6, 9, 17]
    rp = region_paths(meta, paths, off, shp)
    with pytest.raises(O.OracleError) as eo:
        store_read(meta, rp, off, shp)
    with pytest.raises(ZhError) as ed:
        files_read(dev, meta, rp, off, shp)
    assert str(ed.value) == str(eo.value)
    assert str(ed.value).startswith("The checksum of the sharding index is invalid. Stored: 0 ")


@pytest.mark.skipif(os.geteuid() == 0, reason="root reads files regardless of their mode")
def test_files_unreadable_is_store_exception(dev, tmp_path):
    """A file that exists but cannot be read: ZH_EIO → StoreException (readFailed)."""
    meta, arr, shards = make_case("sharded", seed=67)
    paths = write_store(tmp_path, meta, shards)
    os.chmod(paths[0], 0)
    try:
        off, shp = [0, 0, 0], [8, 16, 24]
        with pytest.raises(ZhError) as ed:
            files_read(dev, meta, region_paths(meta, paths, off, shp), off, shp,
                       store=tmp_path)
        assert ed.value.status == A.ZH_EIO
        # StoreException.readFailed (StoreException.java:17-21): the store, the key below it,
        # and the cause's text (an AccessDeniedException carries the file)
        key = os.path.relpath(paths[0], tmp_path)
        assert str(ed.value) == (f"Failed to read from store 'file://{tmp_path}' at key "
                                 f"'{key}': {paths[0]}")
    finally:
        os.chmod(paths[0], stat.S_IRUSR | stat.S_IWUSR)


def test_files_device_output(dev, tmp_path, mode):
    meta, arr, shards = make_case("transpose_be", seed=71)
    paths = write_store(tmp_path, meta, shards)
    off, shp = [2, 3, 4], [20, 25, 40]
    nb = int(np.prod(shp)) * 4
    d = dev.malloc(nb)
    try:
        dev.array_read_files(meta, region_paths(meta, paths, off, shp), off, shp, d,
                             A.ZH_OUT_DEVICE)
        got = np.frombuffer(dev.d2h(d, nb), np.uint32).reshape(shp)
    finally:
        dev.free(d)
    np.testing.assert_array_equal(got, oracle_region(meta, shards, off, shp))


def test_files_argument_errors(dev, tmp_path):
    meta, arr, shards = make_case("sharded", seed=73)
    paths = write_store(tmp_path, meta, shards)
    off, shp = [0, 0, 0], [24, 32, 48]
    out = np.empty(shp, np.uint32)
    with pytest.raises(ZhError) as ed:  # one path short
        dev.array_read_files(meta, region_paths(meta, paths, off, shp)[:-1], off, shp,
                             out.ctypes.data)
    assert ed.value.status == A.ZH_EINVAL
    with pytest.raises(ZhError) as ed:
        dev.array_read_files(meta, region_paths(meta, paths, off, shp), off, shp,
                             out.ctypes.data, A.ZH_SRC_DEVICE)
    assert ed.value.status == A.ZH_EINVAL
    with pytest.raises(ZhError) as ed:  # M/core/Array.java:386-390
        dev.array_read_files(meta, region_paths(meta, paths, off, shp), [1, 0, 0], shp,
                             out.ctypes.data)
    assert str(ed.value) == "Requested data is outside of the array's domain."


def _rchar():
    with open("/proc/self/io") as f:
        for line in f:
            if line.startswith("rchar:"):
                return int(line.split()[1])
    return None


def test_files_read_only_referenced_bytes(dev, tmp_path, mode):
    """StoreHandleDataProvider semantics: a sub-shard part reads the index and the ranges it
    references, not the shard (bytes read by this process's read calls, /proc/self/io)."""
    shape = [64, 64, 32]
    meta = A.make_meta(shape, [64, 64, 32], 4, sharded=True, inner_chunk_shape=[8, 8, 8],
                       endian=A.ZH_ENDIAN_BIG)
    arr = rand_array(shape, 4, seed=79, fill_frac=0.0, fill=0)
    shards = encode_oracle(meta, arr)
    paths = write_store(tmp_path, meta, shards)
    if _rchar() is None:
        pytest.skip("no /proc/self/io")
    off, shp = [5, 9, 3], [10, 12, 6]
    r0 = _rchar()
    got = files_read(dev, meta, paths, off, shp)
    used = _rchar() - r0
    np.testing.assert_array_equal(got, arr[5:15, 9:21, 3:9])
    assert used < len(shards[0]) / 4, used
    r0 = _rchar()
    np.testing.assert_array_equal(files_read(dev, meta, paths, [0, 0, 0], shape), arr)
    assert _rchar() - r0 >= len(shards[0])


@pytest.mark.parametrize("inner", [[1, 16, 16, 16], [1, 32, 32, 32]])
def test_array_read_goes_through_files(dev, tmp_path, monkeypatch, inner):
    """zarrhip.Array.read over a FilesystemStore hands the files to the library (a region of
    96 MiB: the default pipelined thresholds), with the result of the mirror's own store reads
    (ZH_FILES=0) and of the written data."""
    shape = [1, 256, 384, 256]
    m = (z.ArrayMetadataBuilder().withShape(*shape).withDataType(z.DataType.UINT32)
         .withChunkShape(1, 128, 128, 128).withFillValue(0)
         .withCodecs(lambda c: c.withSharding(
             inner, lambda c1: c1.withTranspose([0, 3, 2, 1]).withBytes("BIG")))
         .build())
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("f"), m)
    data = np.random.default_rng(83).integers(0, 2 ** 32, shape, dtype=np.uint32)
    a.write(None, data)
    b = z.Array.open(z.FilesystemStore(tmp_path).resolve("f"))
    got = b.read()
    assert b.last_read_timing.get("files") is True
    np.testing.assert_array_equal(got, data)
    off, shp = [0, 17, 33, 5], [1, 200, 300, 250]
    part = b.read(off, shp)
    np.testing.assert_array_equal(part, data[:, 17:217, 33:333, 5:255])
    monkeypatch.setenv("ZH_FILES", "0")
    np.testing.assert_array_equal(b.read(off, shp), part)
    assert b.last_read_timing.get("files") is None


def _outcome(fn):
    try:
        return ("ok", fn())
    except Exception as e:  # noqa: BLE001 - compared by type and message
        return (type(e).__name__, str(e))


@pytest.mark.parametrize("sharded", [False, True])
def test_empty_chunk_file_same_as_store_reads(dev, tmp_path, monkeypatch, sharded):
    """A chunk file of zero bytes (it exists: FilesystemStore.exists is true, get returns an
    empty buffer) fails or reads exactly as it does through the mirror's own store reads
    (ZH_FILES=0): for a shard, smaller than its index; for an unsharded chunk, the bytes
    codec's length check."""
    shape = [32, 32, 48]
    b = (z.ArrayMetadataBuilder().withShape(*shape).withDataType(z.DataType.UINT32)
         .withChunkShape(16, 32, 24).withFillValue(0))
    if sharded:
        b = b.withCodecs(lambda c: c.withSharding([8, 8, 8], lambda c1: c1.withBytes("LITTLE")))
    else:
        b = b.withCodecs(lambda c: c.withBytes("BIG"))
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("e"), b.build())
    data = np.random.default_rng(127).integers(1, 2 ** 32, shape, dtype=np.uint32)
    a.write(None, data)
    victim = tmp_path / "e" / "c" / "1" / "0" / "1"
    assert victim.is_file()
    victim.write_bytes(b"")
    a = z.Array.open(z.FilesystemStore(tmp_path).resolve("e"))
    kinds = []
    for off, shp in (([0, 0, 0], shape), ([16, 0, 24], [16, 32, 24]), ([3, 1, 2], [9, 30, 20])):
        files = _outcome(lambda: a.read(off, shp).copy())
        monkeypatch.setenv("ZH_FILES", "0")
        mirror = _outcome(lambda: a.read(off, shp).copy())
        monkeypatch.delenv("ZH_FILES")
        assert files[0] == mirror[0], (files, mirror)
        if files[0] == "ok":
            np.testing.assert_array_equal(files[1], mirror[1])
        else:
            assert files[1] == mirror[1]
        kinds.append(files[0])
    # the regions with chunk (1, 0, 1) fail; the last one avoids it and reads the data
    assert kinds[0] != "ok" and kinds[1] != "ok" and kinds[2] == "ok", kinds


@pytest.mark.parametrize("sharded", [False, True])
def test_read_chunk_goes_through_files(dev, tmp_path, monkeypatch, sharded):
    """zarrhip.Array.readChunk (M/core/Array.java:167-182) over a FilesystemStore: the chunk's
    file read by the library (the chunk viewed as a one-chunk array); a boundary chunk keeps
    its padding, a missing chunk is fill — the same as the mirror's own store reads."""
    shape = [40, 56, 24]
    b = (z.ArrayMetadataBuilder().withShape(*shape).withDataType(z.DataType.UINT32)
         .withChunkShape(16, 32, 24).withFillValue(3))
    if sharded:
        b = b.withCodecs(lambda c: c.withSharding(
            [8, 8, 8], lambda c1: c1.withTranspose([2, 0, 1]).withBytes("BIG")))
    else:
        b = b.withCodecs(lambda c: c.withBytes("BIG"))
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("r"), b.build())
    data = np.random.default_rng(89).integers(0, 2 ** 32, shape, dtype=np.uint32)
    data[32:, 32:, :] = 3  # chunk (2, 1, 0) all fill: deleted on write
    a.write(None, data)
    for c in [(0, 0, 0), (2, 0, 0), (1, 1, 0), (2, 1, 0)]:
        got = a.readChunk(list(c))
        monkeypatch.setenv("ZH_FILES", "0")
        want = a.readChunk(list(c))
        monkeypatch.delenv("ZH_FILES")
        np.testing.assert_array_equal(got, want)
        sl = tuple(slice(ci * cs, min((ci + 1) * cs, n)) for ci, cs, n in zip(c, [16, 32, 24], shape))
        np.testing.assert_array_equal(got[tuple(slice(0, s.stop - s.start) for s in sl)], data[sl])


@pytest.fixture(scope="module")
def three_ctxs():
    from zarrhip._lib import DeviceContext
    cs = [DeviceContext(0) for _ in range(3)]
    yield cs
    for c in cs:
        c.close()


@pytest.mark.parametrize("ndev", [2, 3])
@pytest.mark.parametrize("out_dev", [False, True])
def test_files_multi_context(three_ctxs, tmp_path, mode, ndev, out_dev):
    """zh_array_read_files_multi: one slab per context (here contexts on one device), each
    reading the files of its slab; host-terminated slices, or the root's device buffer (the
    other slabs decoded by plans that read their file bytes into host buffers first)."""
    from zarrhip._lib import array_read_files_multi
    shape = [1, 96, 64, 80]
    meta = A.make_meta(shape, [1, 32, 32, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 8, 16, 16], transpose_order=[0, 3, 2, 1])
    arr = rand_array(shape, 4, seed=97)
    shards = encode_oracle(meta, arr)
    shards[1] = None
    paths = write_store(tmp_path, meta, shards)
    cs = three_ctxs[:ndev]
    for off, shp in [([0, 0, 0, 0], shape), ([0, 5, 3, 7], [1, 83, 50, 61])]:
        want = oracle_region(meta, shards, off, shp)
        rp = region_paths(meta, paths, off, shp)
        nb = int(np.prod(shp)) * 4
        if out_dev:
            d = cs[0].malloc(nb)
            try:
                routes = array_read_files_multi(cs, meta, rp, off, shp, d, A.ZH_OUT_DEVICE)
                got = np.frombuffer(cs[0].d2h(d, nb), np.uint32).reshape(shp)
            finally:
                cs[0].free(d)
            assert routes[1] == 3  # ZH_ROUTE_SAME: decoded on its context, copied to the root
        else:
            got = np.empty(shp, np.uint32)
            routes = array_read_files_multi(cs, meta, rp, off, shp, got.ctypes.data, 0)
            assert all(r == 0 for r in routes)  # every slab straight into its host slice
        np.testing.assert_array_equal(got, want)


# ---- the write side: zh_array_write_files ------------------------------------------------
WCHAINS = {
    "sharded_t": dict(sharded=True, inner_chunk_shape=[4, 8, 8], transpose_order=[2, 0, 1],
                      endian=A.ZH_ENDIAN_BIG),
    "start_crc": dict(sharded=True, inner_chunk_shape=[4, 8, 8], inner_crc32c=True,
                      index_location=A.ZH_INDEX_START),
    "nested": dict(sharded=True, inner_chunk_shape=[8, 8, 8], nested_chunk_shape=[4, 4, 8]),
    "bytes": dict(endian=A.ZH_ENDIAN_BIG),
}


@pytest.fixture(params=["one_window", "windows"])
def wmode(request, monkeypatch):
    """windows: 64 KiB ring windows over 3 lanes, so every chunk file is written in many
    pwrite windows by several lanes."""
    if request.param == "windows":
        monkeypatch.setenv("ZH_PIPE_CHUNK_KB", "64")
        monkeypatch.setenv("ZH_PIPE_THREADS", "3")
    return request.param


@pytest.mark.parametrize("chain", list(WCHAINS))
def test_write_files_matches_oracle(dev, tmp_path, wmode, chain):
    """Each chunk file holds exactly the oracle's encoded bytes (ShardingIndexedCodec.encode /
    BytesCodec.encode); an all-fill chunk's existing file is deleted (writeChunk → delete); the
    parent directories are created (FilesystemStore.set)."""
    shape = [24, 32, 48]
    meta = A.make_meta(shape, [8, 16, 24], 4, fill=(7).to_bytes(4, "little"), **WCHAINS[chain])
    arr = rand_array(shape, 4, seed=101, fill_frac=0.1, fill=7)
    arr[8:16, 0:16, 24:48] = 7  # chunk (1, 0, 1): all fill → deleted
    want = encode_oracle(meta, arr)
    coords = chunk_coords(meta, [0, 0, 0], shape)
    paths = [str(tmp_path / "w" / "c" / "/".join(map(str, c))) for c in coords]
    k = coords.index((1, 0, 1))
    assert want[k] is None
    os.makedirs(os.path.dirname(paths[k]), exist_ok=True)
    with open(paths[k], "wb") as f:
        f.write(b"stale")
    sizes = dev.array_write_files(meta, arr.ctypes.data, [0, 0, 0], shape, paths)
    for p, w, sz in zip(paths, want, sizes):
        if w is None:
            assert sz == 0 and not os.path.exists(p)
        else:
            assert sz == len(w)
            assert open(p, "rb").read() == w
    # and read back through the files
    got = files_read(dev, meta, paths, [0, 0, 0], shape)
    np.testing.assert_array_equal(got, arr)


@pytest.mark.parametrize("chain", list(WCHAINS))
def test_write_files_random_regions(dev, tmp_path, wmode, chain):
    """Seeded random regions of whole chunks (the array boundary clips the last ones), written
    one after another into the same store: every chunk file the region covers holds exactly the
    oracle's encoding of that region (ShardingIndexedCodec.encode / BytesCodec.encode)."""
    shape = [20, 40, 56]
    cs = [8, 16, 24]
    meta = A.make_meta(shape, cs, 4, fill=(5).to_bytes(4, "little"), **WCHAINS[chain])
    rng = np.random.default_rng(149)
    grid = [-(-s // c) for s, c in zip(shape, cs)]
    for k in range(6):
        c0 = [int(rng.integers(0, g)) for g in grid]
        c1 = [int(rng.integers(a + 1, g + 1)) for a, g in zip(c0, grid)]
        off = [a * c for a, c in zip(c0, cs)]
        shp = [min(b * c, s) - o for b, c, s, o in zip(c1, cs, shape, off)]
        arr = rand_array(shp, 4, seed=151 + k, fill_frac=0.2, fill=5)
        want = O.array_write(meta, arr.tobytes(), off, shp)
        coords = chunk_coords(meta, off, shp)
        paths = [str(tmp_path / "r" / "c" / "/".join(map(str, c))) for c in coords]
        sizes = dev.array_write_files(meta, arr.ctypes.data, off, shp, paths)
        for p, w, sz in zip(paths, want, sizes):
            if w is None:
                assert sz == 0 and not os.path.exists(p)
            else:
                assert sz == len(w) and open(p, "rb").read() == w, (off, shp, p)


def test_write_files_windows_of_one_file(dev, tmp_path, monkeypatch):
    """Chunk files of several ring windows (here 64 KiB, three lanes), so the lanes write
    windows of the same file at once: each file holds exactly the oracle's bytes, a longer stale
    file is cut to the new size, and no chunk's size is a multiple of the window."""
    monkeypatch.setenv("ZH_PIPE_CHUNK_KB", "64")
    monkeypatch.setenv("ZH_PIPE_THREADS", "3")
    shape = [40, 64, 72]
    meta = A.make_meta(shape, [32, 64, 72], 4, sharded=True, inner_chunk_shape=[8, 16, 24],
                       inner_crc32c=True, transpose_order=[1, 2, 0], endian=A.ZH_ENDIAN_BIG)
    arr = rand_array(shape, 4, seed=109, fill_frac=0.05)
    want = encode_oracle(meta, arr)
    coords = chunk_coords(meta, [0, 0, 0], shape)
    paths = [str(tmp_path / "m" / "c" / "/".join(map(str, c))) for c in coords]
    assert all(len(w) > 64 << 10 and len(w) % (64 << 10) for w in want)
    os.makedirs(os.path.dirname(paths[0]), exist_ok=True)
    with open(paths[0], "wb") as f:
        f.write(b"\xab" * (2 * len(want[0])))
    sizes = dev.array_write_files(meta, arr.ctypes.data, [0, 0, 0], shape, paths)
    assert list(sizes) == [len(w) for w in want]
    for p, w in zip(paths, want):
        assert open(p, "rb").read() == w
    np.testing.assert_array_equal(files_read(dev, meta, paths, [0, 0, 0], shape), arr)


def test_write_files_device_source_and_errors(dev, tmp_path):
    shape = [24, 32, 48]
    meta = A.make_meta(shape, [8, 16, 24], 4, **WCHAINS["sharded_t"])
    arr = rand_array(shape, 4, seed=103)
    want = encode_oracle(meta, arr)
    coords = chunk_coords(meta, [0, 0, 0], shape)
    paths = [str(tmp_path / "d" / "_".join(map(str, c))) for c in coords]
    d = dev.malloc(arr.nbytes)
    try:
        dev.h2d(d, arr.tobytes())
        dev.array_write_files(meta, d, [0, 0, 0], shape, paths, A.ZH_SRC_DEVICE)
    finally:
        dev.free(d)
    assert [open(p, "rb").read() for p in paths] == want
    # a region that cuts chunks: the binding's read-modify-write
    with pytest.raises(ZhError) as ed:
        dev.array_write_files(meta, arr.ctypes.data, [0, 0, 1], [8, 16, 24], paths[:1])
    assert ed.value.status == A.ZH_EUNSUPPORTED
    # a parent path that is a file: the directories cannot be created → StoreException
    blocker = tmp_path / "blocker"
    blocker.write_bytes(b"x")
    bad = [str(blocker / "c" / str(i)) for i in range(len(paths))]
    with pytest.raises(ZhError) as ed:
        dev.array_write_files(meta, arr.ctypes.data, [0, 0, 0], shape, bad, store=tmp_path)
    assert ed.value.status == A.ZH_EIO
    # StoreException.writeFailed with FilesystemStore.set's cause (FilesystemStore.java:107-115)
    assert str(ed.value) == (f"Failed to write to store 'file://{tmp_path}' at key "
                             f"'blocker/c/0': Failed to create parent directories for path: "
                             f"{blocker}/c")


def _nofile_headroom(extra):
    """Lower this process's RLIMIT_NOFILE soft limit to the descriptors open now + extra; returns
    the old limits (restore them with resource.setrlimit)."""
    import resource
    old = resource.getrlimit(resource.RLIMIT_NOFILE)
    used = len(os.listdir("/proc/self/fd"))
    resource.setrlimit(resource.RLIMIT_NOFILE, (used + extra, old[1]))
    return old


def test_files_read_more_chunks_than_descriptors(dev, tmp_path, mode):
    """A region of more chunk files than the process may open at once (RLIMIT_NOFILE lowered
    to 24 beyond what is open): the reference opens one file per get(); the library keeps at
    most a bounded number of descriptors (closing idle ones, reopening by path), so the read
    completes and equals the oracle's."""
    import resource
    shape = [40, 40, 40]
    meta = A.make_meta(shape, [4, 4, 8], 4, endian=A.ZH_ENDIAN_BIG)  # 10*10*5 = 500 files
    arr = rand_array(shape, 4, seed=171)
    chunks = encode_oracle(meta, arr)
    paths = write_store(tmp_path, meta, chunks)
    off, shp = [0, 0, 0], shape
    old = _nofile_headroom(24)
    try:
        got = files_read(dev, meta, region_paths(meta, paths, off, shp), off, shp)
    finally:
        resource.setrlimit(resource.RLIMIT_NOFILE, old)
    np.testing.assert_array_equal(got, arr)
    # sharded parts too: 500 shards, each read as index + ranges
    meta = A.make_meta(shape, [4, 4, 8], 4, sharded=True, inner_chunk_shape=[2, 2, 4])
    shards = encode_oracle(meta, arr)
    paths = write_store(tmp_path, meta, shards, tag="s")
    off, shp = [1, 1, 1], [38, 38, 38]
    old = _nofile_headroom(24)
    try:
        got = files_read(dev, meta, region_paths(meta, paths, off, shp), off, shp)
    finally:
        resource.setrlimit(resource.RLIMIT_NOFILE, old)
    np.testing.assert_array_equal(got, arr[1:39, 1:39, 1:39])


def test_array_write_goes_through_files(dev, tmp_path, monkeypatch):
    """zarrhip.Array.write over a FilesystemStore: the library writes the chunk files; the
    files equal the ones the mirror's own store writes make (ZH_FILES=0)."""
    shape = [1, 64, 96, 80]
    m = (z.ArrayMetadataBuilder().withShape(*shape).withDataType(z.DataType.UINT32)
         .withChunkShape(1, 32, 32, 64).withFillValue(0)
         .withCodecs(lambda c: c.withSharding(
             [1, 8, 16, 16], lambda c1: c1.withTranspose([0, 3, 2, 1]).withBytes("BIG")))
         .build())
    data = np.random.default_rng(107).integers(0, 2 ** 32, shape, dtype=np.uint32)
    data[0, 32:, 32:64, :] = 0  # two all-fill shards
    a = z.Array.create(z.FilesystemStore(tmp_path / "lib").resolve("a"), m)
    a.write(None, data)
    monkeypatch.setenv("ZH_FILES", "0")
    b = z.Array.create(z.FilesystemStore(tmp_path / "mirror").resolve("a"), m)
    b.write(None, data)
    monkeypatch.delenv("ZH_FILES")
    for root, _, files in os.walk(tmp_path / "mirror" / "a"):
        for fn in files:
            rel = os.path.relpath(os.path.join(root, fn), tmp_path / "mirror")
            assert open(tmp_path / "lib" / rel, "rb").read() == \
                open(tmp_path / "mirror" / rel, "rb").read(), rel
    n_lib = sum(len(f) for _, _, f in os.walk(tmp_path / "lib"))
    n_mir = sum(len(f) for _, _, f in os.walk(tmp_path / "mirror"))
    assert n_lib == n_mir
    np.testing.assert_array_equal(z.Array.open(z.FilesystemStore(tmp_path / "lib").resolve("a"))
                                  .read(), data)


def _tmp_leftovers(root):
    return [os.path.join(d, f) for d, _, fs in os.walk(root) for f in fs if ".zhtmp" in f]


def test_write_files_more_chunks_than_descriptors(dev, tmp_path, wmode):
    """More chunk files than the process may open at once (RLIMIT_NOFILE lowered to 24 beyond
    what is open): the reference opens, writes and closes one file per set(); the library keeps
    at most 3 files per lane open, so the write completes with the oracle's bytes and leaves
    no temporary files."""
    import resource
    shape = [40, 40, 48]
    meta = A.make_meta(shape, [4, 4, 8], 4, **WCHAINS["sharded_t"] | dict(
        inner_chunk_shape=[2, 2, 4]))  # 10*10*6 = 600 chunk files
    arr = rand_array(shape, 4, seed=173, fill_frac=0.0)
    want = encode_oracle(meta, arr)
    coords = chunk_coords(meta, [0, 0, 0], shape)
    paths = [str(tmp_path / "n" / "c" / "/".join(map(str, c))) for c in coords]
    old = _nofile_headroom(24)
    try:
        dev.array_write_files(meta, arr.ctypes.data, [0, 0, 0], shape, paths)
    finally:
        resource.setrlimit(resource.RLIMIT_NOFILE, old)
    assert [open(p, "rb").read() for p in paths] == want
    assert not _tmp_leftovers(tmp_path)


def test_write_files_failure_leaves_unfinished_chunks_intact(dev, tmp_path, wmode):
    """A write that fails part-way (one chunk's path is a directory, so its file cannot be put
    in place): the call raises StoreException.writeFailed's text for that chunk; every other
    chunk file holds either its old bytes or its new bytes, whole — a chunk the failure did not
    let finish is never truncated or half-written (each chunk goes to a temporary file renamed
    over the old one once complete) — and no temporary file is left behind."""
    shape = [24, 32, 48]
    meta = A.make_meta(shape, [8, 16, 24], 4, **WCHAINS["sharded_t"])
    old_arr = rand_array(shape, 4, seed=179, fill_frac=0.0)
    new_arr = rand_array(shape, 4, seed=181, fill_frac=0.0)
    old_enc, new_enc = encode_oracle(meta, old_arr), encode_oracle(meta, new_arr)
    coords = chunk_coords(meta, [0, 0, 0], shape)
    paths = [str(tmp_path / "f" / "c" / "/".join(map(str, c))) for c in coords]
    dev.array_write_files(meta, old_arr.ctypes.data, [0, 0, 0], shape, paths)
    k = len(paths) // 2
    os.remove(paths[k])
    os.makedirs(os.path.join(paths[k], "x"))  # a non-empty directory at the chunk's key
    with pytest.raises(ZhError) as ed:
        dev.array_write_files(meta, new_arr.ctypes.data, [0, 0, 0], shape, paths,
                              store=tmp_path / "f")
    assert ed.value.status == A.ZH_EIO
    key = "c/" + "/".join(map(str, coords[k]))
    assert str(ed.value) == (f"Failed to write to store 'file://{tmp_path}/f' at key '{key}': "
                             f"Failed to write {len(new_enc[k])} bytes to file: {paths[k]}")
    for i, p in enumerate(paths):
        if i == k:
            assert os.path.isdir(p)
            continue
        b = open(p, "rb").read()
        assert b in (old_enc[i], new_enc[i]), (i, len(b))
    assert not _tmp_leftovers(tmp_path)


@pytest.mark.parametrize("loc", ["end", "start"])
def test_mirror_and_library_store_reads_agree_on_truncated_shards(dev, tmp_path, monkeypatch,
                                                                   loc):
    """zarrhip.Array.read over a FilesystemStore whose shard file lost its tail, through the
    library's own file reads (ZH_FILES=1) and through the mirror's store reads (ZH_FILES=0:
    FilesystemStore.get(keys, start, end) zero-padded in store.py, the shard size bounding
    nothing in Array._stage_shard, as ShardPieces.part does in Java): both equal the oracle's
    read of the same files — a part decodes, a whole shard fails with the same message."""
    shape = [1, 32, 32, 48]
    m = (z.ArrayMetadataBuilder().withShape(*shape).withDataType(z.DataType.UINT32)
         .withChunkShape(1, 16, 32, 48).withFillValue(0)
         .withCodecs(lambda c: c.withSharding([1, 8, 8, 16], lambda c1: c1.withTranspose(
             [0, 3, 2, 1]).withBytes("BIG"), loc)).build())
    data = np.random.default_rng(193).integers(0, 2 ** 32, shape, dtype=np.uint32)
    a = z.Array.create(z.FilesystemStore(tmp_path).resolve("t"), m)
    a.write(None, data)
    f = tmp_path / "t" / "c" / "0" / "0" / "0" / "0"
    whole = f.read_bytes()
    isz = 16 * (2 * 4 * 3) + 4
    f.write_bytes(whole[:-3000 - isz] + whole[-isz:] if loc == "end" else whole[:-3000])
    p1 = str(tmp_path / "t" / "c" / "0" / "1" / "0" / "0")
    for off, shp, whole_shard in (([0, 1, 2, 3], [1, 14, 29, 40], False),
                                  ([0, 0, 0, 0], [1, 16, 32, 48], True)):
        b = z.Array.open(z.FilesystemStore(tmp_path).resolve("t"))
        paths = [str(f)] + ([p1] if off[1] + shp[1] > 16 else [])
        try:
            want = store_read(b.zmeta, paths, off, shp)
        except O.OracleError as eo:
            assert whole_shard
            for files in ("1", "0"):
                monkeypatch.setenv("ZH_FILES", files)
                with pytest.raises(z.ZarrException) as ez:
                    z.Array.open(z.FilesystemStore(tmp_path).resolve("t")).read(off, shp)
                assert str(ez.value) == str(eo), files
            continue
        assert not whole_shard
        for files in ("1", "0"):
            monkeypatch.setenv("ZH_FILES", files)
            got = z.Array.open(z.FilesystemStore(tmp_path).resolve("t")).read(off, shp)
            np.testing.assert_array_equal(got, want, err_msg=f"ZH_FILES={files}")


def test_truncated_whole_shard_with_host_codec(dev, tmp_path):
    """a whole shard with an inner host codec (zstd) whose file was cut short is
    the file as it is (decodePartial → chunkHandle.read() → ByteBufferDataProvider,
    ShardingIndexedCodec.java:246-251, 301-331): the entry beyond its bytes is an error — the
    device's "Could not load byte data for chunk [..]" (DESIGN quirk Q14) — never a
    zero-padded range decoded on the host.  A part of the same shard still reads its other
    inner chunks."""
    import zarrhip as z
    data = np.arange(16 * 16 * 16, dtype=np.uint32).reshape(16, 16, 16) + 1
    m = (z.ArrayMetadataBuilder().withShape(16, 16, 16).withDataType(z.DataType.UINT32)
         .withChunkShape(8, 8, 8).withFillValue(0)
         .withCodecs(lambda c: c.withSharding([4, 8, 8], lambda c1: c1.withZstd(),
                                              index_location="start")).build())
    h = z.FilesystemStore(tmp_path).resolve("a")
    z.Array.create(h, m).write(None, data)
    a = z.Array.open(h)
    p = tmp_path / "a" / "c" / "0" / "0" / "0"
    assert p.exists()
    os.truncate(p, os.path.getsize(p) - 3)  # the last inner chunk's zstd frame loses 3 bytes
    with pytest.raises(z.ZarrException) as e:
        a.read([0, 0, 0], [8, 8, 8])
    assert str(e.value).startswith("Could not load byte data for chunk [")
    np.testing.assert_array_equal(a.read([0, 0, 0], [4, 8, 8]), data[0:4, 0:8, 0:8])


def test_write_files_symlink_mode_and_stale_temporaries(dev, tmp_path, wmode):
    """ADVICE r05 / DESIGN Q15: FilesystemStore.set opens the chunk's path and writes it in place
    (FilesystemStore.java:116-121); the library writes a temporary file and renames it, and so
    (a) a chunk path that is a symlink is written through — the link stays, its target gets the
    bytes; (b) an existing chunk file keeps its permission bits; (c) a temporary file a dead
    writer left beside a chunk is removed when that chunk is written next (it would otherwise
    show up in FilesystemStore.list), while one of a live process is left alone."""
    import subprocess
    shape = [16, 16, 24]
    meta = A.make_meta(shape, [8, 16, 24], 4, **WCHAINS["sharded_t"])
    arr = rand_array(shape, 4, seed=191, fill_frac=0.0)
    want = encode_oracle(meta, arr)
    coords = chunk_coords(meta, [0, 0, 0], shape)
    paths = [str(tmp_path / "s" / "c" / "/".join(map(str, c))) for c in coords]
    for p in paths:
        os.makedirs(os.path.dirname(p), exist_ok=True)
    real = tmp_path / "elsewhere"
    real.write_bytes(b"old")
    os.symlink(real, paths[0])                      # (a)
    with open(paths[1], "wb") as f:                 # (b)
        f.write(b"old")
    os.chmod(paths[1], 0o640)
    dead = subprocess.Popen(["true"])
    dead.wait()
    stale = paths[1] + f".zhtmp{dead.pid}.0"        # (c) a dead writer's leftover
    live = paths[1] + f".zhtmp{os.getppid()}.0"     # a live process's: not ours to remove
    for q in (stale, live):
        with open(q, "wb") as f:
            f.write(b"partial")
    dev.array_write_files(meta, arr.ctypes.data, [0, 0, 0], shape, paths)
    assert os.path.islink(paths[0]) and real.read_bytes() == want[0]
    assert open(paths[1], "rb").read() == want[1]
    assert (os.stat(paths[1]).st_mode & 0o777) == 0o640
    assert not os.path.exists(stale) and os.path.exists(live)
    os.unlink(live)
    assert not _tmp_leftovers(tmp_path)
