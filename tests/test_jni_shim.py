"""The JNI shim (zarr-java_amd/java/jni/zarrhip_jni.c) executed: compiled against the test-only
stand-in jni.h and driven through a fake JNIEnv (tests/jni/, tests/jni_harness.py).  No JDK
exists here or on the GPU box, so this is the shim's only execution; it checks what a JVM would
hold the shim to and what zarr-java's callers see:
  - every entry point's results equal the oracle (GPU cases);
  - each GetPrimitiveArrayCritical has its Release, no JNI call happens inside a critical
    section, sources are released with JNI_ABORT (and, in copy mode, never written), the
    result with mode 0;
  - the critical windows follow the slab policy (ZH_JNI_SLAB_MB: one window per slab);
  - ZH_EDATA surfaces as dev.zarr.zarrjava.ZarrException with the reference's text,
    ZH_EINVAL as IllegalArgumentException, other failures as RuntimeException.
Reference surface: core.Array.read (M/core/Array.java:378-441), ShardingIndexedCodec.decode /
decodePartial (M/v3/codec/core/ShardingIndexedCodec.java:98-103, 245-255), Crc32cCodec.decode
(M/v3/codec/core/Crc32cCodec.java:24-48)."""
import ctypes as C
import os
import struct

import numpy as np
import pytest

import oracle as O
from helpers import NP_DT, chunk_coords, encode_oracle, jni_fetch, rand_array
from jni_harness import FakeJVM, JavaException, jni_lib
from zarrhip import _abi as A
from zarrhip._lib import lib, shard_ranges

ZE = "dev/zarr/zarrjava/ZarrException"
IAE = "java/lang/IllegalArgumentException"
RTE = "java/lang/RuntimeException"


def _case(chain="c4", shape=(24, 32, 48), seed=3, dsize=4):
    kw = {"c3": dict(sharded=True, inner_chunk_shape=[4, 8, 8], endian=A.ZH_ENDIAN_BIG),
          "c4": dict(sharded=True, inner_chunk_shape=[4, 8, 8], transpose_order=[2, 0, 1],
                     endian=A.ZH_ENDIAN_BIG),
          "crc": dict(sharded=True, inner_chunk_shape=[4, 8, 8], inner_crc32c=True,
                      transpose_order=[1, 2, 0], endian=A.ZH_ENDIAN_BIG),
          "start": dict(sharded=True, inner_chunk_shape=[4, 8, 8],
                        index_location=A.ZH_INDEX_START, index_endian=A.ZH_ENDIAN_BIG),
          "nested": dict(sharded=True, inner_chunk_shape=[8, 8, 8], nested_chunk_shape=[4, 4, 8]),
          "bytes": dict(endian=A.ZH_ENDIAN_BIG)}[chain]
    shape = list(shape)
    meta = A.make_meta(shape, [8, 16, 24], dsize, fill=(7).to_bytes(dsize, "little"), **kw)
    arr = rand_array(shape, dsize, seed=seed, fill_frac=0.2, fill=0)
    if kw.get("sharded"):
        arr[:4, :8, :8] = 0  # an all-zero inner chunk: Q1 through a missing entry
    return meta, arr, encode_oracle(meta, arr)


def _oracle(meta, shards, off, shp):
    n = meta.ndim
    allc = chunk_coords(meta, [0] * n, [meta.shape[d] for d in range(n)])
    pos = {c: i for i, c in enumerate(allc)}
    srcs = [shards[pos[c]] for c in chunk_coords(meta, off, shp)]
    return np.frombuffer(O.array_read(meta, srcs, off, shp), NP_DT[meta.dtype_size]).reshape(shp)


def _region_chunks(meta, shards, off, shp):
    n = meta.ndim
    allc = chunk_coords(meta, [0] * n, [meta.shape[d] for d in range(n)])
    pos = {c: i for i, c in enumerate(allc)}
    return [shards[pos[c]] for c in chunk_coords(meta, off, shp)]


def _write_store(tmp_path, shards):
    paths = []
    for i, s in enumerate(shards):
        p = str(tmp_path / f"c{i}")
        if s is not None:
            with open(p, "wb") as f:
                f.write(s)
        paths.append(p if s is not None else None)
    return paths


def _index_of(meta, shard):
    isz = lib().zh_shard_index_size(C.byref(meta))
    return shard[:isz] if meta.chain.index_location == A.ZH_INDEX_START else shard[-isz:]


@pytest.fixture
def slab_mb(monkeypatch):
    def set_(mb):
        if mb is None:
            monkeypatch.delenv("ZH_JNI_SLAB_MB", raising=False)
        else:
            monkeypatch.setenv("ZH_JNI_SLAB_MB", str(mb))
    return set_


# ---- CPU: the shim without a device ---------------------------------------------------------
def test_shim_exports_every_native_method():
    """Every native method ZarrHip.java declares has its JNI symbol in the shim."""
    src = open(os.path.join(os.path.dirname(__file__), "..", "zarr-java_amd", "java", "src",
                            "main", "java", "dev", "zarr", "zarrjava", "hip", "ZarrHip.java")).read()
    import re
    names = re.findall(r"static native \S+ (\w+)\(", src)
    assert len(names) >= 9
    L = jni_lib()
    for n in names:
        assert hasattr(L, "Java_dev_zarr_zarrjava_hip_ZarrHip_" + n), n


@pytest.mark.parametrize("chain", ["c3", "start", "nested"])
def test_shard_ranges_through_the_shim(chain):
    """shardRanges (ShardPieces.part's call) returns zh_shard_ranges' ranges, reads the index
    outside any critical section, and with checkIndex fails a corrupt index with the
    reference's ZarrException before any range is named."""
    meta, arr, shards = _case(chain)
    idx = _index_of(meta, shards[0])
    size = len(shards[0])
    jvm = FakeJVM()
    for lo, hi, run in [([0, 0, 0], [8, 16, 24], 1 << 20), ([1, 3, 5], [7, 11, 20], 0)]:
        assert jvm.shard_ranges(meta, idx, size, lo, hi, run) == \
            shard_ranges(meta, idx, size, lo, hi, run)
        assert jvm.shard_ranges(meta, idx, -1, lo, hi, run, check=True) == \
            shard_ranges(meta, idx, -1, lo, hi, run)
    bad = bytearray(shards[0])
    pos = 3 if chain == "start" else len(bad) - len(idx) + 3
    bad[pos] ^= 0x40
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, [bytes(bad)], [0, 0, 0], [8, 16, 24])
    with pytest.raises(JavaException) as ej:
        jvm.shard_ranges(meta, _index_of(meta, bytes(bad)), -1, [0, 0, 0], [8, 16, 24], 0,
                         check=True)
    assert ej.value.cls == ZE and ej.value.msg == str(eo.value)
    # without the check the shim never reads the index's crc32c (the device does)
    assert jvm.shard_ranges(meta, _index_of(meta, bytes(bad)), -1, [0, 0, 0], [8, 16, 24], 0)
    s = jvm.check_rules()
    assert s.gets == 0  # shardRanges copies the index: no critical section at all


def test_error_mapping_without_device(slab_mb):
    """Status → exception class: a bad transpose order (ZH_EINVAL from zh_validate_meta) →
    IllegalArgumentException; an output array of the wrong length → IllegalArgumentException
    before anything is held; no GPU context → RuntimeException from ctxCreate when no device
    is visible."""
    meta, arr, shards = _case("c4")
    jvm = FakeJVM()
    bad = A.make_meta([24, 32, 48], [8, 16, 24], 4, sharded=True, inner_chunk_shape=[4, 8, 8],
                      transpose_order=[0, 0, 1])
    with pytest.raises(JavaException) as e:
        jvm.array_read_pieces([0], bad, [None], [0, 0, 0], [8, 16, 24])
    assert e.value.cls in (IAE, ZE)
    # wrong output length: the JNI checks it against the region
    nel = 8 * 16 * 24
    out = jvm.output(4, nel - 1)
    args = jvm.meta_args(meta) + (jvm.objs([None], b"[B"), jvm.longs([0, 0, 0]),
                                  jvm.longs([8, 16, 24]), out)
    rc = jvm._fn("arrayRead")(C.c_void_p(jvm.env), None, C.c_int64(0), *map(C.c_void_p, args))
    exc = jvm.exception()
    assert exc is not None and exc.cls == IAE and "does not match" in exc.msg and rc != 0
    s = jvm.check_rules()
    assert s.gets == 0
    jvm.outputs.clear()


@pytest.mark.parametrize("mb", [None, 1])
def test_pieces_critical_bookkeeping_without_device(slab_mb, mb):
    """arrayReadPieces with no context (status ZH_EINVAL from the library): the shim still
    collects the first slab's arrays, enters and leaves every critical section (sources
    JNI_ABORT, the result 0), stops at that slab and throws IllegalArgumentException."""
    slab_mb(mb)
    shape = [64, 64, 96]  # 1.5 MiB of uint32: two slabs at ZH_JNI_SLAB_MB=1
    meta, arr, shards = _case("c4", shape=shape, seed=5)
    fetched = [(None, len(s), [(0, s)]) if s is not None else None
               for s in _region_chunks(meta, shards, [0, 0, 0], shape)]
    jvm = FakeJVM()
    with pytest.raises(JavaException) as e:
        jvm.array_read_pieces([0], meta, fetched, [0, 0, 0], shape)
    assert e.value.cls == IAE
    s = jvm.check_rules()
    assert s.windows == 1 and s.gets >= 2


@pytest.mark.parametrize("mb", [None, 1])
def test_files_critical_bookkeeping_without_device(tmp_path, slab_mb, mb):
    """arrayReadFiles with no context: every path string is converted and released before the
    first critical section, only the result is held (mode 0) and the library's ZH_EINVAL
    surfaces as IllegalArgumentException."""
    slab_mb(mb)
    shape = [64, 64, 96]
    meta, arr, shards = _case("c4", shape=shape, seed=5)
    paths = _write_store(tmp_path, _region_chunks(meta, shards, [0, 0, 0], shape))
    jvm = FakeJVM()
    with pytest.raises(JavaException) as e:
        jvm.array_read_files(0, meta, paths, [0, 0, 0], shape)
    assert e.value.cls == IAE
    s = jvm.check_rules()
    assert s.windows == 1 and s.gets == 1
    assert s.string_gets == sum(p is not None for p in paths)


def test_array_write_declines_a_mismatched_array():
    """arrayWrite returns null (the caller keeps core.Array.write) when the Java array's length
    is not the region's, without entering a critical section."""
    meta, arr, shards = _case("c3")
    jvm = FakeJVM()
    data = jvm.prim(b"I", np.zeros(10, np.int32))
    args = jvm.meta_args(meta) + (jvm.longs([0, 0, 0]), jvm.longs([24, 32, 48]), data)
    r = jvm._fn("arrayWrite")(C.c_void_p(jvm.env), None, C.c_int64(0), *map(C.c_void_p, args))
    assert not r and jvm.exception() is None
    assert jvm.check_rules().gets == 0


# ---- GPU: every entry point against the oracle -----------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("chain", ["c3", "c4", "crc", "start", "nested"])
@pytest.mark.parametrize("mb", [None, 1])
def test_array_read_pieces_via_shim(dev, tmp_path, slab_mb, chain, mb):
    """HipArray.read's sharded path: ShardPieces' store I/O (jni_fetch), then arrayReadPieces;
    whole shards, sub-shard parts, a missing shard, one element.  ZH_JNI_SLAB_MB=1 cuts the
    64×32×48 region into slabs (one critical window each)."""
    slab_mb(mb)
    shape = [64, 32, 48]
    meta, arr, shards = _case(chain, shape=shape, seed=7)
    shards[1] = None
    paths = _write_store(tmp_path, shards)
    n = meta.ndim
    allc = chunk_coords(meta, [0] * n, shape)
    pos = {c: i for i, c in enumerate(allc)}
    jvm = FakeJVM()
    windows = 0
    for off, shp in [([0, 0, 0], shape), ([3, 5, 7], [57, 20, 33]), ([9, 17, 0], [1, 1, 1])]:
        rp = [paths[pos[c]] for c in chunk_coords(meta, off, shp)]
        fetched = jni_fetch(meta, rp, off, shp, max_run=64 << 20)
        rc, got = jvm.array_read_pieces([dev.h.value], meta, fetched, off, shp)
        assert rc == 0
        np.testing.assert_array_equal(got, _oracle(meta, shards, off, shp))
        s = jvm.check_rules()
        slabs = s.windows - windows
        windows = s.windows
        row = 4 * int(np.prod(shp[1:]))
        if mb == 1 and shp[0] * row > (1 << 20):
            assert slabs > 1
        else:
            assert slabs == 1


@pytest.mark.gpu
@pytest.mark.parametrize("chain", ["c3", "c4", "crc", "start", "nested", "bytes"])
@pytest.mark.parametrize("mb", [None, 1])
def test_array_read_files_via_shim(dev, tmp_path, slab_mb, chain, mb):
    """HipArray.read over a FilesystemStore: the chunk keys' paths go to arrayReadFiles and the
    library reads the files (zh_array_read_files); whole shards, parts, a missing file, a null
    path, one element.  Only the result is held critical, one window per slab."""
    slab_mb(mb)
    shape = [64, 32, 48]
    meta, arr, shards = _case(chain, shape=shape, seed=13)
    shards[1] = None
    paths = _write_store(tmp_path, shards)
    paths[2] = str(tmp_path / "absent")  # a key without a file: fill, as a null path
    shards[2] = None
    n = meta.ndim
    allc = chunk_coords(meta, [0] * n, shape)
    pos = {c: i for i, c in enumerate(allc)}
    jvm = FakeJVM()
    windows = 0
    for off, shp in [([0, 0, 0], shape), ([3, 5, 7], [57, 20, 33]), ([9, 17, 0], [1, 1, 1])]:
        rp = [paths[pos[c]] for c in chunk_coords(meta, off, shp)]
        rc, got = jvm.array_read_files(dev.h.value, meta, rp, off, shp)
        assert rc == 0
        np.testing.assert_array_equal(got, _oracle(meta, shards, off, shp))
        s = jvm.check_rules()
        assert s.gets == s.windows  # the result only
        slabs = s.windows - windows
        windows = s.windows
        row = 4 * int(np.prod(shp[1:]))
        if mb == 1 and shp[0] * row > (1 << 20):
            assert slabs > 1
        else:
            assert slabs == 1


@pytest.mark.gpu
@pytest.mark.parametrize("chain", ["c4", "start", "nested"])
def test_codec_decode_partial_files_via_shim(dev, tmp_path, chain):
    """HipShardingIndexedCodec.decodePartial over a FilesystemStore: arrayReadFiles on the shard
    viewed as a one-chunk array (shape = the shard shape), one path, a shard-local part."""
    meta, arr, shards = _case(chain, seed=19)
    paths = _write_store(tmp_path, shards)
    sm = A.zh_array_meta.from_buffer_copy(meta)
    for d in range(meta.ndim):
        sm.shape[d] = meta.chunk_shape[d]
    jvm = FakeJVM()
    for lo, part in [([0, 0, 0], [8, 16, 24]), ([1, 3, 5], [6, 9, 17])]:
        rc, got = jvm.array_read_files(dev.h.value, sm, [paths[0]], lo, part)
        assert rc == 0
        want = np.frombuffer(O.array_read(sm, [shards[0]], lo, part),
                             NP_DT[meta.dtype_size]).reshape(part)
        np.testing.assert_array_equal(got, want)
    jvm.check_rules()


@pytest.mark.gpu
def test_array_read_files_errors_via_shim(dev, tmp_path):
    """A corrupt shard index → ZarrException with the reference's CRC text; an unreadable file
    (when not root) → StoreException."""
    meta, arr, shards = _case("c4", seed=17)
    bad = list(shards)
    b = bytearray(bad[0])
    b[-2] ^= 0x10
    bad[0] = bytes(b)
    paths = _write_store(tmp_path, bad)
    off, shp = [0, 0, 0], [8, 16, 24]
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, [bad[0]], off, shp)
    jvm = FakeJVM()
    with pytest.raises(JavaException) as ej:
        jvm.array_read_files(dev.h.value, meta, [paths[0]], off, shp)
    assert ej.value.cls == ZE and ej.value.msg == str(eo.value)
    if os.geteuid() != 0:
        os.chmod(paths[0], 0)
        try:
            with pytest.raises(JavaException) as ej:
                jvm.array_read_files(dev.h.value, meta, [paths[0]], off, shp,
                                     store=(str(tmp_path), f"file://{tmp_path}"))
            assert ej.value.cls == "dev/zarr/zarrjava/store/StoreException"
            key = os.path.relpath(paths[0], tmp_path)
            # StoreException.readFailed (StoreException.java:17-21): store, key, cause
            assert ej.value.msg == (f"Failed to read from store 'file://{tmp_path}' at key "
                                    f"'{key}': {paths[0]}")
        finally:
            os.chmod(paths[0], 0o600)
    jvm.check_rules()


@pytest.mark.gpu
def test_array_read_pieces_host_decoded_via_shim(dev):
    """Pieces whose host stages were undone (DeviceChain.innerHost): the stored lengths and the
    held payloads differ; one range per inner chunk (maxRun 0)."""
    meta, arr, shards = _case("c4", seed=23)
    isz = lib().zh_shard_index_size(C.byref(meta))
    raw = shards[0]
    body = raw[-isz:-4]
    ents = [struct.unpack("<QQ", body[16 * k:16 * k + 16]) for k in range(len(body) // 16)]
    framed, new, p = b"", [], 0
    for o, nb in ents:
        if o == 2 ** 64 - 1:
            new.append((o, nb))
            continue
        fr = b"FRAME!!!" + raw[o:o + nb]  # a stand-in codec frame around each payload
        new.append((p, len(fr)))
        framed += fr
        p += len(fr)
    nbody = b"".join(struct.pack("<QQ", *e) for e in new)
    nidx = nbody + struct.pack("<I", O.crc32c(nbody))
    size = len(framed) + len(nidx)
    off, shp = [2, 3, 4], [5, 11, 17]
    jvm = FakeJVM()
    rs = jvm.shard_ranges(meta, nidx, size, off, [a + b for a, b in zip(off, shp)], 0, check=True)
    pieces = [(o, framed[o + 8:o + nb]) for o, nb in rs]
    rc, got = jvm.array_read_pieces([dev.h.value], meta, [(nidx, size, pieces)], off, shp,
                                    stored_lens=[[nb for _, nb in rs]])
    assert rc == 0
    np.testing.assert_array_equal(got, _oracle(meta, shards, off, shp))
    jvm.check_rules()


@pytest.mark.gpu
@pytest.mark.parametrize("chain", ["c3", "c4", "bytes", "nested"])
@pytest.mark.parametrize("mb", [None, 1])
def test_array_read_via_shim(dev, slab_mb, chain, mb):
    """arrayRead (whole stored chunks from the store; the unsharded path of HipArray.read)."""
    slab_mb(mb)
    shape = [64, 32, 48]
    meta, arr, shards = _case(chain, shape=shape, seed=11)
    jvm = FakeJVM()
    for off, shp in [([0, 0, 0], shape), ([5, 1, 2], [50, 30, 40])]:
        rc, got = jvm.array_read(dev.h.value, meta, _region_chunks(meta, shards, off, shp), off,
                                 shp)
        assert rc == 0
        np.testing.assert_array_equal(got, _oracle(meta, shards, off, shp))
    jvm.check_rules()


@pytest.mark.gpu
@pytest.mark.parametrize("chain", ["c4", "crc", "nested"])
def test_shard_decode_via_shim(dev, slab_mb, chain):
    """HipShardingIndexedCodec's two calls: shardDecodePartial over a whole shard's bytes and
    shardDecodePieces over its index + ranges, for a part of the shard, in slabs."""
    slab_mb(1)
    shape = [64, 32, 48]
    meta, arr, shards = _case(chain, shape=shape, seed=13)
    meta1 = meta
    raw = shards[0]
    lo, part = [1, 2, 3], [7, 13, 20]
    want = np.empty(part, NP_DT[4])
    err = C.create_string_buffer(1024)
    rb = (C.c_char * len(raw)).from_buffer_copy(raw)
    st = O.lib().zo_sharding_decode_partial(C.byref(meta1), rb, len(raw), (C.c_int64 * 3)(*lo),
                                            (C.c_int32 * 3)(*part), C.c_void_p(want.ctypes.data),
                                            1, err, 1024)
    assert st == 0, err.value
    jvm = FakeJVM()
    rc, got = jvm.shard_decode_partial(dev.h.value, meta, raw, lo, part)
    assert rc == 0
    np.testing.assert_array_equal(got, want)
    idx = _index_of(meta, raw)
    rs = shard_ranges(meta, idx, len(raw), lo, [a + b for a, b in zip(lo, part)], 1 << 20)
    rc, got = jvm.shard_decode_pieces(dev.h.value, meta, idx, len(raw),
                                      [(o, raw[o:o + nb]) for o, nb in rs], lo, part)
    assert rc == 0
    np.testing.assert_array_equal(got, want)
    jvm.check_rules()


@pytest.mark.gpu
@pytest.mark.parametrize("chain", ["c3", "c4", "crc", "nested", "bytes"])
def test_array_write_via_shim(dev, slab_mb, chain):
    """HipArray.write → arrayWrite: the region copied out of the heap in slab windows, the
    encoded chunk objects equal the oracle's (null where a chunk is all fill_value)."""
    slab_mb(1)
    shape = [64, 64, 96]  # 1.5 MiB of uint32: two copy windows at ZH_JNI_SLAB_MB=1
    meta, arr, shards = _case(chain, shape=shape, seed=17)
    arr[0:8, 0:16, 0:24] = 7  # one chunk all fill_value: deleted (null)
    want = encode_oracle(meta, arr)
    jvm = FakeJVM()
    got = jvm.array_write(dev.h.value, meta, arr, [0, 0, 0])
    assert got == want and got[0] is None
    s = jvm.check_rules()
    assert s.windows == -(-arr.nbytes // (1 << 20)) == 2


@pytest.mark.gpu
@pytest.mark.parametrize("chain", ["c3", "c4", "crc", "nested", "bytes"])
@pytest.mark.parametrize("mb", [None, 1])
def test_array_write_files_via_shim(dev, tmp_path, slab_mb, chain, mb):
    """HipArray.write over a FilesystemStore: arrayWriteFiles copies the region out of the heap
    in slab windows and the library writes each chunk file (all-fill chunks deleted); the files
    hold the oracle's encoded bytes."""
    slab_mb(mb)
    shape = [64, 32, 48]
    meta, arr, shards = _case(chain, shape=shape, seed=37)
    coords = chunk_coords(meta, [0, 0, 0], shape)
    paths = [str(tmp_path / "s" / "c" / "/".join(map(str, c))) for c in coords]
    jvm = FakeJVM()
    rc = jvm.array_write_files(dev.h.value, meta, arr, [0, 0, 0], paths)
    assert rc == 0
    for p, w in zip(paths, shards):
        if w is None:
            assert not os.path.exists(p)
        else:
            assert open(p, "rb").read() == w
    s = jvm.check_rules()
    nbytes = arr.nbytes
    assert s.windows == (1 if mb is None else -(-nbytes // (1 << 20)))
    # a region that cuts chunks: 3 (the caller's read-modify-write), nothing written
    sub = np.ascontiguousarray(arr[1:9, :16, :24])
    assert jvm.array_write_files(dev.h.value, meta, sub, [1, 0, 0],
                                 [str(tmp_path / "x")]) == 3
    assert not os.path.exists(tmp_path / "x")
    jvm.check_rules()


@pytest.mark.gpu
def test_array_write_files_store_error_via_shim(dev, tmp_path):
    """A chunk path whose parent directory cannot be created (a file is in the way): ZH_EIO →
    dev.zarr.zarrjava.store.StoreException with the store's message; the region's primitive
    array is released (JNI_ABORT) and no critical section stays open."""
    shape = [64, 32, 48]
    meta, arr, shards = _case("c4", shape=shape, seed=41)
    coords = chunk_coords(meta, [0, 0, 0], shape)
    blocker = tmp_path / "blocker"
    blocker.write_bytes(b"x")
    paths = [str(blocker / "c" / "/".join(map(str, c))) for c in coords]
    jvm = FakeJVM()
    with pytest.raises(JavaException) as ej:
        jvm.array_write_files(dev.h.value, meta, arr, [0, 0, 0], paths,
                              store=(str(tmp_path), "file://" + str(tmp_path)))
    assert ej.value.cls == "dev/zarr/zarrjava/store/StoreException"
    # StoreException.writeFailed with FilesystemStore.set's cause (FilesystemStore.java:
    # 107-115): the parent directory that could not be created
    key = os.path.relpath(paths[0], tmp_path)
    assert ej.value.msg == (f"Failed to write to store 'file://{tmp_path}' at key '{key}': "
                            "Failed to create parent directories for path: "
                            f"{os.path.dirname(paths[0])}")
    jvm.check_rules()


@pytest.mark.gpu
def test_data_errors_become_zarr_exceptions(dev, tmp_path):
    """ZH_EDATA → dev.zarr.zarrjava.ZarrException with the oracle's (the reference's) text:
    a corrupt stored index on the device, a missing range ("Could not load byte data")."""
    meta, arr, shards = _case("c4", seed=19)
    bad = bytearray(shards[0])
    bad[len(bad) - 30] ^= 0x04
    shards_bad = [bytes(bad)] + shards[1:]
    paths = _write_store(tmp_path, shards_bad)
    off, shp = [0, 0, 0], [8, 16, 24]
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, [shards_bad[0]], off, shp)
    fetched = jni_fetch(meta, [paths[0]], [1, 0, 0], [7, 16, 24])
    jvm = FakeJVM()
    with pytest.raises(JavaException) as ej:
        jvm.array_read_pieces([dev.h.value], meta, fetched, [1, 0, 0], [7, 16, 24])
    assert ej.value.cls == ZE and ej.value.msg == str(eo.value)
    paths2 = _write_store(tmp_path, shards)
    fetched = jni_fetch(meta, [paths2[0]], [1, 0, 0], [7, 16, 24], drop={(0, 0)})
    with pytest.raises(JavaException) as ej:
        jvm.array_read_pieces([dev.h.value], meta, fetched, [1, 0, 0], [7, 16, 24])
    assert ej.value.cls == ZE and ej.value.msg.startswith("Could not load byte data for chunk")
    jvm.check_rules()


@pytest.mark.gpu
def test_multi_context_reads_via_shim(dev, tmp_path, slab_mb):
    """arrayReadPieces, arrayReadMulti and arrayReadFiles with several contexts (ZarrHip.ctxs()
    under ZH_DEVICES: zh_array_read_pieces_multi / zh_array_read_multi /
    zh_array_read_files_multi, one slab per context); two
    extra contexts on the box's one GPU, slabs of 1 MiB per context."""
    from zarrhip._lib import DeviceContext
    slab_mb(1)
    shape = [64, 32, 48]
    meta, arr, shards = _case("c4", shape=shape, seed=31)
    paths = _write_store(tmp_path, shards)
    c1, c2 = DeviceContext(0), DeviceContext(0)
    try:
        ctxs = [dev.h.value, c1.h.value, c2.h.value]
        jvm = FakeJVM()
        off, shp = [2, 3, 4], [60, 27, 40]
        n = meta.ndim
        allc = chunk_coords(meta, [0] * n, shape)
        pos = {c: i for i, c in enumerate(allc)}
        rp = [paths[pos[c]] for c in chunk_coords(meta, off, shp)]
        fetched = jni_fetch(meta, rp, off, shp, max_run=64 << 20)
        rc, got = jvm.array_read_pieces(ctxs, meta, fetched, off, shp)
        assert rc == 0
        np.testing.assert_array_equal(got, _oracle(meta, shards, off, shp))
        rc, got = jvm.array_read(None, meta, _region_chunks(meta, shards, off, shp), off, shp,
                                 ctxs=ctxs)
        assert rc == 0
        np.testing.assert_array_equal(got, _oracle(meta, shards, off, shp))
        # arrayReadFiles over the same contexts (zh_array_read_files_multi)
        rc, got = jvm.array_read_files(ctxs, meta, rp, off, shp)
        assert rc == 0
        np.testing.assert_array_equal(got, _oracle(meta, shards, off, shp))
        jvm.check_rules()
    finally:
        c1.close()
        c2.close()
