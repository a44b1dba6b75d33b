"""Concurrent codec-path calls (the reference's ForkJoin threads call the sharding codec once
per shard, M/core/Array.java:403-407): threads decoding different shards through a pool of
contexts on one GPU (the Java side's ZH_CODEC_CONTEXTS pool, ZarrHip.codecCtx) and through one
shared context (calls serialise on its mutex) give the oracle's bytes."""
import ctypes as C
import threading

import numpy as np
import pytest

import oracle as O
from helpers import encode_oracle, rand_array
from zarrhip import _abi as A
from zarrhip._lib import DeviceContext, i32arr, i64arr

pytestmark = pytest.mark.gpu


def _decode_partial(ctx, meta, shard, off, shp):
    out = (C.c_char * (int(np.prod(shp)) * 4))()
    buf = (C.c_char * len(shard)).from_buffer_copy(shard)
    err = C.create_string_buffer(512)
    st = ctx.L.zh_sharding_decode_partial(ctx.h, C.byref(meta), buf, len(shard), i64arr(off),
                                          i32arr(shp), out, 0, None, err, 512)
    assert st == 0, err.value
    return np.frombuffer(bytes(out), np.uint32).reshape(shp)


@pytest.mark.parametrize("ncontexts", [1, 4])
def test_threads_decode_shards_concurrently(dev, ncontexts):
    shape = [1, 64, 64, 64]
    meta = A.make_meta(shape, [1, 32, 32, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 8, 8, 16], transpose_order=[0, 3, 2, 1])
    arr = rand_array(shape, 4, seed=31)
    shards = encode_oracle(meta, arr)
    smeta = A.zh_array_meta.from_buffer_copy(meta)
    for d in range(4):
        smeta.shape[d] = meta.chunk_shape[d]
    ctxs = [dev] + [DeviceContext(0) for _ in range(ncontexts - 1)]
    jobs = [(i, [0, 3 * (k % 5), 2 * (k % 7), k % 9], [1, 20, 20, 40])
            for k, i in enumerate(list(range(len(shards))) * 4)]
    results, errors = {}, []

    def work(t):
        try:
            ctx = ctxs[t % len(ctxs)]
            for j in range(t, len(jobs), 8):
                i, off, shp = jobs[j]
                results[j] = _decode_partial(ctx, smeta, shards[i], off, shp)
        except Exception as e:  # surfaced below
            errors.append(e)
    th = [threading.Thread(target=work, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for c in ctxs[1:]:
        c.close()
    assert not errors, errors
    for j, (i, off, shp) in enumerate(jobs):
        want = np.frombuffer(O.array_read(smeta, [shards[i]], off, shp), np.uint32).reshape(shp)
        np.testing.assert_array_equal(results[j], want)


def test_gather_blocks(dev):
    """zh_gather_blocks (the bench's shuffled-layout helper) against numpy indexing."""
    rng = np.random.default_rng(5)
    nb, bb = 37, 4096
    src_h = rng.integers(0, 256, nb * bb, dtype=np.uint8)
    perm = rng.permutation(nb)
    src, dst = dev.malloc(nb * bb), dev.malloc(nb * bb)
    dev.h2d(src, src_h.tobytes())
    dev.gather_blocks(dst, src, bb, perm.tolist())
    got = np.frombuffer(dev.d2h(dst, nb * bb), np.uint8).reshape(nb, bb)
    dev.free(src)
    dev.free(dst)
    np.testing.assert_array_equal(got, src_h.reshape(nb, bb)[perm])


@pytest.mark.parametrize("ncontexts", [1, 4])
@pytest.mark.parametrize("pipelined", [False, True])
def test_threads_read_files_concurrently(dev, tmp_path, monkeypatch, ncontexts, pipelined):
    """HipShardingIndexedCodec.decodePartial over a FilesystemStore from eight threads
    (zh_array_read_files on the shard viewed as a one-chunk array): the process-wide file table
    and the contexts' pipelines under concurrent calls give the oracle's bytes."""
    if pipelined:
        monkeypatch.setenv("ZH_PIPE_MIN_KB", "1")
        monkeypatch.setenv("ZH_PIPE_SLAB_KB", "16")
        monkeypatch.setenv("ZH_PIPE_CHUNK_KB", "64")
        monkeypatch.setenv("ZH_PIPE_THREADS", "2")
    shape = [1, 64, 64, 64]
    meta = A.make_meta(shape, [1, 32, 32, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 8, 8, 16], transpose_order=[0, 3, 2, 1])
    arr = rand_array(shape, 4, seed=37)
    shards = encode_oracle(meta, arr)
    paths = []
    for i, s in enumerate(shards):
        p = str(tmp_path / f"s{i}")
        with open(p, "wb") as f:
            f.write(s)
        paths.append(p)
    smeta = A.zh_array_meta.from_buffer_copy(meta)
    for d in range(4):
        smeta.shape[d] = meta.chunk_shape[d]
    ctxs = [dev] + [DeviceContext(0) for _ in range(ncontexts - 1)]
    jobs = [(i, [0, 3 * (k % 5), 2 * (k % 7), k % 9], [1, 20, 20, 40])
            for k, i in enumerate(list(range(len(shards))) * 4)]
    results, errors = {}, []

    def work(t):
        try:
            ctx = ctxs[t % len(ctxs)]
            for j in range(t, len(jobs), 8):
                i, off, shp = jobs[j]
                out = np.empty(shp, np.uint32)
                ctx.array_read_files(smeta, [paths[i]], off, shp, out.ctypes.data)
                results[j] = out
        except Exception as e:  # surfaced below
            errors.append(e)
    th = [threading.Thread(target=work, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for c in ctxs[1:]:
        c.close()
    assert not errors, errors
    for j, (i, off, shp) in enumerate(jobs):
        want = np.frombuffer(O.array_read(smeta, [shards[i]], off, shp), np.uint32).reshape(shp)
        np.testing.assert_array_equal(results[j], want)


@pytest.mark.parametrize("sharded", [False, True])
def test_concurrent_writes_different_chunks(tmp_path, sharded):
    """ParallelWriteTest.testConcurrentWritesDifferentChunks (ParallelWriteTest.java:91-153):
    eight threads call write on one Array instance, each a different 50² chunk (sharded: a
    different 50² shard of 25² inner chunks) with its own value; the array then reads back
    every chunk's value, and every element, through the library's file writes and reads."""
    from concurrent.futures import ThreadPoolExecutor
    import zarrhip as z
    n, cs = 10, 50
    b = (z.ArrayMetadataBuilder().withShape(n * cs, n * cs).withDataType(z.DataType.INT32)
         .withChunkShape(cs, cs).withFillValue(-1))
    if sharded:
        b = b.withCodecs(lambda c: c.withSharding([25, 25], lambda c1: c1.withBytes("LITTLE")))
    arr = z.Array.create(z.FilesystemStore(tmp_path).resolve("concurrent_write_safety"), b.build())

    def task(ij):
        i, j = ij
        arr.write([i * cs, j * cs], np.full((cs, cs), i * n + j, np.int32), False)

    with ThreadPoolExecutor(8) as ex:
        list(ex.map(task, [(i, j) for i in range(n) for j in range(n)]))
    got = arr.read()
    want = np.repeat(np.repeat(np.arange(n * n, dtype=np.int32).reshape(n, n), cs, 0), cs, 1)
    np.testing.assert_array_equal(got, want)
