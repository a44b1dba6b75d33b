"""zh_array_read_multi (one region read split over several device contexts in one process)
vs the oracle, bit-exact.  The box has one GPU, so the contexts are several zh_ctx on
device 0: the split, the per-slab chunk selection, the concurrent host threads, the
host-terminated slices and the root gather (hipMemcpyPeerAsync, here within one device)
are exercised; on a node the same contexts sit on different GPUs."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from helpers import chunk_coords, encode_oracle, rand_array, shape_of
from zarrhip import _abi as A
from zarrhip._lib import DeviceContext, ZhError, array_read_multi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    cs = [DeviceContext(0) for _ in range(3)]
    yield cs
    for c in cs:
        c.close()


def _meta():
    return A.make_meta([1, 96, 64, 80], [1, 32, 32, 64], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 8, 16, 16], transpose_order=[0, 3, 2, 1])


def _sources(meta, shards, off, shp):
    pos = {c: i for i, c in enumerate(chunk_coords(meta, [0] * meta.ndim, shape_of(meta)))}
    return [shards[pos[c]] for c in chunk_coords(meta, off, shp)]


def _host_srcs(srcs):
    keep = [(C.c_char * len(s)).from_buffer_copy(s) if s is not None else None for s in srcs]
    return keep, [(C.addressof(k), len(s)) if s is not None else (None, 0)
                  for k, s in zip(keep, srcs)]


REGIONS = [([0, 0, 0, 0], [1, 96, 64, 80]), ([0, 5, 3, 7], [1, 83, 50, 61]),
           ([0, 40, 0, 0], [1, 2, 64, 80])]


@pytest.mark.parametrize("region", range(len(REGIONS)))
@pytest.mark.parametrize("ndev", [1, 2, 3])
def test_multi_host_terminated(ctxs, region, ndev):
    meta = _meta()
    arr = rand_array(shape_of(meta), 4, seed=71)
    arr[0, 0:8, 0:16, 0:16] = 0
    shards = encode_oracle(meta, arr)
    shards[1] = None
    off, shp = REGIONS[region]
    srcs = _sources(meta, shards, off, shp)
    want = np.frombuffer(O.array_read(meta, srcs, off, shp), np.uint32).reshape(shp)
    keep, hs = _host_srcs(srcs)
    out = (C.c_char * (int(np.prod(shp)) * 4))()
    array_read_multi(ctxs[:ndev], meta, hs, off, shp, C.addressof(out), 0)
    np.testing.assert_array_equal(np.frombuffer(bytes(out), np.uint32).reshape(shp), want)


@pytest.mark.parametrize("root", [0, 2])
@pytest.mark.parametrize("src_device", [False, True])
def test_multi_root_gather_on_device(ctxs, root, src_device):
    meta = _meta()
    arr = rand_array(shape_of(meta), 4, seed=73)
    shards = encode_oracle(meta, arr)
    off, shp = [0, 3, 1, 2], [1, 90, 60, 77]
    srcs = _sources(meta, shards, off, shp)
    want = np.frombuffer(O.array_read(meta, srcs, off, shp), np.uint32).reshape(shp)
    dev = ctxs[root]
    nbytes = int(np.prod(shp)) * 4
    out = dev.malloc(nbytes)
    bufs = []
    if src_device:
        for s in srcs:
            b = dev.malloc(len(s))
            dev.h2d(b, s)
            bufs.append((b, len(s)))
        flags = A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE
        array_read_multi(ctxs, meta, bufs, off, shp, out, flags, root=root)
    else:
        keep, hs = _host_srcs(srcs)
        array_read_multi(ctxs, meta, hs, off, shp, out, A.ZH_OUT_DEVICE, root=root)
    got = np.frombuffer(dev.d2h(out, nbytes), np.uint32).reshape(shp)
    dev.free(out)
    for b, _ in bufs:
        dev.free(b)
    np.testing.assert_array_equal(got, want)


def test_multi_error_is_first_failing_slab(ctxs):
    """A corrupt index in a shard only the last slab reads: the oracle's message."""
    meta = _meta()
    arr = rand_array(shape_of(meta), 4, seed=79)
    shards = encode_oracle(meta, arr)
    off, shp = [0, 0, 0, 0], [1, 96, 64, 80]
    srcs = _sources(meta, shards, off, shp)
    bad = bytearray(srcs[-1])
    bad[-10] ^= 0x40                     # inside the index (at the end), under its crc32c
    srcs[-1] = bytes(bad)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, srcs, off, shp)
    keep, hs = _host_srcs(srcs)
    out = (C.c_char * (int(np.prod(shp)) * 4))()
    with pytest.raises(ZhError) as ed:
        array_read_multi(ctxs, meta, hs, off, shp, C.addressof(out), 0)
    assert str(ed.value) == str(eo.value)
