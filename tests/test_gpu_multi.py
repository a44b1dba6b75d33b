"""zh_array_read_multi (one region read split over several device contexts in one process)
vs the oracle, bit-exact.  On a one-GPU box the contexts are several zh_ctx on device 0:
the split, the per-slab chunk selection, the concurrent host threads, the host-terminated
slices and the root gather (a same-device copy, or the no-peer staged route when forced)
are exercised.  When the box has several GPUs, test_multi_distinct_devices puts one context
on each and asserts the xGMI (or staged) route that ran."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from helpers import chunk_coords, encode_oracle, rand_array, shape_of
from zarrhip import _abi as A
from zarrhip._lib import DeviceContext, ZhError, array_read_multi, device_count

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
        routes = array_read_multi(ctxs, meta, bufs, off, shp, out, flags, root=root)
    else:
        keep, hs = _host_srcs(srcs)
        routes = array_read_multi(ctxs, meta, hs, off, shp, out, A.ZH_OUT_DEVICE, root=root)
    # one device: the root slab decodes in place, the others copy within the device
    assert routes == [A.ZH_ROUTE_DIRECT if r == root else A.ZH_ROUTE_SAME for r in range(3)]
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
    # zh_last_data_error: the failing shard's grid coords, the index crc32c's key (~0)
    last = chunk_coords(meta, off, shp)[-1]
    assert ed.value.position == (tuple(last), 2 ** 64 - 1)


def test_data_error_position_is_the_sequential_first(ctxs):
    """Two corrupt shards, one plan and one multi-context read: the error raised and its
    position (zh_last_data_error: what the multi-rank API orders ranks by) are the first
    corrupt shard's in C order, as the oracle's sequential read reports."""
    meta = _meta()
    arr = rand_array(shape_of(meta), 4, seed=83)
    shards = encode_oracle(meta, arr)
    off, shp = [0, 0, 0, 0], [1, 96, 64, 80]
    cc = chunk_coords(meta, off, shp)
    srcs = _sources(meta, shards, off, shp)
    for k in (4, 2):
        bad = bytearray(srcs[k])
        bad[-10] ^= 0x40
        srcs[k] = bytes(bad)
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, srcs, off, shp)
    keep, hs = _host_srcs(srcs)
    nb = int(np.prod(shp)) * 4
    out = (C.c_char * nb)()
    dev = ctxs[0]
    with pytest.raises(ZhError) as e1:
        dev.array_read(meta, hs, off, shp, C.addressof(out), 0)
    with pytest.raises(ZhError) as e3:
        array_read_multi(ctxs, meta, hs, off, shp, C.addressof(out), 0)
    for e in (e1, e3):
        assert str(e.value) == str(eo.value)
        assert e.value.position == (tuple(cc[2]), 2 ** 64 - 1)
    # reported once: a later error without a position does not inherit this one
    from zarrhip._lib import last_data_error
    assert last_data_error() is None


@pytest.mark.parametrize("src_device", [False, True])
def test_multi_forced_staged_route(ctxs, src_device, monkeypatch):
    """The no-peer fallback (D2H into pinned host memory, H2D on a fresh stream of the root
    device; device sources staged to the slab's device first), forced on one GPU."""
    monkeypatch.setenv("ZH_MULTI_FORCE_STAGED", "1")
    meta = _meta()
    arr = rand_array(shape_of(meta), 4, seed=83)
    shards = encode_oracle(meta, arr)
    off, shp = [0, 1, 2, 3], [1, 94, 61, 70]
    srcs = _sources(meta, shards, off, shp)
    want = np.frombuffer(O.array_read(meta, srcs, off, shp), np.uint32).reshape(shp)
    dev = ctxs[0]
    nbytes = int(np.prod(shp)) * 4
    out = dev.malloc(nbytes)
    dev.memset(out, 0xA5, nbytes)
    bufs = []
    if src_device:
        for s in srcs:
            b = dev.malloc(len(s))
            dev.h2d(b, s)
            bufs.append((b, len(s)))
        routes = array_read_multi(ctxs, meta, bufs, off, shp, out,
                                  A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
    else:
        keep, hs = _host_srcs(srcs)
        routes = array_read_multi(ctxs, meta, hs, off, shp, out, A.ZH_OUT_DEVICE)
    got = np.frombuffer(dev.d2h(out, nbytes), np.uint32).reshape(shp)
    dev.free(out)
    for b, _ in bufs:
        dev.free(b)
    np.testing.assert_array_equal(got, want)
    src_flag = A.ZH_ROUTE_SRC_STAGED if src_device else 0
    assert routes == [A.ZH_ROUTE_DIRECT] + [A.ZH_ROUTE_STAGED | src_flag] * 2


@pytest.mark.skipif(device_count() < 2, reason="one GPU on this box (the node run covers it)")
@pytest.mark.parametrize("peer", ["1", "0"])
def test_multi_distinct_devices(peer, monkeypatch):
    """One context per visible GPU (up to 8): root gather of a region read with device
    sources on the root, vs the oracle; the non-root slabs must report the xGMI route when
    the pair has peer access (peer=1) and the staged route when it is forced off
    (ZH_MULTI_FORCE_STAGED=1)."""
    monkeypatch.setenv("ZH_MULTI_FORCE_STAGED", "0" if peer == "1" else "1")
    nd = min(8, device_count())
    cs = [DeviceContext(d) for d in range(nd)]
    try:
        meta = A.make_meta([1, 128, 64, 80], [1, 32, 32, 64], 4, endian=A.ZH_ENDIAN_BIG,
                           sharded=True, inner_chunk_shape=[1, 8, 16, 16],
                           transpose_order=[0, 3, 2, 1])
        arr = rand_array(shape_of(meta), 4, seed=89)
        shards = encode_oracle(meta, arr)
        off, shp = [0, 0, 1, 2], [1, 128, 60, 77]
        srcs = _sources(meta, shards, off, shp)
        want = np.frombuffer(O.array_read(meta, srcs, off, shp), np.uint32).reshape(shp)
        root = cs[0]
        nbytes = int(np.prod(shp)) * 4
        out = root.malloc(nbytes)
        bufs = []
        for s in srcs:
            b = root.malloc(len(s))
            root.h2d(b, s)
            bufs.append((b, len(s)))
        routes = array_read_multi(cs, meta, bufs, off, shp, out,
                                  A.ZH_SRC_DEVICE | A.ZH_OUT_DEVICE)
        got = np.frombuffer(root.d2h(out, nbytes), np.uint32).reshape(shp)
        root.free(out)
        for b, _ in bufs:
            root.free(b)
        np.testing.assert_array_equal(got, want)
        assert routes[0] == A.ZH_ROUTE_DIRECT
        for r in routes[1:]:
            if peer == "0":
                assert r == A.ZH_ROUTE_STAGED | A.ZH_ROUTE_SRC_STAGED
            else:
                assert r in (A.ZH_ROUTE_PEER | A.ZH_ROUTE_SRC_PEER,
                             A.ZH_ROUTE_STAGED | A.ZH_ROUTE_SRC_STAGED)
        # host-terminated over the same devices (each slab over its own link)
        keep, hs = _host_srcs(srcs)
        hout = (C.c_char * nbytes)()
        routes = array_read_multi(cs, meta, hs, off, shp, C.addressof(hout), 0)
        assert routes == [A.ZH_ROUTE_DIRECT] * nd
        np.testing.assert_array_equal(np.frombuffer(bytes(hout), np.uint32).reshape(shp), want)
    finally:
        for c in cs:
            c.close()
