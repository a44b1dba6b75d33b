"""The product's multi-GPU read on one GPU (zarrhip.parallel).

- `Array.read_device` (ZH_OUT_DEVICE) through each store form — the library's own file reads,
  the mirror's store reads, a MemoryStore — equals `Array.read` and the written array;
- `RegionGather` over an NCCL (= RCCL) group of one rank: the device-tensor branch — the root's
  pieces decoded on the side stream by `PlanDecoder` (one plan per piece over device-resident
  shards, on torch's current stream) or `array_decoder` (store reads into device memory),
  assembled in a CUDA byte tensor, and a second run reusing the same plans and buffers.
The point-to-point exchange itself runs on gloo at world sizes 2 and 3 in
tests/test_distributed.py (the same code), and over RCCL in the driver's 8-GPU bench; RCCL
cannot put two ranks on one card."""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if __name__ == "__main__":  # the child process: the paths conftest.py sets for pytest
    for _p in (os.path.join(ROOT, "zarr-java_amd"), os.path.join(ROOT, "oracle"), ROOT,
               os.path.join(ROOT, "tests")):
        sys.path.insert(0, _p)
    import torch  # noqa: F401  before zarrhip loads its library (one HIP runtime)

import numpy as np
import pytest

import oracle as O
import zarrhip as z
from helpers import chunk_coords, encode_oracle, rand_array, shape_of
from zarrhip import _abi as A
from zarrhip import parallel as P

pytestmark = pytest.mark.gpu

SHAPE = [1, 48, 40, 56]


def _metadata():
    return (z.ArrayMetadataBuilder().withShape(*SHAPE).withDataType(z.DataType.UINT32)
            .withChunkShape(1, 16, 40, 32).withFillValue(0)
            .withCodecs(lambda c: c.withSharding(
                [1, 8, 8, 16], lambda c1: c1.withTranspose([0, 3, 2, 1]).withBytes("BIG")))
            .build())


@pytest.fixture
def written(tmp_path):
    data = np.random.default_rng(191).integers(0, 2 ** 32, SHAPE, dtype=np.uint32)
    data[0, 16:32, :, 32:] = 0  # an all-fill shard (deleted on write): reads fill_value
    stores = {"files": z.FilesystemStore(tmp_path / "f"), "mirror": z.FilesystemStore(tmp_path / "m"),
              "memory": z.MemoryStore()}
    for st in stores.values():
        z.Array.create(st.resolve("a"), _metadata()).write(None, data)
    return data, stores


REGIONS = [([0, 0, 0, 0], SHAPE), ([0, 3, 5, 7], [1, 41, 30, 45]), ([0, 20, 1, 33], [1, 1, 1, 1])]


@pytest.mark.parametrize("kind", ["files", "mirror", "memory"])
def test_read_device_matches_read(dev, written, monkeypatch, kind):
    data, stores = written
    if kind == "mirror":
        monkeypatch.setenv("ZH_FILES", "0")
    a = z.Array.open(stores[kind].resolve("a"))
    for off, shp in REGIONS:
        nb = int(np.prod(shp)) * 4
        d = dev.malloc(nb)
        try:
            a.read_device(off, shp, d, dev)
            got = np.frombuffer(dev.d2h(d, nb), np.uint32).reshape(shp)
        finally:
            dev.free(d)
        want = data[tuple(slice(o, o + s) for o, s in zip(off, shp))]
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(got, a.read(off, shp))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_region_gather_nccl_one_rank(written, tmp_path):
    """RegionGather's device branch over an RCCL group of one rank, in a child process that
    imports torch before zarrhip loads its library (one shared HIP runtime, INTEGRATION.md §4;
    this test process loaded the library first): the region in pieces of 8 rows, each decoded
    by its own plan (PlanDecoder over device-resident shards) into its place of the root's CUDA
    region on the side stream, equal to the oracle's read, twice with the same plans and
    buffers; the same region through array_decoder (the files read straight into device
    memory).  In this process (library first): the gloo form, and RegionGather's refusal of a
    device group with a clear message instead of torch's failing CUDA init."""
    import subprocess
    import sys
    import torch.distributed as dist
    data, stores = written
    np.save(tmp_path / "data.npy", data)
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "child", str(tmp_path),
                        str(stores["files"].path), str(_free_port())],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert r.stdout.strip().endswith("child ok"), r.stdout[-2000:]
    from zarrhip import _lib
    _lib.lib()  # loaded by this process's earlier device tests, before torch
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1)
    try:
        g = P.RegionGather([0] * 4, SHAPE, 4, align=8)  # gloo: host tensors, no torch HIP
        assert not g.on_device
        if not _lib.LOADED_AFTER_TORCH:  # a device group here would meet a second HIP runtime
            real = dist.get_backend
            dist.get_backend = lambda group=None: "nccl"
            try:
                with pytest.raises(RuntimeError, match="loaded before torch"):
                    P.RegionGather([0] * 4, SHAPE, 4, align=8)
            finally:
                dist.get_backend = real
    finally:
        dist.destroy_process_group()


def _child(tmp, files_root, port):
    """The child of test_region_gather_nccl_one_rank (torch first)."""
    import torch
    import torch.distributed as dist
    torch.cuda.init()
    torch.cuda.set_device(0)
    from zarrhip import _lib
    from zarrhip._lib import DeviceContext
    data = np.load(os.path.join(tmp, "data.npy"))
    dev = DeviceContext(0)
    assert _lib.LOADED_AFTER_TORCH
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    group = dist.group.WORLD
    meta = A.make_meta(SHAPE, [1, 16, 40, 32], 4, sharded=True, inner_chunk_shape=[1, 8, 8, 16],
                       transpose_order=[0, 3, 2, 1], endian=A.ZH_ENDIAN_BIG)
    shards = encode_oracle(meta, data)
    allc = chunk_coords(meta, [0] * 4, shape_of(meta))
    pos = {c: i for i, c in enumerate(allc)}
    bufs = {}
    for c, s in zip(allc, shards):
        if s is not None:
            p = dev.malloc(len(s))
            dev.h2d(p, s)
            bufs[c] = (p, len(s))

    def sources(po, ps):
        return [bufs.get(c, (None, 0)) for c in chunk_coords(meta, po, ps)]
    for off, shp in REGIONS[:2]:
        g = P.RegionGather(off, shp, 4, group=group, align=8,
                           piece_bytes=8 * shp[2] * shp[3] * 4, device=0)
        assert g.on_device and g.region.is_cuda and len(g.pieces()) > 1
        dec = P.PlanDecoder(dev, meta, sources)
        want = np.frombuffer(O.array_read(meta, [shards[pos[c]] for c in
                                                 chunk_coords(meta, off, shp)], off, shp),
                             np.uint32).reshape(shp)
        for _ in range(2):
            g.region.zero_()
            got = g.run(dec).cpu().numpy().view(np.uint32).reshape(shp)
            np.testing.assert_array_equal(got, want)
        assert len(dec.plans) == len(g.pieces())  # one plan per piece, reused
        dec.close()
    a = z.Array.open(z.FilesystemStore(files_root).resolve("a"))
    off, shp = REGIONS[1]
    out = P.distributed_read(P.array_decoder(a, dev), off, shp, np.uint32, group=group, align=8,
                             piece_bytes=8 * 30 * 45 * 4, device=0)
    assert isinstance(out, torch.Tensor) and out.is_cuda
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(shp),
                                  data[tuple(slice(o, o + s) for o, s in zip(off, shp))])
    # error parity: two shards with a corrupt index crc32c.  Every piece's
    # plan defers its device error to wait(); RegionGather collects them all and raises the one
    # a sequential read meets first — the oracle's text, placed by zh_last_data_error
    corrupt = [c for c in allc if c in bufs][1:3]
    bad_shards = list(shards)
    cbufs = dict(bufs)
    for c in corrupt:
        b = bytearray(shards[pos[c]])
        b[-2] ^= 0x77
        bad_shards[pos[c]] = bytes(b)
        p = dev.malloc(len(b))
        dev.h2d(p, bytes(b))
        cbufs[c] = (p, len(b))
    try:
        O.array_read(meta, [bad_shards[pos[c]] for c in allc], [0] * 4, SHAPE)
        raise AssertionError("the oracle read a corrupt index")
    except O.OracleError as e:
        want_msg = str(e)
    assert want_msg.startswith("The checksum of the sharding index is invalid.")
    g = P.RegionGather([0] * 4, SHAPE, 4, group=group, align=8,
                       piece_bytes=8 * SHAPE[2] * SHAPE[3] * 4, device=0)
    bad_dec = P.PlanDecoder(dev, meta, lambda po, ps: [cbufs.get(c, (None, 0))
                                                       for c in chunk_coords(meta, po, ps)])
    try:
        g.run(bad_dec)
        raise AssertionError("RegionGather returned a region with corrupt shards")
    except _lib.ZhError as e:
        assert str(e) == want_msg, (str(e), want_msg)
        assert e.position == (tuple(corrupt[0]), 2 ** 64 - 1), e.position
    bad_dec.close()
    dec = P.PlanDecoder(dev, meta, sources)  # the group and buffers serve the next read
    got = g.run(dec).cpu().numpy().view(np.uint32).reshape(SHAPE)
    np.testing.assert_array_equal(got, data)
    dec.close()
    for c in corrupt:
        dev.free(cbufs[c][0])
    for p, _ in bufs.values():
        dev.free(p)
    dist.destroy_process_group()
    print("child ok", flush=True)


if __name__ == "__main__" and len(__import__("sys").argv) > 1 and \
        __import__("sys").argv[1] == "child":
    import sys
    _child(sys.argv[2], sys.argv[3], int(sys.argv[4]))


def test_shared_host_region_one_rank(dev, written, tmp_path):
    """SharedHostRegion on the GPU (a gloo group of one rank: no torch HIP involved): the slice
    page-locked with zh_host_register, the slab read by array_host_decoder (Array.read_into: the
    library's pipelined read DMA-ing straight into the pinned slice), equal to the array; the
    buffer removed on close."""
    import torch.distributed as dist
    data, stores = written
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1)
    try:
        a = z.Array.open(stores["files"].resolve("a"))
        for off, shp in REGIONS[:2]:
            name = str(tmp_path / "region")
            h = P.SharedHostRegion(off, shp, 4, dev=dev, align=8, name=name)
            try:
                h.read(P.array_host_decoder(a, dev))
                np.testing.assert_array_equal(
                    h.array(np.uint32), data[tuple(slice(o, o + s) for o, s in zip(off, shp))])
            finally:
                h.close()
            assert not os.path.exists(name)
    finally:
        dist.destroy_process_group()
