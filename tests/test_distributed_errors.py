"""Error parity of the multi-rank read: when any rank's part
of a RegionGather / SharedHostRegion read fails, EVERY rank — the root included — raises the
error one sequential core.Array.read would have thrown (the reference throws out of read() when a
chunk fails: M/core/Array.java:403-407, 436-438; Crc32cCodec.java:39-44), within a bounded time,
and no rank returns a region holding the failed slab.  gloo at world 2 and 3 on CPU; the
per-rank decode is the oracle (test infrastructure), once synchronous (array_decoder's form)
and once deferring its errors to wait() (PlanDecoder's form)."""
import os
import socket

import numpy as np
import pytest

from zarrhip import parallel as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPE = [1, 24, 20, 12]
CHUNK = [1, 8, 8, 8]


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# --- pick_error: the choice every rank agrees on ------------------------------------------
def rec(msg, pos=None, cls="ZarrException", module="zarrhip.errors"):
    return {"cls": cls, "module": module, "msg": msg, "status": None, "pos": pos}


def test_pick_error_orders_placed_errors_like_a_sequential_read():
    """All errors placed: the first in the reference's order (chunk coords in C order; inside a
    chunk the larger key, i.e. the index crc32c (~0) before any inner chunk) wins, whichever
    rank met it."""
    assert P.pick_error([[], []]) is None
    recs = [[rec("a", ((0, 2, 0, 0), 7))], [rec("b", ((0, 1, 1, 0), 1))],
            [rec("c", ((0, 1, 0, 1), 3)), rec("d", ((0, 1, 0, 1), 2 ** 64 - 1))]]
    assert P.pick_error(recs) == (2, 1)  # (0,1,0,1) < (0,1,1,0); the index crc first
    recs[2] = []
    assert P.pick_error(recs) == (1, 0)


def test_pick_error_unplaced_falls_back_to_the_first_failing_rank():
    """Any error without a position (a host-side failure): the first failing rank's first error
    — the slabs are contiguous in C order, as zh_array_read_multi picks its slabs."""
    recs = [[], [rec("b", ((0, 2, 0, 0), 1))], [rec("c", None, "StoreException", "zarrhip.store")]]
    assert P.pick_error(recs) == (1, 0)


def test_rebuild_error_keeps_class_message_and_position():
    from zarrhip.errors import ZarrException
    from zarrhip.store import StoreException
    e = P.rebuild_error(rec("The checksum of the sharding index is invalid. Stored: 1 "
                            "Computed: 2", ((0, 1), 5)))
    assert type(e) is ZarrException and e.position == ((0, 1), 5)
    assert str(e).startswith("The checksum of the sharding index is invalid.")
    assert type(P.rebuild_error(rec("x", None, "StoreException", "zarrhip.store"))) is StoreException
    assert type(P.rebuild_error(rec("y", None, "ValueError", "builtins"))) is ValueError
    assert type(P.rebuild_error(rec("z", None, "Weird", "elsewhere"))) is RuntimeError
    r = P.error_record(ValueError("v"))
    assert r["cls"] == "ValueError" and r["module"] == "builtins" and r["pos"] is None


# --- multi-process: the collective raises the same error on every rank ---------------------
def _setup(rank, world, port):
    import sys
    for p in (os.path.join(ROOT, "zarr-java_amd"), os.path.join(ROOT, "oracle"), ROOT,
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _encoded(seed):
    import oracle as O
    from helpers import encode_oracle, rand_array
    from zarrhip import _abi as A
    meta = A.make_meta(SHAPE, CHUNK, 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 4, 4, 4], transpose_order=[0, 3, 2, 1])
    arr = rand_array(SHAPE, 4, seed=seed)
    shards = encode_oracle(meta, arr)
    allc = O.compute_chunk_coords(SHAPE, CHUNK, [0] * 4, SHAPE)
    return meta, arr, shards, allc


def _corrupt_rank1_shard(world, shards, allc):
    """Flip a byte of the stored index crc32c of a shard that only rank 1's slab reads."""
    lo, hi = [(o[1], o[1] + s[1]) for o, s in P.slab_partition([0] * 4, SHAPE, world, 4)][1]
    target = next(c for c in allc if lo <= c[1] * 8 and (c[1] + 1) * 8 <= hi)
    k = allc.index(target)
    b = bytearray(shards[k])
    b[-1] ^= 0x5A
    shards[k] = bytes(b)
    return target


def _oracle_decoders(meta, shards, allc):
    import oracle as O
    from zarrhip.errors import ZarrException
    pos = {c: i for i, c in enumerate(allc)}

    def raw(po, ps):
        sel = O.compute_chunk_coords(SHAPE, CHUNK, po, ps)
        try:
            return O.array_read(meta, [shards[pos[c]] for c in sel], po, ps)
        except O.OracleError as e:  # the reference's text, as zarrhip.Array raises it
            raise ZarrException(str(e.args[1] if len(e.args) > 1 else e)) from None

    def sync(po, ps, dst):
        dst.numpy()[:] = np.frombuffer(raw(po, ps), np.uint8)

    class Deferred:  # PlanDecoder's form: errors surface only in wait()
        def __init__(self):
            self.errs = []

        def __call__(self, po, ps, dst):
            try:
                dst.numpy()[:] = np.frombuffer(raw(po, ps), np.uint8)
            except ZarrException as e:
                dst.numpy()[:] = 0xEE  # what a failed device decode leaves: garbage
                self.errs.append(e)

        def wait(self):
            errs, self.errs = self.errs, []
            if errs:
                raise errs[0]

    def host(po, ps, addr):
        import ctypes
        b = raw(po, ps)
        ctypes.memmove(addr, b, len(b))

    return raw, sync, Deferred, host


def _err_worker(rank, world, port, tmp):
    import json
    dist = _setup(rank, world, port)
    from zarrhip import parallel as PP
    meta, arr, shards, allc = _encoded(31)
    target = _corrupt_rank1_shard(world, shards, allc)
    raw, sync, Deferred, host = _oracle_decoders(meta, shards, allc)
    out = {"target": list(target)}
    if rank == 0:
        try:
            raw([0] * 4, SHAPE)
            out["sequential"] = None
        except Exception as e:
            out["sequential"] = str(e)
    for name, dec in (("sync", sync), ("deferred", Deferred())):
        g = PP.RegionGather([0] * 4, SHAPE, 4, align=4, piece_bytes=2 * 20 * 12 * 4)
        try:
            g.run(dec)
            out[name] = ["returned", None]
        except Exception as e:
            out[name] = [type(e).__name__, str(e)]
    try:
        h = PP.SharedHostRegion([0] * 4, SHAPE, 4, align=4)
        try:
            h.read(host)
            out["host"] = ["returned", None]
        except Exception as e:
            out["host"] = [type(e).__name__, str(e)]
        finally:
            h.close()
    except Exception as e:  # noqa: BLE001
        out["host"] = ["setup", repr(e)]
    # the group is still usable after a failed read: a read that avoids the bad shard works
    lo = [0, 0, 0, 0]
    shp = [1, 8, 20, 12]
    g = PP.RegionGather(lo, shp, 4, align=4, piece_bytes=2 * 20 * 12 * 4)
    got = g.run(sync)
    if rank == 0:
        out["after_ok"] = bool(np.array_equal(got.numpy().view(np.uint32).reshape(shp),
                                              arr[:, 0:8]))
    with open(os.path.join(tmp, f"err{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_corrupt_shard_on_rank1_raises_on_every_rank(tmp_path, world):
    """A corrupt shard index read only by rank 1: with a synchronous decoder, a deferred-error
    decoder (wait()) and the host-terminated SharedHostRegion, every rank raises ZarrException
    with exactly the message a single sequential read of the region gives (the oracle's
    "The checksum of the sharding index is invalid. Stored: .. Computed: .."), nobody hangs (the
    test is time-bounded), and the same group then serves a good read."""
    import json
    import torch.multiprocessing as mp
    mp.spawn(_err_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [json.load(open(tmp_path / f"err{r}.json")) for r in range(world)]
    want = res[0]["sequential"]
    assert want and want.startswith("The checksum of the sharding index is invalid. Stored: ")
    for r in range(world):
        for form in ("sync", "deferred", "host"):
            assert res[r][form] == ["ZarrException", want], (r, form, res[r][form])
    assert res[0]["after_ok"] is True


def _placed_worker(rank, world, port, tmp):
    import json
    dist = _setup(rank, world, port)
    from zarrhip import parallel as PP
    from zarrhip.errors import ZarrException
    from zarrhip.store import StoreException
    out = {}

    def make(plan):
        def dec(po, ps, dst):
            kind = plan.get(rank)
            if kind is None:
                dst.numpy()[:] = 0
                return
            if kind[0] == "store":
                raise StoreException(kind[1])
            e = ZarrException(kind[1])
            e.position = kind[2]
            raise e
        return dec

    cases = {
        # rank 0 fails later in the sequential order than rank 1: rank 1's error everywhere
        "placed": {0: ("data", "late", ((0, 2, 0, 0), 5)), 1: ("data", "early", ((0, 1, 0, 0), 3))},
        # an unplaced (store) failure anywhere: the first failing rank's error
        "unplaced": {0: ("data", "r0", ((0, 2, 0, 0), 5)), 1: ("store", "r1 store")},
        "root_only": {0: ("data", "root", ((0, 0, 0, 0), 1))},
    }
    for name, plan in cases.items():
        g = PP.RegionGather([0] * 4, SHAPE, 4, align=4, piece_bytes=4 * 20 * 12 * 4)
        try:
            g.run(make(plan))
            out[name] = ["returned", None]
        except (ZarrException, StoreException) as e:
            out[name] = [type(e).__name__, str(e)]
    with open(os.path.join(tmp, f"placed{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_errors_of_several_ranks_resolve_to_the_sequential_first(tmp_path, world):
    """Several ranks fail: all raise the error that sits first in the sequential read's order
    when every error is placed (positions from zh_last_data_error), else the first failing
    rank's; an error on the root alone reaches the peers too."""
    import json
    import torch.multiprocessing as mp
    mp.spawn(_placed_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        res = json.load(open(tmp_path / f"placed{r}.json"))
        assert res["placed"] == ["ZarrException", "early"]
        assert res["unplaced"] == ["ZarrException", "r0"]
        assert res["root_only"] == ["ZarrException", "root"]


def _shm_worker(rank, world, port, tmp):
    import json
    dist = _setup(rank, world, port)
    from zarrhip import parallel as PP
    out = {}
    a = PP.SharedHostRegion([0, 0], [8, 16], 4)
    b = PP.SharedHostRegion([0, 0], [4, 16], 4)  # alive at once: its own file
    out["distinct"] = a.name != b.name
    if rank == 0:
        a.array(np.uint32)[:] = 7
    dist.barrier()
    if rank == 0:
        b.array(np.uint32)[:] = 3
    dist.barrier()
    out["a_intact"] = bool((a.array(np.uint32) == 7).all())
    # a view still held on rank 1: its close raises there, and nobody hangs in the barrier
    held = b.array(np.uint32) if rank == 1 else None
    try:
        b.close()
        out["close_b"] = "ok"
    except BufferError:
        out["close_b"] = "BufferError"
    del held
    a.close()
    # a caller-chosen name that already exists: every rank raises
    path = os.path.join(tmp, "taken")
    if rank == 0:
        open(path, "w").close()
    dist.barrier()
    try:
        PP.SharedHostRegion([0], [16], 4, name=path)
        out["taken"] = "created"
    except FileExistsError:
        out["taken"] = "FileExistsError"
    with open(os.path.join(tmp, f"shm{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_shared_region_names_and_close_barrier(tmp_path):
    """two regions alive at once get distinct /dev/shm files (rank 0 creates each
    exclusively), so neither clobbers the other; close() reaches the barrier on every rank even
    when a rank still holds array()'s view (it raises BufferError there, afterwards); an
    existing caller-chosen name fails on every rank."""
    import json
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_shm_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [json.load(open(tmp_path / f"shm{r}.json")) for r in range(world)]
    for r in range(world):
        assert res[r]["distinct"] and res[r]["a_intact"] and res[r]["taken"] == "FileExistsError"
    assert res[0]["close_b"] == "ok" and res[1]["close_b"] == "BufferError"
