"""Multi-process (world_size 2 and 3, gloo on CPU) coverage of the N>1 paths: bench.py's
barrier / max-over-ranks harness and zarrhip.parallel's slab partition and region gather
(RegionGather / distributed_read, the same code that runs over RCCL on GPUs).  The per-rank
decode here is the oracle (test infrastructure); on GPUs it is the HIP path (PlanDecoder /
array_decoder)."""
import os
import socket

import numpy as np
import pytest

from zarrhip import parallel as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("shape,world,align", [([1, 4096, 4096, 1536], 8, 32),
                                               ([1, 4096, 4096, 1536], 2, 32),
                                               ([100, 7], 3, 1), ([1, 1, 64, 5], 4, 16),
                                               ([50], 4, 32)])
def test_slab_partition_covers_region(shape, world, align):
    off = [0] * len(shape)
    parts = P.slab_partition(off, shape, world, align)
    ax = P.slab_axis(shape, world)
    assert len(parts) == world
    pos = off[ax]
    for o, s in parts:
        assert o[ax] == pos
        for d in range(len(shape)):
            if d != ax:
                assert o[d] == off[d] and s[d] == shape[d]
        pos += s[ax]
    assert pos == off[ax] + shape[ax]
    if shape == [1, 4096, 4096, 1536] and world == 8:
        assert [s[1] for _, s in parts] == [512] * 8  # 512-row slabs
    # host-terminated read: each slab's slice of the region buffer starts where the
    # previous one ends (contiguous C-order slabs tile the buffer)
    pos_b = 0
    for o, s in parts:
        assert P.slab_byte_offset(shape, o, 4) == pos_b
        pos_b += 4 * int(np.prod(s))
    assert pos_b == 4 * int(np.prod(shape))


def _worker(rank, world, port, tmp):
    import sys
    for p in (os.path.join(ROOT, "zarr-java_amd"), os.path.join(ROOT, "oracle"), ROOT,
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    import bench
    import oracle as O
    from helpers import encode_oracle, rand_array
    from zarrhip import _abi as A
    from zarrhip import parallel as PP
    d = bench.Dist(world)  # init_process_group("gloo") from the env, as under torchrun
    d.barrier()
    mx = d.max(float(rank + 1))
    shape = [1, 24, 20, 12]
    meta = A.make_meta(shape, [1, 8, 8, 8], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 4, 4, 4], transpose_order=[0, 3, 2, 1])
    arr = rand_array(shape, 4, seed=99)
    shards = encode_oracle(meta, arr)
    allc = O.compute_chunk_coords(shape, [1, 8, 8, 8], [0] * 4, shape)
    pos = {c: i for i, c in enumerate(allc)}
    calls = []

    def decode(po, ps, dst):  # the oracle stands in for the device decode (CPU test)
        calls.append((list(po), list(ps)))
        sel = O.compute_chunk_coords(shape, [1, 8, 8, 8], po, ps)
        raw = O.array_read(meta, [shards[pos[c]] for c in sel], po, ps)
        dst.numpy()[:] = np.frombuffer(raw, np.uint8)

    # the product's distributed read: slabs on the inner-chunk grid, pieces of 2 rows
    full = PP.distributed_read(decode, [0] * 4, shape, np.uint32, align=4,
                               piece_bytes=2 * 20 * 12 * 4)
    # an unaligned region at an offset: the same gather, region-relative placement
    off2, shp2 = [0, 3, 2, 1], [1, 19, 15, 9]
    part = PP.distributed_read(decode, off2, shp2, np.uint32, align=1,
                               piece_bytes=3 * 15 * 9 * 4)
    if rank == 0:
        np.save(os.path.join(tmp, "full.npy"), full)
        np.save(os.path.join(tmp, "part.npy"), part)
        np.save(os.path.join(tmp, "want.npy"), arr)
    with open(os.path.join(tmp, f"max{rank}.txt"), "w") as f:
        f.write(str(mx))
    with open(os.path.join(tmp, f"calls{rank}.txt"), "w") as f:
        f.write(repr(calls))
    d.close()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_distributed_read_and_bench_harness(tmp_path, world):
    """zarrhip.parallel.distributed_read (RegionGather: bounded pieces, decode(k) before
    send(k), the root's own slab decoded into place) with gloo at world sizes 2 and 3: the
    assembled region equals the array for the whole region and for an unaligned part at an
    offset; each rank decoded exactly its own pieces, in order; bench.Dist's max over ranks."""
    import ast
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    want = np.load(tmp_path / "want.npy")
    np.testing.assert_array_equal(np.load(tmp_path / "full.npy"), want)
    np.testing.assert_array_equal(np.load(tmp_path / "part.npy"), want[:, 3:22, 2:17, 1:10])
    for r in range(world):
        assert float(open(tmp_path / f"max{r}.txt").read()) == float(world)
    shape = [1, 24, 20, 12]
    for (off, shp, align, cap) in (([0] * 4, shape, 4, 2 * 20 * 12 * 4),
                                   ([0, 3, 2, 1], [1, 19, 15, 9], 1, 3 * 15 * 9 * 4)):
        parts = P.slab_partition(off, shp, world, align)
        rel = [([o - b for o, b in zip(po, off)], ps) for po, ps in parts]
        sched = P.gather_pieces(shp, rel, 4, cap, align)
        for r in range(world):
            calls = ast.literal_eval(open(tmp_path / f"calls{r}.txt").read())
            mine = [([a + b for a, b in zip(po, off)], ps) for po, ps, _, _ in sched[r]]
            assert all(c in calls for c in mine)
            idx = [calls.index(c) for c in mine]
            assert idx == sorted(idx) and len(mine) > 1  # in order, several pieces


def _host_worker(rank, world, port, tmp):
    import ctypes
    import sys
    for p in (os.path.join(ROOT, "zarr-java_amd"), os.path.join(ROOT, "oracle"), ROOT,
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist
    import oracle as O
    from helpers import encode_oracle, rand_array
    from zarrhip import _abi as A
    from zarrhip import parallel as PP
    dist.init_process_group("gloo", rank=rank, world_size=world)
    shape = [1, 24, 20, 12]
    meta = A.make_meta(shape, [1, 8, 8, 8], 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=[1, 4, 4, 4], transpose_order=[0, 3, 2, 1])
    arr = rand_array(shape, 4, seed=97)
    shards = encode_oracle(meta, arr)
    allc = O.compute_chunk_coords(shape, [1, 8, 8, 8], [0] * 4, shape)
    pos = {c: i for i, c in enumerate(allc)}
    seen = []

    def decode(po, ps, addr):  # the oracle stands in for the device read (CPU test)
        seen.append((list(po), list(ps)))
        sel = O.compute_chunk_coords(shape, [1, 8, 8, 8], po, ps)
        raw = O.array_read(meta, [shards[pos[c]] for c in sel], po, ps)
        ctypes.memmove(addr, raw, len(raw))

    for off, shp in (([0] * 4, shape), ([0, 3, 2, 1], [1, 19, 15, 9])):
        h = PP.SharedHostRegion(off, shp, 4, group=None, align=4 if off == [0] * 4 else 1,
                                name=os.path.join(tmp, f"region_{port}"))
        h.read(decode)
        got = h.array(np.uint32).copy()  # every rank sees the whole region
        h.close()
        want = arr[tuple(slice(o, o + s) for o, s in zip(off, shp))]
        np.save(os.path.join(tmp, f"host{rank}_{off[1]}.npy"), got)
        np.save(os.path.join(tmp, f"want_{off[1]}.npy"), want)
        assert not os.path.exists(os.path.join(tmp, f"region_{port}")) or rank != 0
    with open(os.path.join(tmp, f"seen{rank}.txt"), "w") as f:
        f.write(repr(seen))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_shared_host_region(tmp_path, world):
    """zarrhip.parallel.SharedHostRegion (the host-terminated multi-GPU read, no gather): every
    rank decodes exactly its slab into its slice of one shared buffer, and every rank then sees
    the whole region — for the whole array and an unaligned part at an offset; rank 0 removes
    the buffer on close."""
    import ast
    import torch.multiprocessing as mp
    mp.spawn(_host_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    for y in (0, 3):
        want = np.load(tmp_path / f"want_{y}.npy")
        for r in range(world):
            np.testing.assert_array_equal(np.load(tmp_path / f"host{r}_{y}.npy"), want)
    shape = [1, 24, 20, 12]
    for r in range(world):
        seen = [tuple(map(list, c)) for c in
                ast.literal_eval(open(tmp_path / f"seen{r}.txt").read())]
        assert seen == [tuple(P.slab_partition([0] * 4, shape, world, 4)[r]),
                        tuple(P.slab_partition([0, 3, 2, 1], [1, 19, 15, 9], world, 1)[r])]
    assert not [f for f in os.listdir(tmp_path) if f.startswith("region_")]


@pytest.mark.parametrize("seed", range(12))
def test_c_slab_partition_matches_python(seed):
    """zh_slab_partition (the C-ABI multi-GPU read's split) == zarrhip.parallel.slab_partition."""
    from zarrhip._lib import ZhError, slab_partition
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 5))
    lead = int(rng.integers(0, n))
    shape = [1] * lead + [int(rng.integers(1, 300)) for _ in range(n - lead)]
    off = [int(rng.integers(0, 50)) for _ in range(n)]
    world = int(rng.integers(1, 9))
    align = int(rng.choice([1, 4, 16, 32]))
    try:
        want = P.slab_partition(off, shape, world, align)
    except ValueError:
        with pytest.raises(ZhError):
            slab_partition(off, shape, world, align)
        return
    assert slab_partition(off, shape, world, align) == want


def test_bench_self_launches_ranks_without_a_launcher():
    """`python bench.py --gpus 2` with no WORLD_SIZE starts its two ranks itself (before any
    GPU call, as child processes) and rank 0 prints exactly one JSON line with n_gpus 2 and
    strong scaling; --dry-run keeps it off the GPU so the harness runs here."""
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dry-run", "--steps", "2", "--warmup", "1"], capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["dry_run"] is True
    assert d["config"]["slab_rows_max"] == 2048
    # the overlapped gather's schedule: 2048 rows of 24 MiB per rank in 1 GiB-capped pieces of
    # 32 rows (inner-chunk aligned) = 64 pieces of 768 MiB each
    assert d["config"]["gather_pieces_per_rank"] == [64, 64]
    assert d["config"]["gather_max_piece_bytes"] == 32 * 4096 * 1536 * 4


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("cap_mb,align", [(1024, 32), (100, 32), (10, 32), (64, 1), (1, 7)])
def test_gather_piece_schedule(world, cap_mb, align):
    """zarrhip.parallel.gather_pieces (bench.py's bounded, overlapped RCCL gather): every rank's
    pieces tile its slab exactly once, in order, as contiguous byte ranges of the C-order
    region; none exceeds the cap unless one row does; boundaries fall on the `align` grid when
    `align` rows fit the cap."""
    shape = [1, 4096, 4096, 1536]
    row = 4096 * 1536 * 4
    cap = cap_mb << 20
    parts = P.slab_partition([0] * 4, shape, world, align=32)
    sched = P.gather_pieces(shape, parts, 4, cap, align=align)
    assert len(sched) == world
    covered = 0
    for (so, ss), pieces in zip(parts, sched):
        b0 = P.slab_byte_offset(shape, so, 4)
        pos = b0
        y = so[1]
        for po, ps, b, nb in pieces:
            assert po[0] == 0 and po[2:] == [0, 0] and ps[2:] == [4096, 1536] and ps[0] == 1
            assert po[1] == y and ps[1] > 0 and b == pos and nb == ps[1] * row
            if row <= cap:
                assert nb <= cap
            else:
                assert ps[1] == 1
            if align > 1 and align * row <= cap and po[1] + ps[1] < so[1] + ss[1]:
                assert (po[1] + ps[1]) % align == 0
            pos += nb
            y += ps[1]
        assert y == so[1] + ss[1] and pos == b0 + ss[1] * row
        covered += pos - b0
    assert covered == 4096 * row


def test_gather_piece_schedule_small_regions():
    """Ragged slabs of a small region and an empty slab: same tiling rules."""
    shape = [1, 1, 37, 5]
    parts = P.slab_partition([0] * 4, shape, 3, align=1)
    sched = P.gather_pieces(shape, parts, 2, 3 * 5 * 2, align=1)
    got = [(po[2], ps[2]) for pieces in sched for po, ps, _, _ in pieces]
    assert got[0] == (0, 3) and sum(n for _, n in got) == 37
    assert [b for pieces in sched for _, _, b, _ in pieces] == [o * 10 for o, _ in got]
    empty = P.gather_pieces([1, 2, 8], [([0, 0, 0], [1, 2, 8]), ([0, 2, 0], [1, 0, 8])], 4,
                            1 << 20)
    assert len(empty[0]) == 1 and empty[1] == []


def _pieces_worker(rank, world, port, tmp):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "zarr-java_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    from zarrhip import parallel as PP
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grp = dist.new_group(backend="gloo")
    shape = [1, 40, 6, 5]
    full = np.arange(int(np.prod(shape)) * 4, dtype=np.int64).astype(np.uint8)
    parts = PP.slab_partition([0] * 4, shape, world, align=4)
    sched = PP.gather_pieces(shape, parts, 4, 5 * 6 * 5 * 4, align=4)  # pieces of 4 rows
    so, ss = parts[rank]
    b0 = PP.slab_byte_offset(shape, so, 4)
    nb = 4 * int(np.prod(ss))
    region = torch.zeros(full.size, dtype=torch.uint8)
    region[b0:b0 + nb] = torch.from_numpy(full[b0:b0 + nb])  # the root's own slab in place
    send = torch.from_numpy(full[b0:b0 + nb].copy())
    decoded = []
    for w in PP.gather_pieces_p2p(dist, grp, rank, world, sched, send, region,
                                  decode=lambda k: decoded.append(k)):
        w.wait()
    if rank == 0:
        np.save(os.path.join(tmp, "region.npy"), region.numpy())
        np.save(os.path.join(tmp, "full.npy"), full)
    with open(os.path.join(tmp, f"decoded{rank}.txt"), "w") as f:
        f.write(",".join(map(str, decoded)) + "|" + str(len(sched[rank])))
    dist.destroy_process_group()


def test_pieced_gather_p2p_three_ranks(tmp_path):
    """gather_pieces_p2p (bench.py strong mode's gather) on gloo with three ranks: bounded pieces
    of every peer's slab land in their places of the root's region (batched on both sides), and a
    peer calls decode(k) once per piece, in order, before sending it."""
    import torch.multiprocessing as mp
    world = 3
    mp.spawn(_pieces_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    np.testing.assert_array_equal(np.load(tmp_path / "region.npy"), np.load(tmp_path / "full.npy"))
    for r in range(1, world):
        dec, n = open(tmp_path / f"decoded{r}.txt").read().split("|")
        assert int(n) > 1 and dec == ",".join(map(str, range(int(n))))
