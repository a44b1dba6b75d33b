"""Multi-GPU readiness without the hardware (BASELINE
configs[4]; the reference's ForkJoin chunk loop, M/core/Array.java:403-407).

- bench.py's strong-mode geometry (strong_slab) and memory plan (strong_memory_plan) at the
  FULL 1x4096x4096x1536 c4 size and N = 8: every rank's slab, the shards it must hold and its
  device memory — the root's assembled 96 GiB region included — fit one MI355X's 288 GB.
- The same code path at world 8 over gloo on a scaled array with the same 8-slab geometry
  (each slab half a shard row, 4 shard columns, a half-filled boundary shard along x; the
  c4 chain): each rank holds only the shards strong_slab names, decodes its pieces (the
  oracle stands in for the HIP decode on CPU) before sending them through
  zarrhip.parallel.RegionGather, and the root's assembled region equals the array."""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_BYTES = 288 * 10 ** 9  # MI355X HBM3E (MI355X_MICROARCH.md)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_full_size_strong_memory_plan_n8():
    """N = 8 on the full c4 array: 512-row slabs on the 32-row inner-chunk grid; every rank
    holds one shard row (8 shards: 4 along y-x, 2 along z, the second half-filled); the root's
    plan (its 24 GiB cover box as output and encode source, its 24 GiB of shards, the 96 GiB
    region RCCL assembles into, 4 GiB headroom) and every peer's (plus its 12 GiB send buffer)
    fit 288 GB, with room to spare for RCCL's own buffers."""
    import bench
    from zarrhip import _abi as A
    from zarrhip._lib import lib
    L = lib()
    meta = bench.build_meta(A, "c4")
    GiB = 1 << 30
    seen_rows = 0
    for rank in range(8):
        geo = bench.strong_slab(L, meta, 8, rank)
        assert geo["ss"] == [1, 512, 4096, 1536] and geo["so"][1] == 512 * rank
        assert geo["lo"][1] == (512 * rank // 1024) * 1024 and geo["ext"][1] == 1024
        assert len(geo["cover"]) == 8
        caps = bench.chunk_capacities(meta, geo["cover"])
        _, tot = bench.slab_layout(caps)
        plan = bench.strong_memory_plan(geo, tot, rank, "nccl")
        assert plan["output"] == 24 * GiB and 24 * GiB <= plan["shards"] < 24 * GiB + (64 << 20)
        if rank == 0:
            assert plan["region"] == 96 * GiB and plan["send_buffer"] == 0
            assert plan["total"] < 150 * GiB
        else:
            assert plan["region"] == 0 and plan["send_buffer"] == 12 * GiB
            assert plan["total"] < 66 * GiB
        assert plan["total"] <= HBM_BYTES
        seen_rows += geo["ss"][1]
    assert seen_rows == 4096
    # the gloo form keeps the region on the host: no device region on the root
    geo = bench.strong_slab(L, meta, 8, 0)
    caps = bench.chunk_capacities(meta, geo["cover"])
    assert bench.strong_memory_plan(geo, bench.slab_layout(caps)[1], 0, "gloo")["region"] == 0


SCALED = [1, 256, 256, 96]      # full / 16 along y and x, 1536 / 16 along z
SCALED_CHUNK = [1, 64, 64, 64]  # 4 shard rows, 4 shard columns, 1.5 shards along z
SCALED_INNER = [1, 4, 4, 4]     # 16 inner rows per shard row; a slab = 8 inner rows


def _scaled_meta():
    from zarrhip import _abi as A
    return A.make_meta(SCALED, SCALED_CHUNK, 4, endian=A.ZH_ENDIAN_BIG, sharded=True,
                       inner_chunk_shape=SCALED_INNER, transpose_order=[0, 3, 2, 1],
                       index_endian=A.ZH_ENDIAN_LITTLE, index_crc32c=True,
                       index_location=A.ZH_INDEX_END)


def _world8_worker(rank, world, port, tmp):
    import json
    import sys
    for p in (os.path.join(ROOT, "zarr-java_amd"), os.path.join(ROOT, "oracle"), ROOT,
              os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    import oracle as O
    from helpers import rand_array
    from zarrhip import parallel as PP
    from zarrhip._lib import lib
    d = bench.Dist(world)  # init_process_group("gloo") from the env, as under torchrun
    L = lib()
    meta = _scaled_meta()
    arr = rand_array(SCALED, 4, seed=2026)
    geo = bench.strong_slab(L, meta, world, rank)
    lo, ext = geo["lo"], geo["ext"]
    box = np.ascontiguousarray(arr[tuple(slice(l, l + e) for l, e in zip(lo, ext))])
    held = dict(zip(geo["cover"], O.array_write(meta, box.tobytes(), lo, ext)))  # my shards only
    caps = bench.chunk_capacities(meta, geo["cover"])
    assert [len(held[c]) for c in geo["cover"]] == caps  # the bench's slab sizes hold
    plan = bench.strong_memory_plan(geo, bench.slab_layout(caps)[1], rank, "gloo")
    decoded = []

    def decode(po, ps, dst):  # decode-before-send; the oracle stands in for the HIP decode
        sel = O.compute_chunk_coords(SCALED, SCALED_CHUNK, po, ps)
        missing = [c for c in sel if c not in held]
        assert not missing, f"rank {rank} needs shards it does not hold: {missing}"
        dst.numpy()[:] = np.frombuffer(O.array_read(meta, [held[c] for c in sel], po, ps),
                                       np.uint8)
        decoded.append((list(po), list(ps)))

    cap = 4 * SCALED[2] * SCALED[3] * 4  # 4 rows per piece: 8 pieces per rank, as 1 GiB at full size
    g = PP.RegionGather([0] * 4, SCALED, 4, align=geo["align"], piece_bytes=cap)
    assert g.parts == geo["parts"]  # the gather cuts the slabs the bench planned
    d.barrier()
    out = g.run(decode)
    mx = d.max(float(len(decoded)))
    res = {"slab": [geo["so"], geo["ss"]], "cover": len(geo["cover"]), "pieces": len(decoded),
           "max_pieces": mx, "plan_total": plan["total"]}
    if rank == 0:
        got = out.numpy().view(np.uint32).reshape(SCALED)
        res["region_equal"] = bool(np.array_equal(got, arr))
    with open(os.path.join(tmp, f"w8_{rank}.json"), "w") as f:
        json.dump(res, f)
    d.close()


@pytest.mark.timeout(600)
def test_world8_strong_mode_rehearsal(tmp_path):
    """bench.py strong mode's geometry and gather at world 8 (gloo, CPU): 8 slabs of 32 rows
    (half a shard row each, as 512 of 1024 at full size), each rank holding the 8 shards of
    its shard row only, 8 pieces of 4 rows per rank decoded before they are sent, the root's
    region equal to the array."""
    import json
    import torch.multiprocessing as mp
    world = 8
    mp.spawn(_world8_worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [json.load(open(tmp_path / f"w8_{r}.json")) for r in range(world)]
    assert res[0]["region_equal"] is True
    for r, x in enumerate(res):
        assert x["slab"] == [[0, 32 * r, 0, 0], [1, 32, 256, 96]]
        assert x["cover"] == 8 and x["pieces"] == 8 and x["max_pieces"] == 8.0
