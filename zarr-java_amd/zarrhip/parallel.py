"""Multi-GPU partitioning of one region read.

Shards and inner chunks are independent, so a read splits into per-rank slabs with no
data-path exchange; ranks own one GPU each (one process per GPU).  A slab along the first
axis that is wider than 1 is contiguous in the region's C order, so a root can assemble
the full region by concatenating the ranks' slabs (RCCL gather over xGMI when the slabs
are device tensors, gloo on host tensors).
"""
import numpy as np


def slab_axis(shape, world):
    """First axis long enough to give every rank a slab (slabs along it are contiguous
    in C order because all earlier axes have extent 1 or are the axis itself)."""
    for d, s in enumerate(shape):
        if s >= world:
            return d
        if s != 1:
            break
    raise ValueError(f"region {list(shape)} cannot be split into {world} contiguous slabs")


def slab_partition(offset, shape, world, align=1):
    """Split [offset, offset+shape) into `world` contiguous slabs along slab_axis.
    Boundaries snap to multiples of `align` (e.g. the inner-chunk extent, so that no inner
    chunk is split between ranks) whenever every rank still gets at least one unit.
    Returns [(slab_offset, slab_shape)] per rank (a rank may get an empty slab)."""
    offset = [int(o) for o in offset]
    shape = [int(s) for s in shape]
    ax = slab_axis(shape, world)
    lo, ext = offset[ax], shape[ax]
    units = ext // align if align > 1 and ext % align == 0 and ext // align >= world else None
    bounds = []
    for r in range(world + 1):
        if units is not None:
            b = lo + (units * r // world) * align
        else:
            b = lo + ext * r // world
        bounds.append(b)
    out = []
    for r in range(world):
        o = list(offset)
        s = list(shape)
        o[ax] = bounds[r]
        s[ax] = bounds[r + 1] - bounds[r]
        out.append((o, s))
    return out


def slab_byte_offset(shape, slab_offset, itemsize):
    """Byte offset of a slab's first element in the C-order region buffer of `shape`: where
    a rank's slice starts in a host-terminated read's shared region buffer."""
    off, st = 0, 1
    for d in range(len(shape) - 1, -1, -1):
        off += int(slab_offset[d]) * st
        st *= int(shape[d])
    return off * itemsize


def gather_pieces(shape, parts, itemsize, cap_bytes, align=1):
    """The bounded, overlapped gather's schedule (bench.py strong mode): every
    rank's slab cut, in order, into pieces of at most `cap_bytes` along the slab's first axis
    of extent >= 2 (all earlier axes have extent 1, so each piece is one contiguous C-order
    part of the region, sent into its place in the root's buffer as its decode finishes).
    Piece boundaries fall on multiples of `align` rows (the inner-chunk extent: no inner chunk
    is decoded twice) whenever `align` rows fit the cap; a single row larger than the cap is
    one piece.  Returns, per rank, [(piece_offset, piece_shape, region_byte_offset, nbytes)]."""
    out = []
    for so, ss in parts:
        so, ss = [int(v) for v in so], [int(v) for v in ss]
        pieces = []
        if all(v > 0 for v in ss):
            ax = next((d for d, v in enumerate(ss) if v >= 2), len(ss) - 1)
            if any(ss[d] != 1 for d in range(ax)):
                raise ValueError(f"slab {ss} is not one contiguous C-order part of {shape}")
            row = int(itemsize)
            for d in range(ax + 1, len(ss)):
                row *= ss[d]
            per = max(1, int(cap_bytes) // row)
            if align > 1 and per >= align:
                per = per // align * align
            lo, end = so[ax], so[ax] + ss[ax]
            while lo < end:
                hi = min(end, lo + per)
                if align > 1 and hi < end and hi % align:  # snap to the unit grid
                    snapped = hi // align * align
                    hi = snapped if snapped > lo else hi
                po, ps = list(so), list(ss)
                po[ax], ps[ax] = lo, hi - lo
                nb = (hi - lo) * row
                pieces.append((po, ps, slab_byte_offset(shape, po, itemsize), nb))
                lo = hi
        out.append(pieces)
    return out


def gather_pieces_p2p(tdist, grp, rank, world, sched, send_buf, region, decode=None):
    """The point-to-point part of the pieced gather into rank 0's region buffer (bench.py strong
    mode; gloo on CPU tensors in tests/test_distributed.py).  `sched` = gather_pieces(...);
    `send_buf` holds this rank's slab (byte tensor, piece k at its offset within the slab),
    `region` the root's whole region (byte tensor).  Rank 0 posts round k of every peer as one
    batch (the peers' links in parallel); a peer sends piece k as a batch of one, after calling
    decode(k) when given (the send then waits only for that piece's decode).  Every op, batched
    on both sides, runs on the group's communicator.  Returns the works to wait on."""
    works = []
    if rank == 0:
        for k in range(max((len(p) for p in sched), default=0)):
            ops = [tdist.P2POp(tdist.irecv, region[sched[r][k][2]:sched[r][k][2] + sched[r][k][3]],
                               r, grp)
                   for r in range(1, world) if k < len(sched[r])]
            if ops:
                works += tdist.batch_isend_irecv(ops)
        return works
    mine = sched[rank]
    base = mine[0][2] if mine else 0
    for k, (_, _, b, nb) in enumerate(mine):
        if decode is not None:
            decode(k)
        works += tdist.batch_isend_irecv(
            [tdist.P2POp(tdist.isend, send_buf[b - base:b - base + nb], 0, grp)])
    return works


def assemble(slabs, shape, axis):
    """Concatenate per-rank slabs (in rank order) into the full region."""
    parts = [np.asarray(s) for s in slabs if np.asarray(s).size]
    full = np.concatenate(parts, axis=axis) if parts else np.zeros(shape)
    assert list(full.shape) == list(shape)
    return full


def distributed_read(decode, offset, shape, dist, root=0, align=1):
    """Each rank decodes its slab with `decode(offset, shape) -> np.ndarray` (the device
    read, e.g. zarrhip.Array.read); the root gathers and returns the full region (other
    ranks return their slab).  `dist` is an initialised torch.distributed module."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    parts = slab_partition(offset, shape, world, align)
    ax = slab_axis(shape, world)
    so, ss = parts[rank]
    mine = decode(so, ss) if all(s > 0 for s in ss) else None
    # gather as flat byte tensors of the largest slab (gather needs equal sizes)
    sizes = [int(np.prod(s)) for _, s in parts]
    dts = [None] * world
    dist.all_gather_object(dts, None if mine is None else np.dtype(mine.dtype).str)
    dt = np.dtype(next(d for d in dts if d is not None))
    itemsize = dt.itemsize
    nmax = max(sizes) * itemsize
    buf = torch.zeros(nmax, dtype=torch.uint8)
    if mine is not None:
        buf[: mine.nbytes] = torch.from_numpy(np.ascontiguousarray(mine).view(np.uint8).ravel())
    gl = [torch.zeros(nmax, dtype=torch.uint8) for _ in range(world)] if rank == root else None
    dist.gather(buf, gl, dst=root)
    if rank != root:
        return mine
    slabs = [gl[r][: sizes[r] * itemsize].numpy().view(dt).reshape(parts[r][1])
             for r in range(world)]
    return assemble(slabs, shape, ax)
