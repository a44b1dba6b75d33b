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
