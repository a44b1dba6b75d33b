"""Shared test helpers: random arrays, oracle round trips, device round trips."""
import ctypes as C
import json
import os
import struct

import numpy as np

import oracle as O
from zarrhip import _abi as A
from zarrhip._lib import lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")

NP_DT = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}


def rand_array(shape, dsize, seed=0, fill_frac=0.0, fill=0):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 2 ** (8 * dsize) - 1, size=shape, dtype=np.uint64).astype(NP_DT[dsize])
    if fill_frac > 0:
        mask = rng.random(shape) < fill_frac
        a[mask] = fill
    return a


def shape_of(meta):
    return [meta.shape[d] for d in range(meta.ndim)]


def chunk_coords(meta, offset, shape):
    return O.compute_chunk_coords(shape_of(meta), [meta.chunk_shape[d] for d in range(meta.ndim)],
                                  offset, shape)


def encode_oracle(meta, arr):
    """Whole-array write through the oracle → list of chunk bytes (None = deleted)."""
    n = meta.ndim
    return O.array_write(meta, arr.tobytes(), [0] * n, shape_of(meta))


def device_read(dev, meta, sources, offset, shape):
    """Host bytes in → zh_array_read (H2D inside) → host numpy out."""
    n = meta.ndim
    nel = int(np.prod(shape))
    out = (C.c_char * max(1, nel * meta.dtype_size))()
    keep = []
    srcs = []
    for s in sources:
        if s is None:
            srcs.append((None, 0))
        else:
            b = (C.c_char * max(1, len(s))).from_buffer_copy(s if len(s) else b"\0")
            keep.append(b)
            srcs.append((C.addressof(b), len(s)))
    dev.array_read(meta, srcs, offset, shape, C.addressof(out), 0)
    return np.frombuffer(bytes(out), dtype=NP_DT[meta.dtype_size]).reshape(shape)


def device_write(dev, meta, arr):
    """Device encode of the whole array → list of chunk bytes (None = deleted)."""
    n = meta.ndim
    shape = shape_of(meta)
    src = dev.malloc(max(1, arr.nbytes))
    dev.h2d(src, arr.tobytes())
    coords = chunk_coords(meta, [0] * n, shape)
    cap = lib().zh_array_encoded_bound(C.byref(meta))
    bufs = [dev.malloc(cap) for _ in coords]
    for b in bufs:  # poison: every byte of the result must be written by the encode
        dev.memset(b, 0xA5, cap)
    sizes = dev.array_write(meta, src, [0] * n, shape, [(b, cap) for b in bufs])
    out = []
    for b, sz in zip(bufs, sizes):
        out.append(dev.d2h(b, sz) if sz else None)
        dev.free(b)
    dev.free(src)
    return out


def unwrap_blosc_memcpyed_shard(b, n_inner, index_location):
    """Host hand-off for the reference fixtures' inner `blosc` codec: its frames carry the
    MEMCPYED flag, so the raw bytes follow a 16-byte header.  Returns an equivalent shard
    without the blosc stage (new index + crc32c)."""
    isz = 16 * n_inner + 4
    idx = b[:isz] if index_location == "start" else b[-isz:]
    ents = [struct.unpack("<QQ", idx[16 * i:16 * i + 16]) for i in range(n_inner)]
    payload = b""
    newents = []
    for off, nb in ents:
        if off == 2 ** 64 - 1:
            newents.append((off, nb))
            continue
        fr = b[off:off + nb]
        assert fr[2] & 0x02, "only MEMCPYED blosc frames can be unwrapped without a codec"
        raw = fr[16:]
        newents.append((len(payload) + (isz if index_location == "start" else 0), len(raw)))
        payload += raw
    ib = b"".join(struct.pack("<QQ", *e) for e in newents)
    ib += struct.pack("<I", O.crc32c(ib))
    return ib + payload if index_location == "start" else payload + ib


def load_reference_fixture(loc):
    """tests/golden/sharding_index_location/<loc> (copied from the reference testdata)."""
    base = os.path.join(GOLDEN, "sharding_index_location", loc)
    meta_json = json.load(open(os.path.join(base, "zarr.json")))
    m = A.make_meta([16, 16, 16], [16, 8, 8], 4, sharded=True, inner_chunk_shape=[8, 4, 8],
                    transpose_order=[2, 1, 0],
                    index_location=A.ZH_INDEX_START if loc == "start" else A.ZH_INDEX_END)
    srcs = []
    for c in O.compute_chunk_coords([16, 16, 16], [16, 8, 8], [0, 0, 0], [16, 16, 16]):
        raw = open(os.path.join(base, "c", *map(str, c)), "rb").read()
        srcs.append(unwrap_blosc_memcpyed_shard(raw, 4, loc))
    return meta_json, m, srcs


# ---- the JNI shim's call sequence for HipArray.read (java/jni/zarrhip_jni.c) ------------
def shard_part(meta, coords, offset, shape):
    """Shard-local [lo, hi) of the region inside the shard at `coords`."""
    n = meta.ndim
    lo, hi = [], []
    for d in range(n):
        c0 = coords[d] * meta.chunk_shape[d]
        lo.append(max(offset[d], c0) - c0)
        hi.append(min(offset[d] + shape[d], c0 + meta.chunk_shape[d]) - c0)
    return lo, hi


def jni_fetch(meta, paths, offset, shape, max_run=64 << 20, size_known=True, drop=None,
              pad=False):
    """HipArray.read's store I/O (FilesystemStore): per shard of the region either the whole
    object (part == shard) or the stored index by one prefix/suffix read, zh_shard_ranges, and
    one range read per returned range.  Returns [(index bytes|None, shard size, [(offset,
    bytes)])] in computeChunkCoords order (None = missing key).  `drop`: (shard, range) pairs
    whose store read "fails" (returns null: the piece is not passed on).  `pad`: a range
    past the end of the file reads zero-padded, as FilesystemStore.get(keys, start, end) does
    (M/store/FilesystemStore.java:43-75)."""
    from zarrhip._lib import shard_ranges
    n = meta.ndim
    isz = lib().zh_shard_index_size(C.byref(meta))
    start = meta.chain.index_location == A.ZH_INDEX_START
    out = []
    for si, (c, path) in enumerate(zip(chunk_coords(meta, offset, shape), paths)):
        if path is None or not os.path.exists(path):
            out.append(None)
            continue
        size = os.path.getsize(path)
        lo, hi = shard_part(meta, c, offset, shape)
        with open(path, "rb") as f:
            if lo == [0] * n and hi == [meta.chunk_shape[d] for d in range(n)]:
                out.append((None, size, [(0, f.read())]))
                continue
            f.seek(0 if start else size - isz)
            idx = f.read(isz)
            rs = shard_ranges(meta, idx, size if size_known else -1, lo, hi, max_run)
            pieces = []
            for k, (o, nb) in enumerate(rs):
                if drop and (si, k) in drop:
                    continue
                if pad:  # pread: no seek (an offset beyond the file system's largest file)
                    b = os.pread(f.fileno(), nb, o)
                    pieces.append((o, b + bytes(nb - len(b))))
                    continue
                f.seek(o)
                pieces.append((o, f.read(nb)))
        out.append((idx, size if size_known else -1, pieces))
    return out


def jni_read(dev, meta, fetched, offset, shape):
    """The JNI marshalling of arrayReadPieces (java/jni/zarrhip_jni.c): no copy on the binding
    side.  Every index and piece byte[] (here: one host buffer each, as the store returned it)
    and the result's primitive array (allocated zeroed, as the JVM does) are passed to
    zh_array_read_pieces as they are; the library's pipelined read copies the sources once into
    its page-locked ring and the region straight into the result."""
    from zarrhip._lib import ShardSource
    nel = int(np.prod(shape))
    keep, shards = [], []
    for s in fetched:
        if s is None:
            shards.append(None)
            continue
        idx, size, pieces = s
        ip = None
        if idx is not None:
            ib = (C.c_char * max(1, len(idx))).from_buffer_copy(idx or b"\0")
            keep.append(ib)
            ip = C.addressof(ib)
        ps = []
        for o, b in pieces:
            pb = (C.c_char * max(1, len(b))).from_buffer_copy(b or b"\0")
            keep.append(pb)
            ps.append((o, len(b), C.addressof(pb), len(b)))
        shards.append(ShardSource(ip, len(idx) if idx is not None else 0, size, ps))
    out = np.zeros(nel, NP_DT[meta.dtype_size])
    dev.array_read_pieces(meta, shards, offset, shape, out.ctypes.data, 0)
    return out.reshape(shape)


def shard_from_pieces(meta, ss):
    """A shard the oracle can read, rebuilt from a sub-shard form (zarrhip ShardSource): the
    stored index plus the pieces at their offsets (bytes no piece holds stay zero).  Pieces
    whose host stages were undone (held bytes != stored bytes) go into a fresh raw layout
    with the index rewritten to them (+ its crc32c)."""
    isz = lib().zh_shard_index_size(C.byref(meta))
    idx = C.string_at(ss.index_ptr, ss.index_nbytes)
    start = meta.chain.index_location == A.ZH_INDEX_START
    idx = idx[:isz] if start else idx[len(idx) - isz:]
    fmt = ">QQ" if meta.chain.index_endian == A.ZH_ENDIAN_BIG else "<QQ"
    if all(nb == held for _, nb, _, held in ss.pieces):
        end = max([o + nb for o, nb, _, _ in ss.pieces] + [0])
        size = ss.shard_nbytes if ss.shard_nbytes >= 0 else end + (0 if start else isz)
        buf = bytearray(size)
        for o, nb, ptr, _ in ss.pieces:
            buf[o:o + nb] = C.string_at(ptr, nb)
        if start:
            buf[:isz] = idx
        else:
            buf[size - isz:] = idx
        return bytes(buf)
    held = {o: C.string_at(ptr, h) for o, nb, ptr, h in ss.pieces}
    ents = [struct.unpack(fmt, idx[16 * k:16 * k + 16]) for k in range((isz - 4) // 16)]
    payload, new = b"", []
    base = isz if start else 0
    for o, nb in ents:
        if o in held:
            new.append((base + len(payload), len(held[o])))
            payload += held[o]
        else:
            new.append((2 ** 64 - 1, 2 ** 64 - 1))
    body = b"".join(struct.pack(fmt, *e) for e in new)
    ib = body + struct.pack("<I", O.crc32c(body))
    return ib + payload if start else payload + ib
