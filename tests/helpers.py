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
