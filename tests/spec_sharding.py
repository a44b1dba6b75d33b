"""Independent numpy restatement of the Zarr v3 `sharding_indexed` byte format (SURVEY.md
Appendix B; ShardingIndexedCodec.java:105-168 encode, :183-243 decode), recursive so that a
level's inner codec may itself be sharding.  Test infrastructure only: it pins the C oracle's
nested-sharding path, for which the reference holds no fixture (its only nested case,
ZarrPythonTests "sharding_nested", needs zarr-python, which is not installed).

A level is a dict: {"chunk": [...], "index_be": bool, "crc": bool, "start": bool}; the leaf
codec is bytes(endian) without transpose.  Layout is C order over non-fill chunks (the
reference's order is nondeterministic, Q7; decode is index-driven either way).
"""
import struct

import numpy as np

MISSING = 2 ** 64 - 1


def crc32c(data):
    """Bitwise CRC-32C (reflected 0x82F63B78), CRC32C.java:14-164."""
    c = 0xFFFFFFFF
    for b in bytes(data):
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
    return c ^ 0xFFFFFFFF


def _index_size(shape, level):
    n = int(np.prod([s // c for s, c in zip(shape, level["chunk"])]))
    return 16 * n + (4 if level["crc"] else 0)


def encode(arr, levels, leaf_be=False, fill=0):
    """Encode the chunk `arr` (shape = the outer chunk) through len(levels) sharding levels."""
    lv = levels[0]
    shape = arr.shape
    cs = lv["chunk"]
    grid = [s // c for s, c in zip(shape, cs)]
    isz = _index_size(shape, lv)
    fmt = ">QQ" if lv["index_be"] else "<QQ"
    entries, payload, pos = [], [], isz if lv["start"] else 0
    for ic in np.ndindex(*grid):
        sub = arr[tuple(slice(i * c, (i + 1) * c) for i, c in zip(ic, cs))]
        if np.all(sub == fill):
            entries.append((MISSING, MISSING))
            continue
        if len(levels) > 1:
            b = encode(sub, levels[1:], leaf_be, fill)
        else:
            b = sub.astype(sub.dtype.newbyteorder(">" if leaf_be else "<")).tobytes()
        entries.append((pos, len(b)))
        payload.append(b)
        pos += len(b)
    idx = b"".join(struct.pack(fmt, *e) for e in entries)
    if lv["crc"]:
        idx += struct.pack("<I", crc32c(idx))
    pb = b"".join(payload)
    return idx + pb if lv["start"] else pb + idx


def decode(buf, shape, levels, dtype, leaf_be=False):
    """Decode one shard of `shape`; missing chunks at any level read as 0 (Q1)."""
    lv = levels[0]
    cs = lv["chunk"]
    grid = [s // c for s, c in zip(shape, cs)]
    isz = _index_size(shape, lv)
    idx = buf[:isz] if lv["start"] else buf[len(buf) - isz:]
    if lv["crc"]:
        stored = struct.unpack("<I", idx[-4:])[0]
        if crc32c(idx[:-4]) != stored:
            raise ValueError("The checksum of the sharding index is invalid.")
    fmt = ">QQ" if lv["index_be"] else "<QQ"
    out = np.zeros(shape, dtype)
    for k, ic in enumerate(np.ndindex(*grid)):
        off, nb = struct.unpack(fmt, idx[16 * k:16 * k + 16])
        if off == MISSING or nb == MISSING:
            continue
        b = buf[off:off + nb]
        sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(ic, cs))
        if len(levels) > 1:
            out[sl] = decode(b, cs, levels[1:], dtype, leaf_be)
        else:
            dt = np.dtype(dtype).newbyteorder(">" if leaf_be else "<")
            out[sl] = np.frombuffer(b, dt).reshape(cs)
    return out
