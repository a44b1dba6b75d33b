"""zh_shard_ranges (host, no GPU): the byte ranges of a stored shard a sub-shard part needs —
the I/O of StoreHandleDataProvider (ShardingIndexedCodec.java:190-230, 333-357) that the
JNI shim performs before zh_array_read_pieces.  Checked against a plain-Python model of the
same rule on oracle-encoded shards and on hand-made indexes."""
import ctypes as C
import struct

import numpy as np
import pytest

import oracle as O
from helpers import encode_oracle, rand_array
from zarrhip import _abi as A
from zarrhip._lib import lib, shard_ranges

M1 = 2 ** 64 - 1


def model_ranges(meta, index, size, lo, hi, max_run, unit=None):
    """The rule restated: entries of the part's box (C order), missing (-1) dropped, unreadable
    ones dropped, sorted, overlaps united, adjacent ranges merged up to max_run."""
    n = meta.ndim
    unit = unit or [meta.chain.inner_chunk_shape[d] for d in range(n)]
    cps = [meta.chunk_shape[d] // unit[d] for d in range(n)]
    fmt = ">QQ" if meta.chain.index_endian == A.ZH_ENDIAN_BIG else "<QQ"
    ents = []
    for c in np.ndindex(*[(hi[d] - 1) // unit[d] - lo[d] // unit[d] + 1 for d in range(n)]):
        cc = [lo[d] // unit[d] + c[d] for d in range(n)]
        lin = int(np.ravel_multi_index(cc, cps))
        off, nb = struct.unpack(fmt, index[16 * lin:16 * lin + 16])
        if off == M1 or nb == M1 or nb == 0 or off >= 2 ** 63 or nb > 2 ** 31 - 1:
            continue
        if size >= 0 and (off > size or nb > size - off):
            continue
        ents.append((off, nb))
    out = []
    for off, nb in sorted(ents):
        if out and max_run <= 0:  # one range per entry (host-decoded chains): duplicates once
            if (off, nb) != out[-1]:
                out.append((off, nb))
            continue
        if out and off < out[-1][0] + out[-1][1]:
            o0, n0 = out[-1]
            if off + nb <= o0 + n0:
                continue
            if off + nb - o0 <= 2 ** 31 - 1:
                out[-1] = (o0, off + nb - o0)
            else:  # a union longer than one Java read: continue from the previous end
                out.append((o0 + n0, off + nb - o0 - n0))
        elif out and off == out[-1][0] + out[-1][1] and max_run > 0 and out[-1][1] + nb <= max_run:
            out[-1] = (out[-1][0], out[-1][1] + nb)
        else:
            out.append((off, nb))
    return out


def index_of(meta, shard):
    isz = lib().zh_shard_index_size(C.byref(meta))
    return shard[:isz] if meta.chain.index_location == A.ZH_INDEX_START else shard[-isz:]


@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
@pytest.mark.parametrize("be", [A.ZH_ENDIAN_LITTLE, A.ZH_ENDIAN_BIG])
def test_ranges_match_model_on_oracle_shards(loc, be):
    shape = [32, 48, 40]
    meta = A.make_meta(shape, [16, 24, 40], 4, sharded=True, inner_chunk_shape=[4, 8, 10],
                       index_location=loc, index_endian=be, endian=A.ZH_ENDIAN_BIG)
    arr = rand_array(shape, 4, seed=5, fill_frac=0.3)
    arr[:4, :8, :10] = 0  # one all-fill inner chunk: a missing (-1) entry
    shards = encode_oracle(meta, arr)
    shard = shards[0]
    idx = index_of(meta, shard)
    for lo, hi, run in [([0, 0, 0], [16, 24, 40], 1 << 30), ([1, 3, 5], [9, 20, 33], 0),
                        ([4, 8, 0], [8, 16, 40], 1 << 20), ([0, 0, 0], [16, 24, 40], 4000)]:
        got = shard_ranges(meta, idx, len(shard), lo, hi, run)
        assert got == model_ranges(meta, idx, len(shard), lo, hi, run)
        for o, nb in got:  # every range lies inside the shard
            assert 0 <= o and o + nb <= len(shard)


def test_ranges_skip_unreadable_entries_and_unknown_size():
    meta = A.make_meta([8, 8], [8, 8], 1, sharded=True, inner_chunk_shape=[4, 4])
    ents = [(0, 16), (16, 16), (1 << 40, 16), (M1, M1)]  # the third lies beyond the shard
    body = b"".join(struct.pack("<QQ", *e) for e in ents)
    idx = body + struct.pack("<I", O.crc32c(body))
    size = 32 + len(idx)
    assert shard_ranges(meta, idx, size, [0, 0], [8, 8], 1 << 20) == [(0, 32)]
    # size unknown (StoreHandle.getSize() == -1): the far entry is kept (the store read decides)
    assert shard_ranges(meta, idx, -1, [0, 0], [8, 8], 0) == [(0, 16), (16, 16), (1 << 40, 16)]
    # a Java array holds < 2^31 bytes: longer entries are never fetched
    big = struct.pack("<QQ", 0, 1 << 31) + body[16:]
    assert shard_ranges(meta, big + idx[-4:], -1, [0, 0], [8, 8], 0)[0] == (16, 16)


def test_ranges_nested_cells_are_read_whole():
    shape = [16, 16]
    meta = A.make_meta(shape, [16, 16], 2, sharded=True, inner_chunk_shape=[8, 8],
                       nested_chunk_shape=[4, 4])
    shard = encode_oracle(meta, rand_array(shape, 2, seed=9))[0]
    idx = index_of(meta, shard)
    got = shard_ranges(meta, idx, len(shard), [1, 9], [6, 13], 0)
    assert got == model_ranges(meta, idx, len(shard), [1, 9], [6, 13], 0)
    assert len(got) == 1  # the one level-1 cell (sub-shard) the part touches, whole
    assert got[0][1] > 16 * 4  # a whole sub-shard: leaves + its own index


def test_ranges_errors():
    meta = A.make_meta([8, 8], [8, 8], 1, sharded=True, inner_chunk_shape=[4, 4])
    L = lib()
    buf = (C.c_char * 68)()
    lo = (C.c_int64 * 2)(0, 0)
    hi = (C.c_int64 * 2)(8, 8)
    assert L.zh_shard_ranges(C.byref(meta), buf, 60, 100, lo, hi, 0, None, 0) == -A.ZH_EINVAL
    bad = (C.c_int64 * 2)(8, 9)
    assert L.zh_shard_ranges(C.byref(meta), buf, 68, 100, lo, bad, 0, None, 0) == -A.ZH_EINVAL
    un = A.make_meta([8, 8], [8, 8], 1)
    assert L.zh_shard_ranges(C.byref(un), buf, 68, 100, lo, hi, 0, None, 0) == -A.ZH_EINVAL


def _index(ents, fmt="<QQ"):
    body = b"".join(struct.pack(fmt, *e) for e in ents)
    return body + struct.pack("<I", O.crc32c(body))


def test_ranges_overlapping_entries():
    """Entries that share stored bytes (a writer may point several inner chunks at one payload):
    raw reads (max_run > 0) unite them into one range; host-decoded chains (max_run == 0) read
    and decode each entry on its own, as StoreHandleDataProvider does, so every distinct entry
    is its own range and exact duplicates are read once."""
    meta = A.make_meta([8, 8], [8, 8], 1, sharded=True, inner_chunk_shape=[4, 4])
    idx = _index([(0, 16), (0, 16), (8, 16), (40, 8)])
    assert shard_ranges(meta, idx, -1, [0, 0], [8, 8], 1 << 20) == [(0, 24), (40, 8)]
    assert shard_ranges(meta, idx, -1, [0, 0], [8, 8], 0) == [(0, 16), (8, 16), (40, 8)]
    for run in (0, 1 << 20):
        assert shard_ranges(meta, idx, -1, [0, 0], [8, 8], run) == \
            model_ranges(meta, idx, -1, [0, 0], [8, 8], run)


def test_ranges_union_never_exceeds_a_java_read():
    """Two overlapping entries of 2^30 + 2^29 bytes each, 2^30 apart: their union (2^31 + 2^29)
    would not fit one byte[]; the second range continues from the first one's end."""
    meta = A.make_meta([8, 8], [8, 8], 1, sharded=True, inner_chunk_shape=[4, 4])
    a, b = (0, 3 << 29), (1 << 30, 3 << 29)
    idx = _index([a, b, (M1, M1), (M1, M1)])
    got = shard_ranges(meta, idx, -1, [0, 0], [8, 8], 1 << 40)
    assert got == [(0, 3 << 29), (3 << 29, (1 << 30) + (3 << 29) - (3 << 29))]
    assert all(nb <= 2 ** 31 - 1 for _, nb in got)
    assert got == model_ranges(meta, idx, -1, [0, 0], [8, 8], 1 << 40)


@pytest.mark.parametrize("loc", [A.ZH_INDEX_END, A.ZH_INDEX_START])
def test_shard_index_check_matches_the_oracle_message(loc):
    """zh_shard_index_check (Crc32cCodec.decode of the index on the host, for reads whose host
    work the index decides): an intact index passes, a flipped byte fails with exactly the
    message the oracle's read raises, a chain without an index crc32c is never checked."""
    from zarrhip._lib import ZhError, shard_index_check
    shape = [16, 16]
    meta = A.make_meta(shape, [16, 16], 4, sharded=True, inner_chunk_shape=[4, 8],
                       index_location=loc, endian=A.ZH_ENDIAN_BIG)
    shard = encode_oracle(meta, rand_array(shape, 4, seed=3))[0]
    idx = index_of(meta, shard)
    shard_index_check(meta, idx)
    shard_index_check(meta, b"junk" + idx if loc == A.ZH_INDEX_END else idx + b"junk")
    isz = len(idx)
    pos = 5 if loc == A.ZH_INDEX_START else len(shard) - isz + 5
    bad = bytearray(shard)
    bad[pos] ^= 0x10
    with pytest.raises(O.OracleError) as eo:
        O.array_read(meta, [bytes(bad)], [0, 0], shape)
    with pytest.raises(ZhError) as ed:
        shard_index_check(meta, index_of(meta, bytes(bad)))
    assert ed.value.status == A.ZH_EDATA
    assert str(ed.value) == str(eo.value)
    assert str(ed.value).startswith("The checksum of the sharding index is invalid. Stored: ")
    nocrc = A.make_meta(shape, [16, 16], 4, sharded=True, inner_chunk_shape=[4, 8],
                        index_location=loc, index_crc32c=False)
    shard_index_check(nocrc, b"\xff" * lib().zh_shard_index_size(C.byref(nocrc)))
