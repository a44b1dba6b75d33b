"""Seeded corrupt shard indexes on the HIP path vs the oracle (SURVEY §8(c) edge cases:
erasures, collisions, out-of-range and wrapping entries).

The shard index carries no crc32c here (one chain: a recomputed, valid one), so every corrupt
entry reaches the code that interprets it: the device's resolve kernel (memory shards: ByteBufferDataProvider slices,
ShardingIndexedCodec.java:215-231, 323-330) and the library's host planner over files
(sub-shard reads: StoreHandleDataProvider.read → FilesystemStore.get, zero-padded past the end
of the file, ShardingIndexedCodec.java:340-356; whole-shard reads slice the file's bytes).
A fourth form reads the region in slabs over three contexts (zh_array_read_multi).
The third form is the Java drop-in's: HipArray.read's store reads (the stored index, then
zh_shard_ranges' ranges, zero-padded past the end of the file) handed to zh_array_read_pieces.
ZH_FUZZ_TRIALS / ZH_FUZZ_SEED widen the search (default 48 trials, seed 0).
Each trial corrupts a few entries of one or two shards with one of the mutations below and
reads a random region (or the whole array) both ways:
- both succeed → the outputs are equal, bit for bit;
- both fail → "Could not load byte data for chunk [...]" and index-checksum texts are equal;
  a wrong inner-chunk length is the documented Q12 divergence (same first words, the device
  names the chunk instead of the two lengths).
The nested chain keeps its sub-shard index crc32c, so an outer entry that moves a sub-shard
fails that checksum with the same Stored/Computed values on both sides."""
import os
import struct

import numpy as np
import pytest

import oracle as O
from helpers import (NP_DT, chunk_coords, device_read, encode_oracle, jni_fetch, jni_read,
                     rand_array)
from test_gpu_files import files_read, store_read, three_ctxs  # noqa: F401 (fixture)
from test_gpu_pieces import CHAINS, region_paths, write_store
from zarrhip import _abi as A
from zarrhip._lib import ZhError

pytestmark = pytest.mark.gpu

U64 = (1 << 64) - 1
MUTATIONS = ["missing_off", "missing_nb", "huge_off", "negative_off", "straddle_end", "nb_off_by",
             "nb_zero", "nb_huge", "wrap", "collide", "into_index"]


def _layout(meta):
    ch = meta.chain
    cps = 1
    for d in range(meta.ndim):
        cps *= meta.chunk_shape[d] // ch.inner_chunk_shape[d]
    isz = 16 * cps + (4 if ch.index_has_crc32c else 0)
    fmt = ">QQ" if ch.index_endian == A.ZH_ENDIAN_BIG else "<QQ"
    return cps, isz, ch.index_location == A.ZH_INDEX_START, fmt


def corrupt(rng, meta, shard, nbad, huge=1 << 62):
    """`shard` with `nbad` index entries mutated; returns (bytes, [mutation names]).  `huge`
    bounds the far-out offsets of huge_off."""
    cps, isz, start, fmt = _layout(meta)
    total = len(shard)
    ib = 0 if start else total - isz
    ents = [list(struct.unpack(fmt, shard[ib + 16 * k:ib + 16 * k + 16])) for k in range(cps)]
    live = [k for k in range(cps) if ents[k][0] != U64]
    names = []
    for k in rng.choice(cps, size=min(nbad, cps), replace=False):
        off, nb = ents[k]
        want = nb if off != U64 else int(np.prod(meta.chain.inner_chunk_shape[:meta.ndim])) * \
            meta.dtype_size
        mu = MUTATIONS[int(rng.integers(len(MUTATIONS)))]
        names.append(mu)
        if mu == "missing_off":
            ents[k] = [U64, int(rng.integers(0, 1 << 40))]
        elif mu == "missing_nb":
            ents[k] = [int(rng.integers(0, 1 << 40)), U64]
        elif mu == "huge_off":
            ents[k] = [int(rng.integers(total + 1, huge)), want]
        elif mu == "negative_off":
            ents[k] = [(1 << 63) + int(rng.integers(0, 1 << 40)), want]
        elif mu == "straddle_end":
            ents[k] = [max(0, total - want + int(rng.integers(1, 9))), want]
        elif mu == "nb_off_by":
            ents[k] = [off if off != U64 else 0, max(0, want + int(rng.choice([-5, -1, 1, 3])))]
        elif mu == "nb_zero":
            ents[k] = [off if off != U64 else 0, 0]
        elif mu == "nb_huge":
            ents[k] = [0, (1 << 63) + int(rng.integers(0, 1 << 20))]
        elif mu == "wrap":  # off + nb overflows 64 bits
            ents[k] = [U64 - want // 2, want]
        elif mu == "collide" and live:  # another chunk's payload: read twice, no error
            ents[k] = list(ents[int(rng.choice(live))])
        else:  # into_index (or collide with nothing live): the index bytes read as data
            ents[k] = [ib, want]
    idx = b"".join(struct.pack(fmt, *e) for e in ents)
    if meta.chain.index_has_crc32c:
        c = O.crc32c(idx)
        if rng.random() < 0.15:
            names.append("index_crc")
            c ^= 1 << int(rng.integers(32))
        idx += struct.pack("<I", c)
    out = bytearray(shard[:ib] + idx + shard[ib + isz:])
    assert len(out) == total
    if total > isz and rng.random() < 0.4:  # one payload byte flipped (a chunk crc32c, a
        names.append("flip")                 # sub-shard index, or data both sides read alike)
        k = int(rng.integers(0, total - isz)) + (isz if start else 0)
        out[k] ^= 1 << int(rng.integers(8))
    return bytes(out), names


# test_gpu_pieces' chains, plus leaves with a crc32c under nested sharding (the sub-shard
# decode checks every leaf of a referenced cell, inside the requested part or not), plus the
# shard index with its crc32c (corrupt entries under a recomputed, valid crc; sometimes the
# crc itself broken: the index checksum is then reported first)
FUZZ_CHAINS = dict(CHAINS, nested_crc=dict(sharded=True, inner_chunk_shape=[8, 8, 8],
                                           nested_chunk_shape=[4, 4, 8], inner_crc32c=True),
                   index_crc=dict(sharded=True, inner_chunk_shape=[4, 8, 8], index_crc32c=True,
                                  inner_crc32c=True, index_location=A.ZH_INDEX_START))


def make_case(chain, seed):
    shape = [24, 32, 48]
    kw = dict(index_crc32c=False)
    kw.update(FUZZ_CHAINS[chain])
    meta = A.make_meta(shape, [8, 16, 24], 4, fill=(7).to_bytes(4, "little"), **kw)
    arr = rand_array(shape, 4, seed=seed, fill_frac=0.2, fill=0)
    arr[:4, :8, :8] = 0  # an inner chunk of zeros: a missing entry
    return meta, arr


def _multi_read(ctxs, meta, src, off, shp):
    import ctypes as C
    from zarrhip import _lib
    keep = [None if b is None else (C.c_char * max(1, len(b))).from_buffer_copy(b or b"\0")
            for b in src]
    sources = [(None, 0) if k is None else (C.addressof(k), len(b)) for k, b in zip(keep, src)]
    out = np.zeros(shp, NP_DT[meta.dtype_size])
    _lib.array_read_multi(ctxs, meta, sources, off, shp, out.ctypes.data, 0)
    return out


def _outcome(fn):
    try:
        return "ok", fn()
    except (ZhError, O.OracleError) as e:
        return "err", str(e)


def _same(got, want, ctx):
    assert got[0] == want[0], (ctx, got if got[0] == "err" else "ok",
                               want if want[0] == "err" else "ok")
    if got[0] == "ok":
        np.testing.assert_array_equal(got[1], want[1], err_msg=str(ctx))
        return
    g, w = got[1], want[1]
    if w.startswith("unexpected inner chunk byte length"):  # Q12
        assert g.startswith("unexpected inner chunk byte length"), (ctx, g, w)
    else:
        assert g == w, ctx


def _region(rng, shape):
    if rng.random() < 0.4:
        return [0] * len(shape), list(shape)
    off = [int(rng.integers(0, s)) for s in shape]
    return off, [int(rng.integers(1, s - o + 1)) for s, o in zip(shape, off)]


@pytest.mark.parametrize("small_one", ["0", "1"])
@pytest.mark.parametrize("pipelined", [False, True])
@pytest.mark.parametrize("form", ["memory", "files", "pieces", "multi"])
@pytest.mark.parametrize("chain", list(FUZZ_CHAINS))
def test_corrupt_index_entries_match_oracle(dev, three_ctxs, tmp_path, monkeypatch, chain, form,
                                            pipelined, small_one):
    monkeypatch.setenv("ZH_SMALL_ONE", small_one)  # small plans in one launch (conftest)
    if pipelined:  # the reads in slabs through the page-locked rings (test_gpu_files' mode)
        for k, v in (("ZH_PIPE_MIN_KB", "1"), ("ZH_PIPE_SLAB_KB", "4"),
                     ("ZH_PIPE_CHUNK_KB", "64"), ("ZH_PIPE_THREADS", "3")):
            monkeypatch.setenv(k, v)
    meta, arr = make_case(chain, seed=211)
    shards = encode_oracle(meta, arr)
    shape = [meta.shape[d] for d in range(meta.ndim)]
    allc = chunk_coords(meta, [0] * meta.ndim, shape)
    pos = {c: i for i, c in enumerate(allc)}
    seed = int(os.environ.get("ZH_FUZZ_SEED", "0"))
    rng = np.random.default_rng(sum(map(ord, chain + form)) + 7919 * seed)
    kinds = {"ok": 0, "err": 0}
    for t in range(int(os.environ.get("ZH_FUZZ_TRIALS", "48"))):
        bad = list(shards)
        muts = []
        for i in rng.choice(len(bad), size=int(rng.integers(1, 3)), replace=False):
            if bad[i] is not None:
                bad[i], m = corrupt(rng, meta, bad[i], int(rng.integers(1, 4)))
                muts += m
        off, shp = _region(rng, shape)
        sel = chunk_coords(meta, off, shp)
        ctx = (chain, form, t, muts, off, shp)
        if form in ("memory", "multi"):
            src = [bad[pos[c]] for c in sel]
            want = _outcome(lambda: np.frombuffer(O.array_read(meta, src, off, shp),
                                                  NP_DT[meta.dtype_size]).reshape(shp))
            if form == "memory":
                got = _outcome(lambda: device_read(dev, meta, src, off, shp))
            else:  # zh_array_read_multi: the region in slabs over three contexts
                got = _outcome(lambda: _multi_read(three_ctxs, meta, src, off, shp))
        else:
            paths = write_store(tmp_path, meta, bad, tag=f"t{t}")
            rp = region_paths(meta, paths, off, shp)
            want = _outcome(lambda: store_read(meta, rp, off, shp))
            if form == "files":
                got = _outcome(lambda: files_read(dev, meta, rp, off, shp))
            else:  # HipArray.read's pieces over a FilesystemStore (size unknown: -1)
                got = _outcome(lambda: jni_read(
                    dev, meta, jni_fetch(meta, rp, off, shp, size_known=False, pad=True),
                    off, shp))
        _same(got, want, ctx)
        kinds[want[0]] += 1
    assert kinds["ok"] and kinds["err"], kinds  # both outcomes exercised


@pytest.mark.parametrize("form", ["memory", "files"])
def test_unsharded_crc_chunk_of_wrong_length(dev, tmp_path, form):
    """A whole chunk with a crc32c whose stored length is wrong: the reference's pipeline checks
    the checksum first (so the checksum fails, with its stored and computed values) unless the
    stored crc happens to match the bytes, then the length (Q12).  Device and oracle agree on
    which error and on its text, in chunk order."""
    shape = [16, 24]
    meta = A.make_meta(shape, [8, 8], 4, transpose_order=[1, 0], inner_crc32c=True)
    arr = rand_array(shape, 4, seed=227)
    chunks = encode_oracle(meta, arr)
    rng = np.random.default_rng(229)
    cases = []
    # appended bytes (checksum over the longer body fails), a truncated chunk, a chunk whose
    # longer body carries a matching crc (then the length is reported)
    longer = bytearray(chunks[1]) + bytes(8)
    cases.append({1: bytes(longer)})
    cases.append({4: chunks[4][:-12]})
    body = bytes(rng.integers(0, 256, 8 * 8 * 4 + 16, dtype=np.uint8))
    cases.append({2: body + struct.pack("<I", O.crc32c(body)), 5: chunks[5][:-1]})
    for k, mod in enumerate(cases):
        bad = [mod.get(i, c) for i, c in enumerate(chunks)]
        off, shp = [0, 0], shape
        if form == "memory":
            want = _outcome(lambda: O.array_read(meta, bad, off, shp))
            got = _outcome(lambda: device_read(dev, meta, bad, off, shp))
        else:
            paths = write_store(tmp_path, meta, bad, tag=f"u{k}")
            want = _outcome(lambda: store_read(meta, paths, off, shp))
            got = _outcome(lambda: files_read(dev, meta, paths, off, shp))
        assert want[0] == got[0] == "err", (k, want, got)
        if want[1].startswith("unexpected inner chunk byte length"):
            assert got[1].startswith("unexpected inner chunk byte length"), (k, got, want)
            assert k == 2 and got[1].endswith("for chunk [0, 2]"), got
        else:
            assert got[1] == want[1], (k, got, want)


@pytest.mark.parametrize("loc", ["end", "start"])
def test_corrupt_shard_files_through_the_array_api(dev, tmp_path, monkeypatch, loc):
    """The same corrupt entries in the shard files of an array written through the Array API
    (index [bytes, crc32c], recomputed valid over the corrupt entries), read through
    Array.read with the library's file reads (ZH_FILES=1) and with the mirror's store reads
    (ZH_FILES=0): both equal the oracle's store read — the same array or the same message.
    Huge offsets stay below 2^40 here, under every file system's largest file (Q18)."""
    import os
    import zarrhip as z
    shape = [24, 32, 48]
    data = np.random.default_rng(233).integers(0, 2 ** 32, shape, dtype=np.uint32)
    data[:8, :16, :24] = 0
    m = (z.ArrayMetadataBuilder().withShape(*shape).withDataType(z.DataType.UINT32)
         .withChunkShape(8, 16, 24).withFillValue(0)
         .withCodecs(lambda c: c.withSharding([4, 8, 8], lambda c1: c1.withTranspose([2, 0, 1])
                                              .withBytes("BIG"), loc)).build())
    z.Array.create(z.FilesystemStore(tmp_path).resolve("a"), m).write(None, data)
    a = z.Array.open(z.FilesystemStore(tmp_path).resolve("a"))
    meta = a.zmeta
    allc = chunk_coords(meta, [0, 0, 0], shape)
    path = {c: os.path.join(tmp_path, "a", "c", *map(str, c)) for c in allc}
    originals = {c: open(p, "rb").read() for c, p in path.items() if os.path.exists(p)}
    rng = np.random.default_rng(239 if loc == "end" else 241)
    for t in range(40):
        for c, b in originals.items():  # fresh files, then corrupt one or two
            with open(path[c], "wb") as f:
                f.write(b)
        for c in [list(originals)[int(i)] for i in
                  rng.choice(len(originals), size=int(rng.integers(1, 3)), replace=False)]:
            bad, _ = corrupt(rng, meta, originals[c], int(rng.integers(1, 4)), huge=1 << 40)
            with open(path[c], "wb") as f:
                f.write(bad)
        off = [int(rng.integers(0, s)) for s in shape]
        shp = [int(rng.integers(1, s - o + 1)) for s, o in zip(shape, off)]
        rp = [path[c] if os.path.exists(path[c]) else None for c in chunk_coords(meta, off, shp)]
        want = _outcome(lambda: store_read(meta, rp, off, shp))
        for files in ("1", "0"):
            monkeypatch.setenv("ZH_FILES", files)
            b = z.Array.open(z.FilesystemStore(tmp_path).resolve("a"))
            try:
                got = ("ok", b.read(off, shp))
            except z.ZarrException as e:
                got = ("err", str(e))
            _same(got, want, (loc, t, files, off, shp))
