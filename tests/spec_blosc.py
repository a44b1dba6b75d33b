"""Test-side restatement of blosc1 framing with simple LZ4 and BloscLZ *encoders*, to
produce valid frames that exercise every decoder path (literal/match length extensions,
overlapping matches, BloscLZ far distances, split and unsplit blocks, byte shuffle,
leftover blocks).  Test infrastructure only; the product decoder is zh_blosc_decompress."""
import struct
import zlib

import numpy as np


def _ext(n):
    out = bytearray()
    while n >= 255:
        out.append(255)
        n -= 255
    out.append(n)
    return bytes(out)


def lz4_compress(src, min_match=4):
    """Greedy LZ4 block encoder (last 5 bytes literal, as the format requires)."""
    src = bytes(src)
    n, i, anchor, out, table = len(src), 0, 0, bytearray(), {}
    limit = n - 5
    while i < limit - 4:
        key = src[i:i + 4]
        cand = table.get(key)
        table[key] = i
        if cand is None or i - cand > 65535:
            i += 1
            continue
        ml = 4
        while i + ml < limit and src[cand + ml] == src[i + ml]:
            ml += 1
        lit = i - anchor
        tok = (min(lit, 15) << 4) | min(ml - min_match, 15)
        out.append(tok)
        if lit >= 15:
            out += _ext(lit - 15)
        out += src[anchor:i]
        out += struct.pack("<H", i - cand)
        if ml - min_match >= 15:
            out += _ext(ml - min_match - 15)
        i += ml
        anchor = i
    lit = n - anchor
    out.append(min(lit, 15) << 4)
    if lit >= 15:
        out += _ext(lit - 15)
    out += src[anchor:]
    return bytes(out)


def blosclz_compress(src):
    """BloscLZ encoder: literal runs of <= 32, matches of length >= 3 at distance up to
    65535 + 8191 (near form below 8191, 16-bit far form above)."""
    src = bytes(src)
    n, i, out, lits, table = len(src), 0, bytearray(), bytearray(), {}

    def flush():
        nonlocal lits
        while lits:
            chunk = lits[:32]
            out.append(len(chunk) - 1)
            out.extend(chunk)
            lits = lits[32:]

    while i < n:
        key = src[i:i + 3]
        cand = table.get(key) if len(key) == 3 else None
        table[key] = i
        if cand is not None:
            dist = i - cand - 1
            ml = 0
            while i + ml < n and src[cand + ml] == src[i + ml] and ml < 600:
                ml += 1
            if ml >= 3 and dist <= 65535 + 8191:
                flush()
                ln = ml - 3
                far = dist >= 8191
                hi = 31 if far else dist >> 8
                if ln < 6:
                    out.append(((ln + 1) << 5) | hi)
                else:
                    out.append((7 << 5) | hi)
                    out += _ext(ln - 6)
                if far:
                    d = dist - 8191
                    out += bytes([255, d >> 8, d & 255])
                else:
                    out.append(dist & 255)
                i += ml
                continue
        lits.append(src[i])
        i += 1
    flush()
    return bytes(out)


def zstd_compress(b, level=3):
    """libzstd (bundled with pyarrow) — an independent zstd encoder for test vectors."""
    import pyarrow as pa
    return pa.Codec("zstd", compression_level=level).compress(bytes(b), asbytes=True)


def bit_shuffle(blk, typesize, version=2):
    """bitshuffle's bshuf_trans_bit_elem layout as blosc's bitshuffle() applies it per block:
    for byte position j and bit k, a row of ne/8 bytes whose bit m of byte q is bit k of byte
    j of element 8q+m.  Blosc format 2 (c-blosc 1.x): only blocks whose element count is a
    multiple of 8 are shuffled (others stored as is); later formats shuffle the multiple-of-8
    prefix and keep the leftover bytes."""
    ne = len(blk) // typesize
    if version <= 2 and ne % 8:
        return bytes(blk)
    ne -= ne % 8
    if ne == 0:
        return bytes(blk)
    a = np.frombuffer(blk[:ne * typesize], np.uint8).reshape(ne, typesize)
    bits = np.unpackbits(a, axis=1, bitorder="little").reshape(ne, typesize, 8)  # [e, j, k]
    rows = bits.transpose(1, 2, 0).reshape(typesize * 8, ne // 8, 8)           # [(j,k), q, m]
    out = np.packbits(rows, axis=2, bitorder="little").ravel()
    return out.tobytes() + bytes(blk[ne * typesize:])


def frame(data, typesize, blocksize, comp="lz4", shuffle=True, split=None, bitshuffle=False,
          version=2):
    """A blosc1 frame of `data` (comp: blosclz / lz4 / zlib / zstd / raw-streams)."""
    data = bytes(data)
    nbytes = len(data)
    code = {"blosclz": 0, "lz4": 1, "zlib": 3, "zstd": 4}[comp]
    if split is None:
        split = comp == "blosclz" and blocksize // typesize >= 128
    if bitshuffle:
        shuffle = False
    flags = (code << 5) | (0x01 if shuffle else 0) | (0x04 if bitshuffle else 0) | \
        (0 if split else 0x10)
    nblocks = -(-nbytes // blocksize) if nbytes else 0
    body, starts = bytearray(), []
    base = 16 + 4 * nblocks
    for k in range(nblocks):
        blk = data[k * blocksize:(k + 1) * blocksize]
        bs = len(blk)
        if shuffle and typesize > 1:
            ne = bs // typesize
            a = np.frombuffer(blk[:ne * typesize], np.uint8).reshape(ne, typesize).T.ravel()
            blk = a.tobytes() + blk[ne * typesize:]
        elif bitshuffle:
            blk = bit_shuffle(blk, typesize, version)
        nsplit = typesize if split and bs == blocksize else 1
        neb = bs // nsplit
        starts.append(base + len(body))
        for s in range(nsplit):
            part = blk[s * neb:(s + 1) * neb]
            c = {"blosclz": blosclz_compress, "lz4": lz4_compress,
                 "zlib": lambda p: zlib.compress(p, 6), "zstd": zstd_compress}[comp](part)
            if len(c) >= len(part):
                c = part  # stored raw (csize == stream size)
            body += struct.pack("<i", len(c)) + c
    hdr = struct.pack("<BBBBIII", version, 1, flags, typesize, nbytes, blocksize,
                      base + len(body))
    return hdr + struct.pack("<%di" % nblocks, *starts) + bytes(body)
