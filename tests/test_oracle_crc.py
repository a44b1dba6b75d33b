"""Chunk-level crc32c codec ([bytes, crc32c]; ZarrPythonTests "crc32c",
ZarrPythonTests.java:180-182) in the C oracle: stored chunk = payload + CRC-32C(payload) LE
(Crc32cCodec.java:50-60); decode verifies with the Crc32cCodec.java:39-44 message.  Pinned to
the bitwise CRC restatement in spec_sharding.py and the CRC-32C check value."""
import struct

import numpy as np
import pytest

import oracle as O
import spec_sharding as spec
from zarrhip import _abi as A


def test_bitwise_crc_check_value():
    assert spec.crc32c(b"123456789") == 0xE3069283 == O.crc32c(b"123456789")


@pytest.mark.parametrize("sharded", [False, True])
def test_oracle_chunk_crc_layout(sharded):
    shape = [8, 12]
    m = A.make_meta(shape, [4, 12], 4, sharded=sharded,
                    inner_chunk_shape=[2, 6] if sharded else None, inner_crc32c=True)
    data = np.arange(96, dtype=np.uint32).reshape(shape) + 1
    enc = O.array_write(m, data.tobytes(), [0, 0], shape)
    if not sharded:
        payload = data[:4].tobytes()
        assert enc[0] == payload + struct.pack("<I", spec.crc32c(payload))
    else:
        shard = enc[0]
        isz = 16 * 4 + 4
        off, nb = struct.unpack("<QQ", shard[len(shard) - isz:len(shard) - isz + 16])
        assert nb == 2 * 6 * 4 + 4
        payload = data[0:2, 0:6].tobytes()
        assert shard[off:off + nb] == payload + struct.pack("<I", spec.crc32c(payload))
    got = np.frombuffer(O.array_read(m, enc, [0, 0], shape), np.uint32).reshape(shape)
    np.testing.assert_array_equal(got, data)


@pytest.mark.parametrize("sharded", [False, True])
def test_oracle_chunk_crc_mismatch_message(sharded):
    shape = [4, 4]
    m = A.make_meta(shape, [4, 4], 4, sharded=sharded, inner_chunk_shape=[2, 2] if sharded else None,
                    inner_crc32c=True)
    data = np.arange(16, dtype=np.uint32).reshape(shape) + 1
    b = bytearray(O.array_write(m, data.tobytes(), [0, 0], shape)[0])
    b[5] ^= 1  # inside the first (inner) chunk's payload
    with pytest.raises(O.OracleError, match=r"The checksum of the sharding index is invalid\. "
                                             r"Stored: -?\d+ Computed: -?\d+"):
        O.array_read(m, [bytes(b)], [0, 0], shape)


@pytest.mark.parametrize("loc,stored_crc", [("end", 0xB756D1D4), ("start", 0x56F05363)])
def test_oracle_inner_chunk_crc_on_reference_bytes(loc, stored_crc):
    """The oracle's inner crc32c encode (Crc32cCodec.encode, Crc32cCodec.java:50-60) of a
    chunk whose payload is the reference fixture's 64-byte index body appends the crc the
    reference stored for those bytes."""
    import os
    import struct
    import numpy as np
    from helpers import GOLDEN, encode_oracle
    from zarrhip import _abi as A
    raw = open(os.path.join(GOLDEN, "sharding_index_location", loc, "c", "0", "0", "0"),
               "rb").read()
    body = raw[:64] if loc == "start" else raw[len(raw) - 68:len(raw) - 4]
    meta = A.make_meta([4, 4], [4, 4], 4, endian=A.ZH_ENDIAN_LITTLE, sharded=True,
                       inner_chunk_shape=[4, 4], inner_crc32c=True)
    shard = encode_oracle(meta, np.frombuffer(body, "<u4").reshape(4, 4))[0]
    assert shard[:64] == body and struct.unpack("<I", shard[64:68])[0] == stored_crc
