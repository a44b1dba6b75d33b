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
