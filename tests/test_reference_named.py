"""ZarrV3Test cases on the path that the other files cover under other names, restated here
under the reference's own names (ZarrV3Test.java): invalid transpose orders, zstd read/write
at several levels with and without the checksum, and sharding over zstd inner chunks."""
import numpy as np
import pytest

import zarrhip as z
from zarrhip.codecs import TransposeCodec


@pytest.mark.parametrize("order", [[1, 0, 0], [1, 2, 3], [1, 2, 3, 0], [1, 2]])
def test_check_invalid_transpose_order(order):
    """testCheckInvalidTransposeOrder (ZarrV3Test.java:81-88, 267-281): encode with such an
    order on a 2x3x3 array throws ZarrException."""
    with pytest.raises(z.ZarrException):
        TransposeCodec(order).validate(3)


def _testdata():
    return np.arange(16 * 16 * 16, dtype=np.uint32).reshape(16, 16, 16)


@pytest.mark.gpu
@pytest.mark.parametrize("level,checksum", [(0, True), (5, False), (22, True)])
def test_zstd_codec_read_write(tmp_path, level, checksum):
    """testZstdCodecReadWrite (ZarrV3Test.java:205-225)."""
    m = (z.ArrayMetadataBuilder().withShape(16, 16, 16).withDataType(z.DataType.UINT32)
         .withChunkShape(2, 4, 8).withFillValue(0)
         .withCodecs(lambda c: c.withZstd(level, checksum)).build())
    h = z.FilesystemStore(tmp_path).resolve("testZstdCodecReadWrite", f"checksum_{checksum}",
                                             f"level_{level}")
    z.Array.create(h, m).write(None, _testdata())
    np.testing.assert_array_equal(z.Array.open(h).read(), _testdata())


@pytest.mark.gpu
def test_sharding_with_zstd_codec_read_write(tmp_path):
    """testShardingWithZstdCodecReadWrite (ZarrV3Test.java:227-246): shards 8³ of 2x4x8 inner
    chunks, inner codecs [zstd] (bytes auto-inserted)."""
    m = (z.ArrayMetadataBuilder().withShape(16, 16, 16).withDataType(z.DataType.UINT32)
         .withChunkShape(8, 8, 8).withFillValue(0)
         .withCodecs(lambda c: c.withSharding([2, 4, 8], lambda c1: c1.withZstd())).build())
    h = z.FilesystemStore(tmp_path).resolve("testShardingWithZstdCodecReadWrite")
    z.Array.create(h, m).write(None, _testdata())
    np.testing.assert_array_equal(z.Array.open(h).read(), _testdata())
