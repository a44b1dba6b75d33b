"""reshape codec (M/v3/codec/core/ReshapeCodec.java) in the host mirror: the reference's
ReshapeCodecTest cases (valid / invalid configurations, resolveArrayMetadata grids), and the
fold of [transpose | reshape]* into one chunk-dim permutation checked against a numpy model
of the codec semantics (encode applies the array→array codecs in order; bytes is C order)."""
import numpy as np
import pytest

import zarrhip as z
from zarrhip.codecs import _aa_order

VALID = [  # ReshapeCodecTest.validReshapes
    ([2, 3, 4], [[0, 1], [2]], [6, 4]),
    ([2, 3, 4], [[0, 1, 2]], [24]),
    ([2, 3, 4], [-1], [24]),
    ([4, 5, 6, 3], [[0, 1], [2], 3], [20, 6, 3]),
    ([6, 4], [2, 3, 4], [2, 3, 4]),
    ([4, 4], [1, [0], [1]], [1, 4, 4]),
    ([2, 3, 4], [6, -1], [6, 4]),
    ([2, 3, 4], [[0], -1], [2, 12]),
    ([2, 3, 4], [[0], [1], [2]], [2, 3, 4]),
    ([2, 3], [[0], [1], 1], [2, 3, 1]),
    ([2, 2, 2, 2, 2], [-1], [32]),
]
INVALID = [  # ReshapeCodecTest.invalidReshapes
    ([2, 3], [5]), ([2, 3, 4], [7, -1]), ([2, 3, 4], [-1, -1]), ([2, 3], [0, 6]),
    ([2, 3], [-2, 3]), ([2, 3], [[1], [0]]), ([2, 3, 4], [[1, 0], [2]]), ([2, 3], [[0, 0]]),
    ([2, 3], [[5]]), ([2, 2, 2], [[2], 4]), ([2, 3], []),
]


@pytest.mark.parametrize("inp,shape,want", VALID)
def test_valid_reshapes(inp, shape, want):
    out, _ = z.ReshapeCodec(shape).resolve(inp)
    assert out == want
    a = np.arange(int(np.prod(inp)))
    assert (a.reshape(inp).reshape(out).ravel() == a).all()


@pytest.mark.parametrize("inp,shape", INVALID)
def test_invalid_reshapes(inp, shape):
    with pytest.raises(z.ZarrException, match="^reshape codec: "):
        z.ReshapeCodec(shape).resolve(inp)


def test_resolve_array_metadata_grids():
    # testResolveArrayMetadataMergesChunkGrid / KeepsGridPerOutputDim
    assert z.ReshapeCodec([[0, 1]]).resolve_array_metadata([8, 6], [4, 3]) == ([48], [12])
    assert z.ReshapeCodec([[0, 1], [2]]).resolve_array_metadata([8, 6, 4], [4, 3, 4]) == \
        ([48, 4], [12, 4])


def test_invalid_reshape_rejected_at_create():
    """testInvalidReshapeFailsOnWrite: product 5 != 16."""
    m = (z.ArrayMetadataBuilder().withShape(4, 4).withDataType(z.DataType.UINT32)
         .withChunkShape(4, 4).withCodecs(lambda c: c.withReshape([5]).withBytes("LITTLE")).build())
    with pytest.raises(z.ZarrException):
        z.Array.create(z.MemoryStore().resolve("r"), m)


def _model_payload(chunk, aa):
    x = chunk
    for c in aa:
        if isinstance(c, z.TransposeCodec):
            x = x.transpose(c.order)
        else:
            x = x.reshape(c.resolve(list(x.shape))[0])
    return np.ascontiguousarray(x).tobytes()


FOLDS = [
    ([4, 5, 6], [z.ReshapeCodec([[0, 1], [2]])]),
    ([4, 5, 6], [z.ReshapeCodec([2, 2, 5, 6])]),
    ([4, 5, 6], [z.TransposeCodec([2, 1, 0]), z.ReshapeCodec([[0, 1], [2]])]),
    ([4, 4, 4], [z.TransposeCodec([2, 1, 0]), z.ReshapeCodec([[0, 1], [2]])]),
    ([4, 5, 6], [z.ReshapeCodec([[0, 1], [2]]), z.TransposeCodec([1, 0])]),
    ([4, 5, 6, 3], [z.ReshapeCodec([[0, 1], [2], 3]), z.TransposeCodec([2, 0, 1])]),
    ([4, 5, 6], [z.ReshapeCodec([1, [0], [1, 2]]), z.TransposeCodec([2, 0, 1])]),
    ([2, 3, 4], [z.TransposeCodec([1, 2, 0]), z.ReshapeCodec([[0, 1], [2]]),
                 z.TransposeCodec([1, 0])]),
    ([3, 1, 4], [z.ReshapeCodec([3, 4]), z.TransposeCodec([1, 0])]),
]


@pytest.mark.parametrize("shape,aa", FOLDS)
def test_fold_matches_codec_semantics(shape, aa):
    chunk = np.arange(int(np.prod(shape)), dtype=np.uint32).reshape(shape)
    order = _aa_order(aa, len(shape), shape)
    got = chunk.transpose(order if order is not None else list(range(len(shape))))
    assert np.ascontiguousarray(got).tobytes() == _model_payload(chunk, aa)


def test_split_then_transpose_is_unsupported():
    with pytest.raises(z.UnsupportedChainError):
        _aa_order([z.ReshapeCodec([2, 2, 5, 6]), z.TransposeCodec([3, 2, 1, 0])], 3, [4, 5, 6])


def test_reshape_json_roundtrip():
    c = z.ReshapeCodec([[0, 1], [2], 3])
    j = c.to_json()
    assert j == {"name": "reshape", "configuration": {"shape": [[0, 1], [2], 3]}}
    assert z.CodecRegistry.codec_from_json(j).shape == [[0, 1], [2], 3]
