"""The C-ABI library (libzarrhip.so) loads without a GPU, exports every symbol the header
declares, and its host-side planner matches the reference's known-answer tests."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import oracle as O
from helpers import ROOT
from zarrhip import _abi as A
from zarrhip._lib import declared_symbols, i32arr, i64arr, lib


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "zarrhip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(zh_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    L = lib()
    syms = header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(declared_symbols()) == syms


def test_struct_layout_matches_compiler():
    out = (C.c_int64 * 4)()
    assert lib().zh_abi_sizes(out, 4) == 4
    assert list(out) == [C.sizeof(A.zh_codec_chain), C.sizeof(A.zh_array_meta),
                         C.sizeof(A.zh_chunk_src), C.sizeof(A.zh_chunk_dst)]


def test_struct_layout():
    assert C.sizeof(A.zh_codec_chain) == 4 * (1 + 8 + 1 + 8 + 4 + 1 + 8 + 3 + 1)
    assert C.sizeof(A.zh_array_meta) == (16 + 64 + 32 + 8 + C.sizeof(A.zh_codec_chain) + 7) // 8 * 8
    assert C.sizeof(A.zh_chunk_src) == 16 and C.sizeof(A.zh_chunk_dst) == 24


def test_host_crc_matches_oracle():
    L = lib()
    assert L.zh_crc32c(0, b"123456789", 9) == 0xE3069283
    rng = np.random.default_rng(0)
    for n in (0, 1, 7, 8, 9, 1000, 65537):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert L.zh_crc32c(0, b, n) == O.crc32c(b)


def test_planner_kats():
    L = lib()

    def coords(ashape, cshape, off, shp):
        n = len(ashape)
        num = L.zh_compute_chunk_coords(n, i64arr(ashape), i32arr(cshape), i64arr(off),
                                        i64arr(shp), None, 0)
        out = (C.c_int64 * (num * n))()
        L.zh_compute_chunk_coords(n, i64arr(ashape), i32arr(cshape), i64arr(off), i64arr(shp),
                                  out, num)
        return [tuple(out[i * n:(i + 1) * n]) for i in range(num)]
    assert coords([100, 100], [30, 30], [50, 20], [20, 1]) == [(1, 0), (2, 0)]
    assert coords([1, 52], [1, 17], [0, 32], [1, 20]) == [(0, 1), (0, 2), (0, 3)]
    assert L.zh_compute_chunk_coords(2, i64arr([100000] * 2), i32arr([1, 1]), i64arr([0, 0]),
                                     i64arr([100000] * 2), None, 0) == -1
    co, oo, ps = i32arr([0, 0]), i32arr([0, 0]), i32arr([0, 0])
    assert L.zh_compute_projection(2, i64arr([0, 2]), i64arr([1, 52]), i32arr([1, 17]),
                                   i64arr([0, 32]), i64arr([1, 20]), co, oo, ps) == 0
    assert (list(co), list(oo), list(ps)) == ([0, 0], [0, 2], [1, 17])
    inv = i32arr([0, 0, 0])
    assert L.zh_inverse_permutation(3, i32arr([1, 2, 0]), inv) == 0 and list(inv) == [2, 0, 1]
    assert L.zh_is_permutation(3, i32arr([0, 1, 1])) == 0


@pytest.mark.parametrize("seed", range(20))
def test_planner_matches_oracle_random(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 5))
    ashape = [int(rng.integers(1, 60)) for _ in range(n)]
    cshape = [int(rng.integers(1, 20)) for _ in range(n)]
    off = [int(rng.integers(0, a)) for a in ashape]
    shp = [int(rng.integers(1, a - o + 1)) for a, o in zip(ashape, off)]
    want = O.compute_chunk_coords(ashape, cshape, off, shp)
    L = lib()
    num = L.zh_compute_chunk_coords(n, i64arr(ashape), i32arr(cshape), i64arr(off), i64arr(shp),
                                    None, 0)
    assert num == len(want)
    for c in want:
        co, oo, ps = i32arr([0] * n), i32arr([0] * n), i32arr([0] * n)
        L.zh_compute_projection(n, i64arr(c), i64arr(ashape), i32arr(cshape), i64arr(off),
                                i64arr(shp), co, oo, ps)
        assert (list(co)[:n], list(oo)[:n], list(ps)[:n]) == \
            tuple(O.compute_projection(c, ashape, cshape, off, shp))


def test_validate_meta_messages():
    L = lib()
    err = C.create_string_buffer(512)
    m = A.make_meta([16, 16], [16, 16], 4, sharded=True, inner_chunk_shape=[5, 4])
    assert L.zh_validate_meta(C.byref(m), err, 512) == A.ZH_EDATA
    assert err.value.decode() == ("Sharding inner chunk shape [5, 4] does not evenly divide the "
                                  "outer chunk size [16, 16]")
    m = A.make_meta([4, 4], [4, 4], 4, transpose_order=[0, 0])
    assert L.zh_validate_meta(C.byref(m), err, 512) == A.ZH_EDATA
    assert err.value.decode() == "Order is no permutation array"
    m = A.make_meta([4, 4], [4, 4], 4, sharded=True, inner_chunk_shape=[2, 2], index_location=7)
    assert L.zh_validate_meta(C.byref(m), err, 512) == A.ZH_EDATA
    assert err.value.decode() == 'Only index_location "start" or "end" are supported.'
    m = A.make_meta([4, 4], [4, 4], 4, sharded=True, inner_chunk_shape=[2, 2])
    assert L.zh_validate_meta(C.byref(m), err, 512) == A.ZH_OK
    assert L.zh_shard_index_size(C.byref(m)) == 16 * 4 + 4


def test_no_gpu_means_loud_failure():
    """Without a visible GPU the product refuses (no silent CPU fallback)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); from zarrhip._lib import DeviceContext\n"
            "try:\n    DeviceContext(0)\nexcept Exception as e:\n    print('raised', type(e).__name__)\n"
            "else:\n    print('ok')" % os.path.join(ROOT, "zarr-java_amd"))
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                       timeout=120)
    assert "raised ZhError" in r.stdout
