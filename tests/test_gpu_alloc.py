"""Device allocator: views of a ZH_MALLOC_SCATTER arena (its physical chunks mapped again at a
fresh virtual range, zh_device_scatter_view) and the store-only write probe
(zh_device_write_rate), DESIGN §4 "Placement".  Small arenas of 2 MiB chunks."""
import numpy as np
import pytest

from zarrhip import _abi as A
from zarrhip._lib import ZhError

pytestmark = pytest.mark.gpu

MB2 = 2 << 20


def _chunks(dev, ptr, n):
    raw = np.frombuffer(dev.d2h(ptr, n * MB2), dtype=np.uint32)
    return [raw[i * MB2 // 4:(i + 1) * MB2 // 4].copy() for i in range(n)]


@pytest.mark.parametrize("n", [2, 5, 7])
def test_views_alias_the_same_chunks(dev, monkeypatch, n):
    monkeypatch.setenv("ZH_SCATTER_MB", "2")
    p = dev.malloc(n * MB2, A.ZH_MALLOC_SCATTER | A.ZH_MALLOC_REQUIRE)
    views = []
    try:
        dev.synth_fill(p, n * MB2 // 4, 4, 0, 77)
        dev.sync()
        before = _chunks(dev, p, n)
        keys = {c[0]: i for i, c in enumerate(before)}  # the first word tells the chunks apart
        assert len(keys) == n
        perms = set()
        for order in (0, 1, 2, 3):
            v = dev.scatter_view(p, order)
            views.append(v)
            assert v != p
            after = _chunks(dev, v, n)
            perm = [keys[c[0]] for c in after]
            assert sorted(perm) == list(range(n))  # a permutation of the same physical chunks
            for slot, src in enumerate(perm):
                assert np.array_equal(after[slot], before[src])
            if order == 0:
                assert perm == list(range(n))
            perms.add(tuple(perm))
        assert len(perms) > 1  # the orders differ
        # a store through a view is seen through the allocation (aliasing, not a copy)
        dev.memset(views[0], 0xAB, 4096)
        dev.sync()
        assert dev.d2h(p, 4096) == b"\xab" * 4096
    finally:
        for v in views:
            dev.free(v)
        dev.free(p)


def test_view_rejects_plain_allocations_and_views(dev, monkeypatch):
    p = dev.malloc(1 << 20, 0)
    try:
        with pytest.raises(ZhError):
            dev.scatter_view(p, 1)
    finally:
        dev.free(p)
    monkeypatch.setenv("ZH_SCATTER_MB", "2")
    q = dev.malloc(2 * MB2, A.ZH_MALLOC_SCATTER | A.ZH_MALLOC_REQUIRE)
    v = dev.scatter_view(q, 1)
    try:
        with pytest.raises(ZhError):
            dev.scatter_view(v, 0)
    finally:
        dev.free(v)
        dev.free(q)


@pytest.mark.parametrize("pattern", [0, 1])
def test_write_rate_probe(dev, pattern):
    nb = 64 << 20
    p = dev.malloc(nb, 0)
    try:
        g = dev.write_rate(p, nb, pattern, 3)
        assert 10.0 < g < 20000.0  # GB/s, plausible for HBM
        with pytest.raises(ZhError):
            dev.write_rate(p, nb, 2, 3)
    finally:
        dev.free(p)


def test_freed_ranges_are_not_handed_out_again(dev, monkeypatch):
    """A freed scatter range is never reserved again: a new allocation mapped at a reused
    address was partly written through the old translations on ROCm 7.2 (kernel stores went
    elsewhere, a D2H copy then read zeros)."""
    monkeypatch.setenv("ZH_SCATTER_MB", "2")
    seen = set()
    for rnd, n in enumerate((2, 5, 3, 7, 4)):
        p = dev.malloc(n * MB2, A.ZH_MALLOC_SCATTER | A.ZH_MALLOC_REQUIRE)
        try:
            assert p not in seen
            seen.add(p)
            nel = n * MB2 // 4
            dev.synth_fill(p, nel, 4, 0, 100 + rnd)
            dev.sync()
            assert dev.synth_verify(p, [nel], [0], [nel], 4, 100 + rnd) == 0
            host = np.frombuffer(dev.d2h(p, n * MB2), dtype=np.uint32)
            q = dev.malloc(n * MB2, 0)
            dev.memcpy(q, p, n * MB2, 2)  # device to device, then checked by the kernel
            assert dev.synth_verify(q, [nel], [0], [nel], 4, 100 + rnd) == 0
            dev.free(q)
            assert np.count_nonzero(host == 0) < nel // 1000  # no chunk read back as zeros
        finally:
            dev.free(p)


def test_calibrated_arena(dev, monkeypatch):
    """ZH_MALLOC_CALIBRATE: two candidate arenas probed, the faster kept, the other freed; the
    kept arena holds data like any other."""
    tries = 2
    monkeypatch.setenv("ZH_SCATTER_MB", "2")
    n = 9 * MB2 + 4096  # ten chunks, the last one partly used
    p = dev.malloc(n, A.ZH_MALLOC_SCATTER | A.ZH_MALLOC_CALIBRATE | A.ZH_MALLOC_REQUIRE)
    try:
        probes, chosen = dev.alloc_probes(p)
        assert len(probes) == tries and 0 <= chosen < tries
        assert probes[chosen] == max(probes) and min(probes) > 0
        nel = n // 4
        dev.synth_fill(p, nel, 4, 0, 5)
        assert dev.synth_verify(p, [nel], [0], [nel], 4, 5) == 0
    finally:
        dev.free(p)
    q = dev.malloc(MB2, A.ZH_MALLOC_SCATTER | A.ZH_MALLOC_REQUIRE)
    try:
        assert dev.alloc_probes(q) == ([], -1)
    finally:
        dev.free(q)


def test_default_kind_by_size(dev):
    """zh_device_malloc's default kind (flags 0): a buffer of 1 GiB or more is built from 1 GiB
    physical chunks (a scatter allocation: scatter_view accepts it), a smaller one and
    ZH_MALLOC_PLAIN are hipMalloc'd (scatter_view refuses them); data round-trips in each."""
    big = dev.malloc((1 << 30) + 4096, 0)
    small = dev.malloc(64 << 20, 0)
    plain = dev.malloc(1 << 30, A.ZH_MALLOC_PLAIN)
    try:
        v = dev.scatter_view(big, 0)
        dev.free(v)
        for p in (small, plain):
            with pytest.raises(ZhError):
                dev.scatter_view(p, 0)
        for p, nb in ((big, (1 << 30) + 4096), (small, 64 << 20), (plain, 1 << 30)):
            nel = nb // 4
            dev.synth_fill(p, nel, 4, 0, 77)
            assert dev.synth_verify(p, [nel], [0], [nel], 4, 77) == 0
    finally:
        for p in (big, small, plain):
            dev.free(p)
