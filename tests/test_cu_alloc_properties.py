"""Properties of the XCD-balanced CU allocator (device/amd/cu_alloc.py).

No reference equivalent (the reference converts gpucores % to a count and
stops, pkg/device/amd/device.go:333-344); these pin the invariants the device
plugin relies on when it turns ranges into ``HSA_CU_MASK``: grants never
overlap, every grant covers each XCD equally, grants are whole granules, and
allocation succeeds exactly when enough granules are free."""

import pytest
from hypothesis import given, settings, strategies as st

from k8s_vgpu_scheduler_amd.device.amd import cu_alloc as A

TOPOS = [A.CUTopology(), A.CUTopology(layout="blocked"), A.CUTopology(total=64, xcds=8),
         A.CUTopology(total=32, xcds=4)]


@settings(max_examples=120, deadline=None)
@given(st.sampled_from(TOPOS), st.lists(st.integers(1, 96), max_size=12))
def test_sequential_grants_are_disjoint_balanced_and_complete(topo, requests):
    used = 0
    for n in requests:
        free_granules = sum(1 for k in range(topo.granules) if A._granule_free(used, topo, k))
        need = -(-n // topo.xcds)
        got = A.pick(used, n, topo)
        if need > free_granules:
            assert got is None
            continue
        assert got is not None
        bm = A.bitmap_from_ranges(got)
        assert bm & used == 0                                   # disjoint
        assert bin(bm).count("1") == A.round_up_cus(n, topo)    # whole granules
        assert A.is_balanced(got, topo)                         # same count on every XCD
        assert all(0 <= a <= b < topo.total for a, b in got)
        used |= bm
        assert A.free_cus(used, topo) == topo.total - bin(used).count("1")


@settings(max_examples=80, deadline=None)
@given(st.sampled_from(TOPOS), st.integers(1, 8))
def test_contiguous_run_preferred(topo, need):
    """On an empty GPU a grant is one contiguous run of granules."""
    need = min(need, topo.granules)
    got = A.pick(0, need * topo.xcds, topo)
    ks = sorted({g for g in range(topo.granules)
                 if A.bitmap_from_ranges(got) & A._granule_masks(topo)[g]})
    assert ks == list(range(ks[0], ks[0] + need))


def test_best_fit_keeps_the_large_hole():
    topo = A.CUTopology()
    # granules 0..31; occupy 2 and 10..31 except a 3-hole at 5..7 -> free: 0,1,3,4,5,6,7,8,9
    used = 0
    for k in [2] + list(range(10, 32)):
        used |= A._granule_masks(topo)[k]
    got = A.pick(used, 2 * topo.xcds, topo)
    ks = sorted({g for g in range(topo.granules) if A.bitmap_from_ranges(got) & A._granule_masks(topo)[g]})
    assert ks == [0, 1]          # the 2-run, not a slice of the 7-run 3..9


def test_fragmented_falls_back_to_lowest_free():
    topo = A.CUTopology()
    used = 0
    for k in range(1, 32, 2):      # every odd granule taken
        used |= A._granule_masks(topo)[k]
    got = A.pick(used, 3 * topo.xcds, topo)
    assert A.is_balanced(got, topo) and A.bitmap_from_ranges(got) & used == 0


@pytest.mark.parametrize("n,want", [(0, 0), (-3, 0), (1, 8), (8, 8), (9, 16), (64, 64), (255, 256), (999, 256)])
def test_round_up(n, want):
    assert A.round_up_cus(n, A.CUTopology()) == want


def test_too_large_request_refused():
    assert A.pick(0, 257, A.CUTopology()) is None
    assert A.pick(0, 0, A.CUTopology()) == []


@settings(max_examples=80, deadline=None)
@given(st.sets(st.integers(0, 255), max_size=60))
def test_ranges_bitmap_round_trip(cus):
    r = A.ranges_from_cus(cus)
    bm = A.bitmap_from_ranges(r)
    assert {i for i in range(256) if bm >> i & 1} == cus


def test_interleaved_granule_is_one_cu_per_xcd():
    topo = A.CUTopology()
    for k in (0, 5, 31):
        assert sorted(topo.xcd_of(c) for c in topo.granule_cus(k)) == list(range(8))
    blocked = A.CUTopology(layout="blocked")
    assert sorted(blocked.xcd_of(c) for c in blocked.granule_cus(3)) == list(range(8))


def test_unbalanced_mask_detected():
    topo = A.CUTopology()
    assert not A.is_balanced([(0, 3)], topo)      # XCDs 0..3 only
    assert not A.is_balanced([], topo)
    assert A.is_balanced([(0, 7)], topo)


def test_whole_gpu_share_unit_on_a_304_cu_part():
    """cuShareUnit's default means the whole GPU, not 256 CUs.  On
    a 304-CU part the pool range covers every CU, so the device plugin emits
    no HSA_CU_MASK for a pooled pod: the shim's governor time-slices it, and
    host truth treats a shimless one as ungoverned."""
    from k8s_vgpu_scheduler_amd.deviceplugin.allocate import PluginConfig, container_env
    from k8s_vgpu_scheduler_amd.device.amd.device import AMDConfig
    from k8s_vgpu_scheduler_amd.device.types import ContainerDevice
    from k8s_vgpu_scheduler_amd.smi import GPUInfo
    topo = A.CUTopology(total=304, xcds=8)
    assert AMDConfig().cu_share_unit == A.WHOLE_GPU
    assert A.share_unit(topo, A.WHOLE_GPU) == 304 and A.share_unit(topo, 512) == 304
    assert A.share_unit(A.CUTopology(), A.WHOLE_GPU) == 256
    assert A.share_unit(topo, 0) == 72 and A.share_unit(topo, 64) == 64
    r = A.pick_shared(0, {}, 32, topo, A.WHOLE_GPU)
    assert A.bitmap_from_ranges(r) == (1 << 304) - 1
    g = GPUInfo(index=0, uuid="GPU-x", rocr_id="GPU-x", name="MI355X", memory_mib=294912, cus=304)
    d = ContainerDevice(idx=0, uuid="GPU-x", type="AMD", usedmem=8192, usedcores=32,
                        custominfo={"cu_ranges": r})
    env = container_env([d], {"GPU-x": g}, PluginConfig(hook_path="/tmp/none"), "/tmp/none/x.cache")
    assert "HSA_CU_MASK" not in env and env["HIP_DEVICE_CORE_LIMIT"]
