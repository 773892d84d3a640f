"""Differential tests: the shim's C++ parsers (libmivgpu.so, exported for
tests) against the monitor's Python ones (monitor/feedback.py), which must
agree because the monitor reconciles each region against the same grant the
shim parsed (``expected_region``)."""

import ctypes

from hypothesis import given, settings, strategies as st

from k8s_vgpu_scheduler_amd.monitor import feedback as F

rng = st.tuples(st.integers(0, 255), st.integers(0, 63)).map(lambda t: f"{t[0]}-{t[0] + t[1]}" if t[1] else str(t[0]))
dev_mask = st.tuples(st.integers(0, 7), st.lists(rng, min_size=1, max_size=4)).map(
    lambda t: f"{t[0]}:{','.join(t[1])}")
mask = st.lists(dev_mask, max_size=4, unique_by=lambda s: s.split(":")[0]).map(";".join)


def _lib(native_build):
    lib = ctypes.CDLL(str(native_build["shim"]))
    lib.mivgpu_parse_size.restype = ctypes.c_ulonglong
    lib.mivgpu_parse_size.argtypes = [ctypes.c_char_p]
    lib.mivgpu_parse_cu_mask_count.argtypes = [ctypes.c_char_p, ctypes.c_int]
    return lib


@settings(max_examples=200, deadline=None)
@given(mask, st.integers(0, 7))
def test_cu_mask_count_agrees(native_build, m, idx):
    lib = _lib(native_build)
    assert lib.mivgpu_parse_cu_mask_count(m.encode(), idx) == F.mask_count(m, idx), (m, idx)


@settings(max_examples=200, deadline=None)
@given(st.integers(1, 10 ** 6), st.sampled_from(["", "k", "m", "g", "K", "M", "G"]))
def test_parse_size_agrees(native_build, n, suf):
    lib = _lib(native_build)
    s = f"{n}{suf}"
    assert lib.mivgpu_parse_size(s.encode()) == F.parse_size(s), s


@settings(max_examples=100, deadline=None)
@given(st.lists(st.integers(1, 31), min_size=1, max_size=3))
def test_device_plugin_mask_counted_by_the_shim(native_build, granules):
    """A grant built by the scheduler's allocator and the device plugin's env
    writer is counted by the shim as exactly the CUs granted, per device."""
    from k8s_vgpu_scheduler_amd.device.amd import cu_alloc
    from k8s_vgpu_scheduler_amd.device.types import ContainerDevice
    from k8s_vgpu_scheduler_amd.deviceplugin.allocate import PluginConfig, container_env

    lib = _lib(native_build)
    topo = cu_alloc.CUTopology()
    devs = []
    for i, g in enumerate(granules):
        ranges = cu_alloc.pick(0, g * 8, topo)
        devs.append(ContainerDevice(uuid=f"GPU-{i}", type="AMD", usedmem=10, usedcores=g * 8,
                                    custominfo={"cu_ranges": ranges}))
    env = container_env(devs, {}, PluginConfig(), "/tmp/x.cache")
    for i, g in enumerate(granules):
        assert lib.mivgpu_parse_cu_mask_count(env["HSA_CU_MASK"].encode(), i) == g * 8


pct_text = st.one_of(
    st.integers(0, 1000).map(str),
    st.tuples(st.integers(0, 999), st.integers(0, 10 ** 6), st.integers(0, 6)).map(
        lambda t: f"{t[0]}.{str(t[1]).zfill(t[2])[:t[2]]}"),
    st.text(alphabet="0123456789.+- x", max_size=8))


@settings(max_examples=300, deadline=None)
@given(pct_text)
def test_core_limit_ppm_agrees(native_build, s):
    lib = _lib(native_build)
    lib.mivgpu_parse_pct_ppm.restype = ctypes.c_uint
    lib.mivgpu_parse_pct_ppm.argtypes = [ctypes.c_char_p]
    lib.mivgpu_pct_of_ppm.argtypes = [ctypes.c_uint]
    got = lib.mivgpu_parse_pct_ppm(s.encode())
    assert got == F.core_limit_ppm(s), s
    assert lib.mivgpu_pct_of_ppm(got) == F.pct_of_ppm(got), s
