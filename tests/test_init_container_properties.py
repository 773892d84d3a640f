"""Properties of init-container-aware accounting (device/init_container.py,
reference pkg/device/initContainer.go and docs/develop/initContainer-design.md):
for every device the collapsed footprint is max(peak init, sum app), never
below the app-only footprint, and its CU ranges are the union of all
containers' ranges."""

from hypothesis import given, settings, strategies as st

from k8s_vgpu_scheduler_amd.device.codec import merge_ranges
from k8s_vgpu_scheduler_amd.device.init_container import (app_containers_only_device_usage,
                                                          collapse_init_container_usage)
from k8s_vgpu_scheduler_amd.device.types import ContainerDevice
from k8s_vgpu_scheduler_amd.k8s.fake import make_pod

UUIDS = ["GPU-0", "GPU-1", "GPU-2"]
entry = st.tuples(st.sampled_from(UUIDS), st.integers(0, 1000), st.integers(0, 256),
                  st.lists(st.tuples(st.integers(0, 255), st.integers(0, 15)), max_size=2))
ctr = st.lists(entry, max_size=3, unique_by=lambda e: e[0])


def _build(containers):
    out = []
    for c in containers:
        devs = []
        for u, m, cu, rs in c:
            ranges = [(a, a + w) for a, w in rs]
            devs.append(ContainerDevice(uuid=u, type="AMD", usedmem=m, usedcores=cu,
                                        custominfo={"cu_ranges": ranges} if ranges else {}))
        out.append(devs)
    return out


@settings(max_examples=150, deadline=None)
@given(st.lists(ctr, max_size=3), st.lists(ctr, min_size=1, max_size=4))
def test_collapse_is_max_of_init_peak_and_app_sum(init, app):
    pod = make_pod("p", containers=[{"name": f"a{i}"} for i in range(len(app))],
                   init_containers=[{"name": f"i{i}"} for i in range(len(init))])
    raw = {"AMD": _build(init) + _build(app)}
    eff = {d.uuid: d for d in collapse_init_container_usage(pod, raw)["AMD"][0]}
    only = {d.uuid: d for d in app_containers_only_device_usage(pod, raw)["AMD"][0]}
    for u in UUIDS:
        peak_m = max([m for c in init for uu, m, _, _ in c if uu == u], default=0)
        peak_c = max([cu for c in init for uu, _, cu, _ in c if uu == u], default=0)
        sum_m = sum(m for c in app for uu, m, _, _ in c if uu == u)
        sum_c = sum(cu for c in app for uu, _, cu, _ in c if uu == u)
        n_app = sum(1 for c in app for uu, *_ in c if uu == u)
        used_anywhere = any(uu == u for c in init + app for uu, *_ in c)
        assert (u in eff) == used_anywhere
        if not used_anywhere:
            continue
        d = eff[u]
        assert d.usedmem == max(peak_m, sum_m) and d.usedcores == max(peak_c, sum_c)
        assert d.slots == max(n_app, 1)
        if u in only:
            assert only[u].usedmem == sum_m <= d.usedmem and only[u].slots == n_app
        all_ranges = [(a, a + w) for c in init + app for uu, _, _, rs in c if uu == u for a, w in rs]
        assert (d.custominfo or {}).get("cu_ranges", []) == merge_ranges(all_ranges)


def test_none_passes_through():
    pod = make_pod("p")
    assert collapse_init_container_usage(pod, None) is None
    assert app_containers_only_device_usage(pod, None) is None
