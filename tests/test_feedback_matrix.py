"""Priority-feedback and grant-reconciliation tables (monitor/feedback.py;
reference cmd/vGPUmonitor/feedback.go:40-165 and its tests).  Containers are
stubs exposing the region accessors ``observe`` uses, so each case states the
tenants on each GPU (priority, recent_kernel) and the expected decisions."""

import pytest

from k8s_vgpu_scheduler_amd.monitor import feedback as F
from k8s_vgpu_scheduler_amd.monitor.region import MAX_DEVICES


class StubRegion:
    def __init__(self, uuids, prio, rk, sw=0):
        self._u, self._p, self._rk, self._sw = list(uuids), prio, rk, sw

    def device_num(self):
        return len(self._u)

    def uuid(self, i):
        return self._u[i]

    def is_valid_uuid(self, i):
        return bool(self._u[i])

    def priority(self):
        return self._p

    def recent_kernel(self):
        return self._rk

    def utilization_switch(self):
        return self._sw

    def set_recent_kernel(self, v):
        self._rk = v

    def set_utilization_switch(self, v):
        self._sw = v


class StubContainer:
    def __init__(self, region):
        self.region = region


class StubLister:
    def __init__(self, cs):
        self.cs = cs

    def list_containers(self):
        return self.cs


def run(tenants):
    """tenants: [(uuids, priority, recent_kernel)] -> [(recent_kernel, switch)] after one pass."""
    cs = [StubContainer(StubRegion(u, p, rk)) for u, p, rk in tenants]
    F.observe(StubLister(cs))
    return [(c.region._rk, c.region._sw) for c in cs]


@pytest.mark.parametrize("name,tenants,want", [
    ("idle tenant alone", [(["g0"], 1, 0)], [(0, 0)]),
    ("active tenant alone decays, no switch", [(["g0"], 1, 2)], [(1, 0)]),
    ("high priority active blocks low priority on the same GPU",
     [(["g0"], 0, 2), (["g0"], 1, 2)], [(1, 0), (-1, 1)]),
    ("high priority on another GPU blocks nothing",
     [(["g0"], 0, 2), (["g1"], 1, 2)], [(1, 0), (1, 0)]),
    ("two active tenants of the same priority: both governed, none blocked",
     [(["g0"], 1, 2), (["g0"], 1, 2)], [(1, 1), (1, 1)]),
    ("a tenant whose counter decays to 0 this pass is not counted",
     [(["g0"], 0, 1), (["g0"], 1, 2)], [(0, 0), (1, 0)]),
    ("blocked tenant is released once the high-priority tenant is idle",
     [(["g0"], 0, 0), (["g0"], 1, -1)], [(0, 0), (0, 0)]),
    ("multi-GPU tenant blocked through any of its GPUs",
     [(["g1"], 0, 2), (["g0", "g1"], 2, 2)], [(1, 0), (-1, 1)]),
    ("negative priority never counted",
     [(["g0"], -1, 2), (["g0"], 1, 2)], [(1, 0), (1, 0)]),
    ("order does not matter: the high-priority tenant listed second blocks the first",
     [(["g0"], 2, 2), (["g0"], 0, 2)], [(-1, 1), (1, 0)]),
    ("three levels: the middle one is blocked by the top and governs nothing else",
     [(["g0"], 0, 2), (["g0"], 1, 2), (["g0"], 2, 2)], [(1, 0), (-1, 1), (-1, 1)]),
])
def test_observe(name, tenants, want):
    assert run(tenants) == want, name


def test_switch_turns_off_when_contention_ends():
    r = StubRegion(["g0"], 1, 2, sw=1)
    F.observe(StubLister([StubContainer(r)]))
    assert r._sw == 0


@pytest.mark.parametrize("v,want", [
    (None, 0), ("", 0), ("4096m", 4096 << 20), ("36g", 36 << 30), ("1T", 1 << 40), ("512k", 512 << 10),
    ("12345", 12345), ("1.5g", int(1.5 * (1 << 30))), ("xm", 0), ("m", 0),
])
def test_parse_size(v, want):
    assert F.parse_size(v) == want


@pytest.mark.parametrize("mask,idx,want", [
    ("0:0-63", 0, 64), ("0:0-63", 1, 0), ("0:0-7,16-23;1:8-15", 0, 16), ("0:0-7,16-23;1:8-15", 1, 8),
    ("0:5", 0, 1), (None, 0, 0), ("", 0, 0), ("0:a-b", 0, 0), ("junk", 0, 0),
])
def test_mask_count(mask, idx, want):
    assert F.mask_count(mask, idx) == want


def test_expected_region_from_a_slice_grant():
    e = F.expected_region({"HIP_DEVICE_MEMORY_LIMIT_0": "36864m", "HIP_DEVICE_CORE_LIMIT": "25",
                           "HSA_CU_MASK": "0:0-63", "GPU_CORE_UTILIZATION_POLICY": "force",
                           "HIP_TASK_PRIORITY": "0"})
    assert e["mem_limit"][0] == 36864 << 20 and e["mem_limit"][1] == 0
    assert e["cu_limit"][0] == 25 and e["cu_limit"][MAX_DEVICES - 1] == 25
    assert e["cu_mask"][0] == 64 and e["core_policy"] == 1 and e["priority"] == 0
    assert len(e["mem_limit"]) == len(e["cu_mask"]) == MAX_DEVICES


@pytest.mark.parametrize("grant,field,want", [
    ({}, "cu_limit", 100), ({"HIP_DEVICE_CORE_LIMIT": "0"}, "cu_limit", 100),
    ({"HIP_DEVICE_CORE_LIMIT": "250"}, "cu_limit", 100), ({"HIP_DEVICE_CORE_LIMIT": "x"}, "cu_limit", 100),
    ({"GPU_CORE_UTILIZATION_POLICY": "DISABLE"}, "core_policy", 2),
    ({"GPU_CORE_UTILIZATION_POLICY": "default"}, "core_policy", 0),
    ({}, "priority", 1), ({"HIP_TASK_PRIORITY": "nope"}, "priority", 1),
])
def test_expected_region_defaults(grant, field, want):
    got = F.expected_region(grant)[field]
    assert (got[0] if isinstance(got, list) else got) == want


def test_per_device_core_limits_in_the_grant():
    """HIP_DEVICE_CORE_LIMIT_<i> overrides the all-devices key for one device."""
    e = F.expected_region({"HIP_DEVICE_CORE_LIMIT": "25", "HIP_DEVICE_CORE_LIMIT_0": "25",
                           "HIP_DEVICE_CORE_LIMIT_1": "100", "HIP_DEVICE_CORE_LIMIT_2": "bad"})
    assert e["cu_limit"][:4] == [25, 100, 25, 25]


def test_global_memory_limit_applies_to_every_device():
    e = F.expected_region({"HIP_DEVICE_MEMORY_LIMIT": "1g", "HIP_DEVICE_MEMORY_LIMIT_1": "2g"})
    assert e["mem_limit"][0] == 1 << 30 and e["mem_limit"][1] == 2 << 30 and e["mem_limit"][2] == 1 << 30
