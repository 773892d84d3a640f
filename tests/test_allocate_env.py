"""Device-plugin Allocate environment tables (deviceplugin/allocate.py).

Model: the reference's plugin/util_test.go and alloc_refactor_test.go, which
pin the env a container receives for each allocation shape (memory limit per
device, core limit, visible devices, oversubscription, disable-core-limit).
Here the grant also carries the XCD-balanced ``HSA_CU_MASK`` and the HW-queue
cap for shared GPUs, and it is written to a read-only grant file that the
shim prefers over the environment (``grant_text`` / ``parse_grant``)."""

import pytest
from hypothesis import given, settings, strategies as st

from k8s_vgpu_scheduler_amd.deviceplugin import allocate as A
from k8s_vgpu_scheduler_amd.device.types import ContainerDevice
from k8s_vgpu_scheduler_amd.smi import GPUInfo

G0 = GPUInfo(index=0, uuid="GPU-a", rocr_id="GPU-00000000000000aa")
G1 = GPUInfo(index=1, uuid="GPU-b", rocr_id="GPU-00000000000000bb")
GPUS = {g.uuid: g for g in (G0, G1)}
WHOLE = 294912


def cd(uuid="GPU-a", mem=WHOLE, cus=256, ranges=None):
    return ContainerDevice(uuid=uuid, type="AMD", usedmem=mem, usedcores=cus,
                           custominfo={"cu_ranges": ranges} if ranges else {})


def env(devs, **cfg):
    return A.container_env(devs, GPUS, A.PluginConfig(**cfg), "/tmp/vgpu/x.cache")


@pytest.mark.parametrize("name,devs,cfg,want,absent", [
    ("whole card exclusive", [cd()], {},
     {"HIP_DEVICE_MEMORY_LIMIT_0": f"{WHOLE}m", "ROCR_VISIBLE_DEVICES": G0.rocr_id, "HIP_DEVICE_CORE_LIMIT": "100",
      "MIVGPU_DEVICE_UUIDS": "GPU-a"}, ["HSA_CU_MASK", "GPU_MAX_HW_QUEUES", "MIVGPU_OVERSUBSCRIBE"]),
    ("64-CU slice", [cd(mem=36864, cus=64, ranges=[(0, 63)])], {},
     {"HIP_DEVICE_MEMORY_LIMIT_0": "36864m", "HSA_CU_MASK": "0:0-63", "HIP_DEVICE_CORE_LIMIT": "25",
      "GPU_MAX_HW_QUEUES": "2"}, []),
    ("time-shared (no cores)", [cd(mem=1000, cus=0)], {},
     {"HIP_DEVICE_CORE_LIMIT": "0", "GPU_MAX_HW_QUEUES": "2"}, ["HSA_CU_MASK"]),
    ("two GPUs, second masked", [cd(), cd("GPU-b", mem=5000, cus=128, ranges=[(64, 191)])], {},
     {"ROCR_VISIBLE_DEVICES": f"{G0.rocr_id},{G1.rocr_id}", "HSA_CU_MASK": "1:64-191",
      "HIP_DEVICE_MEMORY_LIMIT_1": "5000m", "MIVGPU_DEVICE_UUIDS": "GPU-a,GPU-b"}, []),
    ("unknown GPU falls back to its uuid", [cd("GPU-zz", mem=10)], {},
     {"ROCR_VISIBLE_DEVICES": "GPU-zz"}, []),
    ("oversubscription", [cd(mem=1000, cus=0)], {"device_memory_scaling": 2.0},
     {"MIVGPU_OVERSUBSCRIBE": "true"}, []),
    ("disable core limit", [cd(mem=1000, cus=64, ranges=[(0, 63)])], {"disable_core_limit": True},
     {"GPU_CORE_UTILIZATION_POLICY": "disable"}, []),
    ("log level passed", [cd()], {"log_level": "3"}, {"MIVGPU_LOG_LEVEL": "3"}, []),
    ("queue cap off", [cd(mem=1000, cus=0)], {"hw_queues_shared": 0}, {}, ["GPU_MAX_HW_QUEUES"]),
    ("full-card ranges are no mask", [cd(ranges=[(0, 255)])], {}, {}, ["HSA_CU_MASK"]),
])
def test_container_env(name, devs, cfg, want, absent):
    e = env(devs, **cfg)
    for k, v in want.items():
        assert e.get(k) == v, (name, k, e)
    for k in absent:
        assert k not in e, (name, k, e)
    assert e["MIVGPU_SHARED_CACHE"] == "/tmp/vgpu/x.cache"


@pytest.mark.parametrize("cus,want", [(1, "0.391"), (8, "3.125"), (32, "12.5"), (64, "25"), (128, "50"),
                                      (77, "30.078"), (255, "99.609"), (256, "100")])
def test_core_limit_percent_rounding(cus, want):
    assert env([cd(mem=10, cus=cus)])["HIP_DEVICE_CORE_LIMIT"] == want


def test_grant_text_keeps_only_grant_keys():
    e = env([cd(mem=36864, cus=64, ranges=[(0, 63)])], log_level="2")
    e["PATH"] = "/bin"
    text = A.grant_text(e)
    got = A.parse_grant(text)
    assert "PATH" not in got and "MIVGPU_LOG_LEVEL" not in got
    assert got["HSA_CU_MASK"] == "0:0-63" and got["HIP_DEVICE_MEMORY_LIMIT_0"] == "36864m"
    assert text.splitlines() == sorted(text.splitlines())


@settings(max_examples=80, deadline=None)
@given(st.dictionaries(st.sampled_from(list(A.GRANT_KEYS) + ["HIP_DEVICE_MEMORY_LIMIT_3", "OTHER"]),
                       st.text(alphabet=st.characters(min_codepoint=0x20, max_codepoint=0x7e), max_size=20)))
def test_grant_round_trip(e):
    """Grant values are printable ASCII (limits, masks, paths, uuids)."""
    got = A.parse_grant(A.grant_text(e))
    assert got == {k: v for k, v in e.items() if k != "OTHER"}


def test_parse_grant_skips_comments_and_junk():
    assert A.parse_grant("# HSA_CU_MASK=0:0-7\nnot a line\nHSA_CU_MASK=0:8-15\n=x\n") == {"HSA_CU_MASK": "0:8-15"}


def test_limits_host_path():
    assert A.limits_host_path("/usr/local/vgpu", "uid1", "main") == "/usr/local/vgpu/vgpu/limits/uid1_main.conf"
