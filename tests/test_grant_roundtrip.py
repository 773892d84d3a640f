"""Webhook -> Allocate -> grant file -> shim region, and the tenant opt-outs.

ADVICE r2 (high): the grant file was built from container_env() alone, which
never holds HIP_TASK_PRIORITY or GPU_CORE_UTILIZATION_POLICY (the webhook
writes both into the container spec, device/amd/device.py:mutate_admission);
the shim takes both from the grant file only, and the monitor's reconcile pass
put the region back to priority 1 / policy default every 5 s.  These tests run
the whole chain.

VERDICT r2 weak #3b: MIVGPU_DISABLE_CONTROL=true (or policy disable) in a
fractional pod's own spec dropped every limit.  The webhook denies it; the
device plugin ignores it for pods that bypassed the webhook.
"""

from __future__ import annotations

import pytest

from k8s_vgpu_scheduler_amd.device.amd.device import AMDDevices, AMDConfig
from k8s_vgpu_scheduler_amd.device.devices import AdmissionError
from k8s_vgpu_scheduler_amd.device.types import ContainerDevice
from k8s_vgpu_scheduler_amd.deviceplugin.allocate import (GRANT_KEYS, PluginConfig, allocate_container, grant_text,
                                                          parse_grant)
from k8s_vgpu_scheduler_amd.monitor.feedback import expected_region
from k8s_vgpu_scheduler_amd.smi import FakeBackend
from k8s_vgpu_scheduler_amd.testing import amd_container, amd_pod


def _gpus():
    return {g.uuid: g for g in FakeBackend(n=2).gpus()}


def _allocate(ctr, devs, cfg=None, tmp_path=None):
    pod = amd_pod("p", containers=[ctr])
    cfg = cfg or PluginConfig(hook_path=str(tmp_path))
    return allocate_container(pod, ctr, devs, _gpus(), cfg, make_dirs=False)


def _slice(uuid="GPU-0000", mem=36864, cores=64, ranges=None):
    return ContainerDevice(idx=0, uuid=uuid, type="MI355X", usedmem=mem, usedcores=cores,
                           custominfo={"cu_ranges": ranges} if ranges else {})


@pytest.mark.parametrize("policy", ["force", "default"])
def test_priority_and_policy_survive_webhook_allocate_grant_region(tmp_path, policy):
    dev = AMDDevices(AMDConfig(gpu_core_policy=policy))
    ctr = amd_container(mem=36864, cores=25, priority=0)
    pod = amd_pod("p", containers=[ctr])
    assert dev.mutate_admission(ctr, pod)
    env = {e["name"]: e["value"] for e in ctr["env"]}
    assert env["HIP_TASK_PRIORITY"] == "0"
    out = _allocate(ctr, [_slice()], tmp_path=tmp_path)
    grant = parse_grant(grant_text(out["envs"]))
    assert grant["HIP_TASK_PRIORITY"] == "0"
    if policy == "force":
        assert grant["GPU_CORE_UTILIZATION_POLICY"] == "force"
    want = expected_region(grant)
    assert want["priority"] == 0
    assert want["core_policy"] == (1 if policy == "force" else 0)


def test_priority_comes_from_the_resource_not_a_forged_env(tmp_path):
    ctr = amd_container(mem=1000, cores=25)             # no amd.com/priority resource
    ctr["env"] = [{"name": "HIP_TASK_PRIORITY", "value": "0"}]
    grant = parse_grant(grant_text(_allocate(ctr, [_slice()], tmp_path=tmp_path)["envs"]))
    assert grant["HIP_TASK_PRIORITY"] == "1"             # may lower itself, never raise
    ctr["env"] = [{"name": "HIP_TASK_PRIORITY", "value": "3"}]
    grant = parse_grant(grant_text(_allocate(ctr, [_slice()], tmp_path=tmp_path)["envs"]))
    assert grant["HIP_TASK_PRIORITY"] == "3"


@pytest.mark.parametrize("cfg_kw,spec_policy,fractional,want", [
    ({}, "disable", True, None),                         # a shared slice cannot switch its governor off
    ({}, "disable", False, "disable"),                   # a whole GPU may
    ({"allow_tenant_opt_out": True}, "disable", True, "disable"),
    ({"disable_core_limit": True}, "force", True, "disable"),   # --disable-core-limit wins
    ({}, "bogus", True, None),
])
def test_core_policy_in_the_grant(tmp_path, cfg_kw, spec_policy, fractional, want):
    ctr = amd_container(mem=1000 if fractional else 294912, cores=25 if fractional else 100)
    ctr["env"] = [{"name": "GPU_CORE_UTILIZATION_POLICY", "value": spec_policy}]
    dev = _slice(mem=1000, cores=64, ranges=[[0, 63]]) if fractional else _slice(mem=294912, cores=256)
    cfg = PluginConfig(hook_path=str(tmp_path), **cfg_kw)
    grant = parse_grant(grant_text(_allocate(ctr, [dev], cfg=cfg)["envs"]))
    assert grant.get("GPU_CORE_UTILIZATION_POLICY") == want


def test_grant_carries_the_queue_cap_and_per_device_core_limits(tmp_path):
    """A container holding a 25 % slice of GPU 0 and all of GPU 1: one core
    limit per device, and the shared-pod queue cap, all in the grant."""
    ctr = amd_container(gpu=2, mem=1000, cores=25)
    devs = [_slice("GPU-0000", mem=36864, cores=64, ranges=[[0, 63]]),
            ContainerDevice(idx=1, uuid="GPU-0001", type="MI355X", usedmem=294912, usedcores=256)]
    out = _allocate(ctr, devs, tmp_path=tmp_path)
    grant = parse_grant(grant_text(out["envs"]))
    assert grant["GPU_MAX_HW_QUEUES"] == "2"
    assert grant["HIP_DEVICE_CORE_LIMIT_0"] == "25" and grant["HIP_DEVICE_CORE_LIMIT_1"] == "100"
    assert expected_region(grant)["cu_limit"][:2] == [25, 100]
    assert "GPU_MAX_HW_QUEUES" in GRANT_KEYS


OPT_OUTS = [("MIVGPU_DISABLE_CONTROL", "true"), ("MIVGPU_DISABLE_CONTROL", "1"),
            ("GPU_CORE_UTILIZATION_POLICY", "disable"), ("GPU_CORE_UTILIZATION_POLICY", "DISABLE")]


@pytest.mark.parametrize("name,value", OPT_OUTS)
@pytest.mark.parametrize("req,fractional", [
    (dict(mem=1000, cores=25), True), (dict(mem=1000), True), (dict(mem_pct=50), True), (dict(cores=30), True),
    (dict(), False), (dict(mem_pct=100), False), (dict(cores=100, mem_pct=100), False),
])
def test_webhook_denies_opt_out_on_fractional_pods(name, value, req, fractional):
    dev = AMDDevices(AMDConfig())
    ctr = amd_container(**req)
    ctr["env"] = [{"name": name, "value": value}]
    pod = amd_pod("p", containers=[ctr])
    if fractional:
        with pytest.raises(AdmissionError, match="opting out"):
            dev.mutate_admission(ctr, pod)
    else:
        assert dev.mutate_admission(ctr, pod)
    # the operator can allow it
    ctr2 = amd_container(**req)
    ctr2["env"] = [{"name": name, "value": value}]
    assert AMDDevices(AMDConfig(allow_tenant_opt_out=True)).mutate_admission(ctr2, amd_pod("p", containers=[ctr2]))


def test_webhook_opt_out_falsy_values_allowed():
    dev = AMDDevices(AMDConfig())
    for v in ("false", "0", ""):
        ctr = amd_container(mem=1000, cores=25)
        ctr["env"] = [{"name": "MIVGPU_DISABLE_CONTROL", "value": v}]
        assert dev.mutate_admission(ctr, amd_pod("p", containers=[ctr]))


def test_webhook_own_policy_is_not_a_tenant_opt_out():
    """gpuCorePolicy: disable in the device config is the operator's choice:
    the webhook writes it itself, after the tenant check."""
    dev = AMDDevices(AMDConfig(gpu_core_policy="disable"))
    ctr = amd_container(mem=1000, cores=25)
    assert dev.mutate_admission(ctr, amd_pod("p", containers=[ctr]))
    assert {"name": "GPU_CORE_UTILIZATION_POLICY", "value": "disable"} in ctr["env"]
