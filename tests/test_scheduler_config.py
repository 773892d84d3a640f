"""Scheduler configuration tables (model: pkg/scheduler/config/config_test.go):
flag parsing, device-config YAML merging (a HAMi ConfigMap with other vendor
sections is accepted, only ``amd`` is honoured), and registry init."""

import argparse

import pytest

from k8s_vgpu_scheduler_amd.device import devices as D
from k8s_vgpu_scheduler_amd.device.amd.device import AMDConfig
from k8s_vgpu_scheduler_amd.scheduler import config as C


def parse(*argv):
    ap = argparse.ArgumentParser()
    C.add_flags(ap)
    return C.from_args(ap.parse_args(list(argv)))


def test_defaults_match_the_dataclass():
    cfg = parse()
    ref = C.SchedulerConfig()
    for f in ("http_bind", "scheduler_name", "node_scheduler_policy", "gpu_scheduler_policy",
              "metrics_bind_address", "kube_qps", "kube_burst", "node_lock_timeout",
              "force_overwrite_default_scheduler", "leader_elect", "legacy_metrics"):
        assert getattr(cfg, f) == getattr(ref, f), f
    assert cfg.hostname


@pytest.mark.parametrize("argv,field,want", [
    (["--scheduler-name", "hami-scheduler"], "scheduler_name", "hami-scheduler"),
    (["--node-scheduler-policy", "spread"], "node_scheduler_policy", "spread"),
    (["--gpu-scheduler-policy", "binpack,numa"], "gpu_scheduler_policy", "binpack,numa"),
    (["--node-label-selector", "gpu=on, zone = a"], "node_label_selector", {"gpu": "on", "zone": "a"}),
    (["--node-label-selector", "junk,,k=v"], "node_label_selector", {"k": "v"}),
    (["--node-label-selector", ""], "node_label_selector", {}),
    (["--force-overwrite-default-scheduler", "false"], "force_overwrite_default_scheduler", False),
    (["--force-overwrite-default-scheduler", "1"], "force_overwrite_default_scheduler", True),
    (["--force-overwrite-default-scheduler", "TRUE"], "force_overwrite_default_scheduler", True),
    (["--leader-elect"], "leader_elect", True),
    (["--legacy-metrics"], "legacy_metrics", True),
    (["--kube-qps", "7.5"], "kube_qps", 7.5),
    (["--node-lock-timeout", "60"], "node_lock_timeout", 60.0),
])
def test_flag(argv, field, want):
    assert getattr(parse(*argv), field) == want


def test_invalid_node_policy_rejected():
    with pytest.raises(SystemExit):
        parse("--node-scheduler-policy", "random")


def test_no_file_gives_defaults():
    assert C.load_device_config(None) == C.DEFAULT_DEVICE_CONFIG
    assert C.load_device_config("") == C.DEFAULT_DEVICE_CONFIG


def test_amd_section_merged_over_defaults(tmp_path):
    p = tmp_path / "device-config.yaml"
    p.write_text("amd:\n  deviceSplitCount: 4\n  gpuCorePolicy: force\n"
                 "nvidia:\n  resourceCountName: nvidia.com/gpu\n")
    cfg = C.load_device_config(str(p))
    assert cfg["amd"]["deviceSplitCount"] == 4 and cfg["amd"]["gpuCorePolicy"] == "force"
    assert cfg["amd"]["resourceCountName"] == "amd.com/gpu"   # default kept
    assert "nvidia" not in cfg                                # other vendors ignored
    assert C.DEFAULT_DEVICE_CONFIG["amd"]["deviceSplitCount"] == 8   # defaults not mutated


@pytest.mark.parametrize("text", ["", "amd:\n", "other: 1\n"])
def test_empty_or_foreign_files(tmp_path, text):
    p = tmp_path / "c.yaml"
    p.write_text(text)
    assert C.load_device_config(str(p))["amd"] == C.DEFAULT_DEVICE_CONFIG["amd"]


def test_registry_init_registers_amd_only():
    C.init_devices_with_config(gpu_policy="binpack")
    assert list(D.get_devices()) == ["AMD"]
    assert D.GPU_SCHEDULER_POLICY[0] == "binpack"
    C.init_devices_with_config()
    assert D.GPU_SCHEDULER_POLICY[0] == "spread"


def test_custom_resource_names_reach_the_backend():
    cfg = {"amd": {**C.DEFAULT_DEVICE_CONFIG["amd"], "resourceCountName": "example.com/vgpu",
                   "resourceMemoryName": "example.com/vmem"}}
    C.init_devices_with_config(cfg)
    names = D.get_devices()["AMD"].get_resource_names()
    assert names.count == "example.com/vgpu" and names.memory == "example.com/vmem"
    C.init_devices_with_config()


@pytest.mark.parametrize("d,field,want", [
    ({"defaultMemory": 1024}, "default_memory", 1024),
    ({"defaultCores": 25}, "default_cores", 25),
    ({"memoryFactor": 2}, "memory_factor", 2),
    ({"cuLayout": "blocked"}, "cu_layout", "blocked"),
    ({"deviceMemoryScaling": 1.5}, "device_memory_scaling", 1.5),
    ({"unknownKey": 1}, "default_gpu_num", 1),
])
def test_amd_config_keys(d, field, want):
    assert getattr(AMDConfig.from_dict(d), field) == want


def test_amd_config_rejects_bad_core_policy():
    with pytest.raises(ValueError, match="gpuCorePolicy"):
        AMDConfig.from_dict({"gpuCorePolicy": "sometimes"})
