"""Scheduler configuration: flags, device-config YAML, device registry init.

Reference: pkg/scheduler/config/config.go:76-497 (``Config``,
``InitDevicesWithConfig``, ``InitDefaultDevices``, ``GlobalFlagSet``,
``LoadConfig``) and cmd/scheduler/main.go:62-91 (flags).  Only the AMD
section of the device config is honoured in this version (north star: no
multi-vendor dispatch); other vendor sections are accepted and ignored so a
HAMi device ConfigMap can be reused verbatim.
"""

from __future__ import annotations

import argparse
import logging
from dataclasses import dataclass, field
from pathlib import Path

import yaml

from k8s_vgpu_scheduler_amd.device import devices as D
from k8s_vgpu_scheduler_amd.device.amd.device import AMDConfig, init_amd_device

log = logging.getLogger(__name__)

DEFAULT_DEVICE_CONFIG = {
    "amd": {
        "resourceCountName": "amd.com/gpu",
        "resourceMemoryName": "amd.com/gpumem",
        "resourceCoreName": "amd.com/gpucores",
        "resourceMemoryPercentageName": "amd.com/gpumem-percentage",
        "resourcePriorityName": "amd.com/priority",
        "defaultMemory": 0,
        "defaultCores": 0,
        "defaultGPUNum": 1,
        "gpuCorePolicy": "default",
        "xcdsPerDevice": 8,
        "cuLayout": "interleaved",
        "deviceSplitCount": 8,
    }
}


@dataclass
class SchedulerConfig:
    http_bind: str = "127.0.0.1:8080"
    cert_file: str = ""
    key_file: str = ""
    scheduler_name: str = ""
    node_scheduler_policy: str = "binpack"
    gpu_scheduler_policy: str = "spread"
    metrics_bind_address: str = ":9395"
    node_label_selector: dict = field(default_factory=dict)
    kube_qps: float = 50.0
    kube_burst: int = 100
    kube_timeout: float = 30.0
    profiling: bool = False
    node_lock_timeout: float = 300.0
    node_lock_retry_timeout: float = 28.0
    force_overwrite_default_scheduler: bool = True
    leader_elect: bool = False
    leader_elect_resource_name: str = "hami-scheduler"
    leader_elect_resource_namespace: str = "kube-system"
    legacy_metrics: bool = False
    device_config_file: str = ""
    debug: bool = False
    hostname: str = ""


def _parse_selector(s: str) -> dict:
    out = {}
    for part in (s or "").split(","):
        if "=" in part:
            k, v = part.split("=", 1)
            out[k.strip()] = v.strip()
    return out


def add_flags(ap: argparse.ArgumentParser):
    ap.add_argument("--http_bind", default="127.0.0.1:8080")
    ap.add_argument("--cert_file", default="")
    ap.add_argument("--key_file", default="")
    ap.add_argument("--scheduler-name", default="")
    ap.add_argument("--node-scheduler-policy", default="binpack", choices=["binpack", "spread"])
    ap.add_argument("--gpu-scheduler-policy", default="spread")
    ap.add_argument("--metrics-bind-address", default=":9395")
    ap.add_argument("--node-label-selector", default="")
    ap.add_argument("--kube-qps", type=float, default=50.0)
    ap.add_argument("--kube-burst", type=int, default=100)
    ap.add_argument("--kube-timeout", type=float, default=30.0)
    ap.add_argument("--profiling", action="store_true")
    ap.add_argument("--node-lock-timeout", type=float, default=300.0)
    ap.add_argument("--node-lock-retry-timeout", type=float, default=28.0)
    ap.add_argument("--force-overwrite-default-scheduler", default="true")
    ap.add_argument("--leader-elect", action="store_true")
    ap.add_argument("--leader-elect-resource-name", default="hami-scheduler")
    ap.add_argument("--leader-elect-resource-namespace", default="kube-system")
    ap.add_argument("--legacy-metrics", action="store_true")
    ap.add_argument("--device-config-file", default="")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-v", type=int, default=2, help="log verbosity (klog-style)")


def from_args(a) -> SchedulerConfig:
    import socket
    return SchedulerConfig(
        http_bind=a.http_bind, cert_file=a.cert_file, key_file=a.key_file, scheduler_name=a.scheduler_name,
        node_scheduler_policy=a.node_scheduler_policy, gpu_scheduler_policy=a.gpu_scheduler_policy,
        metrics_bind_address=a.metrics_bind_address, node_label_selector=_parse_selector(a.node_label_selector),
        kube_qps=a.kube_qps, kube_burst=a.kube_burst, kube_timeout=a.kube_timeout, profiling=a.profiling,
        node_lock_timeout=a.node_lock_timeout, node_lock_retry_timeout=a.node_lock_retry_timeout,
        force_overwrite_default_scheduler=str(a.force_overwrite_default_scheduler).lower() in ("1", "true"),
        leader_elect=a.leader_elect, leader_elect_resource_name=a.leader_elect_resource_name,
        leader_elect_resource_namespace=a.leader_elect_resource_namespace, legacy_metrics=a.legacy_metrics,
        device_config_file=a.device_config_file, debug=a.debug, hostname=socket.gethostname())


def load_device_config(path: str | None) -> dict:
    if not path:
        return dict(DEFAULT_DEVICE_CONFIG)
    data = yaml.safe_load(Path(path).read_text()) or {}
    merged = dict(DEFAULT_DEVICE_CONFIG)
    if "amd" in data:
        merged["amd"] = {**DEFAULT_DEVICE_CONFIG["amd"], **(data.get("amd") or {})}
    return merged


def init_devices_with_config(device_config: dict | None = None, gpu_policy: str = "spread"):
    """(Re)build the registry: one MI355X backend under type "AMD"."""
    cfg = device_config or DEFAULT_DEVICE_CONFIG
    D.reset_registry()
    D.GPU_SCHEDULER_POLICY[0] = gpu_policy
    amd = init_amd_device(AMDConfig.from_dict(cfg.get("amd") or {}))
    D.DEVICES_MAP["AMD"] = amd
    D.DEVICES_TO_HANDLE.append("AMD")
    return D.DEVICES_MAP
