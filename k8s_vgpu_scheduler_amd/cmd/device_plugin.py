"""``mivgpu-device-plugin``: node agent (registration + kubelet device plugin).

Reference: cmd/device-plugin/nvidia/main.go:53-424 and vgpucfg.go:34-116 (flags
``--device-split-count``, ``--device-memory-scaling``, ``--device-core-scaling``,
``--disable-core-limit``, ``--resource-name``), the per-node override file
``/config/config.json`` (``nodeconfig[]``, server.go:128-169) and
docker/vgpu-init.sh (install the shim under the hook path and write
``ld.so.preload``).
"""

from __future__ import annotations

import argparse
import json
import logging
import os
import shutil
import signal
import threading
from pathlib import Path

from k8s_vgpu_scheduler_amd.deviceplugin import api
from k8s_vgpu_scheduler_amd.deviceplugin.allocate import PluginConfig, ld_so_preload_contents
from k8s_vgpu_scheduler_amd.deviceplugin.register import Registrar
from k8s_vgpu_scheduler_amd.deviceplugin.server import AMDDevicePlugin, run_with_restarts
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.shim import DEFAULT_SHIM
from k8s_vgpu_scheduler_amd.smi import detect
from k8s_vgpu_scheduler_amd.utils.logsetup import setup_logging

log = logging.getLogger("mivgpu.device-plugin")


def apply_node_config(cfg: PluginConfig, path: str, node: str) -> PluginConfig:
    """Per-node overrides: {"nodeconfig": [{"name": ..., "devicesplitcount": ...}]}."""
    p = Path(path)
    if not p.exists():
        return cfg
    data = json.loads(p.read_text() or "{}")
    for nc in data.get("nodeconfig") or []:
        if nc.get("name") != node:
            continue
        if "devicesplitcount" in nc:
            cfg.device_split_count = int(nc["devicesplitcount"])
        if "devicememoryscaling" in nc:
            cfg.device_memory_scaling = float(nc["devicememoryscaling"])
        if "devicecorescaling" in nc:
            cfg.device_core_scaling = float(nc["devicecorescaling"])
        if "hwqueues" in nc:
            cfg.hw_queues_shared = int(nc["hwqueues"])
        if "partitions" in nc:
            cfg.partitions = {int(k): str(v).upper() for k, v in (nc["partitions"] or {}).items()}
        if "enablegetpreferredallocation" in nc:
            cfg.enable_preferred_allocation = bool(nc["enablegetpreferredallocation"])
        fd = nc.get("filterdevices") or {}
        cfg.filter_uuids = tuple(fd.get("uuid") or ())
        cfg.filter_indexes = tuple(int(i) for i in (fd.get("index") or ()))
    return cfg


def install_shim(hook_path: str, src: Path = DEFAULT_SHIM):
    """vgpu-init.sh: copy libmivgpu.so into <hook>/vgpu and (re)write ld.so.preload."""
    dst = Path(hook_path) / "vgpu"
    dst.mkdir(parents=True, exist_ok=True)
    if src.exists():
        tmp = dst / "libmivgpu.so.tmp"
        shutil.copy2(src, tmp)
        os.replace(tmp, dst / "libmivgpu.so")
    (dst / "ld.so.preload").write_text(ld_so_preload_contents())
    (dst / "containers").mkdir(exist_ok=True)


def main(argv=None):
    ap = argparse.ArgumentParser("mivgpu-device-plugin")
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME", ""))
    ap.add_argument("--resource-name", default="amd.com/gpu")
    ap.add_argument("--device-split-count", type=int, default=8)
    ap.add_argument("--device-memory-scaling", type=float, default=1.0)
    ap.add_argument("--device-core-scaling", type=float, default=1.0)
    ap.add_argument("--disable-core-limit", action="store_true")
    ap.add_argument("--hw-queues", type=int, default=2, help="GPU_MAX_HW_QUEUES for shared pods (0 = HIP default)")
    ap.add_argument("--allow-tenant-opt-out", action="store_true",
                    help="honour MIVGPU_DISABLE_CONTROL / GPU_CORE_UTILIZATION_POLICY=disable in the spec of "
                         "fractional (shared) containers (default: only whole-GPU containers may opt out)")
    ap.add_argument("--hook-path", default=os.environ.get("HOOK_PATH", "/usr/local/vgpu"))
    ap.add_argument("--kubelet-socket", default=api.KUBELET_SOCKET)
    ap.add_argument("--socket-dir", default=api.DEVICE_PLUGIN_PATH)
    ap.add_argument("--node-config", default="/config/config.json")
    ap.add_argument("--log-level", default="", help="MIVGPU_LOG_LEVEL injected into containers")
    ap.add_argument("--smi-backend", default=None, choices=[None, "amdsmi", "sysfs", "fake"])
    ap.add_argument("--enable-numa-topology", action="store_true")
    ap.add_argument("--device-list-strategy", default="envvar", choices=["envvar", "cdi-annotations", "cdi-cri"])
    ap.add_argument("--cdi-spec-dir", default="/var/run/cdi")
    ap.add_argument("--enable-partition-manager", action="store_true",
                    help="reconcile compute-partition modes from mivgpu.io/partition-request")
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("-v", type=int, default=2)
    a = ap.parse_args(argv)
    setup_logging(a.v)
    if not a.node_name:
        raise SystemExit("--node-name / NODE_NAME is required")
    from k8s_vgpu_scheduler_amd.k8s.rest import RestClient
    init_global_client(RestClient.from_env(a.kubeconfig))
    cfg = PluginConfig(hook_path=a.hook_path, resource_name=a.resource_name, device_split_count=a.device_split_count,
                       device_memory_scaling=a.device_memory_scaling, device_core_scaling=a.device_core_scaling,
                       disable_core_limit=a.disable_core_limit, log_level=a.log_level, hw_queues_shared=a.hw_queues,
                       enable_numa_topology=a.enable_numa_topology, node_name=a.node_name,
                       device_list_strategy=a.device_list_strategy, allow_tenant_opt_out=a.allow_tenant_opt_out)
    cfg = apply_node_config(cfg, a.node_config, a.node_name)
    install_shim(a.hook_path)
    backend = detect(a.smi_backend)
    if cfg.device_list_strategy != "envvar":
        from k8s_vgpu_scheduler_amd.deviceplugin import cdi
        log.info("wrote CDI spec %s", cdi.write_spec(cdi.build_spec(backend.gpus(), cfg.cdi_kind), a.cdi_spec_dir))
    reg = Registrar(backend, cfg, a.node_name)
    threading.Thread(target=reg.watch_and_register, name="register", daemon=True).start()
    reload = threading.Event()
    # SIGHUP: re-register with the kubelet (reference: main.go:305-337)
    signal.signal(signal.SIGHUP, lambda *_: reload.set())
    if a.enable_partition_manager or cfg.partitions:
        from k8s_vgpu_scheduler_amd.deviceplugin.partition import PartitionManager

        pm = PartitionManager(backend, a.node_name, static=cfg.partitions)

        def on_change():
            reg.register_once()
            reload.set()
        threading.Thread(target=pm.watch, args=(on_change,), name="partitions", daemon=True).start()
    run_with_restarts(lambda: AMDDevicePlugin(backend, cfg, a.node_name, a.socket_dir), a.kubelet_socket,
                      reload=reload)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
