"""Container environment, mounts and device nodes for an allocated vGPU slice.

Reference contract: Allocate in pkg/device-plugin/nvidiadevice/nvinternal/plugin/
server.go:747-912 (envs :833-847, mounts :848-897) plus the AMD protocol of
docs/develop/amd-vgpu.md:47-104.  MI355X translation:

  env  ROCR_VISIBLE_DEVICES   ROCr ids of the allocated GPUs, in allocation
                              order (= container-local device index)
       HSA_CU_MASK            ``i:ranges;...`` for devices with a CU partition
       HIP_DEVICE_MEMORY_LIMIT_i  ``<MiB>m`` hard limit per local device
       HIP_DEVICE_CORE_LIMIT  CU share in % (first device; the reference's single
                              CUDA_DEVICE_SM_LIMIT, server.go:837), the exact
                              share of the CUs charged ("12.5" for 32 of 256)
       HIP_DEVICE_CORE_LIMIT_i  CU share in % of local device i (a container
                              can hold a compute partition next to a whole GPU)
       GPU_MAX_HW_QUEUES      2 for shared (fractional) pods: HIP's default 4
                              queues/process oversubscribes the HW scheduler
                              when tenants share a GPU (measured, see
                              profiles/README.md §2); part of the grant, so a
                              tenant cannot raise it
       HIP_TASK_PRIORITY, GPU_CORE_UTILIZATION_POLICY  from the container spec
                              (the webhook writes them, device/amd/device.py),
                              carried into the grant
       MIVGPU_SHARED_CACHE    $HOOK_PATH/vgpu/<uuid4>.cache
       MIVGPU_DEVICE_UUIDS, MIVGPU_OVERSUBSCRIBE, MIVGPU_LOG_LEVEL,
       GPU_CORE_UTILIZATION_POLICY=disable (with --disable-core-limit)
       MIVGPU_CONTROL_FILE    /etc/mivgpu/control: the monitor's verdicts (grant key)
  mounts libmivgpu.so (ro), the per-container cache dir (rw), the grant file
       (ro, LIMITS_PATH), the control file (ro, monitor/control.py: block,
       utilization switch and host-measured excess VRAM, written in place by
       the monitor on the host), /etc/ld.so.preload (ro) unless the container
       sets MIVGPU_DISABLE_CONTROL=true

The grant file repeats the policy settings of ``env`` (limits, CU mask, core
limit/policy, visible devices, region path).  It is written on the host and
mounted read-only, and the shim takes the grant from it alone, so a tenant
that unsets or rewrites those variables before the runtime starts still gets
exactly its allocation (the shim re-asserts HSA_CU_MASK / ROCR_VISIBLE_DEVICES
right before ROCr reads them); the monitor reconciles each shared region's
limits against the same host file (monitor/feedback.py).
  devs /dev/kfd and the allocated /dev/dri/renderD<N> (+ card<M>) nodes
"""

from __future__ import annotations

import os
import uuid as _uuid
from dataclasses import dataclass, field

from k8s_vgpu_scheduler_amd.device.codec import format_ranges, ranges_count
from k8s_vgpu_scheduler_amd.monitor.board import (CONTAINER_BOARD_DIR, CONTAINER_FLAGS_DIR, board_host_dir,
                                                  container_flags_dir)
from k8s_vgpu_scheduler_amd.monitor.control import CONTAINER_CONTROL_PATH, control_host_path
from k8s_vgpu_scheduler_amd.monitor.control import create as create_control

CONTAINER_LIB = "/usr/local/vgpu/libmivgpu.so"
LIMITS_PATH = "/etc/mivgpu/limits.conf"     # fixed in the shim (kLimitsPath)
# env keys that form the grant (the shim's is_grant_key list)
GRANT_KEYS = ("HIP_DEVICE_MEMORY_LIMIT", "HIP_DEVICE_CORE_LIMIT", "HSA_CU_MASK", "GPU_CORE_UTILIZATION_POLICY",
              "HIP_TASK_PRIORITY", "MIVGPU_OVERSUBSCRIBE", "MIVGPU_SHARED_CACHE", "MIVGPU_DEVICE_UUIDS",
              "ROCR_VISIBLE_DEVICES", "MIVGPU_ACCOUNT_CONTEXT", "MIVGPU_KFD_SYSFS", "MIVGPU_OCCUPANCY",
              "MIVGPU_OCC_PERIOD_US", "MIVGPU_GATE_INTERVAL_US", "MIVGPU_GATE_BURST_US", "MIVGPU_SHARE_TAU_MS",
              "MIVGPU_DISABLE_CONTROL", "GPU_MAX_HW_QUEUES", "MIVGPU_GATE_MAX_HOLD_US", "MIVGPU_CONTROL_FILE",
              "MIVGPU_BOARD_DIR", "MIVGPU_BOARD_FLAGS_DIR", "MIVGPU_FAIR_LAG_PCT")
# per-device forms of grant keys (HIP_DEVICE_MEMORY_LIMIT_<i>, HIP_DEVICE_CORE_LIMIT_<i>)
GRANT_PREFIXES = ("HIP_DEVICE_MEMORY_LIMIT_", "HIP_DEVICE_CORE_LIMIT_")


def limits_host_path(hook_path: str, pod_uid: str, ctr_name: str) -> str:
    """Host location of a container's grant file (outside the container's rw mounts)."""
    return f"{hook_path}/vgpu/limits/{pod_uid}_{ctr_name}.conf"


def grant_text(env: dict) -> str:
    keys = [k for k in env if k in GRANT_KEYS or k.startswith(GRANT_PREFIXES)]
    return "".join(f"{k}={env[k]}\n" for k in sorted(keys))


def parse_grant(text: str) -> dict:
    out = {}
    for line in text.splitlines():
        k, sep, v = line.partition("=")
        if sep and k and not k.startswith("#"):
            out[k] = v
    return out


@dataclass
class PluginConfig:
    hook_path: str = "/usr/local/vgpu"
    resource_name: str = "amd.com/gpu"
    device_split_count: int = 8
    device_memory_scaling: float = 1.0
    device_core_scaling: float = 1.0
    disable_core_limit: bool = False
    log_level: str = ""
    hw_queues_shared: int = 2
    priority_resource: str = "amd.com/priority"
    # a fractional (shared) container may opt itself out of enforcement
    # (MIVGPU_DISABLE_CONTROL, GPU_CORE_UTILIZATION_POLICY=disable) only when
    # the operator allows it; whole-GPU containers always may
    allow_tenant_opt_out: bool = False
    pass_device_specs: bool = True
    enable_preferred_allocation: bool = True
    filter_uuids: tuple = ()
    filter_indexes: tuple = ()
    enable_numa_topology: bool = False
    node_name: str = ""
    # envvar: device specs in the response; cdi-cri: CDI device names;
    # cdi-annotations: CDI names in a per-container annotation (deviceplugin/cdi.py)
    device_list_strategy: str = "envvar"
    cdi_kind: str = "amd.com/gpu"
    partitions: dict = field(default_factory=dict)   # physical GPU index -> SPX/DPX/QPX/CPX


def _truthy(v) -> bool:
    return str(v).strip().lower() in ("1", "t", "true", "yes")


def is_fractional(devreq: list, gpus: dict, cfg: PluginConfig) -> bool:
    """True if the container shares any of its GPUs (a memory slice, a CU
    share or a CU partition smaller than the device)."""
    for d in devreq:
        g = gpus.get(d.uuid)
        total_cus = g.cus if g else 256
        ranges = (d.custominfo or {}).get("cu_ranges")
        if ranges and ranges_count(ranges) < total_cus:
            return True
        if g and d.usedmem < int(g.memory_mib * cfg.device_memory_scaling):
            return True
        if 0 < d.usedcores < total_cus or d.usedcores == 0:
            return True
    return False


def core_limit_text(cus: int, total: int) -> str:
    """The grant's core limit for ``cus`` charged CUs of ``total``: the exact
    share in percent, up to three decimals ("25", "12.5", "3.125").  Whole
    percents cut a 32-CU charge (gpucores 12 rounded up to whole granules) to
    12 % and left 8 such tenants 4 % of the GPU they were charged for
    (profiles/README.md section 38); the shim parses up to four decimals."""
    if cus <= 0:
        return "0"
    milli = min(100_000, max(1, (cus * 100_000 + total // 2) // total))   # thousandths of a percent
    whole, frac = divmod(milli, 1000)
    return str(whole) if not frac else f"{whole}.{frac:03d}".rstrip("0")


def _core_pct(d, gpus: dict) -> str:
    g = gpus.get(d.uuid)
    return core_limit_text(d.usedcores, g.cus if g else 256)


def container_env(devreq: list, gpus: dict, cfg: PluginConfig, cache_file: str) -> dict:
    """devreq: ContainerDevices of this container; gpus: uuid -> smi.GPUInfo."""
    env = {}
    rocr = []
    masks = []
    shared = is_fractional(devreq, gpus, cfg)
    for i, d in enumerate(devreq):
        g = gpus.get(d.uuid)
        rocr.append(g.rocr_id if g else d.uuid)
        env[f"HIP_DEVICE_MEMORY_LIMIT_{i}"] = f"{d.usedmem}m"
        total_cus = g.cus if g else 256
        ranges = (d.custominfo or {}).get("cu_ranges")
        if ranges and ranges_count(ranges) < total_cus:
            masks.append(f"{i}:{format_ranges(ranges)}")
    env["ROCR_VISIBLE_DEVICES"] = ",".join(rocr)
    if masks:
        env["HSA_CU_MASK"] = ";".join(masks)
    if devreq:
        pcts = [_core_pct(d, gpus) for d in devreq]
        env["HIP_DEVICE_CORE_LIMIT"] = str(pcts[0])
        if any(p != pcts[0] for p in pcts):
            for i, p in enumerate(pcts):
                env[f"HIP_DEVICE_CORE_LIMIT_{i}"] = str(p)
    env["MIVGPU_SHARED_CACHE"] = cache_file
    env["MIVGPU_CONTROL_FILE"] = CONTAINER_CONTROL_PATH
    # the GPU's share board, written by the node sampler only (read-only mount)
    env["MIVGPU_BOARD_DIR"] = CONTAINER_BOARD_DIR
    # this container's own flags directory (not shared with its neighbours)
    env["MIVGPU_BOARD_FLAGS_DIR"] = CONTAINER_FLAGS_DIR
    env["MIVGPU_DEVICE_UUIDS"] = ",".join(d.uuid for d in devreq)
    if cfg.device_memory_scaling > 1:
        env["MIVGPU_OVERSUBSCRIBE"] = "true"
    if cfg.log_level:
        env["MIVGPU_LOG_LEVEL"] = str(cfg.log_level)
    if cfg.disable_core_limit:
        env["GPU_CORE_UTILIZATION_POLICY"] = "disable"
    if shared and cfg.hw_queues_shared:
        env["GPU_MAX_HW_QUEUES"] = str(cfg.hw_queues_shared)
    return env


def allocate_container(pod: dict, ctr: dict, devreq: list, gpus: dict, cfg: PluginConfig,
                       make_dirs: bool = True) -> dict:
    """-> {"envs": {...}, "mounts": [...], "devices": [...]} for one container."""
    hook = cfg.hook_path
    cache_file = f"{hook}/vgpu/{_uuid.uuid4()}.cache"
    envs = container_env(devreq, gpus, cfg, cache_file)
    spec = {e.get("name"): str(e.get("value", "")) for e in ctr.get("env") or [] if e.get("name")}
    opt_out_ok = cfg.allow_tenant_opt_out or not is_fractional(devreq, gpus, cfg)
    envs.update(_spec_policy(ctr, spec, cfg, opt_out_ok))
    uid = (pod.get("metadata") or {}).get("uid", "")
    host_dir = f"{hook}/vgpu/containers/{uid}_{ctr.get('name', '')}"
    limits = limits_host_path(hook, uid, ctr.get("name", ""))
    control = control_host_path(hook, uid, ctr.get("name", ""))
    if make_dirs:
        import shutil
        shutil.rmtree(host_dir, ignore_errors=True)
        os.makedirs(host_dir, exist_ok=True)
        try:
            os.chmod(host_dir, 0o777)
        except OSError:
            pass
        os.makedirs(os.path.dirname(limits), exist_ok=True)
        tmp = limits + ".tmp"
        with open(tmp, "w") as f:
            f.write(grant_text(envs))
        os.chmod(tmp, 0o444)
        os.replace(tmp, limits)
        create_control(control)
        fdir = container_flags_dir(board_host_dir(hook), f"{uid}_{ctr.get('name', '')}")
        shutil.rmtree(fdir, ignore_errors=True)
        os.makedirs(fdir, exist_ok=True)
        try:
            os.chmod(fdir, 0o777)       # the container's uid is not known here
        except OSError:
            pass
    mounts = [
        {"container_path": CONTAINER_LIB, "host_path": f"{hook}/vgpu/libmivgpu.so", "read_only": True},
        {"container_path": f"{hook}/vgpu", "host_path": host_dir, "read_only": False},
        {"container_path": LIMITS_PATH, "host_path": limits, "read_only": True},
        {"container_path": CONTAINER_CONTROL_PATH, "host_path": control, "read_only": True},
        {"container_path": CONTAINER_BOARD_DIR, "host_path": board_host_dir(hook), "read_only": True},
        # this container's held / owing flags: the one board file it writes,
        # in a directory of its own (the node sampler reads a pid's flags only
        # from the directory of the container host truth attributes it to)
        {"container_path": CONTAINER_FLAGS_DIR,
         "host_path": container_flags_dir(board_host_dir(hook), f"{uid}_{ctr.get('name', '')}"),
         "read_only": False},
    ]
    # the pod-spec opt-out drops the preload -- only where opting out is allowed
    # (a fractional pod would otherwise escape every limit; the webhook also
    # denies it, scheduler/webhook.py, this covers pods that bypassed it)
    disabled = opt_out_ok and _truthy(spec.get("MIVGPU_DISABLE_CONTROL", ""))
    if not disabled:
        mounts.append({"container_path": "/etc/ld.so.preload", "host_path": f"{hook}/vgpu/ld.so.preload",
                       "read_only": True})
    devices = []
    cdi_names = []
    if cfg.device_list_strategy in ("cdi-cri", "cdi-annotations"):
        from k8s_vgpu_scheduler_amd.deviceplugin.cdi import qualified_name
        cdi_names = [qualified_name(cfg.cdi_kind, d.uuid) for d in devreq]
    elif cfg.pass_device_specs:
        devices.append({"container_path": "/dev/kfd", "host_path": "/dev/kfd", "permissions": "rw"})
        for d in devreq:
            g = gpus.get(d.uuid)
            if g is None:
                continue
            if g.render_minor >= 0:
                p = f"/dev/dri/renderD{g.render_minor}"
                devices.append({"container_path": p, "host_path": p, "permissions": "rw"})
            if g.card_minor >= 0:
                p = f"/dev/dri/card{g.card_minor}"
                devices.append({"container_path": p, "host_path": p, "permissions": "rw"})
    out = {"envs": envs, "mounts": mounts, "devices": devices}
    if cfg.device_list_strategy == "cdi-cri":
        out["cdi_devices"] = cdi_names
    elif cfg.device_list_strategy == "cdi-annotations":
        from k8s_vgpu_scheduler_amd.deviceplugin.cdi import annotation_key
        out["annotations"] = {annotation_key(ctr.get("name", "")): ",".join(cdi_names)}
    return out


def _spec_policy(ctr: dict, spec: dict, cfg: PluginConfig, opt_out_ok: bool) -> dict:
    """Priority and core policy of the container, for the grant.

    The webhook writes both into the container spec (HIP_TASK_PRIORITY from
    the ``amd.com/priority`` resource, GPU_CORE_UTILIZATION_POLICY from the
    device config, device/amd/device.py:mutate_admission); the shim takes
    them from the grant file alone, so they must be carried into it.  The
    priority resource is the authority (a forged env cannot raise a
    container's priority); policy ``disable`` only where opting out is
    allowed; ``--disable-core-limit`` wins."""
    out = {}
    lim = ((ctr.get("resources") or {}).get("limits") or {}).get(cfg.priority_resource)
    prio = None
    if lim is not None:
        try:
            prio = int(str(lim))
        except ValueError:
            prio = None
    if prio is None and "HIP_TASK_PRIORITY" in spec:
        try:
            # without the resource a container may lower its priority, never raise it
            prio = max(1, int(spec["HIP_TASK_PRIORITY"]))
        except ValueError:
            prio = None
    if prio is not None:
        out["HIP_TASK_PRIORITY"] = str(prio)
    pol = spec.get("GPU_CORE_UTILIZATION_POLICY", "").strip().lower()
    if cfg.disable_core_limit:
        out["GPU_CORE_UTILIZATION_POLICY"] = "disable"
    elif pol in ("force", "default") or (pol == "disable" and opt_out_ok):
        out["GPU_CORE_UTILIZATION_POLICY"] = pol
    return out


def ld_so_preload_contents() -> str:
    return CONTAINER_LIB + "\n"
