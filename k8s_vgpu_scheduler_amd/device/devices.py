"""Device-backend contract and registry (pkg/device/devices.go:34-48, 246-252, 576-738).

``Devices`` is the 13-method backend interface; the registry maps a device
type ("AMD") to its backend plus the pod-annotation keys it reads/writes.
This version registers exactly one backend -- the MI355X AMD backend -- but
keeps the registry shape so scheduler, webhook and quota code stay
backend-agnostic.
"""

from __future__ import annotations

import abc
import datetime as _dt
import logging

from k8s_vgpu_scheduler_amd.k8s import quantity
from k8s_vgpu_scheduler_amd.k8s.client import containers, init_containers
from k8s_vgpu_scheduler_amd.utils import util
from k8s_vgpu_scheduler_amd.utils.types import GPU_POLICY_SPREAD

from .types import ContainerDevice, ContainerDeviceRequest, DeviceInfo, DeviceUsage, NodeInfo, ResourceNames

log = logging.getLogger(__name__)


class AdmissionError(ValueError):
    """MutateAdmission validation failure -> webhook denies the pod."""


class Devices(abc.ABC):
    @abc.abstractmethod
    def common_word(self) -> str: ...

    @abc.abstractmethod
    def mutate_admission(self, ctr: dict, pod: dict) -> bool: ...

    @abc.abstractmethod
    def check_health(self, dev_type: str, node: dict) -> tuple[bool, bool]: ...

    @abc.abstractmethod
    def node_cleanup(self, node_name: str) -> None: ...

    @abc.abstractmethod
    def get_resource_names(self) -> ResourceNames: ...

    @abc.abstractmethod
    def get_node_devices(self, node: dict) -> list[DeviceInfo]: ...

    @abc.abstractmethod
    def lock_node(self, node: dict, pod: dict) -> None: ...

    @abc.abstractmethod
    def release_node_lock(self, node: dict, pod: dict) -> None: ...

    @abc.abstractmethod
    def generate_resource_requests(self, ctr: dict) -> ContainerDeviceRequest: ...

    @abc.abstractmethod
    def patch_annotations(self, pod: dict, annos: dict, pd: dict) -> dict: ...

    @abc.abstractmethod
    def score_node(self, node: dict, pod_single: list, previous: list, policy: str) -> float: ...

    @abc.abstractmethod
    def add_resource_usage(self, pod: dict, dev: DeviceUsage, ctr: ContainerDevice) -> None: ...

    @abc.abstractmethod
    def fit(self, devices: list[DeviceUsage], request: ContainerDeviceRequest, pod: dict,
            node_info: NodeInfo | None, allocated: dict) -> tuple[bool, dict, str]: ...

    # Optional hooks ------------------------------------------------------
    def node_deleted(self, node_name: str) -> None:
        pass

    policy_neutral_score = False  # see scheduler.policy.node_policy.override_score


# ------------------------------------------------------------------ registry
DEVICES_MAP: dict[str, Devices] = {}
IN_REQUEST_DEVICES: dict[str, str] = {}   # type -> "...-devices-to-allocate" annotation
SUPPORT_DEVICES: dict[str, str] = {}      # type -> "...-devices-allocated" annotation
DEVICES_TO_HANDLE: list[str] = []
GPU_SCHEDULER_POLICY = [GPU_POLICY_SPREAD]  # mutable cell (config sets it)
# bumped on every registry rebuild (config reload): caches of Fit results made
# under the old backends (memory factor, CU topology, policies) key on it
REGISTRY_GENERATION = [0]


def get_devices() -> dict[str, Devices]:
    return DEVICES_MAP


def gpu_scheduler_policy() -> str:
    return GPU_SCHEDULER_POLICY[0]


def registry_generation() -> int:
    return REGISTRY_GENERATION[0]


def reset_registry():
    REGISTRY_GENERATION[0] += 1
    DEVICES_MAP.clear()
    IN_REQUEST_DEVICES.clear()
    SUPPORT_DEVICES.clear()
    DEVICES_TO_HANDLE.clear()
    util.HANDSHAKE_ANNOS.clear()


# ------------------------------------------------------------ shared helpers
def resource_value(ctr: dict, name: str, requests_fallback: bool = True):
    """Raw quantity string from limits (then requests), or None."""
    if not name:
        return None
    res = ctr.get("resources") or {}
    lim = res.get("limits") or {}
    if name in lim:
        return lim[name]
    if requests_fallback:
        req = res.get("requests") or {}
        if name in req:
            return req[name]
    return None


def as_int(q) -> tuple[int, bool]:
    return quantity.as_int64(q)


def check_health_handshake(dev_type: str, count_name: str, node: dict) -> tuple[bool, bool]:
    """devices.go:576-615: the device plugin answers ``Requesting_<time>`` by
    re-registering; unhealthy if unanswered for 60 s AND no allocatable left."""
    key = util.HANDSHAKE_ANNOS.get(dev_type)
    annos = (node.get("metadata") or {}).get("annotations") or {}
    handshake = annos.get(key, "") if key else ""
    if "Requesting" in handshake:
        _, _, ts = handshake.partition("_")
        if not ts:
            return True, False
        try:
            former = _dt.datetime.strptime(ts, "%Y-%m-%d %H:%M:%S")
        except ValueError:
            return True, False
        if _dt.datetime.now() < former + _dt.timedelta(seconds=60):
            return True, False
        alloc = ((node.get("status") or {}).get("allocatable") or {}).get(count_name)
        if alloc is not None and quantity.value(alloc) > 0:
            return True, False
        return False, False
    if key:
        try:
            util.patch_node_annotations(
                node["metadata"]["name"],
                {key: "Requesting_" + _dt.datetime.now().strftime("%Y-%m-%d %H:%M:%S")})
        except Exception as e:  # noqa: BLE001
            log.error("handshake patch failed for %s: %s", node["metadata"]["name"], e)
    return True, True


def resource_reqs(pod: dict) -> list[dict]:
    """Per container (init first) map of device type -> request (devices.go:639-691)."""
    out = []
    for ctr in list(init_containers(pod)) + list(containers(pod)):
        m = {}
        for t, dev in get_devices().items():
            r = dev.generate_resource_requests(ctr)
            if r.nums > 0:
                m[t] = r
        out.append(m)
    return out


def check_uuid(annos: dict, dev_id: str, use_key: str, nouse_key: str) -> bool:
    def match(lst):
        return any(u.strip() == dev_id for u in lst.split(","))

    use = annos.get(use_key)
    if use is not None and use.strip() and not match(use):
        return False
    nouse = annos.get(nouse_key)
    if nouse is not None and nouse.strip() and match(nouse):
        return False
    return True


def check_type(annos: dict, card_type: str, use_key: str, nouse_key: str) -> bool:
    ct = card_type.upper()

    def match(lst):
        return any(t.strip() and t.strip().upper() in ct for t in lst.split(","))

    use = annos.get(use_key)
    if use is not None and use.strip() and not match(use):
        return False
    nouse = annos.get(nouse_key)
    if nouse is not None and nouse.strip() and match(nouse):
        return False
    return True
