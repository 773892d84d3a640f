"""AMD (MI355X) kubelet device plugin: ListAndWatch / GetPreferredAllocation / Allocate.

Reference: pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:93-1014
and util.go:94-414.  Protocol kept:
  * the plugin advertises ``split`` replicas per GPU (``<uuid>::<n>``) under
    ``amd.com/gpu`` (optionally with NUMA topology hints);
  * ``Allocate`` is serialised node-wide; the pod is found through the node lock
    / bind-phase annotations (``util.get_pending_pod``); the scheduler's
    decision is decoded from ``hami.io/amd-devices-to-allocate`` (+ CU ranges),
    the next non-empty container entry is popped (init containers first), the
    env/mounts/device nodes are built (:mod:`.allocate`), the popped entries
    are erased from the annotation, and when no AMD entries remain the pod is
    marked ``bind-phase=success`` and the node lock released; any failure marks
    ``failed`` and releases the lock;
  * ``GetPreferredAllocation`` maps the annotated physical GPUs onto replica ids.
``pod_allocation_try_success`` / ``pod_allocation_failed`` / ``get_pending_pod``
are module-level so tests can swap them (server.go:84, util.go:371-407).
"""

from __future__ import annotations

import logging
import os
import threading
import time
from concurrent import futures

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device.amd.device import AMD_DEVICE, CU_RANGES_ANNOS, IN_REQUEST_ANNOS, NODE_LOCK_AMD
from k8s_vgpu_scheduler_amd.k8s.client import containers, get_client, init_containers
from k8s_vgpu_scheduler_amd.smi import Backend, GPUInfo
from k8s_vgpu_scheduler_amd.utils import nodelock, util
from k8s_vgpu_scheduler_amd.utils import types as T

from . import api
from .allocate import PluginConfig, allocate_container
from .register import filtered

log = logging.getLogger(__name__)

REPLICA_SEP = "::"


def physical_id(replica_id: str) -> str:
    return replica_id.split(REPLICA_SEP, 1)[0]


# ----------------------------------------------------- swappable test seams
def get_pending_pod(node_name: str) -> dict:
    return util.get_pending_pod(node_name)


def _update_phase_and_release(node_name: str, pod: dict, phase: str):
    try:
        util.patch_pod_annotations(pod, {T.DEVICE_BIND_PHASE: phase})
    except Exception as e:  # noqa: BLE001
        log.error("failed to patch bind-phase=%s on %s: %s", phase, pod["metadata"]["name"], e)
    try:
        nodelock.release_node_lock(node_name, NODE_LOCK_AMD, pod)
    except Exception as e:  # noqa: BLE001
        log.error("failed to release node lock on %s: %s", node_name, e)


def pod_allocation_try_success(node_name: str, pod: dict):
    """Release the lock only once every device type of the pod is allocated."""
    md = pod["metadata"]
    fresh = get_client().get_pod(md.get("namespace", "default"), md["name"])
    remaining = ((fresh.get("metadata") or {}).get("annotations") or {}).get(IN_REQUEST_ANNOS, "")
    if any(d for ctr in codec.decode_pod_devices({AMD_DEVICE: IN_REQUEST_ANNOS},
                                                 {IN_REQUEST_ANNOS: remaining}).get(AMD_DEVICE, []) for d in ctr):
        return False
    _update_phase_and_release(node_name, fresh, T.DEVICE_BIND_SUCCESS)
    return True


def pod_allocation_failed(node_name: str, pod: dict):
    _update_phase_and_release(node_name, pod, T.DEVICE_BIND_FAILED)


def decode_pod_single_device(pod: dict) -> list:
    annos = (pod.get("metadata") or {}).get("annotations") or {}
    pd = codec.decode_pod_devices({AMD_DEVICE: IN_REQUEST_ANNOS}, annos).get(AMD_DEVICE)
    if pd is None:
        raise LookupError("device request not found")
    return codec.attach_cu_ranges(pd, annos.get(CU_RANGES_ANNOS))


def pop_next_container_devices(pod: dict, single: list):
    """Pop the first non-empty container entry (init containers first)."""
    n_init = len(init_containers(pod))
    for i, ctr in enumerate(single):
        if ctr:
            single[i] = []
            if i < n_init:
                return init_containers(pod)[i], ctr
            j = i - n_init
            if j >= len(containers(pod)):
                raise LookupError(f"container index {i} out of range (init={n_init}, regular={len(containers(pod))})")
            return containers(pod)[j], ctr
    raise LookupError("no pending device allocation found")


def patch_erased_annotation(pod: dict, single: list):
    enc = codec.encode_pod_single_device(single)
    util.patch_pod_annotations(pod, {IN_REQUEST_ANNOS: enc})
    pod["metadata"].setdefault("annotations", {})[IN_REQUEST_ANNOS] = enc


class AllocationError(Exception):
    pass


# --------------------------------------------------------------------- plugin
class AMDDevicePlugin:
    def __init__(self, backend: Backend, cfg: PluginConfig, node_name: str,
                 socket_dir: str = api.DEVICE_PLUGIN_PATH, socket_name: str = "mivgpu-amd.sock"):
        self.backend, self.cfg, self.node = backend, cfg, node_name
        self.gpus: list[GPUInfo] = filtered(backend.gpus(), cfg)
        self.by_uuid = {g.uuid: g for g in self.gpus}
        self.health = {g.uuid: True for g in self.gpus}
        self.event_unhealthy: dict[str, str] = {}    # uuid -> reason, set by device events
        self._cv = threading.Condition()
        self._gen = 0
        self.apply_mutex = threading.Lock()
        self.socket = os.path.join(socket_dir, socket_name)
        self.server = None
        self._stop = threading.Event()

    # ----------------------------------------------------------- devices
    def kubelet_devices(self) -> list:
        out = []
        for g in self.gpus:
            state = api.HEALTHY if self.health.get(g.uuid, True) else api.UNHEALTHY
            for i in range(self.cfg.device_split_count):
                d = api.Device(ID=f"{g.uuid}{REPLICA_SEP}{i}", health=state)
                if self.cfg.enable_numa_topology:
                    d.topology.nodes.add(ID=g.numa)
                out.append(d)
        return out

    def set_health(self, uuid: str, healthy: bool):
        with self._cv:
            if self.health.get(uuid) != healthy:
                self.health[uuid] = healthy
                self._gen += 1
                self._cv.notify_all()

    # event kinds that make a GPU unhealthy by default; "vmfault" is an
    # application fault (the XID 13/31/43 class the reference skips) and only
    # counts when DP_ENABLE_HEALTHCHECKS names it
    FATAL_EVENTS = {"gpu_pre_reset"}
    APP_EVENTS = {"vmfault"}

    def health_loop(self, period: float = 5.0):
        """rm/health.go:checkHealth, AMD form: block up to `period` on amd-smi
        event notifications (the XID event set), then poll RAS/ECC.  A reset
        event on a physical GPU marks it and all of its compute partitions
        unhealthy until the post-reset event; an event the backend cannot place
        marks every GPU.

        DP_DISABLE_HEALTHCHECKS: "all" / "*" or a list of checks ("ecc",
        "events", "reset"); DP_ENABLE_HEALTHCHECKS re-enables listed ones and can
        make application faults fatal ("vmfault") (reference rm/health.go:46-55)."""
        off = {x.strip().lower() for x in os.environ.get("DP_DISABLE_HEALTHCHECKS", "").split(",") if x.strip()}
        on = {x.strip().lower() for x in os.environ.get("DP_ENABLE_HEALTHCHECKS", "").split(",") if x.strip()}
        disabled = bool(off & {"all", "*"}) and not on
        self.backend.skip_checks = (off - on) - {"all", "*"}
        fatal = set(self.FATAL_EVENTS) | (on & self.APP_EVENTS)
        if "reset" in self.backend.skip_checks:
            fatal.discard("gpu_pre_reset")
        use_events = "events" not in self.backend.skip_checks
        from k8s_vgpu_scheduler_amd.deviceplugin.partition import is_applying

        while not self._stop.is_set():
            events, failed = None, False
            if use_events and not disabled:
                try:
                    events = self.backend.wait_health_events(self.gpus, period)
                except Exception as e:  # noqa: BLE001 -- health.go: a failed wait marks all devices
                    log.error("waiting for GPU events failed: %s; marking all devices unhealthy", e)
                    events, failed = [], True
                    for g in self.gpus:
                        self.event_unhealthy[g.uuid] = f"event wait failed: {e}"
                    self._stop.wait(period)
            if events is None and self._stop.wait(period):
                break
            if self._stop.is_set():
                break
            if disabled or is_applying():    # a partition reconfiguration is resetting GPUs
                continue
            if events is not None and not failed:
                # a wait that works again clears the marks a failed one left
                for u in [u for u, r in self.event_unhealthy.items() if r.startswith("event wait failed")]:
                    del self.event_unhealthy[u]
            for ev in events or ():
                self._apply_event(ev, fatal)
            for g in self.gpus:
                ok, why = self.backend.health(g)
                if ok and g.uuid in self.event_unhealthy:
                    ok, why = False, self.event_unhealthy[g.uuid]
                if not ok and self.health.get(g.uuid, True):
                    log.error("GPU %s unhealthy: %s", g.uuid, why)
                self.set_health(g.uuid, ok)

    def _apply_event(self, ev, fatal: set):
        targets = [g for g in self.gpus if ev.physical is None or g.physical == ev.physical]
        if ev.kind == "gpu_post_reset":
            for g in targets:
                if self.event_unhealthy.pop(g.uuid, None) is not None:
                    log.info("GPU %s back after reset", g.uuid)
            return
        if ev.kind not in fatal:
            log.info("skipping GPU event %s on %s: %s", ev.kind,
                     "all" if ev.physical is None else ev.physical, ev.message)
            return
        for g in targets:
            self.event_unhealthy[g.uuid] = f"{ev.kind}: {ev.message}".rstrip(": ")

    # ----------------------------------------------------------- gRPC API
    def GetDevicePluginOptions(self, request, context):  # noqa: N802
        return api.DevicePluginOptions(pre_start_required=False,
                                       get_preferred_allocation_available=self.cfg.enable_preferred_allocation)

    def ListAndWatch(self, request, context):  # noqa: N802
        gen = -1
        while not self._stop.is_set():
            with self._cv:
                if gen == self._gen:
                    self._cv.wait(timeout=1.0)
                if gen == self._gen:
                    if context is not None and not context.is_active():
                        return
                    continue
                gen = self._gen
            yield api.ListAndWatchResponse(devices=self.kubelet_devices())

    def GetPreferredAllocation(self, request, context):  # noqa: N802
        resp = api.PreferredAllocationResponse()
        try:
            pod = get_pending_pod(self.node)
            single = decode_pod_single_device(pod)
        except Exception:  # noqa: BLE001 -- no annotation: fall back to kubelet's order
            pod, single = None, []
        for creq in request.container_requests:
            avail = list(creq.available_deviceIDs)
            chosen = list(creq.must_include_deviceIDs)
            want = []
            for ctr in single:
                if ctr:
                    want = [d.uuid for d in ctr]
                    break
            for u in want:
                if len(chosen) >= creq.allocation_size:
                    break
                for rid in avail:
                    if rid not in chosen and physical_id(rid) == u and \
                            all(physical_id(c) != u for c in chosen):
                        chosen.append(rid)
                        break
            for rid in avail:
                if len(chosen) >= creq.allocation_size:
                    break
                if rid not in chosen:
                    chosen.append(rid)
            resp.container_responses.add(deviceIDs=chosen[:creq.allocation_size])
        return resp

    def PreStartContainer(self, request, context):  # noqa: N802
        return api.PreStartContainerResponse()

    def allocate(self, container_requests: list[list[str]]) -> list[dict]:
        """Core of Allocate; returns per-container dicts (envs/mounts/devices)."""
        with self.apply_mutex:
            pod = get_pending_pod(self.node)
            try:
                single = decode_pod_single_device(pod)
            except Exception as e:
                pod_allocation_failed(self.node, pod)
                raise AllocationError(str(e)) from e
            out = []
            try:
                for ids in container_requests:
                    ctr, devreq = pop_next_container_devices(pod, single)
                    if len(devreq) != len(ids):
                        raise AllocationError("device number not matched")
                    for d in devreq:
                        if d.uuid not in self.by_uuid:
                            raise AllocationError(f"allocated GPU {d.uuid} is not managed by this node")
                        if not self.health.get(d.uuid, True):
                            raise AllocationError(f"allocated GPU {d.uuid} is unhealthy")
                    out.append(allocate_container(pod, ctr, devreq, self.by_uuid, self.cfg,
                                                  make_dirs=not os.environ.get("MIVGPU_DP_DRY_RUN")))
                patch_erased_annotation(pod, single)
            except Exception:
                pod_allocation_failed(self.node, pod)
                raise
            pod_allocation_try_success(self.node, pod)
            return out

    def Allocate(self, request, context):  # noqa: N802
        import grpc

        try:
            res = self.allocate([list(r.devices_ids) for r in request.container_requests])
        except Exception as e:  # noqa: BLE001
            log.error("Allocate failed: %s", e)
            if context is not None:
                context.abort(grpc.StatusCode.UNKNOWN, str(e))
            raise
        resp = api.AllocateResponse()
        for r in res:
            c = resp.container_responses.add()
            for k, v in r["envs"].items():
                c.envs[k] = v
            for m in r["mounts"]:
                c.mounts.add(**m)
            for d in r["devices"]:
                c.devices.add(**d)
            for name in r.get("cdi_devices", ()):
                c.cdi_devices.add(name=name)
            for k, v in r.get("annotations", {}).items():
                c.annotations[k] = v
        return resp

    # --------------------------------------------------------- serve/register
    def serve(self, max_workers: int = 8):
        import grpc

        try:
            os.unlink(self.socket)
        except FileNotFoundError:
            pass
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers))
        api.add_device_plugin_servicer(self.server, self)
        self.server.add_insecure_port(f"unix://{self.socket}")
        self.server.start()
        return self.server

    def register_with_kubelet(self, kubelet_socket: str = api.KUBELET_SOCKET, timeout: float = 10.0):
        import grpc

        with grpc.insecure_channel(f"unix://{kubelet_socket}") as ch:
            grpc.channel_ready_future(ch).result(timeout=timeout)
            api.RegistrationStub(ch).Register(api.RegisterRequest(
                version=api.VERSION, endpoint=os.path.basename(self.socket), resource_name=self.cfg.resource_name,
                options=api.DevicePluginOptions(
                    get_preferred_allocation_available=self.cfg.enable_preferred_allocation)), timeout=timeout)

    def start(self, kubelet_socket: str = api.KUBELET_SOCKET, register: bool = True):
        self.serve()
        if register:
            self.register_with_kubelet(kubelet_socket)
        threading.Thread(target=self.health_loop, name="health", daemon=True).start()
        return self

    def stop(self):
        self._stop.set()
        with self._cv:
            self._cv.notify_all()
        if self.server is not None:
            self.server.stop(grace=1)


def _sock_id(path: str):
    """(inode, ctime) of a socket file, None if absent: a re-created socket
    (kubelet restart) has a new identity even at the same path."""
    try:
        st = os.stat(path)
    except OSError:
        return None
    return (st.st_ino, st.st_ctime_ns)


def run_with_restarts(make_plugin, kubelet_socket: str, max_restarts: int = 5, window_s: float = 3600.0,
                      stop: threading.Event | None = None, reload: threading.Event | None = None,
                      poll_s: float = 1.0, restart_grace_s: float = 10.0, stats: dict | None = None):
    """Keep the plugin registered with the kubelet.

    * A kubelet restart is not a crash (main.go:305-337 restarts the plugins
      when the kubelet socket is re-created): the kubelet wipes the
      device-plugins directory, our socket included, and creates a new
      kubelet.sock; the plugin waits for it and re-registers.
    * ``reload`` (the device list changed, e.g. a new compute-partition mode)
      re-registers without counting as a crash.
    * Anything else that stops the plugin is a crash; more than
      ``max_restarts`` within ``window_s`` is fatal (server.go:518-566).
    ``stats`` (optional) counts crashes / kubelet restarts / reloads."""
    stop = stop or threading.Event()
    reload = reload or threading.Event()
    stats = stats if stats is not None else {}
    for k in ("crashes", "kubelet_restarts", "reloads", "registrations"):
        stats.setdefault(k, 0)
    restarts: list[float] = []
    waiting_logged = False
    while not stop.is_set():
        kubelet_id = _sock_id(kubelet_socket)
        if kubelet_id is None:
            if not waiting_logged:
                log.info("waiting for the kubelet socket %s", kubelet_socket)
                waiting_logged = True
            stop.wait(poll_s)
            continue
        waiting_logged = False
        plugin = make_plugin()
        try:
            plugin.start(kubelet_socket)
            stats["registrations"] += 1
            while not stop.wait(poll_s):
                if reload.is_set():
                    reload.clear()
                    stats["reloads"] += 1
                    log.info("device list changed: re-registering the plugin with the kubelet")
                    break
                if _sock_id(kubelet_socket) != kubelet_id:
                    stats["kubelet_restarts"] += 1
                    log.info("kubelet socket %s gone or re-created (kubelet restart): re-registering",
                             kubelet_socket)
                    break
                if not os.path.exists(plugin.socket):
                    # the kubelet removes plugin sockets when it restarts, possibly
                    # before its own socket is re-created: give it a grace period
                    deadline = time.monotonic() + restart_grace_s
                    while time.monotonic() < deadline and _sock_id(kubelet_socket) == kubelet_id:
                        if stop.wait(min(poll_s, 0.2)):
                            return
                    if _sock_id(kubelet_socket) != kubelet_id:
                        stats["kubelet_restarts"] += 1
                        log.info("kubelet restarted (plugin socket removed, kubelet socket re-created)")
                        break
                    raise RuntimeError("plugin socket disappeared while the kubelet kept running")
        except Exception as e:  # noqa: BLE001
            if _sock_id(kubelet_socket) is None or _sock_id(kubelet_socket) != kubelet_id:
                # registration raced a kubelet restart: not the plugin's fault
                stats["kubelet_restarts"] += 1
                log.info("kubelet went away during registration (%s); waiting for it", e)
            else:
                stats["crashes"] += 1
                log.error("device plugin crashed: %s", e)
                now = time.time()
                restarts = [t for t in restarts if now - t < window_s] + [now]
                if len(restarts) > max_restarts:
                    raise RuntimeError(f"device plugin restarted more than {max_restarts} times within "
                                       f"{window_s}s") from e
                stop.wait(poll_s)
        finally:
            plugin.stop()
