"""Scheduler extender core: caches, registration loop, Filter, simulation Filter, Bind.

Reference: pkg/scheduler/scheduler.go:60-1209.  Behavioural contract kept:
  * informer-driven pod / node / ResourceQuota (and Lease) caches; pods that
    carry ``hami.io/vgpu-node`` are decoded from their allocation annotation,
    collapsed for init containers and added to PodManager + QuotaManager;
  * ``register`` (leader only, 15 s tick + node/leader notifications) reads
    every node's registration annotation, checks backend health (handshake),
    cleans unhealthy/zero-device nodes and marks the cache ``synced``;
  * ``filter`` is idempotent per pod (take-and-delete previous reservation),
    scores every candidate, picks the best node, patches
    ``hami.io/vgpu-node``/``-time`` plus backend annotations and reserves the
    usage immediately;
  * beyond the reference (which re-derives every node's usage from every pod
    and scores nodes in goroutines, score.go:360-419): one usage view per
    node, rebuilt only when that node's pods or registration change, and a
    memo of per-node Fit results keyed by (node usage generation, the pod's
    scheduling-relevant spec, the namespace's quota state).  Between two
    Filters only the node that received the last pod changes, so a Filter
    over N nodes re-fits ~1 node instead of N (Filter p99 at 100 nodes:
    112-152 ms -> see profiles/scheduler_bench_100.json).  Nodes whose
    device state is identical (every empty node of a fresh cluster) share one
    Fit result under device-id renaming, so even a new pod shape fits once per
    distinct node state, not once per node;
  * CA simulation (``Nodes`` given) touches no cache;
  * ``bind`` takes every backend's node lock transactionally (sorted, with
    rollback; PodGroup members retry until --node-lock-retry-timeout), marks
    bind-phase=allocating and creates the Binding.
"""

from __future__ import annotations

import json
import logging
import os
import threading
import time
from collections import OrderedDict

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device import devices as D
from k8s_vgpu_scheduler_amd.device.init_container import (app_containers_only_device_usage,
                                                          collapse_init_container_usage)
from k8s_vgpu_scheduler_amd.device.pods import PodManager
from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.device.types import DeviceUsage, NodeInfo, copy_pod_devices
from k8s_vgpu_scheduler_amd.k8s.client import KubeClient, annotations, name_of, ns_of
from k8s_vgpu_scheduler_amd.k8s.informer import Informer
from k8s_vgpu_scheduler_amd.utils import nodelock, util
from k8s_vgpu_scheduler_amd.utils import types as T
from k8s_vgpu_scheduler_amd.utils.leaderelection import DummyLeaderManager, LeaderManager
from k8s_vgpu_scheduler_amd.utils.weights import weights_for_pod

from . import events as E
from .config import SchedulerConfig
from .nodes import NodeManager
from .policy import DeviceListsScore, DeviceUsageList, NodeScoreList
from .score import NodeUsage, calc_score, record_result, resolve_node_policy, score_node_safe

log = logging.getLogger(__name__)


def _decode_allocation(pod: dict) -> dict:
    """Raw per-container PodDevices from the *-allocated annotations (+ CU ranges)."""
    raw = codec.decode_pod_devices(D.SUPPORT_DEVICES, annotations(pod))
    for t, single in raw.items():
        dev = D.get_devices().get(t)
        key = getattr(dev, "CU_RANGES_ANNOS", None) or "hami.io/amd-cu-ranges"
        codec.attach_cu_ranges(single, annotations(pod).get(key))
    return raw


# Annotations the scheduler / device plugin write as OUTPUT of a Filter or Bind;
# they never influence Fit and are left out of the memo key.
_OUTPUT_ANNOTATIONS = frozenset({T.ASSIGNED_NODE_ANNOTATION, T.ASSIGNED_TIME_ANNOTATION, T.BIND_TIME_ANNOTATION,
                                 T.DEVICE_BIND_PHASE})
_MEMO_MAX = 16384


def _output_annotation(key: str) -> bool:
    if key in _OUTPUT_ANNOTATIONS:
        return True
    if key in D.IN_REQUEST_DEVICES.values() or key in D.SUPPORT_DEVICES.values():
        return True
    return any(getattr(dev, "CU_RANGES_ANNOS", None) == key for dev in D.get_devices().values()) or \
        key == "hami.io/amd-cu-ranges"


def fit_signature(pod: dict) -> str:
    """Everything of ``pod`` that Fit and the node score read: namespace,
    per-container resources (+ init-container restart policy), annotations
    other than the scheduler's own outputs."""
    md = pod.get("metadata") or {}
    spec = pod.get("spec") or {}
    annos = {k: v for k, v in (md.get("annotations") or {}).items() if not _output_annotation(k)}
    return json.dumps([md.get("namespace", "default"), annos,
                       [c.get("resources") for c in spec.get("containers") or []],
                       [(c.get("resources"), c.get("restartPolicy")) for c in spec.get("initContainers") or []]],
                      sort_keys=True, default=str)


class Scheduler:
    def __init__(self, client: KubeClient, cfg: SchedulerConfig | None = None):
        self.client = client
        self.cfg = cfg or SchedulerConfig()
        self.nodes = NodeManager()
        self.pod_manager = PodManager()
        self.quota_manager = get_local_cache()
        self.events = E.EventRecorder(client)
        self.overview: dict[str, NodeUsage] = {}
        self._lock = threading.RLock()
        self.synced = False
        self.started = False
        self._stop = threading.Event()
        self._notify = threading.Event()
        if self.cfg.leader_elect:
            self.leader = LeaderManager(self.cfg.hostname, self.cfg.leader_elect_resource_namespace,
                                        self.cfg.leader_elect_resource_name,
                                        on_started=self._notify.set, on_stopped=self._lost_leadership)
        else:
            self.leader = DummyLeaderManager(True)
        # node -> ((registration gen, pods gen), NodeUsage with policy-free device list)
        self._usage_cache: dict[str, tuple[tuple, NodeUsage]] = {}
        self._score_memo: OrderedDict = OrderedDict()
        self._cache_mu = threading.Lock()
        # Filter's read-usage -> fit -> commit-to-cache section: two overlapping
        # Filters (threaded HTTP server, several scheduler profiles, a retried
        # request) would otherwise both fit against the same free capacity and
        # over-commit a GPU (tests/test_filter_concurrency.py)
        self._decide_mu = threading.Lock()
        # Filters of the SAME pod (an extender-timeout retry, two scheduler
        # profiles) run one at a time from decide through the annotation patch
        # and its rollback: otherwise a rollback could delete the
        # other Filter's live reservation, or the patches land out of order
        self._pod_serial_mu = threading.Lock()
        self._pod_serial: dict[str, list] = {}   # uid -> [lock, users]
        self.memo_hits = 0
        self.memo_misses = 0
        self.memo_class_hits = 0
        self.memoize = True     # False: fit every candidate from scratch (tests compare the two)
        self.pods_inf = Informer(client, "pods")
        self.nodes_inf = Informer(client, "nodes")
        self.quota_inf = Informer(client, "resourcequotas")
        self.lease_inf = Informer(client, "leases", self.cfg.leader_elect_resource_namespace) \
            if self.cfg.leader_elect else None

    # ------------------------------------------------------------ lifecycle
    def _lost_leadership(self):
        with self._lock:
            self.synced = False

    def start(self):
        self.pods_inf.add_event_handler(self.on_add_pod, self.on_update_pod, self.on_del_pod)
        self.nodes_inf.add_event_handler(lambda n: self._notify.set(), self.on_update_node, self.on_del_node)
        self.quota_inf.add_event_handler(self.quota_manager.add_quota,
                                         lambda o, n: self.quota_manager.update_quota(o, n),
                                         self.quota_manager.del_quota)
        self.pods_inf.start()
        self.nodes_inf.start()
        self.quota_inf.start()
        if self.lease_inf is not None:
            self.lease_inf.add_event_handler(self.leader.on_add, self.leader.on_update, self.leader.on_delete)
            self.lease_inf.start()
        self.started = True

    def stop(self):
        self._stop.set()
        self._notify.set()
        for inf in (self.pods_inf, self.nodes_inf, self.quota_inf, self.lease_inf):
            if inf is not None:
                inf.stop()

    def run_register_loop(self, period: float = 15.0):
        """RegisterFromNodeAnnotations (scheduler.go:413-441)."""
        while not self._stop.is_set():
            self._notify.wait(timeout=period)
            self._notify.clear()
            if self._stop.is_set():
                return
            if not self.started:
                continue
            try:
                self.register()
            except Exception:  # noqa: BLE001
                log.exception("register failed")

    @staticmethod
    def _device_annos(node: dict | None) -> dict:
        anns = ((node or {}).get("metadata") or {}).get("annotations") or {}
        return {k: v for k, v in anns.items() if k.startswith("hami.io/node-")}

    def on_update_node(self, old: dict, new: dict):
        """The reference wakes registration on node add only (scheduler.go:371-374) and
        otherwise waits for the 15 s ticker; a changed device-registration or
        handshake annotation wakes it now, so a GPU the device plugin just
        registered is schedulable within one watch event.  Status heartbeats
        do not touch these annotations and do not wake it."""
        if self._device_annos(old) != self._device_annos(new):
            self._notify.set()

    # ------------------------------------------------------------- pod events
    def on_add_pod(self, pod: dict):
        annos = annotations(pod)
        node_id = annos.get(T.ASSIGNED_NODE_ANNOTATION)
        if node_id is None:
            return
        if util.is_pod_terminated(pod):
            pi = self.pod_manager.take_and_delete_pod(pod)
            if pi:
                self.quota_manager.rm_usage(pod, pi.devices)
            return
        if util.is_pod_terminating(pod):
            self.pod_manager.update_pod(pod)
            return
        try:
            raw = _decode_allocation(pod)
        except codec.CodecError as e:
            log.error("failed to decode pod devices %s/%s: %s", ns_of(pod), name_of(pod), e)
            return
        eff = collapse_init_container_usage(pod, raw)
        if self.pod_manager.add_pod(pod, node_id, eff):
            self.quota_manager.add_usage(pod, eff)

    def on_update_pod(self, old: dict, new: dict):
        if T.ASSIGNED_NODE_ANNOTATION not in annotations(new):
            return
        if util.is_pod_terminated(new):
            pi = self.pod_manager.take_and_delete_pod(new)
            if pi:
                self.quota_manager.rm_usage(new, pi.devices)
            return
        if util.is_pod_terminating(new):
            self.pod_manager.update_pod(new)
            return
        pi = self.pod_manager.get_pod(new)
        if pi is None:
            self.on_add_pod(new)
            return
        self.pod_manager.update_pod(new)
        if not pi.init_released and util.all_init_containers_succeeded(new):
            try:
                raw = _decode_allocation(new)
            except codec.CodecError:
                return
            app_only = app_containers_only_device_usage(new, raw)
            old_devs, ok = self.pod_manager.update_pod_device(new, app_only)
            if ok:
                self.quota_manager.replace_usage(new, old_devs, app_only)

    def on_del_pod(self, pod: dict):
        if T.ASSIGNED_NODE_ANNOTATION not in annotations(pod):
            return
        pi = self.pod_manager.take_and_delete_pod(pod)
        if pi:
            self.quota_manager.rm_usage(pod, pi.devices)

    def on_del_node(self, node: dict):
        name = name_of(node)
        nodelock.cleanup_node_lock(name)
        self.nodes.rm_node(name)
        with self._lock:
            self.overview.pop(name, None)
        for dev in D.get_devices().values():
            dev.node_deleted(name)
        self._notify.set()

    # ------------------------------------------------------------ register
    def register(self):
        with self._lock:
            if not self.leader.is_leader():
                return
            self.update_scheduler_label()
            names = []
            for node in self.nodes_inf.list(self.cfg.node_label_selector or None):
                name = name_of(node)
                names.append(name)
                for vendor, dev in D.get_devices().items():
                    err = None
                    try:
                        nodedevs = dev.get_node_devices(node)
                    except Exception as e:  # noqa: BLE001
                        nodedevs, err = [], e
                    healthy, need_update = dev.check_health(vendor, node)
                    if not healthy:
                        try:
                            cur = self.nodes.get_node(name)
                        except LookupError:
                            continue
                        if vendor not in cur.devices:
                            continue
                        log.error("device unhealthy, cleaning up node %s vendor %s", name, vendor)
                        try:
                            dev.node_cleanup(name)
                        except Exception as e:  # noqa: BLE001
                            log.error("node cleanup failed: %s", e)
                        self.nodes.rm_node_devices(name, vendor)
                        continue
                    if err is not None:
                        continue
                    if not nodedevs:
                        try:
                            if vendor in self.nodes.get_node(name).devices:
                                self.nodes.rm_node_devices(name, vendor)
                        except LookupError:
                            pass
                        continue
                    if not need_update:
                        try:
                            self.nodes.get_node(name)
                            continue
                        except LookupError:
                            pass  # not cached yet (e.g. restart): register anyway
                    info = NodeInfo(id=name, node=node, devices={})
                    for d in nodedevs:
                        info.devices.setdefault(d.devicevendor or vendor, []).append(d)
                    self.nodes.add_node(name, info)
            # A delete event can land between the list above and add_node (the
            # reference's register/onDelNode race, register_race_test.go:37-56):
            # the node would be re-added after on_del_node removed it and never
            # leave the cache.  Every pass therefore drops cached nodes the
            # lister no longer returns, so the cache converges on the next pass.
            listed = set(names)
            for stale in [n for n in self.nodes.node_ids() if n not in listed]:
                log.info("dropping node %s: no longer listed", stale)
                self.nodes.rm_node(stale)
                self.overview.pop(stale, None)
            _, overall, _ = self.get_nodes_usage(names, None)
            self.overview = overall
            self.synced = True

    def update_scheduler_label(self):
        ns, me = os.environ.get("POD_NAMESPACE"), os.environ.get("POD_NAME")
        if not ns or not me:
            return
        for pod in self.pods_inf.list({T.COMPONENT_LABEL: T.COMPONENT_SCHEDULER}, namespace=ns):
            want = T.ROLE_LEADER if name_of(pod) == me else T.ROLE_FOLLOWER
            if (pod["metadata"].get("labels") or {}).get(T.ROLE_LABEL) != want:
                try:
                    util.patch_pod_labels(ns, name_of(pod), {T.ROLE_LABEL: want})
                except Exception as e:  # noqa: BLE001
                    log.error("failed to label scheduler pod %s: %s", name_of(pod), e)

    def wait_for_cache_sync(self, timeout: float = 30.0) -> bool:
        deadline = time.time() + timeout
        while time.time() < deadline:
            with self._lock:
                if self.synced:
                    return True
            time.sleep(0.1)
        return False

    def inspect_all_nodes_usage(self) -> dict[str, NodeUsage]:
        with self._lock:
            return {k: v.deepcopy() for k, v in self.overview.items()}

    # --------------------------------------------------------------- usage
    @staticmethod
    def _pod_list_policy(pod: dict | None) -> tuple[str, bool]:
        policy = util.get_gpu_scheduler_policy_by_pod(D.gpu_scheduler_policy(), pod)
        numa = str(annotations(pod or {}).get("amd.com/numa-bind", "")).lower() in ("1", "t", "true")
        return policy, numa

    def build_node_usage(self, info: NodeInfo, pod: dict | None) -> NodeUsage:
        policy, numa = self._pod_list_policy(pod)
        lst = DeviceUsageList([], policy, numa)
        for vendor_devs in info.devices.values():
            for d in vendor_devs:
                ci = dict(d.custominfo or {})
                if d.pair_scores:
                    ci["pair_scores"] = dict(d.pair_scores)
                lst.device_lists.append(DeviceListsScore(DeviceUsage(
                    id=d.id, index=d.index, used=0, count=d.count, usedmem=0, totalmem=d.devmem,
                    totalcore=d.devcore, usedcores=0, mode=d.mode, numa=d.numa, type=d.type, health=d.health,
                    pod_infos=[], custominfo=ci)))
        return NodeUsage(info.node, info, lst)

    @staticmethod
    def _apply_pods(usage: NodeUsage, pods) -> None:
        by_id = {dl.device.id: dl.device for dl in usage.devices.device_lists}
        for p in pods:
            for single in p.devices.values():
                for ctr in single:
                    for cd in ctr:
                        d = by_id.get(cd.uuid)
                        if d is None:
                            log.error("pod %s/%s holds unknown device %s on %s", p.namespace, p.name,
                                      cd.uuid, p.node_id)
                            continue
                        d.used += max(cd.slots, 1)
                        d.usedmem += cd.usedmem
                        d.usedcores += cd.usedcores
                        d.pod_infos.append((p.namespace, p.name, p.uid))
                        r = (cd.custominfo or {}).get("cu_ranges")
                        if r:
                            from k8s_vgpu_scheduler_amd.device.amd.cu_alloc import charge
                            charge(d.custominfo, r, cd.usedcores)

    @staticmethod
    def _shape(usage: NodeUsage) -> tuple[tuple, tuple]:
        """(shape, device ids in list order).  Two nodes with equal shapes are
        interchangeable for Fit up to renaming their device ids: same devices
        in the same order, same usage, CU bitmaps, pair-score matrix (by
        position) and cordons."""
        devs = [dl.device for dl in usage.devices.device_lists]
        pos = {d.id: i for i, d in enumerate(devs)}
        from k8s_vgpu_scheduler_amd.device.amd.device import cordoned_devices
        cordon = cordoned_devices(usage.node_info)
        shape = tuple((d.index, d.type, d.count, d.totalmem, d.totalcore, d.mode, d.numa, d.health, d.used,
                       d.usedmem, d.usedcores, d.custominfo.get("cu_used", 0),
                       tuple(sorted((d.custominfo.get("cu_shared") or {}).items())), d.id in cordon,
                       tuple(sorted((pos.get(k, -1), v) for k, v in (d.custominfo.get("pair_scores") or {}).items())))
                      for d in devs)
        return shape, tuple(d.id for d in devs)

    def _cached_usage(self, node_id: str) -> tuple | None:
        """(generation key, shared base usage, shape, device ids) of a registered
        node, rebuilt only when its registration or its pods changed.  The
        NodeUsage is shared: copy it before fitting into it."""
        ref = self.nodes.get_node_ref(node_id)
        if ref is None:
            return None
        ngen, info = ref
        with self._cache_mu:
            hit = self._usage_cache.get(node_id)
        if hit is not None and hit[0] == (ngen, self.pod_manager.node_generation(node_id)):
            return hit
        pgen, pods = self.pod_manager.pods_on_node(node_id)
        key = (ngen, pgen)
        usage = self.build_node_usage(info, None)
        self._apply_pods(usage, pods)
        shape, ids = self._shape(usage)
        entry = (key, usage, shape, ids)
        with self._cache_mu:
            self._usage_cache[node_id] = entry
        return entry

    @staticmethod
    def _rename(hit: tuple, node_id: str, node: dict, src_ids: tuple, dst_ids: tuple) -> tuple:
        """A class-memo result fitted on an equal-shaped node, moved to ``node_id``."""
        sc, reason = hit
        if sc is None:
            return hit
        m = dict(zip(src_ids, dst_ids))
        devs = copy_pod_devices(sc.devices)
        for single in devs.values():
            for ctr in single:
                for cd in ctr:
                    cd.uuid = m.get(cd.uuid, cd.uuid)
        return type(sc)(node_id, node, devs, sc.score), reason

    def _usage_for_pod(self, base: NodeUsage, pod: dict | None) -> NodeUsage:
        policy, numa = self._pod_list_policy(pod)
        return NodeUsage(base.node, base.node_info,
                         DeviceUsageList([DeviceListsScore(dl.device.deepcopy()) for dl in base.devices.device_lists],
                                         policy, numa))

    def get_nodes_usage(self, node_names: list | None, pod: dict | None):
        overall: dict[str, NodeUsage] = {}
        failed: dict[str, str] = {}
        ids = self.nodes.node_ids()
        for nid in ids:
            c = self._cached_usage(nid)
            if c is not None:
                overall[nid] = self._usage_for_pod(c[1], pod)
        with self._cache_mu:
            for stale in [n for n in self._usage_cache if n not in overall]:
                del self._usage_cache[stale]
        if node_names is None:
            return {}, overall, failed
        cache = {}
        for n in node_names:
            if n not in overall:
                failed[n] = "node unregistered"
                continue
            cache[n] = overall[n]
        return cache, overall, failed

    def score_candidates(self, node_names: list, pod: dict, reqs: list):
        """Fit ``pod`` on every candidate node; per-node results come from the
        memo when neither the node nor the namespace quota changed since the
        same pod shape was last fitted there.
        -> (NodeScoreList, failure reasons, failed nodes)."""
        weights = weights_for_pod(pod)
        policy = resolve_node_policy(pod, self.cfg.node_scheduler_policy)
        res = NodeScoreList(node_list=[], policy=policy)
        failure: dict[str, list] = {}
        failed: dict[str, str] = {}
        sig = (fit_signature(pod), D.gpu_scheduler_policy(), self.cfg.node_scheduler_policy,
               D.registry_generation(),   # a config reload re-creates the backends (ids may be reused)
               self.quota_manager.fit_key((pod.get("metadata") or {}).get("namespace", "default")))
        # UUID selectors name concrete devices: equal-shaped nodes stop being interchangeable
        annos = annotations(pod)
        by_class = not any(k in annos for k in ("amd.com/use-gpu-uuid", "amd.com/nouse-gpu-uuid"))
        for n in node_names:
            c = self._cached_usage(n)
            if c is None:
                failed[n] = "node unregistered"
                continue
            key = (n, c[0], sig)
            ckey = (c[2], sig) if by_class else None
            with self._cache_mu:
                hit = self._score_memo.get(key)
                if hit is not None:
                    self._score_memo.move_to_end(key)
                    self.memo_hits += 1
                elif ckey is not None:
                    tmpl = self._score_memo.get(ckey)
                    if tmpl is not None:
                        self._score_memo.move_to_end(ckey)
                        hit = self._rename(tmpl[0], n, c[1].node, tmpl[1], c[3])
                        self._score_memo[key] = hit
                        self.memo_class_hits += 1
            if hit is None:
                hit = score_node_safe(n, self._usage_for_pod(c[1], pod), reqs, pod, policy, weights)
                with self._cache_mu:
                    self.memo_misses += 1
                    self._score_memo[key] = hit
                    if ckey is not None:
                        self._score_memo[ckey] = (hit, c[3])
                    while len(self._score_memo) > _MEMO_MAX:
                        self._score_memo.popitem(last=False)
            record_result(res, failure, failed, n, hit[0], hit[1])
        return res, failure, failed

    def get_simulation_nodes_usage(self, nodes: list[dict], pod: dict):
        cand, failed = {}, {}
        for node in nodes or []:
            info = NodeInfo(id=name_of(node), node=node, devices={})
            for vendor, dev in D.get_devices().items():
                try:
                    for d in dev.get_node_devices(node):
                        info.devices.setdefault(d.devicevendor or vendor, []).append(d)
                except Exception:  # noqa: BLE001
                    continue
            if not info.devices:
                failed[name_of(node)] = "node unregistered"
                continue
            cand[name_of(node)] = self.build_node_usage(info, pod)
        return cand, failed

    # --------------------------------------------------------------- locks
    def lock_all_devices(self, node: dict, pod: dict):
        acquired = []
        for k in sorted(D.get_devices()):
            dev = D.get_devices()[k]
            try:
                dev.lock_node(node, pod)
            except Exception:
                for a in reversed(acquired):
                    try:
                        a.release_node_lock(node, pod)
                    except Exception as e:  # noqa: BLE001
                        log.error("rollback release failed: %s", e)
                raise
            acquired.append(dev)

    def release_all_devices(self, node: dict, pod: dict):
        for k in sorted(D.get_devices()):
            try:
                D.get_devices()[k].release_node_lock(node, pod)
            except Exception as e:  # noqa: BLE001
                log.error("release node lock failed: %s", e)

    def acquire_node_locks(self, node: dict, pod: dict):
        if not util.is_pod_group_member(pod) or self.cfg.node_lock_retry_timeout <= 0:
            return self.lock_all_devices(node, pod)
        deadline = time.time() + self.cfg.node_lock_retry_timeout
        while True:
            try:
                return self.lock_all_devices(node, pod)
            except nodelock.NodeLockContention:
                if time.time() > deadline:
                    raise nodelock.NodeLockContention(
                        f"timed out after {self.cfg.node_lock_retry_timeout}s waiting for node "
                        f"{name_of(node)} to be unlocked")
                if self._stop.wait(0.1):
                    raise

    # ------------------------------------------------------------------ bind
    def bind(self, args: dict) -> dict:
        pod_name = args.get("PodName") or args.get("podName")
        ns = args.get("PodNamespace") or args.get("podNamespace") or "default"
        uid = args.get("PodUID") or args.get("podUID")
        node_name = args.get("Node") or args.get("node")
        current = self.pods_inf.get(pod_name, ns)
        if current is None:
            try:
                current = self.client.get_pod(ns, pod_name)
            except Exception as e:  # noqa: BLE001
                self._cleanup_stale({"metadata": {"name": pod_name, "namespace": ns, "uid": uid}})
                return {"Error": str(e)}
        node = self.nodes_inf.get(node_name)
        if node is None:
            try:
                node = self.client.get_node(node_name)
            except Exception as e:  # noqa: BLE001
                self.events.binding_result(current, E.BINDING_FAILED, [], f"failed to get node {node_name}")
                self._cleanup_stale(current)
                return {"Error": str(e)}

        def fail(e):
            self.release_all_devices(node, current)
            self.events.binding_result(current, E.BINDING_FAILED, [], e)
            return {"Error": str(e) if e else ""}

        try:
            self.acquire_node_locks(node, current)
        except Exception as e:  # noqa: BLE001
            return fail(e)
        try:
            util.patch_pod_annotations(current, {T.DEVICE_BIND_PHASE: T.DEVICE_BIND_ALLOCATING,
                                                 T.BIND_TIME_ANNOTATION: str(int(time.time()))})
            self.client.bind(ns, pod_name, node_name, uid)
        except Exception as e:  # noqa: BLE001
            return fail(e)
        self.events.binding_result(current, E.BINDING_SUCCEED, [node_name], None)
        return {"Error": ""}

    def _cleanup_stale(self, pod: dict):
        pi = self.pod_manager.take_and_delete_pod(pod)
        if pi and pi.devices:
            self.quota_manager.rm_usage(pod, pi.devices)

    # ---------------------------------------------------------------- filter
    def filter(self, args: dict) -> dict:
        pod = args.get("Pod") or args.get("pod")
        node_names = args.get("NodeNames", args.get("nodenames"))
        nodes = args.get("Nodes", args.get("nodes"))
        reqs = D.resource_reqs(pod)
        if not any(reqs):
            return {"NodeNames": node_names, "FailedNodes": None, "Error": ""}
        if nodes is not None:
            return self._filter_simulation(pod, nodes, reqs)
        uid = (pod.get("metadata") or {}).get("uid") or \
            f"{(pod.get('metadata') or {}).get('namespace', '')}/{(pod.get('metadata') or {}).get('name', '')}"
        with self._pod_serial_mu:
            ent = self._pod_serial.setdefault(uid, [threading.Lock(), 0])
            ent[1] += 1
        ent[0].acquire()
        try:
            return self._filter_one(pod, node_names, reqs)
        finally:
            ent[0].release()
            with self._pod_serial_mu:
                ent[1] -= 1
                if ent[1] == 0:
                    self._pod_serial.pop(uid, None)

    def _filter_one(self, pod: dict, node_names, reqs) -> dict:
        # decide and commit to the caches under the lock; the API writes
        # (events, the allocation patch) happen outside it, serialised per pod
        with self._decide_mu:
            d = self._decide(pod, node_names, reqs)
        if d["best"] is None:
            for reason, ns_ in sorted(d["failure"].items()):
                self.events.filter_result(pod, E.FILTERING_FAILED, "",
                                          f"{len(ns_)} nodes {reason}({','.join(sorted(ns_))})")
            self.events.filter_result(pod, E.FILTERING_FAILED, "",
                                      f"no available node, {len(node_names or [])} nodes do not meet")
            return {"FailedNodes": d["failed"], "NodeNames": None, "Error": ""}
        best, scores = d["best"], d["scores"]
        try:
            util.patch_pod_annotations(pod, d["annos"])
        except Exception as e:  # noqa: BLE001
            self.events.filter_result(pod, E.FILTERING_FAILED, "", e)
            with self._decide_mu:
                # roll back only this decision's reservation (an informer event
                # may have replaced it in the meantime)
                cur = self.pod_manager.get_pod(pod)
                if cur is not None and cur.node_id == best.node_id and cur.devices == d["eff"]:
                    if d["added"]:
                        self.quota_manager.rm_usage(pod, d["eff"])
                    self.pod_manager.del_pod(pod)
            return {"Error": str(e)}
        msg = (f"find fit node({best.node_id}), {len(node_names or []) - len(scores.node_list)} nodes not fit, "
               f"{len(scores.node_list)} nodes fit("
               + ",".join(f"{n.node_id}:{n.score:.2f}" for n in scores.node_list) + ")")
        self.events.filter_result(pod, E.FILTERING_SUCCEED, msg, None)
        return {"NodeNames": [best.node_id], "FailedNodes": d["failed"], "Error": ""}

    def _decide(self, pod: dict, node_names, reqs) -> dict:
        """Fit ``pod`` and, when a node fits, commit its allocation to the pod
        and quota caches (caller holds ``_decide_mu``)."""
        pi = self.pod_manager.take_and_delete_pod(pod)
        if pi:
            self.quota_manager.rm_usage(pod, pi.devices)
        if self.memoize:
            scores, failure, failed = self.score_candidates(list(node_names or []), pod, reqs)
        else:
            usage, _, failed = self.get_nodes_usage(node_names or [], pod)
            scores, failure = calc_score(usage, reqs, pod, failed, self.cfg.node_scheduler_policy)
        if not scores.node_list:
            return {"best": None, "failure": failure, "failed": failed}
        scores.sort()
        best = scores.node_list[-1]
        # memo entries are shared: hand the winner's allocation out as a copy
        best = type(best)(best.node_id, best.node, copy_pod_devices(best.devices), best.score)
        annos = {T.ASSIGNED_NODE_ANNOTATION: best.node_id, T.ASSIGNED_TIME_ANNOTATION: str(int(time.time()))}
        for dev in D.get_devices().values():
            dev.patch_annotations(pod, annos, best.devices)
        eff = collapse_init_container_usage(pod, best.devices)
        added = self.pod_manager.add_pod(pod, best.node_id, eff)
        if added:
            self.quota_manager.add_usage(pod, eff)
        return {"best": best, "scores": scores, "failed": failed, "annos": annos, "eff": eff, "added": added}

    def _filter_simulation(self, pod: dict, nodes, reqs) -> dict:
        items = nodes.get("items", []) if isinstance(nodes, dict) else list(nodes)
        usage, failed = self.get_simulation_nodes_usage(items, pod)
        scores, _ = calc_score(usage, reqs, pod, failed, self.cfg.node_scheduler_policy)
        if not scores.node_list:
            return {"FailedNodes": failed, "Nodes": None, "Error": ""}
        scores.sort()
        best = scores.node_list[-1].node_id
        chosen = [n for n in items if name_of(n) == best][:1]
        return {"Nodes": {"items": chosen}, "FailedNodes": failed, "Error": ""}
