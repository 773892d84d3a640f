"""Escalation for containers that stay over their HBM grant.

A block verdict parks a container's launches through its read-only control
file (monitor/control.py), but a container whose shim is not loaded has no
launches to park, and a blocked tenant still holds the HBM it took.  So the
monitor's ``--over-grant-action`` decides what happens once a container has
been over its grant for ``--over-grant-passes`` consecutive passes:

* ``block`` (default) -- the block verdict only (the reference's behaviour: the
  monitor blocks through the shared region, cmd/vGPUmonitor/feedback.go:74-134);
* ``evict`` -- the pod is evicted through the Eviction API (policy/v1, so
  PodDisruptionBudgets are honoured), once, with a ``VGPUOverGrantEvicted``
  Warning event;
* ``kill`` -- SIGKILL to the pod's host processes that hold VRAM on the
  device (KFD's view), with a ``VGPUOverGrantKilled`` Warning event; again
  every pass the container stays over.

Counts reset as soon as a pass finds the container back under its grant.

A container with NO live shim is a different case: a block verdict cannot
reach it (only the shim reads the control file).  Once it has held VRAM
without a shim for ``passes`` consecutive passes AND is over its HBM grant
or sits on a GPU that only the governor limits (a fractional core limit with
no CU mask, the ``cuPartition: false`` time-sharing mode: nothing bounds its
compute), it is evicted (``shimless_action``, default ``evict``; ``kill``
under ``--over-grant-action kill``) whatever ``action`` is -- the reference
kills such processes from its monitor when they exceed their limit
(pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:866-884 mounts
the tools for it).

Kill lists: a container over its grant through its OWN processes loses those;
a pod over its grant only through processes outside every container's slots
(a hidden process) loses exactly those hidden processes, not the compliant
containers' (ADVICE r4).
"""

from __future__ import annotations

import logging
import os
import signal
import threading
from typing import Callable

log = logging.getLogger(__name__)

ACTIONS = ("block", "evict", "kill")
SHIMLESS_ACTIONS = ("none", "evict", "kill")
EVICTED_REASON = "VGPUOverGrantEvicted"
KILLED_REASON = "VGPUOverGrantKilled"
SHIMLESS_EVICTED_REASON = "VGPUShimlessEvicted"


class OverGrantPolicy:
    """``client``: KubeClient (``evict``) for ``evict``; ``kill``: callable
    ``(pid, sig)`` for ``kill`` (``os.kill`` by default); ``events``:
    EventRecorder-like; ``pod_info``: ``pod_uid -> pod dict``."""

    def __init__(self, action: str = "block", passes: int = 3, client=None, events=None,
                 kill: Callable[[int, int], None] | None = None, shimless_action: str | None = None):
        if action not in ACTIONS:
            raise ValueError(f"over-grant action {action!r} not in {ACTIONS}")
        if shimless_action is None:
            shimless_action = "kill" if action == "kill" else "evict"
        if shimless_action not in SHIMLESS_ACTIONS:
            raise ValueError(f"shimless action {shimless_action!r} not in {SHIMLESS_ACTIONS}")
        self.action = action
        self.shimless_action = shimless_action
        self.shimless: dict[tuple, int] = {}   # (pod_uid, container) -> consecutive passes without a live shim
        self.passes = max(1, int(passes))
        self.client = client
        self.events = events
        self._kill = kill or os.kill
        self._mu = threading.Lock()
        self.count: dict[tuple, int] = {}      # (pod_uid, container) -> consecutive passes over
        self.evicted: set[str] = set()         # pod uids an eviction was issued for
        self.actions: dict[str, int] = {a: 0 for a in ACTIONS}

    def step(self, verdicts: dict, pod_info: Callable | None = None) -> list[tuple]:
        """One pass.  ``verdicts``: ``HostTruth.enforce``'s result.  Returns
        the actions taken: ``[(action, pod_uid, container, detail)]``."""
        taken = []
        with self._mu:
            over = {k for k, v in verdicts.items() if v.over}
            self.count = {k: self.count.get(k, 0) + 1 for k in over}
            due = [k for k, n in self.count.items() if n >= self.passes]
            loose = {k for k, v in verdicts.items() if getattr(v, "no_live_shim", False)}
            self.shimless = {k: self.shimless.get(k, 0) + 1 for k in loose}
            shimless_due = [k for k, n in self.shimless.items()
                            if n >= self.passes and (verdicts[k].over or getattr(verdicts[k], "ungoverned", False))]
        # no live shim: a block verdict cannot reach the container
        if self.shimless_action != "none":
            for key in shimless_due:
                v = verdicts[key]
                why = ("over its HBM grant" if v.over else
                       "on a time-shared GPU with no governor (nothing limits its compute)")
                msg = f"container {key[1]} held VRAM without libmivgpu.so for {self.shimless[key]} passes, {why}"
                if self.shimless_action == "evict":
                    self._evict(key, pod_info, taken, SHIMLESS_EVICTED_REASON, msg + ": pod evicted")
                else:
                    self._kill_pids(key, sorted({p for ps in v.pids.values() for p in ps} | set(v.hidden)),
                                    pod_info, taken, msg)
        if self.action == "block":
            return taken
        for key in due:
            if key in shimless_due and self.shimless_action != "none":
                continue        # handled above
            uid, ctr = key
            if self.action == "evict":
                self._evict(key, pod_info, taken, EVICTED_REASON,
                            f"container {ctr} stayed over its HBM grant for {self.count[key]} passes: pod evicted")
            else:
                v = verdicts[key]
                # its own processes when they hold the excess; the pod's
                # hidden processes when only those put the pod over
                pids = sorted({p for ps in v.pids.values() for p in ps}) if v.own_over or not v.pod_over else []
                pids = sorted(set(pids) | (set(v.hidden) if v.pod_over else set()))
                self._kill_pids(key, pids, pod_info, taken,
                                f"container {ctr} stayed over its HBM grant for {self.count[key]} passes")
        return taken

    def _evict(self, key, pod_info, taken, reason, msg):
        uid, ctr = key
        pod = pod_info(uid) if pod_info is not None else None
        md = (pod or {}).get("metadata") or {}
        name, ns = md.get("name"), md.get("namespace") or "default"
        if uid in self.evicted or not name or self.client is None:
            return
        try:
            self.client.evict(ns, name)
        except Exception as e:  # noqa: BLE001  (a PDB may refuse: retried next pass)
            log.warning("evicting %s/%s failed: %s", ns, name, e)
            return
        self.evicted.add(uid)
        self.actions["evict"] += 1
        taken.append(("evict", uid, ctr, f"{ns}/{name}"))
        self._event(pod, uid, ns, name, reason, msg)

    def _kill_pids(self, key, pids, pod_info, taken, msg):
        uid, ctr = key
        pod = pod_info(uid) if pod_info is not None else None
        md = (pod or {}).get("metadata") or {}
        name, ns = md.get("name"), md.get("namespace") or "default"
        killed = []
        for pid in pids:
            try:
                self._kill(pid, signal.SIGKILL)
                killed.append(pid)
            except ProcessLookupError:
                pass
            except OSError as e:
                log.warning("kill %d (%s/%s) failed: %s", pid, uid, ctr, e)
        if killed:
            self.actions["kill"] += 1
            taken.append(("kill", uid, ctr, killed))
            self._event(pod, uid, ns, name or uid, KILLED_REASON, f"{msg}: killed host pids {killed}")

    def _event(self, pod, uid, ns, name, reason, msg):
        log.warning("%s/%s: %s", ns, name, msg)
        if self.events is not None:
            self.events.event({"kind": "Pod", "metadata": {"name": name, "namespace": ns, "uid": uid}},
                              "Warning", reason, msg)


__all__ = ["OverGrantPolicy", "ACTIONS", "SHIMLESS_ACTIONS", "EVICTED_REASON", "KILLED_REASON",
           "SHIMLESS_EVICTED_REASON"]
