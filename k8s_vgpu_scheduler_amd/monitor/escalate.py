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
"""

from __future__ import annotations

import logging
import os
import signal
import threading
from typing import Callable

log = logging.getLogger(__name__)

ACTIONS = ("block", "evict", "kill")
EVICTED_REASON = "VGPUOverGrantEvicted"
KILLED_REASON = "VGPUOverGrantKilled"


class OverGrantPolicy:
    """``client``: KubeClient (``evict``) for ``evict``; ``kill``: callable
    ``(pid, sig)`` for ``kill`` (``os.kill`` by default); ``events``:
    EventRecorder-like; ``pod_info``: ``pod_uid -> pod dict``."""

    def __init__(self, action: str = "block", passes: int = 3, client=None, events=None,
                 kill: Callable[[int, int], None] | None = None):
        if action not in ACTIONS:
            raise ValueError(f"over-grant action {action!r} not in {ACTIONS}")
        self.action = action
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
        if self.action == "block":
            return taken
        for key in due:
            uid, ctr = key
            pod = pod_info(uid) if pod_info is not None else None
            md = (pod or {}).get("metadata") or {}
            name, ns = md.get("name"), md.get("namespace") or "default"
            if self.action == "evict":
                if uid in self.evicted or not name or self.client is None:
                    continue
                try:
                    self.client.evict(ns, name)
                except Exception as e:  # noqa: BLE001  (a PDB may refuse: retried next pass)
                    log.warning("evicting %s/%s (over its HBM grant) failed: %s", ns, name, e)
                    continue
                self.evicted.add(uid)
                self.actions["evict"] += 1
                taken.append(("evict", uid, ctr, f"{ns}/{name}"))
                self._event(pod, uid, ns, name, EVICTED_REASON,
                            f"container {ctr} stayed over its HBM grant for {self.count[key]} passes: pod evicted")
            else:
                pids = sorted({p for ps in verdicts[key].pids.values() for p in ps})
                killed = []
                for pid in pids:
                    try:
                        self._kill(pid, signal.SIGKILL)
                        killed.append(pid)
                    except ProcessLookupError:
                        pass
                    except OSError as e:
                        log.warning("kill %d (%s/%s over its HBM grant) failed: %s", pid, uid, ctr, e)
                if killed:
                    self.actions["kill"] += 1
                    taken.append(("kill", uid, ctr, killed))
                    self._event(pod, uid, ns, name or uid, KILLED_REASON,
                                f"container {ctr} stayed over its HBM grant for {self.count[key]} passes: "
                                f"killed host pids {killed}")
        return taken

    def _event(self, pod, uid, ns, name, reason, msg):
        log.warning("%s/%s: %s", ns, name, msg)
        if self.events is not None:
            self.events.event({"kind": "Pod", "metadata": {"name": name, "namespace": ns, "uid": uid}},
                              "Warning", reason, msg)


__all__ = ["OverGrantPolicy", "ACTIONS", "EVICTED_REASON", "KILLED_REASON"]
