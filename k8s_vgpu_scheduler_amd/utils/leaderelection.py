"""Passive leader election on the kube-scheduler Lease (pkg/util/leaderelection/leaderelection.go:35-209).

The extender does not run its own election: it watches the Lease that
kube-scheduler (running in the same pod) holds and is leader iff the lease's
``holderIdentity`` starts with this pod's hostname and the lease has not
expired.  Expiry is judged on THIS process's clock -- the local monotonic time
the lease record was last observed to change plus ``leaseDurationSeconds``
(leaderelection.go:100-104,176-181) -- never on the server-written
``renewTime``, so a node whose wall clock is skewed against the API server can
neither keep serving as a stale leader nor refuse as a live one.
``DummyLeaderManager`` is used when election is disabled.
"""

from __future__ import annotations

import logging
import threading
import time

log = logging.getLogger(__name__)


class DummyLeaderManager:
    def __init__(self, is_leader: bool = True):
        self._leader = is_leader

    def is_leader(self) -> bool:
        return self._leader

    def on_lease(self, *a, **k):
        pass


class LeaderManager:
    def __init__(self, hostname: str, namespace: str, name: str, on_started=None, on_stopped=None,
                 clock=time.monotonic):
        self.hostname, self.namespace, self.name = hostname, namespace, name
        self.on_started, self.on_stopped = on_started, on_stopped
        self.clock = clock
        self._lease: dict | None = None
        self._observed = 0.0       # local clock when the lease record was last seen to change
        self._was_leader = False
        self._mu = threading.Lock()

    def _holder(self, lease: dict | None) -> bool:
        holder = ((lease or {}).get("spec") or {}).get("holderIdentity") or ""
        return bool(holder) and holder.startswith(self.hostname)

    def is_leader(self, now: float | None = None) -> bool:
        """``now``: local monotonic seconds (default: the clock now)."""
        now = self.clock() if now is None else now
        with self._mu:
            lease, seen = self._lease, self._observed
        if not lease or not self._holder(lease):
            return False
        dur = (lease.get("spec") or {}).get("leaseDurationSeconds")
        if not dur:
            return False
        return now < seen + int(dur)

    def _update(self, lease: dict | None):
        with self._mu:
            prev = self._lease
            self._lease = lease
            # a record that changed (a renewal bumps renewTime / resourceVersion)
            # restarts the local expiry window; a resync of the same record does not
            if lease is None:
                self._observed = 0.0
            elif prev is None or _record(prev) != _record(lease):
                self._observed = self.clock()
        leader = self.is_leader()
        if leader and not self._was_leader and self.on_started:
            self.on_started()
        if not leader and self._was_leader and self.on_stopped:
            self.on_stopped()
        self._was_leader = leader

    # informer handlers
    def on_add(self, lease: dict):
        if self._mine(lease):
            self._update(lease)

    def on_update(self, old: dict, new: dict):
        if self._mine(new):
            self._update(new)

    def on_delete(self, lease: dict):
        if self._mine(lease):
            self._update(None)

    def _mine(self, lease: dict) -> bool:
        md = lease.get("metadata") or {}
        return md.get("name") == self.name and md.get("namespace", self.namespace) == self.namespace


def _record(lease: dict) -> tuple:
    spec = lease.get("spec") or {}
    md = lease.get("metadata") or {}
    return (spec.get("holderIdentity"), spec.get("renewTime"), spec.get("acquireTime"),
            spec.get("leaseTransitions"), md.get("resourceVersion"))
