"""Passive leader election on the kube-scheduler Lease (pkg/util/leaderelection/leaderelection.go:35-209).

The extender does not run its own election: it watches the Lease that
kube-scheduler (running in the same pod) holds and is leader iff the lease's
``holderIdentity`` starts with this pod's hostname and the lease has not
expired.  ``DummyLeaderManager`` is used when election is disabled.
"""

from __future__ import annotations

import datetime as _dt
import logging
import threading

log = logging.getLogger(__name__)


def _parse_time(s: str | None) -> _dt.datetime | None:
    if not s:
        return None
    s = s.replace("Z", "+00:00")
    try:
        return _dt.datetime.fromisoformat(s)
    except ValueError:
        return None


class DummyLeaderManager:
    def __init__(self, is_leader: bool = True):
        self._leader = is_leader

    def is_leader(self) -> bool:
        return self._leader

    def on_lease(self, *a, **k):
        pass


class LeaderManager:
    def __init__(self, hostname: str, namespace: str, name: str, on_started=None, on_stopped=None):
        self.hostname, self.namespace, self.name = hostname, namespace, name
        self.on_started, self.on_stopped = on_started, on_stopped
        self._lease: dict | None = None
        self._was_leader = False
        self._mu = threading.Lock()

    def _valid(self, lease: dict, now: _dt.datetime) -> bool:
        spec = lease.get("spec") or {}
        holder = spec.get("holderIdentity") or ""
        if not holder.startswith(self.hostname):
            return False
        renew = _parse_time(spec.get("renewTime")) or _parse_time(spec.get("acquireTime"))
        dur = spec.get("leaseDurationSeconds") or 0
        if renew is None:
            return False
        if renew.tzinfo is None:
            renew = renew.replace(tzinfo=_dt.timezone.utc)
        return now <= renew + _dt.timedelta(seconds=int(dur))

    def is_leader(self, now: _dt.datetime | None = None) -> bool:
        now = now or _dt.datetime.now(_dt.timezone.utc)
        with self._mu:
            lease = self._lease
        return bool(lease) and self._valid(lease, now)

    def _update(self, lease: dict | None):
        with self._mu:
            self._lease = lease
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
