"""Namespace ResourceQuota mirror for device memory / cores (pkg/device/quota.go:27-329).

Tracks ``limits.<memory resource>`` and ``limits.<core resource>`` hard limits
per namespace plus the usage of scheduled pods.  ``limit_set`` distinguishes an
explicit limit (including an explicit 0 = block everything) from an entry
created only by usage tracking.  ``update_quota`` swaps limits under one lock
so a check can never observe the zeroed gap between delete and add.
"""

from __future__ import annotations

import logging
import threading
from dataclasses import dataclass

from k8s_vgpu_scheduler_amd.k8s import quantity

from . import devices as D

log = logging.getLogger(__name__)


@dataclass
class Quota:
    used: int = 0
    limit: int = 0
    limit_set: bool = False


class QuotaManager:
    def __init__(self):
        self.quotas: dict[str, dict[str, Quota]] = {}
        self._mu = threading.RLock()

    def fit_quota(self, ns: str, memreq: int, memory_factor: int, coresreq: int, device_name: str) -> bool:
        dev = D.get_devices().get(device_name)
        if dev is None:
            return True
        names = dev.get_resource_names()
        with self._mu:
            dq = self.quotas.get(ns)
            if not dq:
                return True
            mq = dq.get(names.memory)
            if mq is not None:
                limit = mq.limit * memory_factor if memory_factor > 1 else mq.limit
                if mq.limit_set and mq.used + memreq > limit:
                    return False
            cq = dq.get(names.core)
            if cq is not None and cq.limit_set and cq.used + coresreq > cq.limit:
                return False
        return True

    def fit_key(self, ns: str) -> tuple:
        """Everything ``fit_quota`` reads for ``ns``: () when the namespace has
        no explicit limit (every fit passes), else the limited entries.  A
        Filter result computed under one key is valid under an equal key."""
        with self._mu:
            dq = self.quotas.get(ns)
            if not dq:
                return ()
            return tuple(sorted((k, q.used, q.limit) for k, q in dq.items() if q.limit_set))

    @staticmethod
    def _count(pd: dict) -> dict[str, int]:
        res: dict[str, int] = {}
        for dev_name, single in (pd or {}).items():
            dev = D.get_devices().get(dev_name)
            if dev is None:
                continue
            names = dev.get_resource_names()
            # Backends whose allocation unit differs from the quota unit (AMD:
            # CUs allocated, % in the ResourceQuota) convert per device.
            core_units = getattr(dev, "quota_cores", None) or (lambda d: d.usedcores)
            for ctr in single:
                for d in ctr:
                    if names.memory:
                        res[names.memory] = res.get(names.memory, 0) + d.usedmem
                    if names.core:
                        res[names.core] = res.get(names.core, 0) + core_units(d)
        return res

    def _add_locked(self, ns, usage):
        dq = self.quotas.setdefault(ns, {})
        for k, v in usage.items():
            dq.setdefault(k, Quota()).used += v

    def _rm_locked(self, ns, usage):
        dq = self.quotas.get(ns)
        if dq is None:
            return
        for k, v in usage.items():
            q = dq.get(k)
            if q is not None:
                q.used = max(0, q.used - v)

    def add_usage(self, pod: dict, pd: dict):
        usage = self._count(pd)
        if usage:
            with self._mu:
                self._add_locked(pod["metadata"].get("namespace", "default"), usage)

    def rm_usage(self, pod: dict, pd: dict):
        usage = self._count(pd)
        if usage:
            with self._mu:
                self._rm_locked(pod["metadata"].get("namespace", "default"), usage)

    def replace_usage(self, pod: dict, old: dict, new: dict):
        o, n = self._count(old), self._count(new)
        if not o and not n:
            return
        ns = pod["metadata"].get("namespace", "default")
        with self._mu:
            self._rm_locked(ns, o)
            self._add_locked(ns, n)

    @staticmethod
    def is_managed_quota(name: str) -> bool:
        for dev in D.get_devices().values():
            n = dev.get_resource_names()
            if (n.memory and n.memory == name) or (n.core and n.core == name):
                return True
        return False

    @classmethod
    def _managed_name(cls, key: str):
        if not key.startswith("limits."):
            return None
        dn = key[len("limits."):]
        return dn if cls.is_managed_quota(dn) else None

    def _add_quota_locked(self, rq: dict):
        ns = rq["metadata"].get("namespace", "default")
        for key, val in ((rq.get("spec") or {}).get("hard") or {}).items():
            v, ok = quantity.as_int64(val)
            dn = self._managed_name(key)
            if not ok or dn is None:
                continue
            q = self.quotas.setdefault(ns, {}).setdefault(dn, Quota())
            q.limit, q.limit_set = v, True

    def _del_quota_locked(self, rq: dict):
        ns = rq["metadata"].get("namespace", "default")
        for key, val in ((rq.get("spec") or {}).get("hard") or {}).items():
            _, ok = quantity.as_int64(val)
            dn = self._managed_name(key)
            if not ok or dn is None:
                continue
            q = self.quotas.get(ns, {}).get(dn)
            if q is not None:
                q.limit, q.limit_set = 0, False

    def add_quota(self, rq: dict):
        with self._mu:
            self._add_quota_locked(rq)

    def del_quota(self, rq: dict):
        with self._mu:
            self._del_quota_locked(rq)

    def update_quota(self, old: dict | None, new: dict | None):
        with self._mu:
            if old:
                self._del_quota_locked(old)
            if new:
                self._add_quota_locked(new)

    def get_resource_quota(self) -> dict[str, dict[str, Quota]]:
        with self._mu:
            return {ns: {k: Quota(q.used, q.limit, q.limit_set) for k, q in dq.items()}
                    for ns, dq in self.quotas.items()}


_LOCAL = QuotaManager()


def get_local_cache() -> QuotaManager:
    """Process-wide singleton (quota.go:40-55: webhook and scheduler share it)."""
    return _LOCAL
