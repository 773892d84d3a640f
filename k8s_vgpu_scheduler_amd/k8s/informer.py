"""Shared informer + lister over :class:`KubeClient` watches.

Equivalent of the client-go SharedInformerFactory the reference scheduler
builds in pkg/scheduler/scheduler.go:355-407: an initial LIST populates a
thread-safe cache (the lister), then watch events keep it current and fan
out to registered add/update/delete handlers.  Handlers receive deep copies,
matching the reference's deep-copy discipline (nodes.go:71-106).
"""

from __future__ import annotations

import logging
import threading
from typing import Callable, Optional

from k8s_vgpu_scheduler_amd.utils.jcopy import jcopy

from .client import KubeClient, NAMESPACED, match_labels

log = logging.getLogger(__name__)


class Informer:
    def __init__(self, client: KubeClient, kind: str, namespace: str | None = None,
                 field_selector: dict | None = None):
        """``field_selector`` scopes the cache server-side, e.g. the node agents'
        ``{"spec.nodeName": node}`` (pkg/monitor/nvidia/cudevshr.go:308)."""
        self.client, self.kind, self.namespace = client, kind, namespace
        self.field_selector = field_selector
        self._cache: dict[tuple, dict] = {}
        self._mu = threading.RLock()
        self._handlers: list[tuple] = []
        self._synced = False
        self._stop: Optional[Callable] = None

    def add_event_handler(self, on_add=None, on_update=None, on_delete=None):
        self._handlers.append((on_add, on_update, on_delete))
        # Late registration sees the current state as adds (client-go semantics).
        if self._synced and on_add:
            for o in self.list():
                on_add(o)

    def _key(self, obj):
        md = obj.get("metadata") or {}
        return (md.get("namespace") if self.kind in NAMESPACED else "", md.get("name"))

    def _dispatch(self, etype, obj, old):
        key = self._key(obj)
        with self._mu:
            prev = self._cache.get(key)
            if etype == "DELETED":
                self._cache.pop(key, None)
            else:
                self._cache[key] = obj
        for on_add, on_update, on_delete in self._handlers:
            try:
                if etype == "ADDED" and on_add:
                    on_add(jcopy(obj))
                elif etype == "MODIFIED":
                    if prev is None and on_add:
                        on_add(jcopy(obj))
                    elif on_update:
                        on_update(jcopy(prev if prev is not None else old), jcopy(obj))
                elif etype == "DELETED" and on_delete:
                    on_delete(jcopy(prev or obj))
            except Exception:
                log.exception("%s informer handler failed", self.kind)

    def start(self):
        if self._stop:
            return
        # Subscribe first, then list, so no event between the two is lost.
        if self.field_selector:
            self._stop = self.client.watch(self.kind, self._dispatch, self.namespace,
                                           field_selector=self.field_selector)
            listed = self.client.list(self.kind, self.namespace, field_selector=self.field_selector)
        else:
            self._stop = self.client.watch(self.kind, self._dispatch, self.namespace)
            listed = self.client.list(self.kind, self.namespace)
        for o in listed:
            key = self._key(o)
            with self._mu:
                known = key in self._cache
            if not known:
                self._dispatch("ADDED", o, None)
        self._synced = True

    def stop(self):
        if self._stop:
            self._stop()
            self._stop = None

    def has_synced(self) -> bool:
        return self._synced

    # --------------------------------------------------------------- lister
    def get(self, name: str, namespace: str | None = None) -> dict | None:
        with self._mu:
            o = self._cache.get((namespace if self.kind in NAMESPACED else "", name))
            return jcopy(o) if o is not None else None

    def list(self, label_selector: dict | None = None, namespace: str | None = None) -> list[dict]:
        with self._mu:
            items = list(self._cache.items())
        return [jcopy(o) for (ns, _), o in items
                if (namespace is None or ns == namespace) and match_labels(o, label_selector)]
