"""Distributed per-node lock in the node annotation ``hami.io/mutex.lock``.

Semantics of pkg/util/nodelock/nodelock.go:39-318:
  * value ``<RFC3339 time>,<namespace>,<pod>`` (legacy: bare timestamp);
  * acquisition is a resourceVersion-guarded JSON merge patch, retried with
    exponential backoff (5 steps, 100 ms x2, jitter 0.5) on non-contention
    errors; a lost PATCH response is recognised by finding our own owner suffix;
  * expiry after ``HAMI_NODELOCK_EXPIRE`` (Go duration, default 5m);
  * re-entrant for the same pod; dangling owner (pod gone) is broken;
  * release only by the owner (unless ``skip_owner_check``), conflict-safe;
  * an in-process mutex per node serialises this process's own attempts.
"""

from __future__ import annotations

import datetime as _dt
import logging
import os
import random
import re
import threading
import time

from k8s_vgpu_scheduler_amd.k8s.client import get_client, is_not_found
from k8s_vgpu_scheduler_amd.utils.types import NODE_LOCK_KEY, NODE_LOCK_SEP

log = logging.getLogger(__name__)


class NodeLockContention(Exception):
    """The lock is held by another valid pod (retryable for PodGroup members)."""


class NodeLockError(Exception):
    pass


_DUR = re.compile(r"(\d+(?:\.\d+)?)(ns|us|µs|ms|s|m|h)")
_UNITS = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}


def parse_go_duration(s: str) -> float:
    s = s.strip()
    if not s:
        raise ValueError("empty duration")
    pos, total = 0, 0.0
    for m in _DUR.finditer(s):
        if m.start() != pos:
            raise ValueError(f"invalid duration {s!r}")
        total += float(m.group(1)) * _UNITS[m.group(2)]
        pos = m.end()
    if pos != len(s):
        raise ValueError(f"invalid duration {s!r}")
    return total


def _timeout_from_env() -> float:
    v = os.environ.get("HAMI_NODELOCK_EXPIRE")
    if v:
        try:
            return parse_go_duration(v)
        except ValueError:
            log.error("failed to parse HAMI_NODELOCK_EXPIRE=%r, using default", v)
    return 300.0


NODE_LOCK_TIMEOUT = _timeout_from_env()
BACKOFF_STEPS, BACKOFF_BASE, BACKOFF_FACTOR, BACKOFF_JITTER = 5, 0.1, 2.0, 0.5

_locks: dict[str, threading.Lock] = {}
_locks_mu = threading.Lock()


def _node_mutex(node: str) -> threading.Lock:
    with _locks_mu:
        return _locks.setdefault(node, threading.Lock())


def cleanup_node_lock(node: str):
    with _locks_mu:
        _locks.pop(node, None)


def _rfc3339(t: _dt.datetime | None = None) -> str:
    t = (t or _dt.datetime.now().astimezone()).replace(microsecond=0)
    s = t.isoformat()
    return s.replace("+00:00", "Z")


def _parse_rfc3339(s: str) -> _dt.datetime:
    s = s.strip()
    if s.endswith("Z"):
        s = s[:-1] + "+00:00"
    return _dt.datetime.fromisoformat(s)


def pod_ns_name(pod: dict | None, sep: str = NODE_LOCK_SEP) -> str:
    if not pod:
        return ""
    md = pod["metadata"]
    return f"{md.get('namespace', 'default')}{sep}{md['name']}"


def generate_lock_value(pod: dict | None) -> str:
    if pod is None:
        return _rfc3339()
    return f"{_rfc3339()}{NODE_LOCK_SEP}{pod_ns_name(pod)}"


def parse_node_lock(value: str) -> tuple[_dt.datetime, str, str]:
    if NODE_LOCK_SEP not in value:
        return _parse_rfc3339(value), "", ""
    parts = value.split(NODE_LOCK_SEP)
    if len(parts) != 3:
        raise NodeLockError(f"malformed lock annotation: expected 3 parts, got {len(parts)} from {value}")
    return _parse_rfc3339(parts[0]), parts[1], parts[2]


def _retry(fn, retry_on):
    delay = BACKOFF_BASE
    last = None
    for i in range(BACKOFF_STEPS):
        try:
            return fn()
        except Exception as e:  # noqa: BLE001
            last = e
            if not retry_on(e) or i == BACKOFF_STEPS - 1:
                raise
            time.sleep(delay * (1 + BACKOFF_JITTER * random.random()))
            delay *= BACKOFF_FACTOR
    raise last  # pragma: no cover


def set_node_lock(node_name: str, lockname: str, pod: dict):
    with _node_mutex(node_name):
        c = get_client()
        node = c.get_node(node_name)
        if NODE_LOCK_KEY in (node["metadata"].get("annotations") or {}):
            raise NodeLockContention(f"node {node_name} is locked")
        owner = NODE_LOCK_SEP + pod_ns_name(pod)

        def attempt():
            n = c.get_node(node_name)
            cur = (n["metadata"].get("annotations") or {}).get(NODE_LOCK_KEY)
            if cur is not None and NODE_LOCK_SEP in cur and cur.endswith(owner):
                return  # our earlier PATCH landed but its response was lost
            if cur is not None:
                raise NodeLockContention(f"node {node_name} is locked")
            c.patch_node(node_name, {"metadata": {"annotations": {NODE_LOCK_KEY: generate_lock_value(pod)},
                                                  "resourceVersion": n["metadata"]["resourceVersion"]}})

        try:
            _retry(attempt, lambda e: not isinstance(e, NodeLockContention))
        except NodeLockContention:
            raise
        except Exception as e:  # noqa: BLE001
            raise NodeLockError(f"failed to set node lock (node={node_name}): {e}") from e
        log.info("node lock set node=%s pod=%s", node_name, pod["metadata"]["name"])


def release_node_lock(node_name: str, lockname: str, pod: dict, skip_owner_check: bool = False):
    if pod is None:
        raise NodeLockError("cannot release node lock: pod is nil")
    with _node_mutex(node_name):
        c = get_client()
        node = c.get_node(node_name)
        lock_str = (node["metadata"].get("annotations") or {}).get(NODE_LOCK_KEY)
        if lock_str is None:
            return
        owner = NODE_LOCK_SEP + pod_ns_name(pod)
        if not skip_owner_check and NODE_LOCK_SEP in lock_str and not lock_str.endswith(owner):
            log.info("node lock %r is not held by pod %s", lock_str, pod["metadata"]["name"])
            return
        released = [False]

        def attempt():
            n = c.get_node(node_name)
            cur = (n["metadata"].get("annotations") or {}).get(NODE_LOCK_KEY)
            if cur is None:
                return
            if skip_owner_check or NODE_LOCK_SEP not in cur:
                if cur != lock_str:
                    return
            elif not cur.endswith(owner):
                return
            c.patch_node(node_name, {"metadata": {"annotations": {NODE_LOCK_KEY: None},
                                                  "resourceVersion": n["metadata"]["resourceVersion"]}})
            released[0] = True

        try:
            _retry(attempt, lambda e: True)
        except Exception as e:  # noqa: BLE001
            raise NodeLockError(f"failed to release node lock (node={node_name}): {e}") from e
        if released[0]:
            log.info("node lock released node=%s pod=%s", node_name, pod["metadata"]["name"])


def lock_node(node_name: str, lockname: str, pod: dict):
    c = get_client()
    node = c.get_node(node_name)
    annos = node["metadata"].get("annotations") or {}
    if NODE_LOCK_KEY not in annos:
        return set_node_lock(node_name, lockname, pod)
    lock_time, ns, prev = parse_node_lock(annos[NODE_LOCK_KEY])
    skip = False
    now = _dt.datetime.now(lock_time.tzinfo) if lock_time.tzinfo else _dt.datetime.now()
    md = pod["metadata"]
    if (now - lock_time).total_seconds() > NODE_LOCK_TIMEOUT:
        log.info("node lock expired node=%s lockTime=%s", node_name, lock_time)
        skip = True
    elif ns == md.get("namespace", "default") and prev == md["name"]:
        return  # re-entrant: a pod requesting several vendors locks once per vendor
    elif ns and prev:
        try:
            c.get_pod(ns, prev)
        except Exception as e:  # noqa: BLE001
            if not is_not_found(e):
                raise
            log.info("previous lock owner %s/%s not found, releasing", ns, prev)
            skip = True
    if skip:
        release_node_lock(node_name, lockname, pod, skip_owner_check=True)
        return set_node_lock(node_name, lockname, pod)
    raise NodeLockContention(f"node {node_name} has been locked within {NODE_LOCK_TIMEOUT}s")
