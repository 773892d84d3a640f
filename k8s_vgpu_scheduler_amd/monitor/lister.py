"""Discover and map every container's shared region on this node.

Reference: pkg/monitor/nvidia/cudevshr.go:45-331 (``ContainerLister``): scan
``$HOOK_PATH/vgpu/containers/<podUID>_<container>/``, mmap the single
``*.cache`` file, and garbage-collect directories of pods that no longer
exist after ``HAMI_RESYNC_INTERVAL`` (default 5 m).  The pod list comes from
a node-scoped informer (or any callable returning pods).
"""

from __future__ import annotations

import logging
import os
import shutil
import threading
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Callable

from k8s_vgpu_scheduler_amd.utils.nodelock import parse_go_duration

from .control import ControlSet
from .region import SharedRegion

log = logging.getLogger(__name__)


@dataclass
class ContainerUsage:
    pod_uid: str
    container: str
    path: str
    region: SharedRegion
    namespace: str = ""
    pod_name: str = ""
    mtime: float = 0.0


def _resync_interval() -> float:
    v = os.environ.get("HAMI_RESYNC_INTERVAL")
    if v:
        try:
            return parse_go_duration(v)
        except ValueError:
            log.error("bad HAMI_RESYNC_INTERVAL=%r", v)
    return 300.0


class ContainerLister:
    def __init__(self, hook_path: str | None = None, pods: Callable[[], list[dict]] | None = None,
                 resync_interval: float | None = None):
        hook = hook_path or os.environ.get("HOOK_PATH", "/usr/local/vgpu")
        self.base = Path(hook) / "vgpu" / "containers"
        self.pods = pods
        self.resync = _resync_interval() if resync_interval is None else resync_interval
        self.containers: dict[str, ContainerUsage] = {}
        self._mu = threading.Lock()
        self._last_gc = 0.0
        self._pods: dict[str, dict] = {}
        # the host-owned control files next to the regions (monitor/control.py)
        self.controls = ControlSet(str(self.base.parent / "control"))

    def pod(self, uid: str) -> dict | None:
        """The pod with ``uid`` as of the last ``update()`` (None if unknown)."""
        with self._mu:
            return self._pods.get(uid)

    def _pod_index(self) -> dict[str, dict] | None:
        if self.pods is None:
            return None
        try:
            return {(p.get("metadata") or {}).get("uid", ""): p for p in self.pods()}
        except Exception as e:  # noqa: BLE001
            log.warning("pod listing failed: %s", e)
            return None

    def update(self):
        pods = self._pod_index()
        if pods is not None:
            with self._mu:
                self._pods = pods
        if not self.base.exists():
            return
        now = time.time()
        seen = set()
        for d in self.base.iterdir():
            if not d.is_dir() or "_" not in d.name:
                continue
            uid, ctr = d.name.split("_", 1)
            seen.add(d.name)
            pod = pods.get(uid) if pods is not None else None
            if pods is not None and pod is None:
                # pod is gone: drop the mapping now, remove the directory after the resync interval
                with self._mu:
                    cu = self.containers.pop(d.name, None)
                if cu:
                    cu.region.close()
                try:
                    age = now - d.stat().st_mtime
                except OSError:
                    continue
                if age > self.resync:
                    log.info("removing stale container dir %s", d)
                    shutil.rmtree(d, ignore_errors=True)
                    # the container's grant and control files (deviceplugin/allocate.py)
                    for f in (self.base.parent / "limits" / f"{d.name}.conf",
                              self.base.parent / "control" / f"{d.name}.ctl"):
                        try:
                            f.unlink()
                        except OSError:
                            pass
                    # its share-board flags directory (deviceplugin/allocate.py)
                    shutil.rmtree(self.base.parent / "board" / "flags" / d.name, ignore_errors=True)
                continue
            with self._mu:
                known = d.name in self.containers
            if known:
                continue
            caches = sorted(d.glob("*.cache"))
            if not caches:
                continue
            try:
                region = SharedRegion(str(caches[0]))
            except (OSError, ValueError) as e:
                log.debug("skipping %s: %s", caches[0], e)
                continue
            md = (pod or {}).get("metadata") or {}
            cu = ContainerUsage(uid, ctr, str(caches[0]), region, md.get("namespace", ""), md.get("name", ""),
                                caches[0].stat().st_mtime)
            with self._mu:
                self.containers[d.name] = cu
        with self._mu:
            for k in [k for k in self.containers if k not in seen]:
                self.containers.pop(k).region.close()

    def list_containers(self) -> list[ContainerUsage]:
        with self._mu:
            return list(self.containers.values())
