"""Scheduling trace as Kubernetes Events (pkg/scheduler/event.go:33-78)."""

from __future__ import annotations

import datetime as _dt
import logging

log = logging.getLogger(__name__)

FILTERING_FAILED = "FilteringFailed"
FILTERING_SUCCEED = "FilteringSucceed"
BINDING_FAILED = "BindingFailed"
BINDING_SUCCEED = "BindingSucceed"
COMPONENT = "hami-scheduler"


class EventRecorder:
    def __init__(self, client, component: str = COMPONENT):
        self.client, self.component = client, component
        self.recorded: list[tuple] = []   # (reason, type, message) for tests / debug

    def event(self, obj: dict, etype: str, reason: str, message: str):
        self.recorded.append((reason, etype, message))
        if self.client is None:
            return
        md = obj.get("metadata") or {}
        ts = _dt.datetime.now(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
        ev = {"metadata": {"generateName": f"{md.get('name', 'obj')}.", "namespace": md.get("namespace", "default")},
              "involvedObject": {"apiVersion": "v1", "kind": obj.get("kind", "Pod"), "name": md.get("name"),
                                 "namespace": md.get("namespace", "default"), "uid": md.get("uid", "")},
              "reason": reason, "message": message, "type": etype, "count": 1,
              "firstTimestamp": ts, "lastTimestamp": ts, "source": {"component": self.component}}
        try:
            self.client.create("events", ev, md.get("namespace", "default"))
        except Exception as e:  # noqa: BLE001 -- events are best effort
            log.debug("event create failed: %s", e)

    def filter_result(self, pod: dict, reason: str, msg: str, err: Exception | str | None):
        if err:
            self.event(pod, "Warning", reason, str(err))
        else:
            self.event(pod, "Normal", reason, msg)

    def binding_result(self, pod: dict, reason: str, nodes: list, err: Exception | str | None):
        if err:
            self.event(pod, "Warning", reason, str(err))
        else:
            self.event(pod, "Normal", reason, f"Successfully binding node {nodes} to {pod['metadata']['name']}")
