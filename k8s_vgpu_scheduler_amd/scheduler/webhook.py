"""Mutating admission webhook (pkg/scheduler/webhook.go:53-192).

Order of checks (kept from the reference):
  1. deny pods without containers;
  2. pods already owned by another scheduler are allowed untouched (unless
     --force-overwrite-default-scheduler and they use default-scheduler);
  3. every backend's MutateAdmission over init then app containers (validation
     errors -> 500 with the message, as the reference returns Errored);
  4. privileged container + device request -> denied;
  5. set schedulerName; deny if spec.nodeName is pre-set;
  6. quota pre-check with effective = max(sum(app), max(init));
  7. respond with an RFC 6902 JSON patch of the mutations.
"""

from __future__ import annotations

import base64
import json
import logging

from k8s_vgpu_scheduler_amd.device import devices as D
from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.utils.jcopy import jcopy

log = logging.getLogger(__name__)


def _esc(k: str) -> str:
    return k.replace("~", "~0").replace("/", "~1")


def json_patch(a, b, path: str = "") -> list[dict]:
    """Minimal RFC 6902 diff a -> b (dicts recursive, equal-length lists per item)."""
    if a == b:
        return []
    if isinstance(a, dict) and isinstance(b, dict):
        ops = []
        for k in a:
            if k not in b:
                ops.append({"op": "remove", "path": f"{path}/{_esc(k)}"})
        for k, v in b.items():
            p = f"{path}/{_esc(k)}"
            if k not in a:
                ops.append({"op": "add", "path": p, "value": v})
            else:
                ops.extend(json_patch(a[k], v, p))
        return ops
    if isinstance(a, list) and isinstance(b, list) and len(a) == len(b):
        ops = []
        for i, (x, y) in enumerate(zip(a, b)):
            ops.extend(json_patch(x, y, f"{path}/{i}"))
        return ops
    return [{"op": "replace", "path": path or "/", "value": b}]


def _privileged(pod: dict) -> str | None:
    spec = pod.get("spec") or {}
    for c in (spec.get("initContainers") or []) + (spec.get("containers") or []):
        if ((c.get("securityContext") or {}).get("privileged")) is True:
            return c.get("name", "")
    return None


def fit_resource_quota(pod: dict) -> bool:
    ns = (pod.get("metadata") or {}).get("namespace", "default")
    spec = pod.get("spec") or {}
    for name, dev in D.get_devices().items():
        rn = dev.get_resource_names()
        if not rn.memory and not rn.core:
            continue
        app_mem = app_core = init_mem = init_core = 0
        for c in spec.get("containers") or []:
            r = dev.generate_resource_requests(c)
            if r.nums:
                app_mem += r.memreq * r.nums
                app_core += r.coresreq * r.nums
        for c in spec.get("initContainers") or []:
            r = dev.generate_resource_requests(c)
            if r.nums:
                init_mem = max(init_mem, r.memreq * r.nums)
                init_core = max(init_core, r.coresreq * r.nums)
        mem, core = max(app_mem, init_mem), max(app_core, init_core)
        if mem == 0 and core == 0:
            continue
        if not get_local_cache().fit_quota(ns, mem, rn.memory_factor, core, name):
            return False
    return True


class Webhook:
    def __init__(self, scheduler_name: str = "", force_overwrite_default_scheduler: bool = True):
        self.scheduler_name = scheduler_name
        self.force_overwrite = force_overwrite_default_scheduler

    def admit(self, pod: dict) -> tuple[bool, str, dict | None, int]:
        """-> (allowed, message, mutated_pod_or_None, http_code_for_errors)"""
        pod = jcopy(pod)
        spec = pod.setdefault("spec", {})
        if not spec.get("containers"):
            return False, "pod has no containers", None, 403
        sn = spec.get("schedulerName", "")
        if sn and (sn != "default-scheduler" or not self.force_overwrite) and \
                (not self.scheduler_name or sn != self.scheduler_name):
            return True, "pod already has different scheduler assigned", None, 200
        has = False
        for c in (spec.get("initContainers") or []) + spec["containers"]:
            for dev in D.get_devices().values():
                try:
                    has = dev.mutate_admission(c, pod) or has
                except D.AdmissionError as e:
                    return False, str(e), None, 500
        priv = _privileged(pod)
        if priv is not None and has:
            return False, f"container {priv} is privileged", None, 403
        if has and self.scheduler_name:
            spec["schedulerName"] = self.scheduler_name
            if spec.get("nodeName"):
                return False, "pod has node assigned", None, 403
        if not fit_resource_quota(pod):
            return False, "exceeding resource quota", None, 403
        return True, "", pod, 200

    def handle_review(self, review: dict) -> dict:
        req = review.get("request") or {}
        uid = req.get("uid", "")
        pod = req.get("object") or {}
        resp: dict = {"uid": uid}
        try:
            allowed, msg, mutated, code = self.admit(pod)
        except Exception as e:  # noqa: BLE001
            log.exception("webhook failure")
            allowed, msg, mutated, code = False, str(e), None, 500
        resp["allowed"] = allowed
        if msg:
            resp["status"] = {"message": msg, "code": code}
        if allowed and mutated is not None:
            ops = json_patch(pod, mutated)
            if ops:
                resp["patchType"] = "JSONPatch"
                resp["patch"] = base64.b64encode(json.dumps(ops).encode()).decode()
        return {"apiVersion": review.get("apiVersion", "admission.k8s.io/v1"), "kind": "AdmissionReview",
                "response": resp}
