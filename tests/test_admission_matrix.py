"""Table-driven admission and quota matrix (the reference's webhook_test.go
quota tables and mutation cases, re-cast for amd.com resources).

Each case sets the namespace ResourceQuota (``limits.amd.com/gpumem`` /
``limits.amd.com/gpucores``, optionally pre-used), sends one pod through the
mutating webhook and checks allowed / denied with the message, and the
mutations (scheduler name, exclusive-core default, priority env).
"""

from __future__ import annotations

import base64
import json
from dataclasses import dataclass, field

import pytest

from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
from k8s_vgpu_scheduler_amd.scheduler.config import init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.webhook import Webhook
from k8s_vgpu_scheduler_amd.testing import amd_container, amd_pod

QUOTA_EXCEEDED = "exceeding resource quota"


@dataclass
class Case:
    name: str
    pod: dict                               # amd_pod kwargs
    allowed: bool = True
    message: str | None = None
    quota: dict | None = None               # ResourceQuota spec.hard
    namespace: str = "default"
    check: object = None                    # fn(patch ops) -> bool
    privileged: bool = False
    node_name: str | None = None
    scheduler_name: str | None = None


def c(**kw):
    return amd_container(**kw)


def has_env(ops, name, value):
    for o in ops:
        v = o.get("value")
        items = v if isinstance(v, list) else [v]
        for it in items:
            if isinstance(it, dict) and it.get("name") == name and it.get("value") == value:
                return True
    return False


def sets(ops, suffix, value):
    return any(o["path"].endswith(suffix) and o.get("value") == value for o in ops)


CASES = [
    # ------------------------------------------------------------- quota
    Case("memory within quota", dict(mem=1000), quota={"limits.amd.com/gpumem": "2000"}),
    Case("memory over quota", dict(mem=3000), False, QUOTA_EXCEEDED, quota={"limits.amd.com/gpumem": "2000"}),
    Case("multiple GPUs: memory counted per GPU", dict(gpu=2, mem=1500), False, QUOTA_EXCEEDED,
         quota={"limits.amd.com/gpumem": "2000"}),
    Case("multiple GPUs within quota", dict(gpu=2, mem=900), quota={"limits.amd.com/gpumem": "2000"}),
    Case("cores within quota", dict(mem=100, cores=25), quota={"limits.amd.com/gpucores": "50"}),
    Case("cores over quota", dict(mem=100, cores=75), False, QUOTA_EXCEEDED,
         quota={"limits.amd.com/gpucores": "50"}),
    Case("cores per GPU x GPUs over quota", dict(gpu=2, mem=100, cores=30), False, QUOTA_EXCEEDED,
         quota={"limits.amd.com/gpucores": "50"}),
    Case("init containers run sequentially: the max init fits, the sum would not",
         dict(containers=[c(name="a", mem=200), c(name="b", mem=200)],
              init=[c(name="i1", mem=350), c(name="i2", mem=350)]), quota={"limits.amd.com/gpumem": "500"}),
    Case("an init container exceeds the quota on its own",
         dict(containers=[c(name="a", mem=100)], init=[c(name="i", mem=600)]), False, QUOTA_EXCEEDED,
         quota={"limits.amd.com/gpumem": "500"}),
    Case("app containers sum over the quota", dict(containers=[c(name="a", mem=300), c(name="b", mem=300)]),
         False, QUOTA_EXCEEDED, quota={"limits.amd.com/gpumem": "500"}),
    Case("namespace without a quota", dict(mem=10 ** 6), namespace="free", quota={"limits.amd.com/gpumem": "1"}),
    Case("pod without an amd request ignores the quota", dict(containers=[c(gpu=None)]),
         quota={"limits.amd.com/gpumem": "1"}),
    Case("quota of zero blocks any request", dict(mem=1), False, QUOTA_EXCEEDED,
         quota={"limits.amd.com/gpumem": "0"}),
    # ---------------------------------------------------------- mutations
    Case("scheduler name set for an amd pod", dict(mem=1000),
         check=lambda ops: sets(ops, "/schedulerName", "hami-scheduler")),
    Case("no gpucores on a whole-card request: exclusive 100 filled in", dict(gpu=1),
         check=lambda ops: sets(ops, "amd.com~1gpucores", "100")),
    Case("explicit gpucores kept", dict(mem=1000, cores=25),
         check=lambda ops: not any(o["path"].endswith("amd.com~1gpucores") for o in ops)),
    Case("priority 0 becomes HIP_TASK_PRIORITY", dict(containers=[c(mem=1000, priority=0)]),
         check=lambda ops: has_env(ops, "HIP_TASK_PRIORITY", "0")),
    Case("pod with no device request is left alone (no scheduler change)", dict(containers=[c(gpu=None)]),
         check=lambda ops: not any(o["path"] == "/spec/schedulerName" for o in ops)),
    # ------------------------------------------------------------- denials
    Case("gpucores above 100 is a validation error", dict(mem=1000, cores=150), False),
    Case("privileged container with a device request", dict(mem=1000), False, "privileged", privileged=True),
    Case("pod with a pre-assigned node", dict(mem=1000), False, "pod has node assigned", node_name="n1"),
    Case("another scheduler's pod passes untouched", dict(mem=1000), scheduler_name="volcano",
         check=lambda ops: ops == []),
]


@pytest.fixture
def cluster():
    c_ = FakeCluster()
    init_global_client(c_)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    yield c_
    get_local_cache().quotas.clear()


@pytest.mark.parametrize("case", CASES, ids=[x.name for x in CASES])
def test_admission_matrix(cluster, case):
    if case.quota is not None:
        get_local_cache().add_quota({"metadata": {"name": "q", "namespace": "default"},
                                     "spec": {"hard": dict(case.quota)}})
    pod = amd_pod("p", namespace=case.namespace, **case.pod)
    if case.privileged:
        pod["spec"]["containers"][0]["securityContext"] = {"privileged": True}
    if case.node_name:
        pod["spec"]["nodeName"] = case.node_name
    if case.scheduler_name:
        pod["spec"]["schedulerName"] = case.scheduler_name
    review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": {"uid": "u", "object": pod}}
    resp = Webhook("hami-scheduler").handle_review(review)["response"]
    assert resp["allowed"] == case.allowed, (case.name, resp)
    if case.message:
        assert case.message in resp.get("status", {}).get("message", ""), (case.name, resp)
    if case.check is not None:
        ops = json.loads(base64.b64decode(resp["patch"])) if resp.get("patch") else []
        assert case.check(ops), (case.name, ops)
