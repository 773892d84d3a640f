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


# ------------------------------------------------------------ review edges --

def _review(pod):
    return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": {"uid": "u", "object": pod}}


def test_pod_without_containers_denied(cluster):
    resp = Webhook("hami-scheduler").handle_review(_review({"metadata": {"name": "p"}, "spec": {}}))["response"]
    assert not resp["allowed"] and resp["status"]["code"] == 403


@pytest.mark.parametrize("force,want_changed", [(True, True), (False, False)])
def test_default_scheduler_overwrite_flag(cluster, force, want_changed):
    pod = amd_pod("p", mem=1000)
    pod["spec"]["schedulerName"] = "default-scheduler"
    resp = Webhook("hami-scheduler", force_overwrite_default_scheduler=force).handle_review(_review(pod))["response"]
    ops = json.loads(base64.b64decode(resp["patch"])) if resp.get("patch") else []
    assert resp["allowed"]
    assert sets(ops, "/schedulerName", "hami-scheduler") == want_changed


def test_privileged_pod_without_device_request_allowed(cluster):
    pod = amd_pod("p", containers=[c(gpu=None)])
    pod["spec"]["containers"][0]["securityContext"] = {"privileged": True}
    assert Webhook("hami-scheduler").handle_review(_review(pod))["response"]["allowed"]


def test_uid_and_api_version_echoed(cluster):
    out = Webhook("hami-scheduler").handle_review(_review(amd_pod("p", mem=10)))
    assert out["response"]["uid"] == "u" and out["apiVersion"] == "admission.k8s.io/v1"
    assert out["kind"] == "AdmissionReview"


# ---------------------------------------------------------------- json_patch --

from hypothesis import given, settings, strategies as st  # noqa: E402

from k8s_vgpu_scheduler_amd.scheduler.webhook import json_patch  # noqa: E402


def _unesc(k):
    return k.replace("~1", "/").replace("~0", "~")


def _apply(doc, ops):
    """Minimal RFC 6902 applier for add/remove/replace (test oracle)."""
    import copy
    doc = copy.deepcopy(doc)
    for op in ops:
        if op["path"] == "/":
            doc = copy.deepcopy(op["value"])
            continue
        parts = [_unesc(p) for p in op["path"].split("/")[1:]]
        tgt = doc
        for p in parts[:-1]:
            tgt = tgt[int(p)] if isinstance(tgt, list) else tgt[p]
        last = parts[-1]
        if isinstance(tgt, list):
            last = int(last)
        if op["op"] == "remove":
            del tgt[last]
        else:
            tgt[last] = copy.deepcopy(op["value"])
    return doc


keys = st.sampled_from(["a", "b", "c/d", "e~f", "amd.com/gpu"])
json_vals = st.recursive(st.one_of(st.none(), st.booleans(), st.integers(-5, 5), st.text(max_size=3)),
                         lambda ch: st.one_of(st.lists(ch, max_size=3), st.dictionaries(keys, ch, max_size=4)),
                         max_leaves=12)


@settings(max_examples=150, deadline=None)
@given(st.dictionaries(keys, json_vals, max_size=4), st.dictionaries(keys, json_vals, max_size=4))
def test_json_patch_transforms_a_into_b(a, b):
    assert _apply(a, json_patch(a, b)) == b


def test_json_patch_escapes_resource_names():
    ops = json_patch({"r": {}}, {"r": {"amd.com/gpucores": "100"}})
    assert ops == [{"op": "add", "path": "/r/amd.com~1gpucores", "value": "100"}]
