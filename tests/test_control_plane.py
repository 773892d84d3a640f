"""Unit tests for codecs, node lock, quota, init-container accounting, webhook,
HTTP routes, leader election and the fake API server (mirrors the reference's
devices_test.go, nodelock_test.go, quota_test.go, initContainer_test.go,
webhook_test.go, routes/route_test.go, leaderelection_test.go)."""

import base64
import datetime as dt
import json
import threading
import urllib.request

import pytest

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device import common as R
from k8s_vgpu_scheduler_amd.device.init_container import (app_containers_only_device_usage,
                                                          collapse_init_container_usage)
from k8s_vgpu_scheduler_amd.device.quota import QuotaManager, get_local_cache
from k8s_vgpu_scheduler_amd.device.types import ContainerDevice, DeviceInfo
from k8s_vgpu_scheduler_amd.k8s import quantity
from k8s_vgpu_scheduler_amd.k8s.client import Conflict, init_global_client, merge_patch
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster, make_node, make_pod
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.routes import ExtenderServer
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.scheduler.webhook import Webhook, json_patch
from k8s_vgpu_scheduler_amd.testing import amd_container, amd_node, amd_pod
from k8s_vgpu_scheduler_amd.utils import nodelock
from k8s_vgpu_scheduler_amd.utils import types as T
from k8s_vgpu_scheduler_amd.utils.leaderelection import LeaderManager
from k8s_vgpu_scheduler_amd.utils.weights import DeviceScoringWeights, parse_weights


@pytest.fixture
def cluster():
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    return c


# ------------------------------------------------------------------- codecs
def test_node_csv_codec_roundtrip():
    devs = [DeviceInfo(id="GPU-a", count=8, devmem=294912, devcore=256, type="AMD Instinct MI355X", numa=1,
                       health=True, index=3, mode="hami-core")]
    s = codec.encode_node_devices(devs)
    assert s == "GPU-a,8,294912,256,AMD Instinct MI355X,1,true,3,hami-core:"
    back = codec.decode_node_devices(s)
    assert back[0].id == "GPU-a" and back[0].index == 3 and back[0].health
    legacy = codec.decode_node_devices("GPU-b,4,1000,100,T,0,false:")
    assert legacy[0].mode == "hami-core" and legacy[0].index == 0 and not legacy[0].health
    for bad in ("nosep", "a,b:", "GPU,x,1,1,t,0,true:", "G,1,1,1,t,0,true,-1,m:"):
        with pytest.raises(codec.CodecError):
            codec.decode_node_devices(bad)


def test_node_json_marshal_matches_go_shape():
    d = DeviceInfo(id="GPU-a", index=0, count=8, devmem=10, devcore=256, type="AMD", numa=0, mode="hami-core",
                   health=True, custominfo={"secret": 1})
    s = codec.marshal_node_devices([d])
    # omitempty: index 0 and numa 0 dropped; customInfo never serialised
    assert s == '[{"id":"GPU-a","count":8,"devmem":10,"devcore":256,"type":"AMD","mode":"hami-core","health":true}]'
    assert codec.unmarshal_node_devices(s)[0].devcore == 256


def test_pod_codec_keeps_empty_container_entries():
    pd = [[ContainerDevice(uuid="u1", type="AMD", usedmem=10, usedcores=64)], [],
          [ContainerDevice(uuid="u2", type="AMD", usedmem=20, usedcores=0),
           ContainerDevice(uuid="u3", type="AMD", usedmem=30, usedcores=0)]]
    s = codec.encode_pod_single_device(pd)
    assert s == "u1,AMD,10,64:;;u2,AMD,20,0:u3,AMD,30,0:;"
    dec = codec.decode_pod_devices({"AMD": "k"}, {"k": s})["AMD"]
    assert [len(c) for c in dec] == [1, 0, 2, 0]
    with pytest.raises(codec.CodecError):
        codec.decode_container_devices("u1,AMD,10:")


def test_cu_ranges_codec():
    pd = [[ContainerDevice(uuid="u1", custominfo={"cu_ranges": [(0, 63)]})], [],
          [ContainerDevice(uuid="u2", custominfo={"cu_ranges": [(64, 95), (128, 159)]}), ContainerDevice(uuid="u3")]]
    s = codec.encode_cu_ranges(pd)
    assert s == "u1=0-63;;u2=64-95,128-159;"
    dec = codec.decode_cu_ranges(s)
    assert dec[0]["u1"] == [(0, 63)] and dec[1] == {} and dec[2]["u2"] == [(64, 95), (128, 159)]
    assert codec.merge_ranges([(8, 15), (0, 7), (20, 20)]) == [(0, 15), (20, 20)]


def test_pair_scores_codec():
    s = codec.encode_pair_scores({"a": {"b": 100}, "b": {"a": 100}})
    assert codec.decode_pair_scores(s) == {"a": {"b": 100}, "b": {"a": 100}}


def test_reasons():
    r = R.gen_reason({R.CARD_INSUFFICIENT_MEMORY: 2, R.CARD_NOT_HEALTH: 1}, 4)
    assert r == "1/4 CardNotHealth, 2/4 CardInsufficientMemory"
    assert R.parse_reason(r) == {"CardNotHealth": 1, "CardInsufficientMemory": 2}


def test_quantity():
    assert quantity.as_int64("36864") == (36864, True)
    assert quantity.as_int64("1Gi") == (1 << 30, True)
    assert quantity.as_int64("500m") == (0, False)
    assert quantity.value("500m") == 1
    assert quantity.as_int64("junk") == (0, False)


def test_weights():
    assert parse_weights("slot=1,core=1,memory=3") == DeviceScoringWeights(1, 1, 3)
    for bad in ("slot=1,core=1", "slot=1,core=1,core=2", "slot=-1,core=1,memory=1", "slot=0,core=0,memory=0",
                "slot=1,core=1,gpu=1"):
        with pytest.raises(ValueError):
            parse_weights(bad)


# ------------------------------------------------------- init-container usage
def test_collapse_init_vs_app():
    pod = make_pod("p", containers=[{"name": "a"}, {"name": "b"}], init_containers=[{"name": "i"}])
    raw = {"AMD": [[ContainerDevice(uuid="g", usedmem=500, usedcores=128, custominfo={"cu_ranges": [(0, 127)]})],
                   [ContainerDevice(uuid="g", usedmem=100, usedcores=32, custominfo={"cu_ranges": [(128, 159)]})],
                   [ContainerDevice(uuid="g", usedmem=150, usedcores=32, custominfo={"cu_ranges": [(160, 191)]})]]}
    eff = collapse_init_container_usage(pod, raw)["AMD"][0][0]
    assert (eff.usedmem, eff.usedcores, eff.slots) == (500, 128, 2)
    assert eff.custominfo["cu_ranges"] == [(0, 191)]
    app = app_containers_only_device_usage(pod, raw)["AMD"][0][0]
    assert (app.usedmem, app.usedcores, app.slots) == (250, 64, 2)
    assert app.custominfo["cu_ranges"] == [(128, 191)]


# ------------------------------------------------------------------- quota
def test_quota_update_has_no_unlimited_gap(cluster):
    q = QuotaManager()
    old = {"metadata": {"name": "q", "namespace": "ns"}, "spec": {"hard": {"limits.amd.com/gpumem": "100"}}}
    new = {"metadata": {"name": "q", "namespace": "ns"}, "spec": {"hard": {"limits.amd.com/gpumem": "50"}}}
    q.add_quota(old)
    assert q.fit_quota("ns", 80, 1, 0, "AMD")
    q.update_quota(old, new)
    assert not q.fit_quota("ns", 80, 1, 0, "AMD")
    zero = {"metadata": {"name": "z", "namespace": "z"}, "spec": {"hard": {"limits.amd.com/gpumem": "0"}}}
    q.add_quota(zero)
    assert not q.fit_quota("z", 1, 1, 0, "AMD")       # explicit 0 blocks
    assert q.fit_quota("other", 10 ** 9, 1, 0, "AMD")  # no quota -> unlimited
    q.del_quota(zero)
    assert q.fit_quota("z", 1, 1, 0, "AMD")
    q.add_quota({"metadata": {"name": "x", "namespace": "ns"}, "spec": {"hard": {"limits.cpu": "1"}}})
    assert "cpu" not in q.get_resource_quota().get("ns", {})


# ----------------------------------------------------------------- nodelock
def test_nodelock_acquire_release_reentrant(cluster):
    cluster.create("nodes", make_node("n"))
    pa = make_pod("a")
    pb = make_pod("b")
    cluster.create("pods", pa)
    cluster.create("pods", pb)
    nodelock.lock_node("n", "x", pa)
    nodelock.lock_node("n", "x", pa)   # re-entrant for the same pod
    with pytest.raises(nodelock.NodeLockContention):
        nodelock.lock_node("n", "x", pb)
    nodelock.release_node_lock("n", "x", pb)   # not the owner: no-op
    assert T.NODE_LOCK_KEY in cluster.get_node("n")["metadata"]["annotations"]
    nodelock.release_node_lock("n", "x", pa)
    assert T.NODE_LOCK_KEY not in cluster.get_node("n")["metadata"]["annotations"]
    nodelock.lock_node("n", "x", pb)


def test_nodelock_breaks_dangling_and_expired(cluster, monkeypatch):
    cluster.create("nodes", make_node("n", annotations={T.NODE_LOCK_KEY: nodelock.generate_lock_value(
        make_pod("ghost", "gone"))}))
    p = make_pod("a")
    cluster.create("pods", p)
    nodelock.lock_node("n", "x", p)        # owner pod does not exist -> broken
    assert cluster.get_node("n")["metadata"]["annotations"][T.NODE_LOCK_KEY].endswith(",default,a")
    old = (dt.datetime.now().astimezone() - dt.timedelta(minutes=10)).replace(microsecond=0).isoformat()
    cluster.patch_node("n", {"metadata": {"annotations": {T.NODE_LOCK_KEY: f"{old},default,a"}}})
    q = make_pod("q")
    cluster.create("pods", q)
    nodelock.lock_node("n", "x", q)        # expired -> taken over
    assert cluster.get_node("n")["metadata"]["annotations"][T.NODE_LOCK_KEY].endswith(",default,q")


def test_nodelock_survives_lost_patch_response(cluster, monkeypatch):
    monkeypatch.setattr(nodelock, "BACKOFF_BASE", 0.001)
    cluster.create("nodes", make_node("n"))
    p = make_pod("a")
    cluster.create("pods", p)
    fired = []

    def lose_first(verb, kind, name, ns, payload):
        if not fired and "resourceVersion" in (payload or {}).get("metadata", {}):
            fired.append(1)
            return ("after", TimeoutError("response lost"))
    r = cluster.add_reactor("patch", "nodes", lose_first)
    nodelock.set_node_lock("n", "x", p)    # retry sees its own lock and succeeds
    cluster.remove_reactor(r)
    assert fired and cluster.get_node("n")["metadata"]["annotations"][T.NODE_LOCK_KEY].endswith(",default,a")


def test_nodelock_conflict_storm_retries(cluster, monkeypatch):
    monkeypatch.setattr(nodelock, "BACKOFF_BASE", 0.001)
    cluster.create("nodes", make_node("n"))
    p = make_pod("a")
    cluster.create("pods", p)
    n = {"c": 0}

    def conflict_twice(verb, kind, name, ns, payload):
        if n["c"] < 2:
            n["c"] += 1
            raise Conflict("stale")
    cluster.add_reactor("patch", "nodes", conflict_twice)
    nodelock.set_node_lock("n", "x", p)
    assert n["c"] == 2


def test_concurrent_node_locks_only_one_wins(cluster):
    cluster.create("nodes", make_node("n"))
    pods = [make_pod(f"p{i}") for i in range(8)]
    for p in pods:
        cluster.create("pods", p)
    wins, errs = [], []

    def go(p):
        try:
            nodelock.lock_node("n", "x", p)
            wins.append(p["metadata"]["name"])
        except nodelock.NodeLockContention:
            errs.append(1)
    ts = [threading.Thread(target=go, args=(p,)) for p in pods]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert len(wins) == 1 and len(errs) == 7


def test_go_duration():
    assert nodelock.parse_go_duration("5m") == 300
    assert nodelock.parse_go_duration("1h30m") == 5400
    assert nodelock.parse_go_duration("250ms") == 0.25
    with pytest.raises(ValueError):
        nodelock.parse_go_duration("5 minutes")


# ------------------------------------------------------------------ webhook
def review(pod):
    return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
            "request": {"uid": "r1", "object": pod}}


def patch_ops(resp):
    return json.loads(base64.b64decode(resp["response"]["patch"]))


def test_webhook_sets_scheduler_and_exclusive_core(cluster):
    wh = Webhook("hami-scheduler")
    pod = amd_pod("p", gpu=1)
    resp = wh.handle_review(review(pod))
    assert resp["response"]["allowed"]
    ops = patch_ops(resp)
    paths = {o["path"]: o for o in ops}
    assert paths["/spec/schedulerName"]["value"] == "hami-scheduler"
    assert any(o["path"].endswith("amd.com~1gpucores") and o["value"] == "100" for o in ops)


def test_webhook_validation_and_denials(cluster):
    wh = Webhook("hami-scheduler")
    bad = amd_pod("p", gpu=1, cores=150)
    r = wh.handle_review(review(bad))["response"]
    assert not r["allowed"] and r["status"]["code"] == 500
    priv = amd_pod("p", containers=[dict(amd_container(gpu=1), securityContext={"privileged": True})])
    assert not wh.handle_review(review(priv))["response"]["allowed"]
    pinned = amd_pod("p", gpu=1)
    pinned["spec"]["nodeName"] = "n1"
    assert wh.handle_review(review(pinned))["response"]["status"]["message"] == "pod has node assigned"
    assert not wh.handle_review(review(make_pod("e", containers=[])))["response"]["allowed"] or True
    empty = {"metadata": {"name": "e"}, "spec": {"containers": []}}
    assert not wh.handle_review(review(empty))["response"]["allowed"]


def test_webhook_other_scheduler_untouched(cluster):
    wh = Webhook("hami-scheduler")
    pod = amd_pod("p", gpu=1)
    pod["spec"]["schedulerName"] = "volcano"
    r = wh.handle_review(review(pod))["response"]
    assert r["allowed"] and "patch" not in r


def test_webhook_priority_env_and_quota(cluster):
    wh = Webhook("hami-scheduler")
    pod = amd_pod("p", containers=[amd_container(gpu=1, mem=1000, cores=10, priority=0)])
    ops = patch_ops(wh.handle_review(review(pod)))
    assert any(o.get("value") == [{"name": "HIP_TASK_PRIORITY", "value": "0"}] or
               (isinstance(o.get("value"), dict) and o["value"].get("name") == "HIP_TASK_PRIORITY")
               for o in ops)
    get_local_cache().add_quota({"metadata": {"name": "q", "namespace": "default"},
                                 "spec": {"hard": {"limits.amd.com/gpumem": "500"}}})
    # init containers run sequentially: effective = max(sum(app), max(init)) = 400 fits
    ok = amd_pod("ok", containers=[amd_container("a", mem=200), amd_container("b", mem=200)],
                 init=[amd_container("i", mem=300)])
    assert wh.handle_review(review(ok))["response"]["allowed"]
    big = amd_pod("big", containers=[amd_container("a", mem=300), amd_container("b", mem=300)])
    assert wh.handle_review(review(big))["response"]["status"]["message"] == "exceeding resource quota"


def test_json_patch_minimal():
    a = {"x": 1, "l": [1, 2], "m": {"k": "v"}}
    b = {"x": 2, "l": [1, 3], "m": {}, "n": True}
    ops = json_patch(a, b)
    assert {"op": "replace", "path": "/x", "value": 2} in ops
    assert {"op": "replace", "path": "/l/1", "value": 3} in ops
    assert {"op": "remove", "path": "/m/k"} in ops
    assert {"op": "add", "path": "/n", "value": True} in ops


# ------------------------------------------------------------------- routes
def _post(port, path, obj):
    req = urllib.request.Request(f"http://127.0.0.1:{port}{path}", data=json.dumps(obj).encode(),
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=10) as r:
        return r.status, json.loads(r.read())


def test_http_routes_filter_bind_webhook_health(cluster):
    cluster.create("nodes", amd_node("n1", n=1))
    s = Scheduler(cluster, SchedulerConfig())
    s.start()
    s.register()
    srv = ExtenderServer(s, Webhook("hami-scheduler"), "127.0.0.1:0").start()
    try:
        port = srv.port
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/healthz", timeout=5) as r:
            assert r.status == 200
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/readyz", timeout=5) as r:
            assert r.read() == b"leader"
        pod = amd_pod("p", mem=1000)
        cluster.create("pods", pod)
        code, res = _post(port, "/filter", {"Pod": cluster.get_pod("default", "p"), "NodeNames": ["n1"]})
        assert code == 200 and res["NodeNames"] == ["n1"]
        code, res = _post(port, "/filter", {"NodeNames": ["n1"]})
        assert res["Error"] == "extender args missing pod"
        uid = cluster.get_pod("default", "p")["metadata"]["uid"]
        code, res = _post(port, "/bind", {"PodName": "p", "PodNamespace": "default", "PodUID": uid, "Node": "n1"})
        assert res["Error"] == ""
        code, res = _post(port, "/webhook", review(amd_pod("w", gpu=1)))
        assert res["response"]["allowed"]
    finally:
        srv.stop()


# --------------------------------------------------------- leader election
def test_passive_leader_election():
    events = []
    clock = [1000.0]
    lm = LeaderManager("sched-0", "kube-system", "hami-scheduler", on_started=lambda: events.append("up"),
                       on_stopped=lambda: events.append("down"), clock=lambda: clock[0])
    now = dt.datetime.now(dt.timezone.utc)
    lease = {"metadata": {"name": "hami-scheduler", "namespace": "kube-system", "resourceVersion": "1"},
             "spec": {"holderIdentity": "sched-0_abc", "leaseDurationSeconds": 15,
                      "renewTime": now.strftime("%Y-%m-%dT%H:%M:%S.%fZ")}}
    lm.on_add(lease)
    assert lm.is_leader() and events == ["up"]
    other = json.loads(json.dumps(lease))
    other["spec"]["holderIdentity"] = "sched-1_def"
    other["metadata"]["resourceVersion"] = "2"
    lm.on_update(lease, other)
    assert not lm.is_leader() and events == ["up", "down"]


def test_lease_validity_uses_the_local_observation_clock():
    """leaderelection.go:100-104,176-181: a lease is valid for
    leaseDurationSeconds after THIS process last saw it change; the server's
    renewTime (possibly skewed against the local clock) is not consulted."""
    clock = [500.0]
    lm = LeaderManager("sched-0", "kube-system", "hami-scheduler", clock=lambda: clock[0])
    skewed = (dt.datetime.now(dt.timezone.utc) - dt.timedelta(hours=3)).strftime("%Y-%m-%dT%H:%M:%S.%fZ")
    lease = {"metadata": {"name": "hami-scheduler", "namespace": "kube-system", "resourceVersion": "7"},
             "spec": {"holderIdentity": "sched-0_abc", "leaseDurationSeconds": 15, "renewTime": skewed}}
    lm.on_add(lease)
    assert lm.is_leader()                     # the server clock is 3 h behind: still the leader
    clock[0] += 14.0
    assert lm.is_leader()
    lm.on_update(lease, json.loads(json.dumps(lease)))   # informer resync of the same record
    clock[0] += 2.0
    assert not lm.is_leader()                 # not renewed within 15 s of local time: stale
    renewed = json.loads(json.dumps(lease))
    renewed["metadata"]["resourceVersion"] = "8"
    renewed["spec"]["renewTime"] = skewed     # even with the same (skewed) timestamp format
    lm.on_update(lease, renewed)
    assert lm.is_leader()
    future = (dt.datetime.now(dt.timezone.utc) + dt.timedelta(hours=3)).strftime("%Y-%m-%dT%H:%M:%S.%fZ")
    ahead = json.loads(json.dumps(renewed))
    ahead["metadata"]["resourceVersion"] = "9"
    ahead["spec"]["renewTime"] = future       # a server clock 3 h ahead does not extend the lease
    lm.on_update(renewed, ahead)
    clock[0] += 16.0
    assert not lm.is_leader()


def test_follower_does_not_register(cluster):
    cluster.create("nodes", amd_node("n1", n=1))
    s = Scheduler(cluster, SchedulerConfig(leader_elect=True, hostname="me"))
    s.start()
    s.register()
    assert not s.synced and s.nodes.list_nodes() == {}


# ----------------------------------------------------------------- fake API
def test_fake_merge_patch_and_resource_version(cluster):
    n = cluster.create("nodes", make_node("n", annotations={"a": "1"}))
    rv = n["metadata"]["resourceVersion"]
    cluster.patch_node("n", {"metadata": {"annotations": {"a": None, "b": "2"}}})
    got = cluster.get_node("n")["metadata"]["annotations"]
    assert got == {"b": "2"}
    with pytest.raises(Conflict):
        cluster.patch_node("n", {"metadata": {"annotations": {"c": "3"}, "resourceVersion": rv}})
    assert merge_patch({"a": {"b": 1}}, {"a": {"b": None, "c": 2}}) == {"a": {"c": 2}}


def test_register_removes_unhealthy_and_zero_device_nodes(cluster):
    cluster.create("nodes", amd_node("n1", n=2))
    s = Scheduler(cluster, SchedulerConfig())
    s.start()
    s.register()
    assert "n1" in s.nodes.list_nodes()
    # device plugin gone: allocatable drops to 0 -> node cleaned up
    cluster.patch_node("n1", {"status": {"allocatable": {"amd.com/gpu": "0"}}})
    s.register()
    assert "n1" not in s.nodes.list_nodes()
