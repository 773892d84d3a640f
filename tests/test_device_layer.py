"""Device abstraction layer, table-driven (CPU only).

Counterparts of the reference's unit tests:
  pkg/device/devices_test.go        codecs, Resourcereqs, CheckUUID/CheckType, DeepCopy
  pkg/device/nvidia/device_test.go  MutateAdmission / GenerateResourceRequests / Fit cases
                                     (here for the MI355X backend, device/amd/device.py)
  pkg/device/pod_test.go            PodManager
  pkg/device/quota_test.go          QuotaManager
  pkg/device/initContainer_test.go  init-container collapse
  pkg/scheduler/policy/*_test.go    device / node ordering and scores
"""

import pytest

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device import common as R
from k8s_vgpu_scheduler_amd.device import devices as D
from k8s_vgpu_scheduler_amd.device.amd.device import (AMD_DEVICE, AMD_IN_USE, AMD_NO_USE, AMD_NO_USE_UUID,
                                                      AMD_USE_UUID, AMD_VGPU_MODE, AMDConfig, AMDDevices,
                                                      cu_count_for)
from k8s_vgpu_scheduler_amd.device.init_container import (app_containers_only_device_usage,
                                                          collapse_init_container_usage)
from k8s_vgpu_scheduler_amd.device.pods import PodManager
from k8s_vgpu_scheduler_amd.device.quota import QuotaManager, get_local_cache
from k8s_vgpu_scheduler_amd.device.types import (ContainerDevice, ContainerDeviceRequest, DeviceInfo,
                                                 DeviceUsage, NodeInfo)
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster, make_node
from k8s_vgpu_scheduler_amd.scheduler.config import init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.policy import (DeviceListsScore, DeviceUsageList, NodeScore,
                                                     NodeScoreList, sort_key_chain)
from k8s_vgpu_scheduler_amd.testing import MI355X_MEM_MIB, MI355X_TYPE, amd_container, amd_pod
from k8s_vgpu_scheduler_amd.utils import types as T
from k8s_vgpu_scheduler_amd.utils.weights import DeviceScoringWeights


@pytest.fixture(autouse=True)
def registry():
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    yield c
    get_local_cache().quotas.clear()


def amd() -> AMDDevices:
    return D.get_devices()[AMD_DEVICE]


# ======================================================================= codecs
@pytest.mark.parametrize("s,expect", [
    ("gpu0,8,294912,256,MI355X,0,true:", [("gpu0", 8, 294912, 256, "MI355X", 0, True, 0, "hami-core")]),
    ("gpu0,8,1024,256,MI355X,1,false,3,cpx:", [("gpu0", 8, 1024, 256, "MI355X", 1, False, 3, "cpx")]),
    ("a,1,2,3,T,0,1:b,4,5,6,T,1,0,1,hami-core:",
     [("a", 1, 2, 3, "T", 0, True, 0, "hami-core"), ("b", 4, 5, 6, "T", 1, False, 1, "hami-core")]),
    ("a,1,2,3,T,0,True::", [("a", 1, 2, 3, "T", 0, True, 0, "hami-core")]),   # empty segment skipped
])
def test_decode_node_devices_legacy_formats(s, expect):
    got = [(d.id, d.count, d.devmem, d.devcore, d.type, d.numa, d.health, d.index, d.mode)
           for d in codec.decode_node_devices(s)]
    assert got == expect


@pytest.mark.parametrize("bad", [
    "no-separator-at-all",
    "gpu0,8,1024:",                              # too few fields
    "gpu0,8,1024,256,T,0,true,1:",               # 8 fields
    "gpu0,x,1024,256,T,0,true:",                 # count not a number
    "gpu0,8,1024,256,T,0,maybe:",                # health not a Go bool
    "gpu0,8,1024,256,T,0,true,-1,cpx:",          # negative index
    "gpu0,8,99999999999,256,T,0,true:",          # memory beyond int32
    "justtext:",                                 # segment without commas
])
def test_decode_node_devices_rejects(bad):
    with pytest.raises(codec.CodecError):
        codec.decode_node_devices(bad)


def test_encode_decode_node_devices_roundtrip():
    devs = [DeviceInfo(id=f"g{i}", index=i, count=8, devmem=294912, devcore=256, type=MI355X_TYPE, numa=i // 4,
                       mode="hami-core" if i % 2 else "cpx", health=bool(i % 3)) for i in range(8)]
    back = codec.decode_node_devices(codec.encode_node_devices(devs))
    assert [(d.id, d.index, d.count, d.devmem, d.devcore, d.type, d.numa, d.mode, d.health) for d in back] == \
        [(d.id, d.index, d.count, d.devmem, d.devcore, d.type, d.numa, d.mode, d.health) for d in devs]


def test_marshal_node_devices_omits_zero_values_and_custominfo():
    d = DeviceInfo(id="g0", index=0, count=8, devmem=1024, devcore=256, type="T", numa=0, mode="", health=False,
                   custominfo={"secret": 1})
    s = codec.marshal_node_devices([d])
    assert s == '[{"id":"g0","count":8,"devmem":1024,"devcore":256,"type":"T"}]'
    back = codec.unmarshal_node_devices(s)[0]
    assert (back.id, back.count, back.devmem, back.health, back.custominfo) == ("g0", 8, 1024, False, {})


@pytest.mark.parametrize("s,n", [("null", 0), ("[]", 0), ("[{}]", 1)])
def test_unmarshal_node_devices_edge_payloads(s, n):
    assert len(codec.unmarshal_node_devices(s)) == n


@pytest.mark.parametrize("bad", ["{", '{"id":"x"}', "42"])
def test_unmarshal_node_devices_rejects(bad):
    with pytest.raises(codec.CodecError):
        codec.unmarshal_node_devices(bad)


def test_empty_container_and_pod_devices_roundtrip():
    assert codec.decode_container_devices(codec.encode_container_devices([])) == []
    assert codec.encode_pod_devices({AMD_DEVICE: "k"}, {}) == {}
    assert codec.decode_pod_devices({AMD_DEVICE: "k"}, {}) == {}


def test_pod_devices_roundtrip_with_init_and_empty_containers():
    pd = {AMD_DEVICE: [
        [ContainerDevice(uuid="g0", type=AMD_DEVICE, usedmem=1024, usedcores=32)],       # init
        [],                                                                               # app without GPU
        [ContainerDevice(uuid="g1", type=AMD_DEVICE, usedmem=2048, usedcores=64),
         ContainerDevice(uuid="g2", type=AMD_DEVICE, usedmem=2048, usedcores=64)],
    ]}
    annos = codec.encode_pod_devices({AMD_DEVICE: "k"}, pd)
    assert annos == {"k": "g0,AMD,1024,32:;;g1,AMD,2048,64:g2,AMD,2048,64:;"}
    back = codec.decode_pod_devices({AMD_DEVICE: "k"}, annos)[AMD_DEVICE]
    # trailing ';' yields one more empty entry: index == container index is what matters
    assert [[(d.uuid, d.usedmem, d.usedcores) for d in c] for c in back[:3]] == \
        [[("g0", 1024, 32)], [], [("g1", 2048, 64), ("g2", 2048, 64)]]
    assert back[3:] == [[]]


def test_decode_pod_devices_bad_annotation():
    with pytest.raises(codec.CodecError):
        codec.decode_pod_devices({AMD_DEVICE: "k"}, {"k": "g0,AMD,1024:;"})
    with pytest.raises(codec.CodecError):
        codec.decode_pod_devices({AMD_DEVICE: "k"}, {"k": "g0,AMD,lots,32:;"})


def test_encode_container_device_type_filters():
    cd = [ContainerDevice(uuid="a", type="AMD", usedmem=1, usedcores=2),
          ContainerDevice(uuid="b", type="OTHER", usedmem=3, usedcores=4),
          ContainerDevice(uuid="c", type="AMD", usedmem=5, usedcores=6)]
    assert codec.encode_container_device_type(cd, "AMD") == "a,AMD,1,2:c,AMD,5,6"
    assert codec.encode_container_device_type(cd, "NONE") == ""


@pytest.mark.parametrize("ranges,text", [([(0, 7)], "0-7"), ([(0, 0), (8, 15)], "0,8-15"), ([], "")])
def test_cu_range_text(ranges, text):
    assert codec.format_ranges(ranges) == text
    assert codec.parse_ranges(text) == ranges


def test_merge_ranges_and_count():
    assert codec.merge_ranges([(8, 15), (0, 7), (20, 23), (22, 30)]) == [(0, 15), (20, 30)]
    assert codec.ranges_count([(0, 7), (16, 31)]) == 24


# ============================================================ requests / selectors
def test_resource_reqs_init_first_and_empty_entries():
    pod = amd_pod("p", init=[amd_container("i0", gpu=1, mem=1024)],
                  containers=[amd_container("a0", gpu=None), amd_container("a1", gpu=2, cores=50)])
    reqs = D.resource_reqs(pod)
    assert len(reqs) == 3
    assert reqs[0][AMD_DEVICE].nums == 1 and reqs[0][AMD_DEVICE].memreq == 1024
    assert reqs[1] == {}
    assert (reqs[2][AMD_DEVICE].nums, reqs[2][AMD_DEVICE].coresreq) == (2, 50)


def test_resource_reqs_empty_pod_and_no_devices():
    empty = amd_pod("p")
    empty["spec"]["containers"] = []
    assert D.resource_reqs(empty) == []
    assert D.resource_reqs(amd_pod("p", containers=[amd_container(gpu=None)])) == [{}]


@pytest.mark.parametrize("annos,dev,ok", [
    ({}, "g0", True),
    ({AMD_USE_UUID: "g0,g1"}, "g0", True),
    ({AMD_USE_UUID: "g1"}, "g0", False),
    ({AMD_NO_USE_UUID: "g0"}, "g0", False),
    ({AMD_NO_USE_UUID: "g1, g2"}, "g0", True),
    ({AMD_USE_UUID: " g0 "}, "g0", True),
    ({AMD_USE_UUID: "g0", AMD_NO_USE_UUID: "g0"}, "g0", False),
    ({AMD_USE_UUID: ""}, "g0", True),
])
def test_check_uuid(annos, dev, ok):
    assert D.check_uuid(annos, dev, AMD_USE_UUID, AMD_NO_USE_UUID) is ok


@pytest.mark.parametrize("annos,card,ok", [
    ({}, MI355X_TYPE, True),
    ({AMD_IN_USE: "mi355x"}, MI355X_TYPE, True),           # case-insensitive substring
    ({AMD_IN_USE: "MI300X"}, MI355X_TYPE, False),
    ({AMD_IN_USE: "MI300X,MI355"}, MI355X_TYPE, True),
    ({AMD_NO_USE: "instinct"}, MI355X_TYPE, False),
    ({AMD_NO_USE: "MI300"}, MI355X_TYPE, True),
    ({AMD_IN_USE: " , "}, MI355X_TYPE, False),             # non-blank list with no usable entry
])
def test_check_type(annos, card, ok):
    assert D.check_type(annos, card, AMD_IN_USE, AMD_NO_USE) is ok


def test_device_usage_deepcopy_is_independent():
    d = DeviceUsage(id="g0", count=8, totalmem=10, totalcore=256, custominfo={"cu_used": 3, "x": [1]},
                    pod_infos=["p"])
    c = d.deepcopy()
    # custominfo values are replaced, never mutated in place (the Fit path
    # rebinds cu_used; pair scores are read-only): rebinding stays private
    c.custominfo["cu_used"] |= 4
    c.custominfo["x"] = [1, 2]
    c.pod_infos.append("q")
    c.used = 5
    assert d.custominfo == {"cu_used": 3, "x": [1]} and d.pod_infos == ["p"] and d.used == 0


# ==================================================================== admission
def test_mutate_admission_defaults_gpu_and_exclusive_cores():
    ctr = amd_container(gpu=None, mem=None, cores=None, mem_pct=100)
    assert amd().mutate_admission(ctr, amd_pod("p")) is True
    lim = ctr["resources"]["limits"]
    assert lim["amd.com/gpu"] == "1" and lim["amd.com/gpucores"] == "100"


def test_mutate_admission_memory_only_is_shared():
    ctr = amd_container(gpu=1, mem=4096)
    amd().mutate_admission(ctr, amd_pod("p"))
    assert "amd.com/gpucores" not in ctr["resources"]["limits"]


def test_mutate_admission_whole_card_owns_all_cus():
    ctr = amd_container(gpu=2)
    amd().mutate_admission(ctr, amd_pod("p"))
    assert ctr["resources"]["limits"]["amd.com/gpucores"] == "100"


@pytest.mark.parametrize("kw", [{"cores": 101}, {"cores": -1}, {"mem_pct": 150}, {"mem": -5}])
def test_mutate_admission_rejects_out_of_range(kw):
    with pytest.raises(D.AdmissionError):
        amd().mutate_admission(amd_container(gpu=1, **kw), amd_pod("p"))


def test_mutate_admission_priority_env_and_no_request():
    ctr = amd_container(gpu=1, mem=1024, priority=1)
    amd().mutate_admission(ctr, amd_pod("p"))
    assert {"name": T.TASK_PRIORITY_ENV, "value": "1"} in ctr["env"]
    plain = amd_container(gpu=None)
    assert amd().mutate_admission(plain, amd_pod("p")) is False


def test_mutate_admission_runtime_class_and_core_policy():
    dev = AMDDevices(AMDConfig(runtime_class_name="mivgpu", gpu_core_policy="force"))
    pod = amd_pod("p")
    ctr = amd_container(gpu=1, mem=1024, cores=25)
    dev.mutate_admission(ctr, pod)
    assert pod["spec"]["runtimeClassName"] == "mivgpu"
    assert {"name": T.CORE_LIMIT_SWITCH_ENV, "value": "force"} in ctr["env"]


def test_config_rejects_unknown_core_policy():
    with pytest.raises(ValueError):
        AMDConfig.from_dict({"gpuCorePolicy": "sometimes"})


@pytest.mark.parametrize("kw,expect", [
    ({"gpu": 1}, (1, 0, 100, 0)),                               # whole card: 100 % of memory
    ({"gpu": 2, "mem": 36864}, (2, 36864, 101, 0)),
    ({"gpu": 1, "mem_pct": 50}, (1, 0, 50, 0)),
    ({"gpu": 1, "mem_pct": 0}, (1, 0, 100, 0)),                 # 0 % == unset -> whole card
    ({"gpu": 1, "mem_pct": 250}, (1, 0, 100, 0)),               # clamped
    ({"gpu": 1, "cores": 25}, (1, 0, 100, 25)),
    ({"gpu": 0}, (0, 0, 101, 0)),                               # no request
    ({"gpu": 1, "cores": 130}, (1, 0, 100, 100)),               # > 100 clamps to a whole card (device.go:772)
])
def test_generate_resource_requests(kw, expect):
    r = amd().generate_resource_requests(amd_container(**kw))
    assert (r.nums, r.memreq, r.mem_percentage_req, r.coresreq) == expect


def test_generate_resource_requests_memory_factor_and_defaults():
    dev = AMDDevices(AMDConfig(memory_factor=4, default_memory=2048, default_cores=10))
    r = dev.generate_resource_requests(amd_container(gpu=1, mem=1000))
    assert r.memreq == 4000 and r.coresreq == 10
    r = dev.generate_resource_requests(amd_container(gpu=1))
    assert r.memreq == 2048 and r.mem_percentage_req == 101


@pytest.mark.parametrize("pct,total,cus", [(25, 256, 64), (1, 256, 2), (100, 256, 256), (0, 256, 0),
                                           (50, 64, 32), (3, 32, 1)])
def test_cu_count_for(pct, total, cus):
    assert cu_count_for(pct, total) == cus


# =========================================================================== fit
def usage(i, used=0, usedmem=0, usedcores=0, numa=0, count=8, health=True, mode="hami-core",
          typ=MI355X_TYPE, totalmem=MI355X_MEM_MIB, totalcore=256):
    return DeviceUsage(id=f"g{i}", index=i, used=used, count=count, usedmem=usedmem, totalmem=totalmem,
                       totalcore=totalcore, usedcores=usedcores, numa=numa, type=typ, health=health, mode=mode)


def req(nums=1, mem=0, pct=101, cores=0):
    return ContainerDeviceRequest(nums=nums, type=AMD_DEVICE, memreq=mem, mem_percentage_req=pct, coresreq=cores)


def fit(devs, r, annos=None, node_annos=None, pod=None):
    pod = pod or amd_pod("p", annotations=annos)
    node = NodeInfo(id="n", node=make_node("n", annotations=node_annos or {}), devices={})
    return amd().fit(devs, r, pod, node, {})


def test_fit_picks_from_the_end_of_the_sorted_list():
    ok, pd, reason = fit([usage(0), usage(1), usage(2)], req(mem=1024))
    assert ok and [d.uuid for d in pd[AMD_DEVICE]] == ["g2"] and reason == ""


def test_fit_multi_gpu():
    ok, pd, _ = fit([usage(i) for i in range(4)], req(nums=3, mem=1024))
    assert ok and [d.uuid for d in pd[AMD_DEVICE]] == ["g3", "g2", "g1"]


@pytest.mark.parametrize("dev,r,annos,node_annos,reason", [
    (usage(0, health=False), req(), None, None, R.CARD_NOT_HEALTH),
    (usage(0), req(), None, {T.DEVICE_CORDON_ANNOTATION: "g0"}, R.CARD_CORDONED),
    (usage(0), req(), {AMD_IN_USE: "MI300X"}, None, R.CARD_TYPE_MISMATCH),
    (usage(0), req(), {AMD_USE_UUID: "g9"}, None, R.CARD_UUID_MISMATCH),
    (usage(0, used=8), req(mem=1), None, None, R.CARD_TIME_SLICING_EXHAUSTED),
    (usage(0, usedmem=MI355X_MEM_MIB - 100), req(mem=1024), None, None, R.CARD_INSUFFICIENT_MEMORY),
    (usage(0, used=1, usedcores=224), req(mem=1, cores=25), None, None, R.CARD_INSUFFICIENT_CORE),
    (usage(0, used=1, usedmem=10, usedcores=8), req(mem=1, cores=100), None, None, R.CARD_INSUFFICIENT_CORE),
    (usage(0, mode="cpx"), req(), {AMD_VGPU_MODE: "qpx"}, None, R.MODE_NOT_FIT),
])
def test_fit_failure_reasons(dev, r, annos, node_annos, reason):
    ok, _, msg = fit([dev], r, annos=annos, node_annos=node_annos)
    assert not ok
    assert R.parse_reason(msg) == {reason: 1}, msg


def test_fit_exclusive_conflict_when_card_is_shared():
    # 100 % cores on a card that already has a (core-less) tenant
    ok, _, msg = fit([usage(0, used=1, usedmem=10, usedcores=0)], req(mem=1, cores=100))
    assert not ok and R.EXCLUSIVE_DEVICE_ALLOCATE_CONFLICT in R.parse_reason(msg)


def test_fit_memory_percentage_uses_card_capacity():
    ok, pd, _ = fit([usage(0, totalmem=1000)], req(pct=30))
    assert ok and pd[AMD_DEVICE][0].usedmem == 300


def test_fit_cu_ranges_are_disjoint_across_tenants():
    dev = usage(0)
    ok, pd, _ = fit([dev], req(mem=1, cores=25))
    assert ok
    first = pd[AMD_DEVICE][0]
    assert first.usedcores == 64 and codec.ranges_count(first.custominfo["cu_ranges"]) == 64
    amd().add_resource_usage(amd_pod("p"), dev, first)
    ok, pd, _ = fit([dev], req(mem=1, cores=25))
    second = pd[AMD_DEVICE][0]
    a = set().union(*[set(range(x, y + 1)) for x, y in first.custominfo["cu_ranges"]])
    b = set().union(*[set(range(x, y + 1)) for x, y in second.custominfo["cu_ranges"]])
    assert ok and not (a & b)


def test_fit_reports_partial_allocation():
    ok, pd, msg = fit([usage(0), usage(1, health=False)], req(nums=2, mem=1))
    assert not ok
    reasons = R.parse_reason(msg)
    assert reasons[R.ALLOCATED_CARDS_INSUFFICIENT_REQUEST] == 1 and reasons[R.CARD_NOT_HEALTH] == 1


def test_fit_nouse_type_and_mode_selection():
    ok, pd, _ = fit([usage(0, mode="cpx"), usage(1)], req(), annos={AMD_VGPU_MODE: "cpx"})
    assert ok and pd[AMD_DEVICE][0].uuid == "g0"
    ok, _, msg = fit([usage(0)], req(), annos={AMD_NO_USE: "MI355X"})
    assert not ok and R.CARD_TYPE_MISMATCH in R.parse_reason(msg)


def test_fit_respects_namespace_quota():
    get_local_cache().add_quota({"metadata": {"name": "q", "namespace": "default"},
                                 "spec": {"hard": {"limits.amd.com/gpumem": "2048"}}})
    ok, _, msg = fit([usage(0)], req(mem=4096))
    assert not ok and R.RESOURCE_QUOTA_NOT_FIT in R.parse_reason(msg)
    ok, _, _ = fit([usage(0)], req(mem=1024))
    assert ok


def test_reason_histogram_roundtrip():
    s = R.gen_reason({R.CARD_NOT_HEALTH: 2, R.CARD_INSUFFICIENT_MEMORY: 1}, 8)
    assert R.parse_reason(s) == {R.CARD_NOT_HEALTH: 2, R.CARD_INSUFFICIENT_MEMORY: 1}


# =================================================================== PodManager
def test_pod_manager_lifecycle_and_copies():
    pm = PodManager()
    pod = amd_pod("p1")
    devs = {AMD_DEVICE: [[ContainerDevice(uuid="g0", type=AMD_DEVICE, usedmem=1, usedcores=2)]]}
    assert pm.add_pod(pod, "n1", devs)
    devs[AMD_DEVICE][0][0].usedmem = 999           # caller mutation must not leak in
    info = pm.get_pod(pod)
    assert info.node_id == "n1" and info.devices[AMD_DEVICE][0][0].usedmem == 1
    info.devices[AMD_DEVICE][0][0].usedmem = 5      # nor out
    assert pm.get_pod(pod).devices[AMD_DEVICE][0][0].usedmem == 1
    assert len(pm) == 1 and "uid-default-p1" in pm.get_scheduled_pods()
    pm.update_pod_device(pod, {AMD_DEVICE: [[ContainerDevice(uuid="g1", type=AMD_DEVICE)]]})
    assert pm.get_pod(pod).devices[AMD_DEVICE][0][0].uuid == "g1"
    taken = pm.take_and_delete_pod(pod)
    assert taken is not None and pm.get_pod(pod) is None and pm.take_and_delete_pod(pod) is None


def test_pod_manager_delete_and_list():
    pm = PodManager()
    for i in range(3):
        pm.add_pod(amd_pod(f"p{i}"), "n", {})
    pm.del_pod(amd_pod("p1"))
    assert sorted(p.name for p in pm.list_pods_info()) == ["p0", "p2"]


# ================================================================ QuotaManager
def _rq(ns, hard, name="q"):
    return {"metadata": {"name": name, "namespace": ns}, "spec": {"hard": hard}}


def test_quota_fit_memory_and_cores():
    qm = QuotaManager()
    qm.add_quota(_rq("ns", {"limits.amd.com/gpumem": "4096", "limits.amd.com/gpucores": "50"}))
    assert qm.fit_quota("ns", 4096, 1, 50, AMD_DEVICE)
    assert not qm.fit_quota("ns", 4097, 1, 0, AMD_DEVICE)
    assert not qm.fit_quota("ns", 0, 1, 51, AMD_DEVICE)
    assert qm.fit_quota("other-ns", 10 ** 6, 1, 100, AMD_DEVICE)   # no quota there


def test_quota_memory_factor_scales_the_limit():
    qm = QuotaManager()
    qm.add_quota(_rq("ns", {"limits.amd.com/gpumem": "1000"}))
    assert qm.fit_quota("ns", 3000, 4, 0, AMD_DEVICE)
    assert not qm.fit_quota("ns", 5000, 4, 0, AMD_DEVICE)


def test_quota_explicit_zero_blocks_everything():
    qm = QuotaManager()
    qm.add_quota(_rq("ns", {"limits.amd.com/gpumem": "0"}))
    assert not qm.fit_quota("ns", 1, 1, 0, AMD_DEVICE)
    assert qm.fit_quota("ns", 0, 1, 0, AMD_DEVICE)


def test_quota_usage_accounting_and_replace():
    qm = QuotaManager()
    qm.add_quota(_rq("ns", {"limits.amd.com/gpumem": "8192"}))
    pod = amd_pod("p", namespace="ns")
    pd1 = {AMD_DEVICE: [[ContainerDevice(uuid="g0", type=AMD_DEVICE, usedmem=4096, usedcores=64)]]}
    qm.add_usage(pod, pd1)
    assert qm.get_resource_quota()["ns"]["amd.com/gpumem"].used == 4096
    assert not qm.fit_quota("ns", 4097, 1, 0, AMD_DEVICE)
    pd2 = {AMD_DEVICE: [[ContainerDevice(uuid="g0", type=AMD_DEVICE, usedmem=1024, usedcores=64)]]}
    qm.replace_usage(pod, pd1, pd2)
    assert qm.get_resource_quota()["ns"]["amd.com/gpumem"].used == 1024
    qm.rm_usage(pod, pd2)
    qm.rm_usage(pod, pd2)   # never below zero
    assert qm.get_resource_quota()["ns"]["amd.com/gpumem"].used == 0


def test_quota_update_and_delete():
    qm = QuotaManager()
    old = _rq("ns", {"limits.amd.com/gpumem": "100"})
    new = _rq("ns", {"limits.amd.com/gpumem": "200"})
    qm.add_quota(old)
    qm.update_quota(old, new)
    assert qm.fit_quota("ns", 200, 1, 0, AMD_DEVICE) and not qm.fit_quota("ns", 201, 1, 0, AMD_DEVICE)
    qm.del_quota(new)
    assert qm.fit_quota("ns", 10 ** 6, 1, 0, AMD_DEVICE)


def test_managed_quota_names():
    # device resource names (quota.go IsManagedQuota), "limits." stripped by the caller
    assert QuotaManager.is_managed_quota("amd.com/gpumem")
    assert QuotaManager.is_managed_quota("amd.com/gpucores")
    assert not QuotaManager.is_managed_quota("limits.amd.com/gpumem")
    assert not QuotaManager.is_managed_quota("cpu")
    qm = QuotaManager()
    qm.add_quota(_rq("ns", {"requests.amd.com/gpumem": "1", "limits.cpu": "1"}))   # ignored keys
    assert qm.fit_quota("ns", 10 ** 6, 1, 100, AMD_DEVICE)


# =========================================================== init containers
def _cd(uuid, mem, cores, ranges=None):
    return ContainerDevice(uuid=uuid, type=AMD_DEVICE, usedmem=mem, usedcores=cores,
                           custominfo={"cu_ranges": ranges} if ranges else {})


def _pod_with(n_init, n_app):
    return amd_pod("p", init=[amd_container(f"i{i}") for i in range(n_init)],
                   containers=[amd_container(f"a{i}") for i in range(n_app)])


@pytest.mark.parametrize("init,app,expect", [
    # init peak larger than the app sum
    ([[("g0", 8000, 64)]], [[("g0", 1000, 32)], [("g0", 1000, 32)]], {"g0": (8000, 64, 2)}),
    # app sum larger than the init peak
    ([[("g0", 1000, 8)]], [[("g0", 3000, 64)], [("g0", 3000, 64)]], {"g0": (6000, 128, 2)}),
    # several init containers: peak, not sum
    ([[("g0", 5000, 32)], [("g0", 7000, 16)]], [[("g0", 1000, 8)]], {"g0": (7000, 32, 1)}),
    # disjoint devices
    ([[("g0", 5000, 32)]], [[("g1", 1000, 8)]], {"g0": (5000, 32, 1), "g1": (1000, 8, 1)}),
    # no init containers
    ([], [[("g0", 1, 2)], [("g0", 3, 4)], [("g1", 5, 6)]], {"g0": (4, 6, 2), "g1": (5, 6, 1)}),
])
def test_collapse_init_container_usage(init, app, expect):
    pod = _pod_with(len(init), len(app))
    raw = {AMD_DEVICE: [[_cd(*d) for d in ctr] for ctr in init + app]}
    out = collapse_init_container_usage(pod, raw)[AMD_DEVICE][0]
    assert {d.uuid: (d.usedmem, d.usedcores, d.slots) for d in out} == expect


def test_collapse_unions_cu_ranges_and_app_only_drops_init():
    pod = _pod_with(1, 2)
    raw = {AMD_DEVICE: [[_cd("g0", 100, 64, [(0, 63)])], [_cd("g0", 10, 32, [(64, 95)])],
                        [_cd("g0", 10, 32, [(96, 127)])]]}
    col = collapse_init_container_usage(pod, raw)[AMD_DEVICE][0][0]
    assert col.custominfo["cu_ranges"] == [(0, 127)]
    app = app_containers_only_device_usage(pod, raw)[AMD_DEVICE][0][0]
    assert (app.usedmem, app.usedcores, app.slots) == (20, 64, 2)
    assert app.custominfo["cu_ranges"] == [(64, 127)]
    assert collapse_init_container_usage(pod, None) is None


# ====================================================================== policy
def _scored(devs, policy, numa_bind=False, r=None):
    lst = DeviceUsageList([DeviceListsScore(d) for d in devs], policy, numa_bind)
    for s in lst.device_lists:
        s.compute_score({AMD_DEVICE: r or req(mem=1024)}, DeviceScoringWeights())
    lst.sort()
    return [s.device.id for s in lst.device_lists]


def test_binpack_prefers_the_fullest_card_last():
    devs = [usage(0, used=1, usedmem=100000), usage(1), usage(2, used=2, usedmem=200000)]
    assert _scored(devs, T.GPU_POLICY_BINPACK)[-1] == "g2"


def test_spread_prefers_the_emptiest_card_last():
    devs = [usage(0, used=1, usedmem=100000), usage(1), usage(2, used=2, usedmem=200000)]
    assert _scored(devs, T.GPU_POLICY_SPREAD)[-1] == "g1"


def test_mutex_orders_idle_cards_last():
    devs = [usage(0, used=0, numa=1), usage(1, used=3), usage(2, used=0, numa=0)]
    order = _scored(devs, T.GPU_POLICY_MUTEX)
    assert order[0] == "g1" and set(order[1:]) == {"g0", "g2"}


def test_numa_chain_groups_by_numa_then_score():
    devs = [usage(0, numa=1), usage(1, numa=0, used=3, usedmem=300000), usage(2, numa=0), usage(3, numa=1, used=2)]
    order = _scored(devs, "numa,binpack")
    assert order[:2] in (["g2", "g1"], ["g1", "g2"]) and set(order[2:]) == {"g0", "g3"}
    assert order.index("g2") < order.index("g1")   # binpack inside a NUMA node: fuller card later


def test_sort_key_chain_dedups_and_ignores_filters():
    assert sort_key_chain("binpack,numa,binpack,mutex,topology-aware") == ["binpack", "numa"]
    assert sort_key_chain("") == []


def test_device_score_counts_the_pending_request():
    d = usage(0, used=4, usedmem=MI355X_MEM_MIB // 2, usedcores=128)
    s = DeviceListsScore(d)
    s.compute_score({AMD_DEVICE: req(mem=MI355X_MEM_MIB // 2, cores=50)}, DeviceScoringWeights())
    # (5/8 slots + 256/256 cores + 1.0 memory) * 10 with unit weights
    assert s.score == pytest.approx(10 * (5 / 8 + 1.0 + 1.0))


def test_device_score_weights():
    d = usage(0, used=0)
    s = DeviceListsScore(d)
    s.compute_score({AMD_DEVICE: req(mem=MI355X_MEM_MIB)}, DeviceScoringWeights(slot=0, core=0, memory=3))
    assert s.score == pytest.approx(30.0)


def test_zero_capacity_device_scores_zero():
    s = DeviceListsScore(usage(0, totalmem=0))
    s.compute_score({AMD_DEVICE: req()}, DeviceScoringWeights())
    assert s.score == 0.0


def test_node_score_and_ordering():
    a = NodeScore("a", None)
    a.compute_default_score(DeviceUsageList([DeviceListsScore(usage(0, used=8, usedmem=MI355X_MEM_MIB,
                                                                         usedcores=256))]))
    b = NodeScore("b", None)
    b.compute_default_score(DeviceUsageList([DeviceListsScore(usage(0))]))
    assert a.score == pytest.approx(30.0) and b.score == 0.0
    binpack = NodeScoreList([b, a], T.NODE_POLICY_BINPACK)
    binpack.sort()
    assert binpack.node_list[-1].node_id == "a"
    spread = NodeScoreList([a, b], T.NODE_POLICY_SPREAD)
    spread.sort()
    assert spread.node_list[-1].node_id == "b"
