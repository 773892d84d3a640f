"""Property and table tests of the annotation wire codecs (device/codec.py).

Model: the encode/decode tables of the reference's pkg/device/devices_test.go
and pkg/util/util_test.go (DecodeNodeDevices, EncodePodDevices,
DecodePodDevices); the CU-range annotation is AMD-only and has no reference
equivalent.  Hypothesis drives round trips over generated device lists.
"""

import json

import pytest
from hypothesis import given, settings, strategies as st

from k8s_vgpu_scheduler_amd.device import codec as C
from k8s_vgpu_scheduler_amd.device.types import ContainerDevice, DeviceInfo

uuid = st.from_regex(r"GPU-[0-9a-f]{8}", fullmatch=True)
dtype = st.sampled_from(["MI355X", "AMD", "MI300X"])
i32 = st.integers(0, 2 ** 31 - 1)

node_dev = st.builds(DeviceInfo, id=uuid, index=st.integers(0, 63), count=st.integers(0, 64),
                     devmem=i32, devcore=st.integers(0, 512), type=dtype, numa=st.integers(0, 7),
                     mode=st.sampled_from(["hami-core", "cpx", "spx"]), health=st.booleans())
ctr_dev = st.builds(ContainerDevice, uuid=uuid, type=dtype, usedmem=i32, usedcores=st.integers(0, 256))


def _key(d: DeviceInfo):
    return (d.id, d.index, d.count, d.devmem, d.devcore, d.type, d.numa, d.mode, d.health)


@settings(max_examples=80, deadline=None)
@given(st.lists(node_dev, max_size=8))
def test_node_csv_round_trip(devs):
    s = C.encode_node_devices(devs)
    if not devs:
        assert s == ""
        return
    assert [_key(d) for d in C.decode_node_devices(s)] == [_key(d) for d in devs]


@settings(max_examples=80, deadline=None)
@given(st.lists(node_dev, max_size=8))
def test_node_json_round_trip(devs):
    back = C.unmarshal_node_devices(C.marshal_node_devices(devs))
    assert [_key(d) for d in back] == [_key(d) for d in devs]


def test_json_omits_zero_values_and_custominfo():
    d = DeviceInfo(id="GPU-1", count=4, devmem=0, type="MI355X", health=False, custominfo={"x": 1})
    assert json.loads(C.marshal_node_devices([d])) == [{"id": "GPU-1", "count": 4, "type": "MI355X"}]


@pytest.mark.parametrize("s,n", [
    ("GPU-0,10,294912,256,MI355X,0,true:", 1),
    ("GPU-0,10,294912,256,MI355X,0,true,3,cpx:", 1),
    ("GPU-0,10,294912,256,MI355X,0,1:GPU-1,10,294912,256,MI355X,1,F:", 2),
    ("::GPU-0,10,294912,256,MI355X,0,True:", 1),
])
def test_decode_node_legacy_accepts(s, n):
    assert len(C.decode_node_devices(s)) == n


@pytest.mark.parametrize("s,msg", [
    ("GPU-0,10,294912,256,MI355X,0,true", "separator"),
    ("GPU-0:", "malformed"),
    ("GPU-0,10,294912,256,MI355X,0:", "field count"),
    ("GPU-0,10,294912,256,MI355X,0,true,1:", "field count"),
    ("GPU-0,x,294912,256,MI355X,0,true:", "count"),
    ("GPU-0,10,294912,256,MI355X,0,yes:", "health"),
    ("GPU-0,10,99999999999,256,MI355X,0,true:", "int32"),
    ("GPU-0,10,1,256,MI355X,0,true,-1,cpx:", "negative"),
])
def test_decode_node_legacy_rejects(s, msg):
    with pytest.raises(C.CodecError, match=msg):
        C.decode_node_devices(s)


@pytest.mark.parametrize("s", ["{", '{"id": 1}', "3"])
def test_unmarshal_rejects_non_arrays(s):
    with pytest.raises(C.CodecError):
        C.unmarshal_node_devices(s)


def test_unmarshal_null_is_empty():
    assert C.unmarshal_node_devices("null") == []


@settings(max_examples=60, deadline=None)
@given(st.dictionaries(uuid, st.dictionaries(uuid, st.integers(0, 1000), max_size=7), max_size=8))
def test_pair_scores_round_trip(scores):
    assert C.decode_pair_scores(C.encode_pair_scores(scores)) == scores


# ------------------------------------------------------------------ pod side --

def _ckey(c: ContainerDevice):
    return (c.uuid, c.type, c.usedmem, c.usedcores)


@settings(max_examples=80, deadline=None)
@given(st.lists(st.lists(ctr_dev, max_size=4), max_size=5))
def test_pod_devices_round_trip_keeps_container_index(containers):
    """Empty containers survive the round trip, so annotation index == container
    index (init containers first, devices.go:546-551)."""
    checklist = {"MI355X": "hami.io/amd-devices-allocated"}
    annos = C.encode_pod_devices(checklist, {"MI355X": containers})
    back = C.decode_pod_devices(checklist, annos)["MI355X"]
    # encoding terminates every container with ';', decoding keeps the trailing empty entry
    assert len(back) == len(containers) + 1 and back[-1] == []
    assert [[_ckey(c) for c in ctr] for ctr in back[:-1]] == [[_ckey(c) for c in ctr] for ctr in containers]


def test_decode_pod_devices_ignores_absent_keys():
    assert C.decode_pod_devices({"MI355X": "k"}, {"other": "x"}) == {}
    assert C.decode_pod_devices({"MI355X": "k"}, {}) == {}


@pytest.mark.parametrize("s,n", [
    ("", 0),
    ("GPU-0,MI355X,1024,25:", 1),
    ("GPU-0,MI355X,1024,25:GPU-1,MI355X,0,0:", 2),
    ("junk:GPU-0,MI355X,1024,25", 1),
])
def test_decode_container_devices(s, n):
    assert len(C.decode_container_devices(s)) == n


@pytest.mark.parametrize("s", ["GPU-0,MI355X,1024:", "GPU-0,MI355X,x,1:"])
def test_decode_container_devices_rejects(s):
    with pytest.raises(C.CodecError):
        C.decode_container_devices(s)


def test_encode_container_device_type_filters():
    cd = [ContainerDevice(uuid="a", type="MI355X", usedmem=1, usedcores=2),
          ContainerDevice(uuid="b", type="NVIDIA", usedmem=3, usedcores=4),
          ContainerDevice(uuid="c", type="MI355X", usedmem=5, usedcores=6)]
    assert C.encode_container_device_type(cd, "MI355X") == "a,MI355X,1,2:c,MI355X,5,6"


# ------------------------------------------------------------------ CU ranges --

ranges = st.lists(st.tuples(st.integers(0, 255), st.integers(0, 31)).map(lambda t: (t[0], t[0] + t[1])),
                  max_size=8)


@settings(max_examples=100, deadline=None)
@given(ranges)
def test_merge_ranges_is_the_set_union(rs):
    merged = C.merge_ranges(rs)
    want = set()
    for a, b in rs:
        want.update(range(a, b + 1))
    got = set()
    for a, b in merged:
        got.update(range(a, b + 1))
    assert got == want
    assert C.ranges_count(merged) == len(want)
    # sorted, disjoint and non-adjacent
    for (a0, b0), (a1, b1) in zip(merged, merged[1:]):
        assert b0 + 1 < a1
    assert C.merge_ranges(merged) == merged


@settings(max_examples=100, deadline=None)
@given(ranges)
def test_format_parse_round_trip(rs):
    merged = C.merge_ranges(rs)
    assert C.parse_ranges(C.format_ranges(merged)) == merged


@pytest.mark.parametrize("s,want", [
    ("0-63", [(0, 63)]),
    ("5", [(5, 5)]),
    (" 0-3 , 8-11 ,", [(0, 3), (8, 11)]),
    ("", []),
])
def test_parse_ranges(s, want):
    assert C.parse_ranges(s) == want


@pytest.mark.parametrize("s", ["3-1", "-1", "a-b", "1-x"])
def test_parse_ranges_rejects(s):
    with pytest.raises(ValueError):
        C.parse_ranges(s)


@settings(max_examples=60, deadline=None)
@given(st.lists(st.lists(st.tuples(uuid, ranges), max_size=3), max_size=4))
def test_cu_range_annotation_round_trip(spec):
    pd = []
    for ctr in spec:
        devs = []
        for u, rs in ctr:
            merged = C.merge_ranges(rs)
            devs.append(ContainerDevice(uuid=u, type="MI355X",
                                        custominfo={"cu_ranges": merged} if merged else {}))
        pd.append(devs)
    s = C.encode_cu_ranges(pd)
    per = C.decode_cu_ranges(s)
    assert len(per) == len(pd)
    for ctr, got in zip(pd, per):
        want = {}
        for d in ctr:
            if d.custominfo.get("cu_ranges"):
                want[d.uuid] = d.custominfo["cu_ranges"]
        assert got == want
    # attach copies the ranges back onto freshly decoded devices
    fresh = [[ContainerDevice(uuid=d.uuid, type=d.type) for d in ctr] for ctr in pd]
    C.attach_cu_ranges(fresh, s)
    for ctr, got in zip(fresh, per):
        for d in ctr:
            if d.uuid in got:
                assert d.custominfo["cu_ranges"] == got[d.uuid]


def test_attach_cu_ranges_tolerates_missing_annotation():
    pd = [[ContainerDevice(uuid="a")]]
    assert C.attach_cu_ranges(pd, None) is pd
    assert C.attach_cu_ranges(pd, "") is pd
    assert pd[0][0].custominfo == {}
