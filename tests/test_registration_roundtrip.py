"""Registration round trip: what the device plugin publishes for a node
(deviceplugin/register.py, reference plugin/register.go:92-351) is what the
scheduler's backend decodes (AMDDevices.get_node_devices), for generated
split counts, scaling factors and device filters; published xGMI pair scores
are symmetric."""

import pytest
from hypothesis import given, settings, strategies as st

from k8s_vgpu_scheduler_amd.device.amd.device import PAIR_SCORE_ANNOS
from k8s_vgpu_scheduler_amd.device.codec import decode_pair_scores
from k8s_vgpu_scheduler_amd.deviceplugin.allocate import PluginConfig
from k8s_vgpu_scheduler_amd.deviceplugin.register import Registrar
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
from k8s_vgpu_scheduler_amd.scheduler.config import init_devices_with_config
from k8s_vgpu_scheduler_amd.device import devices as D
from k8s_vgpu_scheduler_amd.smi import FakeBackend


@settings(max_examples=40, deadline=None)
@given(st.integers(1, 8), st.integers(1, 16), st.sampled_from([1.0, 1.5, 2.0]), st.sampled_from([1.0, 2.0]),
       st.sets(st.integers(0, 7), max_size=3))
def test_published_devices_decode_identically(n, split, mem_scale, core_scale, hidden):
    init_global_client(FakeCluster())
    init_devices_with_config()
    be = FakeBackend(n=n)
    gpus = be.gpus()
    cfg = PluginConfig(device_split_count=split, device_memory_scaling=mem_scale, device_core_scaling=core_scale,
                       filter_indexes=tuple(hidden))
    annos = Registrar(be, cfg, "node1").annotations(gpus)
    node = {"metadata": {"name": "node1", "annotations": annos}}
    want = [g for g in gpus if g.index not in hidden]
    if not want:            # every GPU filtered out: the node offers none (as the reference)
        with pytest.raises(LookupError, match="no gpu found"):
            D.get_devices()["AMD"].get_node_devices(node)
        return
    got = D.get_devices()["AMD"].get_node_devices(node)
    assert [d.id for d in got] == [g.uuid for g in want]
    for d, g in zip(got, want):
        assert d.count == split and d.devmem == int(g.memory_mib * mem_scale)
        assert d.devcore == int(g.cus * core_scale) and d.numa == g.numa and d.health
    if len(want) > 1:
        scores = decode_pair_scores(annos[PAIR_SCORE_ANNOS])
        assert set(scores) == {g.uuid for g in want}
        for a, row in scores.items():
            assert a not in row
            for b, v in row.items():
                assert scores[b][a] == v
    else:
        assert PAIR_SCORE_ANNOS not in annos
