"""Per-node device-plugin overrides (cmd/device_plugin.apply_node_config;
reference pkg/device-plugin/nvidiadevice/nvinternal/plugin/server.go:128-169,
the ``nodeconfig[]`` list of the device-plugin ConfigMap)."""

import json

import pytest

from k8s_vgpu_scheduler_amd.cmd.device_plugin import apply_node_config
from k8s_vgpu_scheduler_amd.deviceplugin.allocate import PluginConfig


def write(tmp_path, entries):
    p = tmp_path / "config.json"
    p.write_text(json.dumps({"nodeconfig": entries}))
    return str(p)


def test_missing_file_keeps_defaults(tmp_path):
    cfg = apply_node_config(PluginConfig(), str(tmp_path / "absent.json"), "n1")
    assert cfg == PluginConfig()


def test_other_nodes_entries_ignored(tmp_path):
    path = write(tmp_path, [{"name": "n2", "devicesplitcount": 2}])
    assert apply_node_config(PluginConfig(), path, "n1").device_split_count == 8


@pytest.mark.parametrize("entry,field,want", [
    ({"devicesplitcount": 4}, "device_split_count", 4),
    ({"devicesplitcount": "16"}, "device_split_count", 16),
    ({"devicememoryscaling": 1.5}, "device_memory_scaling", 1.5),
    ({"devicecorescaling": 2}, "device_core_scaling", 2.0),
    ({"hwqueues": 0}, "hw_queues_shared", 0),
    ({"enablegetpreferredallocation": False}, "enable_preferred_allocation", False),
    ({"partitions": {"0": "cpx", "3": "dpx"}}, "partitions", {0: "CPX", 3: "DPX"}),
    ({"partitions": None}, "partitions", {}),
    ({"filterdevices": {"uuid": ["GPU-a"], "index": ["2", 5]}}, "filter_uuids", ("GPU-a",)),
    ({"filterdevices": {"uuid": ["GPU-a"], "index": ["2", 5]}}, "filter_indexes", (2, 5)),
])
def test_override(tmp_path, entry, field, want):
    path = write(tmp_path, [{"name": "n1", **entry}])
    assert getattr(apply_node_config(PluginConfig(), path, "n1"), field) == want


def test_later_entries_for_the_same_node_win(tmp_path):
    path = write(tmp_path, [{"name": "n1", "devicesplitcount": 2}, {"name": "n1", "devicesplitcount": 6}])
    assert apply_node_config(PluginConfig(), path, "n1").device_split_count == 6


def test_empty_file_and_empty_list(tmp_path):
    p = tmp_path / "c.json"
    p.write_text("")
    assert apply_node_config(PluginConfig(), str(p), "n1") == PluginConfig()
    p.write_text('{"nodeconfig": null}')
    assert apply_node_config(PluginConfig(), str(p), "n1") == PluginConfig()


def test_malformed_json_is_an_error(tmp_path):
    p = tmp_path / "c.json"
    p.write_text("{nope")
    with pytest.raises(json.JSONDecodeError):
        apply_node_config(PluginConfig(), str(p), "n1")
