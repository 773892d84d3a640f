"""Device identity and partition grouping tables (smi/__init__.py).

One identity whatever the discovery backend: ``GPU-<16 hex>`` from the KFD
unique id, the board's product name (never libdrm's generic "AMD Radeon
Graphics"), partitions of one package numbered inside their physical GPU and
given distinct ids (reference: docs/develop/amd-vgpu.md:174-180 for the ROCr id
form; nvidia MIG uuids play the same role there)."""

import pytest

from k8s_vgpu_scheduler_amd import smi
from k8s_vgpu_scheduler_amd.smi import GPUInfo


@pytest.mark.parametrize("v,want", [
    (0xAE8C1614E27CC400, "GPU-ae8c1614e27cc400"),
    ("ae8c1614e27cc400", "GPU-ae8c1614e27cc400"),
    ("0xAE8C1614E27CC400", "GPU-ae8c1614e27cc400"),
    (1, "GPU-0000000000000001"),
    (None, None), ("", None), (0, None), ("0", None), ("zz", None),
])
def test_rocr_uuid(v, want):
    assert smi.rocr_uuid(v) == want


@pytest.mark.parametrize("cands,dev_id,want", [
    (("AMD Instinct MI355 OAM",), None, "AMD Instinct MI355 OAM"),
    (("AMD Radeon Graphics", "AMD Instinct MI355 OAM"), None, "AMD Instinct MI355 OAM"),
    (("", "N/A", "  "), 0x75A3, "AMD Instinct MI355X"),
    (("unknown",), 0x74A1, "AMD Instinct MI300X"),
    ((None,), None, "AMD Instinct MI355X"),
    (("  Board X  ",), None, "Board X"),
])
def test_canonical_name(cands, dev_id, want):
    assert smi.canonical_name(*cands, device_id=dev_id) == want


def _g(i, bdf, uuid="GPU-a", part="SPX"):
    return GPUInfo(index=i, uuid=uuid, rocr_id=uuid, bdf=bdf, compute_partition=part)


def test_group_physical_spx():
    gs = smi._group_physical([_g(0, "0000:05:00.0"), _g(1, "0000:15:00.0"), _g(2, "0000:65:00.0")])
    assert [g.physical_index for g in gs] == [0, 1, 2]
    assert [g.partition_index for g in gs] == [0, 0, 0]
    assert [g.physical for g in gs] == [0, 1, 2]


def test_group_physical_cpx_partitions_share_the_package():
    gs = [_g(i, f"0000:05:00.{i}", part="CPX") for i in range(4)] + \
         [_g(4 + i, f"0000:15:00.{i}", part="CPX") for i in range(4)]
    smi._group_physical(gs)
    assert [g.physical_index for g in gs] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert [g.partition_index for g in gs] == [0, 1, 2, 3, 0, 1, 2, 3]


def test_group_physical_without_bdf_uses_the_index():
    gs = smi._group_physical([_g(0, ""), _g(1, "")])
    assert [g.physical_index for g in gs] == [0, 1]


def test_duplicate_ids_of_partitions_are_suffixed():
    gs = [_g(i, f"0000:05:00.{i}", uuid="GPU-ae8c1614e27cc400", part="DPX") for i in range(2)] + \
         [_g(2, "0000:15:00.0", uuid="GPU-0000000000000002")]
    smi._group_physical(gs)
    smi._dedupe_partition_ids(gs)
    assert [g.uuid for g in gs] == ["GPU-ae8c1614e27cc400-dpx0", "GPU-ae8c1614e27cc400-dpx1",
                                    "GPU-0000000000000002"]
    assert [g.rocr_id for g in gs] == ["0", "1", "GPU-0000000000000002"]
    assert len({g.uuid for g in gs}) == 3


@pytest.mark.parametrize("h,want", [(None, None), (5, 5), ("7", 7), ("x", None)])
def test_handle_key(h, want):
    assert smi._handle_key(h) == want


def test_handle_key_of_ctypes_pointer():
    import ctypes
    assert smi._handle_key(ctypes.c_void_p(1234)) == 1234
    assert smi._handle_key(ctypes.c_void_p(None)) is None


def test_partition_modes_split_xcds_evenly():
    for mode, n in smi.PARTITION_MODES.items():
        assert 8 % n == 0, mode


def test_fake_backend_identity_is_stable():
    a, b = smi.FakeBackend(n=4).gpus(), smi.FakeBackend(n=4).gpus()
    assert [g.uuid for g in a] == [g.uuid for g in b]
    assert len({g.uuid for g in a}) == 4
