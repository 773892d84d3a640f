"""Shared-region ABI accessors and lister behaviour (pkg/monitor/nvidia/v1/spec_test.go,
cudevshr_test.go counterparts): per-process aggregation over active slots,
procnum clamping, setters visible to a second mapping, read-only mappings,
bad files, concurrent writers, lister remapping and disappearance."""

import os
import threading

import pytest

from k8s_vgpu_scheduler_amd.monitor.lister import ContainerLister
from k8s_vgpu_scheduler_amd.monitor.region import MAX_DEVICES, MAX_PROCS, REGION_SIZE, SharedRegion


@pytest.fixture
def region(tmp_path):
    r = SharedRegion.create(str(tmp_path / "r.cache"), num_devices=2, mem_limit=1 << 30, cu_limit=50)
    yield r
    r.close()


def _proc(r, i, pid, status=1, dev=0, total=0, buffer=0, busy=0, launches=0):
    p = r.r.procs[i]
    p.pid, p.status = pid, status
    p.used[dev].total, p.used[dev].buffer = total, buffer
    p.util[dev].busy_ns, p.util[dev].launches = busy, launches
    r.r.procnum = max(r.r.procnum, i + 1)


def test_create_initialises_header(region):
    assert region.device_num() == 2
    assert region.memory_limit(0) == 1 << 30 and region.memory_limit(15) == 1 << 30
    assert int(region.r.cu_limit[1]) == 50
    assert region.active_procs() == [] and region.memory_total(0) == 0


def test_aggregates_only_active_slots(region):
    _proc(region, 0, 10, total=100, buffer=60, busy=5, launches=2)
    _proc(region, 1, 11, total=200, buffer=150, busy=7, launches=3)
    _proc(region, 2, 12, status=0, total=10 ** 9)          # freed slot: ignored
    _proc(region, 3, 13, dev=1, total=42)
    assert region.memory_total(0) == 300
    assert region.memory_field(0, "buffer") == 210
    assert region.memory_total(1) == 42
    assert region.busy_ns(0) == 12 and region.launches(0) == 5
    assert sorted(region.pids()) == [10, 11, 13]


@pytest.mark.parametrize("procnum", [-5, MAX_PROCS + 100])
def test_corrupt_procnum_is_clamped(region, procnum):
    _proc(region, 0, 10, total=1)
    region.r.procnum = procnum
    n = len(region.active_procs())
    assert n == (0 if procnum < 0 else 1)


def test_device_count_is_clamped(region):
    region.r.num_devices = 999
    assert region.device_num() == MAX_DEVICES


def test_setters_are_visible_to_another_mapping(region, tmp_path):
    other = SharedRegion(region.path, writable=False)
    region.set_recent_kernel(-1)
    region.set_utilization_switch(1)
    region.set_memory_limit(123)
    region.set_cu_limit(25)
    other.refresh()
    assert (other.recent_kernel(), other.utilization_switch()) == (-1, 1)
    assert other.memory_limit(0) == 123 and other.memory_limit(1) == 123
    assert other.memory_limit(2) == 1 << 30          # beyond num_devices: untouched
    assert int(other.r.cu_limit[0]) == 25
    other.close()


def test_read_only_mapping_is_a_snapshot_until_refresh(region):
    ro = SharedRegion(region.path, writable=False)
    region.r.priority = 7
    assert ro.priority() == 0
    ro.refresh()
    assert ro.priority() == 7
    ro.close()


def test_uuid_accessors(region):
    region.r.uuids[0].value = b"GPU-1234"
    assert region.uuid(0) == "GPU-1234" and region.is_valid_uuid(0)
    assert region.uuid(1) == "" and not region.is_valid_uuid(1)


@pytest.mark.parametrize("content", [b"", b"\0" * 100, b"\xff" * REGION_SIZE])
def test_bad_files_are_rejected(tmp_path, content):
    p = tmp_path / "bad.cache"
    p.write_bytes(content)
    with pytest.raises(ValueError):
        SharedRegion(str(p))


def test_concurrent_writers_to_distinct_slots(region):
    """Many threads updating their own slots: no torn totals (8-byte aligned stores)."""
    def work(i):
        for v in range(2000):
            region.r.procs[i].used[0].total = v
        region.r.procs[i].used[0].total = 1000 + i
        region.r.procs[i].status = 1
    for i in range(8):
        region.r.procs[i].pid = 100 + i
    region.r.procnum = 8
    ts = [threading.Thread(target=work, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert region.memory_total(0) == sum(1000 + i for i in range(8))


# ------------------------------------------------------------------ lister
def _mk(base, uid, ctr, name="r.cache"):
    d = base / "vgpu" / "containers" / f"{uid}_{ctr}"
    d.mkdir(parents=True, exist_ok=True)
    r = SharedRegion.create(str(d / name))
    r.close()
    return d


def test_lister_without_pod_source_maps_everything(tmp_path):
    _mk(tmp_path, "u1", "a")
    _mk(tmp_path, "u2", "b")
    lister = ContainerLister(str(tmp_path), None)
    lister.update()
    assert sorted((c.pod_uid, c.container) for c in lister.list_containers()) == [("u1", "a"), ("u2", "b")]


def test_lister_drops_vanished_directories_and_maps_new_ones(tmp_path):
    d1 = _mk(tmp_path, "u1", "a")
    lister = ContainerLister(str(tmp_path), None)
    lister.update()
    assert len(lister.list_containers()) == 1
    for f in d1.iterdir():
        f.unlink()
    d1.rmdir()
    _mk(tmp_path, "u3", "c")
    lister.update()
    assert [c.pod_uid for c in lister.list_containers()] == ["u3"]


def test_lister_ignores_foreign_entries(tmp_path):
    base = tmp_path / "vgpu" / "containers"
    base.mkdir(parents=True)
    (base / "nounderscore").mkdir()
    (base / "file_x").write_text("x")
    (base / "u9_empty").mkdir()
    lister = ContainerLister(str(tmp_path), None)
    lister.update()
    assert lister.list_containers() == []


def test_lister_pod_listing_failure_keeps_mappings(tmp_path):
    _mk(tmp_path, "u1", "a")

    def broken():
        raise RuntimeError("api down")
    lister = ContainerLister(str(tmp_path), broken, resync_interval=0)
    lister.update()
    assert len(lister.list_containers()) == 1
    assert (tmp_path / "vgpu" / "containers" / "u1_a").exists()


def test_lister_missing_hook_path(tmp_path):
    lister = ContainerLister(str(tmp_path / "nope"), None)
    lister.update()
    assert lister.list_containers() == []


def test_region_file_size_matches_struct(tmp_path):
    d = _mk(tmp_path, "u1", "a")
    assert os.path.getsize(d / "r.cache") == REGION_SIZE


def _fake_proc(root, pid, nspids, cgroup):
    d = root / str(pid)
    d.mkdir(parents=True)
    (d / "status").write_text(f"Name:\tpython\nPid:\t{pid}\nNSpid:\t" + "\t".join(map(str, nspids)) + "\n")
    (d / "cgroup").write_text(cgroup)


def test_host_pids_filled_from_nspid_and_pod_cgroup(region, tmp_path):
    """The monitor maps slot pids (container pid namespace) to host pids: the
    NSpid tail must equal the slot pid and the cgroup must name the pod UID."""
    from types import SimpleNamespace

    from k8s_vgpu_scheduler_amd.monitor.hostpid import fill_host_pids

    uid = "3f1c2b7a-0d1e-4a5b-9c8d-112233445566"
    proc = tmp_path / "proc"
    # cgroupfs layout, pid 7 inside the container = host 4107
    _fake_proc(proc, 4107, [4107, 7], f"0::/kubepods/burstable/pod{uid}/abc123\n")
    # systemd layout (dashes -> underscores), pid 8 = host 4108
    _fake_proc(proc, 4108, [4108, 8], f"0::/kubepods.slice/kubepods-pod{uid.replace('-', '_')}.slice/cri-x\n")
    # same container pid 9 in two pods: only the one in our pod may match
    _fake_proc(proc, 4109, [4109, 9], f"0::/kubepods/pod{uid}/c1\n")
    _fake_proc(proc, 5109, [5109, 9], "0::/kubepods/podffffffff-0000-0000-0000-000000000000/c2\n")
    # pid 10 twice in our pod (ambiguous): left unfilled
    _fake_proc(proc, 4110, [4110, 10], f"0::/kubepods/pod{uid}/c1\n")
    _fake_proc(proc, 4210, [4210, 10], f"0::/kubepods/pod{uid}/c3\n")
    (proc / "self").mkdir()
    for i, pid in enumerate((7, 8, 9, 10, 11)):
        _proc(region, i, pid)
    region.r.procs[5].pid, region.r.procs[5].status, region.r.procs[5].hostpid = 12, 1, 999  # already known
    region.r.procnum = 6
    c = SimpleNamespace(pod_uid=uid, region=region)
    assert fill_host_pids([c], proc_root=str(proc)) == 3
    assert [region.r.procs[i].hostpid for i in range(6)] == [4107, 4108, 4109, 0, 0, 999]
    assert fill_host_pids([c], proc_root=str(proc)) == 0      # nothing new to fill
