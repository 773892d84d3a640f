"""sysfs/KFD discovery on a synthetic sysfs tree: one SPX MI355X plus one in
CPX (8 KFD nodes, PCI functions .0-.7 of one device), NUMA/BDF/card minor from
the DRM render node's PCI device, partition grouping, and the partition write."""

import os

from k8s_vgpu_scheduler_amd import smi


def _tree(tmp_path):
    kfd, drm, pci = tmp_path / "kfd", tmp_path / "drm", tmp_path / "pci"
    (kfd / "0").mkdir(parents=True)
    (kfd / "0" / "properties").write_text("cpu_cores_count 96\nsimd_count 0\n")   # the CPU node
    gpus = [("dc", 0, 256, 288 << 30, 128, 0, "SPX")] + \
           [("1b", f, 32, 36 << 30, 136 + f, 1 + f, "CPX") for f in range(8)]
    for i, (bus, fn, cus, mem, minor, card, part) in enumerate(gpus, start=1):
        n = kfd / str(i)
        (n / "mem_banks" / "0").mkdir(parents=True)
        (n / "properties").write_text(f"simd_count {cus * 4}\nsimd_per_cu 4\nunique_id {0x1000 + i}\n"
                                      f"drm_render_minor {minor}\n")
        (n / "mem_banks" / "0" / "properties").write_text(f"heap_type 1\nsize_in_bytes {mem}\n")
        dev = pci / f"0000:{bus}:00.{fn}"
        (dev / "drm" / f"card{card}").mkdir(parents=True)
        (dev / "numa_node").write_text("1\n" if bus == "1b" else "0\n")
        (dev / "current_compute_partition").write_text(part + "\n")
        (dev / "product_name").write_text("AMD Instinct MI355X\n")
        (drm / f"renderD{minor}").mkdir(parents=True)
        os.symlink(dev, drm / f"renderD{minor}" / "device")
    return kfd, drm, pci


def test_sysfs_backend_reads_topology_and_partitions(tmp_path):
    kfd, drm, pci = _tree(tmp_path)
    b = smi.SysfsBackend(kfd, drm)
    gs = b.gpus()
    assert len(gs) == 9
    spx, cpx = gs[0], gs[1:]
    assert (spx.cus, spx.memory_mib, spx.numa, spx.bdf, spx.card_minor, spx.compute_partition) == \
        (256, 288 << 10, 0, "0000:dc:00.0", 0, "SPX")
    assert spx.physical == 0 and spx.partition_index == 0
    assert all(g.physical == 1 and g.cus == 32 and g.numa == 1 and g.compute_partition == "CPX" for g in cpx)
    assert [g.partition_index for g in cpx] == list(range(8))
    assert [g.render_minor for g in cpx] == list(range(136, 144))
    assert len({g.uuid for g in gs}) == 9
    b.set_compute_partition(1, "dpx")
    assert (pci / "0000:1b:00.0" / "current_compute_partition").read_text() == "DPX\n"
    # the event source is amd-smi's; sysfs has none and says so
    assert b.wait_health_events(gs, 0.01) is None


def test_serialized_backend_never_overlaps_calls():
    """The monitor wraps its backend so that scrapes (HTTP thread) and the
    feedback pass (host truth's GPU id map) never call amd-smi at once."""
    import threading
    import time

    from k8s_vgpu_scheduler_amd.smi import FakeBackend, SerializedBackend

    class Probe(FakeBackend):
        inside = 0
        worst = 0

        def gpus(self):
            Probe.inside += 1
            Probe.worst = max(Probe.worst, Probe.inside)
            time.sleep(0.002)
            Probe.inside -= 1
            return super().gpus()

    b = SerializedBackend(Probe(2))
    ths = [threading.Thread(target=lambda: [b.gpus() for _ in range(10)]) for _ in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert Probe.worst == 1 and b.name == "fake" and len(b.gpus()) == 2
