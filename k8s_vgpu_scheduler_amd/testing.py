"""Fixtures for GPU-less tests and demos: fake MI355X nodes and pods.

The reference tests the scheduler with synthetic ``DeviceInfo`` literals and
node annotations on a fake clientset (e.g.
pkg/scheduler/score_test.go:76-3290); these helpers build the same shapes for
MI355X (288 GB = 294912 MiB, 256 CUs, 8 xGMI-connected GPUs per node).
"""

from __future__ import annotations

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device.amd.device import PAIR_SCORE_ANNOS, REGISTER_ANNOS
from k8s_vgpu_scheduler_amd.device.types import DeviceInfo
from k8s_vgpu_scheduler_amd.k8s.fake import container, make_node, make_pod

MI355X_MEM_MIB = 294912
MI355X_CUS = 256
MI355X_TYPE = "AMD Instinct MI355X"


def mi355x_devices(node: str, n: int = 8, split: int = 8, mem: int = MI355X_MEM_MIB, cus: int = MI355X_CUS,
                   numa_per: int = 4, health: bool = True) -> list[DeviceInfo]:
    return [DeviceInfo(id=f"{node}-gpu{i}", index=i, count=split, devmem=mem, devcore=cus, type=MI355X_TYPE,
                       numa=i // numa_per if numa_per else 0, mode="hami-core", health=health)
            for i in range(n)]


def full_mesh_scores(devs: list[DeviceInfo], score: int = 100, degraded: dict | None = None) -> dict:
    """MI355X: every pair is one direct xGMI link; `degraded` overrides pairs."""
    s = {d.id: {o.id: score for o in devs if o.id != d.id} for d in devs}
    for (a, b), v in (degraded or {}).items():
        s[a][b] = v
        s[b][a] = v
    return s


def amd_node(name: str, n: int = 8, split: int = 8, scores: dict | None = None, annotations: dict | None = None,
             labels: dict | None = None, **kw) -> dict:
    devs = mi355x_devices(name, n, split, **kw)
    annos = {REGISTER_ANNOS: codec.marshal_node_devices(devs)}
    if scores is not None:
        annos[PAIR_SCORE_ANNOS] = codec.encode_pair_scores(scores)
    annos.update(annotations or {})
    cap = {"amd.com/gpu": str(n * split)}
    return make_node(name, annotations=annos, labels=labels, capacity=cap, allocatable=cap)


def amd_container(name: str = "main", gpu: int | None = 1, mem: int | None = None, cores: int | None = None,
                  mem_pct: int | None = None, priority: int | None = None) -> dict:
    limits = {}
    if gpu is not None:
        limits["amd.com/gpu"] = gpu
    if mem is not None:
        limits["amd.com/gpumem"] = mem
    if cores is not None:
        limits["amd.com/gpucores"] = cores
    if mem_pct is not None:
        limits["amd.com/gpumem-percentage"] = mem_pct
    if priority is not None:
        limits["amd.com/priority"] = priority
    return container(name, limits=limits)


def amd_pod(name: str, namespace: str = "default", containers: list | None = None, init: list | None = None,
            annotations: dict | None = None, labels: dict | None = None, uid: str | None = None, **ctr_kw) -> dict:
    ctrs = containers if containers is not None else [amd_container(**ctr_kw)]
    return make_pod(name, namespace, containers=ctrs, init_containers=init, annotations=annotations,
                    labels=labels, uid=uid or f"uid-{namespace}-{name}")


def write_mi355x_sysfs(root, n: int = 8, degraded: dict | None = None, pcie_pairs=(), serial_base: int = 0xAE8C1614E27CC400,
                       numa_per: int = 4, product: str = "AMD Instinct MI355 OAM") -> tuple:
    """A KFD topology + DRM/PCI sysfs tree of one 8 x MI355X node, shaped like
    the one measured on the hardware (tests/fixtures/mi355x_8gpu_kfd_links.json):
    CPU nodes 0-1, GPU nodes 2..n+1, each GPU with one PCIe io_link to its
    socket (type 2, weight 20, 64000 MB/s) and one xGMI io_link to every peer
    (type 11, weight 15, 76000 MB/s).  ``degraded`` = {(i, j): MB/s} lowers a
    pair's xGMI bandwidth; ``pcie_pairs`` turns pairs into PCIe peers.
    Returns (kfd_nodes_dir, drm_dir)."""
    import os
    from pathlib import Path

    root = Path(root)
    kfd, drm, pci = root / "kfd" / "topology" / "nodes", root / "drm", root / "pci"
    degraded = {tuple(sorted(k)): v for k, v in (degraded or {}).items()}
    pcie = {tuple(sorted(p)) for p in pcie_pairs}
    buses = [0x05, 0x15, 0x65, 0x75, 0x85, 0x95, 0xE5, 0xF5][:n] + [0x100 + i for i in range(max(0, n - 8))]
    for c in range(2):
        d = kfd / str(c)
        (d / "io_links").mkdir(parents=True)
        (d / "gpu_id").write_text("0\n")
        (d / "properties").write_text("cpu_cores_count 64\nsimd_count 0\nlocation_id 0\ndomain 0\n")
    for i in range(n):
        node = kfd / str(2 + i)
        (node / "mem_banks" / "0").mkdir(parents=True)
        minor = 128 + 8 * i
        (node / "gpu_id").write_text(f"{16000 + 1111 * i}\n")
        (node / "properties").write_text(
            f"cpu_cores_count 0\nsimd_count 1024\nsimd_per_cu 4\nlocation_id {buses[i] << 8}\ndomain 0\n"
            f"unique_id {serial_base + i}\ndevice_id 30115\ndrm_render_minor {minor}\nnum_xcc 8\n")
        (node / "mem_banks" / "0" / "properties").write_text(f"heap_type 1\nsize_in_bytes {288 << 30}\n")
        links = [(i // numa_per if numa_per else 0, 2, 20, 64000)]
        for j in range(n):
            if j == i:
                continue
            key = tuple(sorted((i, j)))
            if key in pcie:
                links.append((2 + j, 2, 40, 64000))
            else:
                bw = degraded.get(key, 76000)
                links.append((2 + j, 11, 15, bw))
        for k, (to, t, w, bw) in enumerate(links):
            ld = node / "io_links" / str(k)
            ld.mkdir(parents=True)
            ld.joinpath("properties").write_text(
                f"type {t}\nnode_from {2 + i}\nnode_to {to}\nweight {w}\nmin_bandwidth {bw if t == 11 else 0}\n"
                f"max_bandwidth {bw}\n")
        dev = pci / f"0000:{buses[i]:02x}:00.0"
        (dev / "drm" / f"card{i}").mkdir(parents=True)
        (dev / "numa_node").write_text(f"{i // numa_per if numa_per else 0}\n")
        (dev / "current_compute_partition").write_text("SPX\n")
        (dev / "product_name").write_text(product + "\n")
        (drm / f"renderD{minor}").mkdir(parents=True)
        os.symlink(dev, drm / f"renderD{minor}" / "device")
    return kfd, drm
