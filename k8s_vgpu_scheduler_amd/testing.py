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
