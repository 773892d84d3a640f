"""Control-plane benchmark: Filter + Bind on a synthetic MI355X cluster (no GPU).

BASELINE.json configs 1 and 5: "scheduler extender filter/score on fake-device
node annotations" and "8 vGPU slices/GPU x 8 MI355X = 64 schedulable vGPUs;
binpack vs spread".  Builds ``--nodes`` nodes of 8 MI355X (split 8 -> 64
vGPUs each, full-mesh xGMI scores) in the in-process fake API server, then
schedules a pod mix until the cluster is full or ``--pods`` is reached.  Each
pod goes through the real path: webhook admission -> /filter -> /bind ->
device-plugin lock release (pod_allocation_try_success).  Reports filter and
bind latency percentiles and placement quality (GPUs / nodes touched,
fragmentation) for each node policy x GPU policy.

    python -m k8s_vgpu_scheduler_amd.bench.scheduler --nodes 8 --out profiles/scheduler_bench.json
"""

from __future__ import annotations

import argparse
import json
import random
import statistics
import time
from pathlib import Path

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device.amd.device import SUPPORT_ANNOS
from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.deviceplugin import server as dp
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.scheduler.webhook import Webhook
from k8s_vgpu_scheduler_amd.testing import amd_container, amd_node, amd_pod, full_mesh_scores, mi355x_devices

# (weight, gpus, gpumem MiB, gpucores %): serving slices, small jobs, 2-GPU TP pods, whole cards
MIX = [(6, 1, 36864, 25), (4, 1, 16384, 12), (2, 1, 73728, 50), (1, 2, 65536, 50), (1, 1, None, 100)]


def _pct(xs, p):
    if not xs:
        return None
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(p / 100.0 * len(xs)))] * 1e3, 3)


def run(nodes: int, pods: int, node_policy: str, gpu_policy: str, seed: int = 0) -> dict:
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config(gpu_policy=gpu_policy)
    get_local_cache().quotas.clear()
    names = [f"node{i}" for i in range(nodes)]
    for n in names:
        c.create("nodes", amd_node(n, scores=full_mesh_scores(mi355x_devices(n))))
    s = Scheduler(c, SchedulerConfig(node_scheduler_policy=node_policy, gpu_scheduler_policy=gpu_policy))
    s.start()
    s.register()
    wh = Webhook("hami-scheduler")
    rng = random.Random(seed)
    weights = [m[0] for m in MIX]
    t_filter, t_bind, placed, rejected = [], [], 0, 0
    for i in range(pods):
        _, g, mem, cores = rng.choices(MIX, weights)[0]
        pod = amd_pod(f"p{i}", containers=[amd_container(gpu=g, mem=mem, cores=cores)])
        rev = wh.handle_review({"request": {"uid": str(i), "object": pod}})
        if not rev["response"]["allowed"]:
            rejected += 1
            continue
        c.create("pods", pod)
        cur = c.get_pod("default", f"p{i}")
        t0 = time.perf_counter()
        res = s.filter({"Pod": cur, "NodeNames": names})
        t_filter.append(time.perf_counter() - t0)
        if not res.get("NodeNames"):
            rejected += 1
            c.delete("pods", f"p{i}", "default")
            if rejected > 20:
                break
            continue
        node = res["NodeNames"][0]
        cur = c.get_pod("default", f"p{i}")
        t0 = time.perf_counter()
        b = s.bind({"PodName": f"p{i}", "PodNamespace": "default", "PodUID": cur["metadata"]["uid"],
                    "Node": node})
        t_bind.append(time.perf_counter() - t0)
        if b["Error"]:
            rejected += 1
            continue
        # device plugin side: everything allocated -> release the node lock
        c.patch_pod("default", f"p{i}", {"metadata": {"annotations": {
            "hami.io/amd-devices-to-allocate": ""}}})
        dp.pod_allocation_try_success(node, c.get_pod("default", f"p{i}"))
        placed += 1
    # placement quality from the allocation annotations
    gpus_used, nodes_used = set(), set()
    mem_used = {}
    for p in c.list_pods():
        ann = (p["metadata"].get("annotations") or {}).get(SUPPORT_ANNOS)
        node = (p.get("spec") or {}).get("nodeName")
        if not ann or not node:
            continue
        nodes_used.add(node)
        for ctr in codec.decode_pod_devices({"AMD": SUPPORT_ANNOS}, {SUPPORT_ANNOS: ann}).get("AMD", []):
            for d in ctr:
                gpus_used.add(d.uuid)
                mem_used[d.uuid] = mem_used.get(d.uuid, 0) + d.usedmem
    total_gpus = nodes * 8
    return {"node_policy": node_policy, "gpu_policy": gpu_policy, "nodes": nodes, "vgpus": nodes * 64,
            "pods_placed": placed, "pods_rejected": rejected,
            "filter_ms_p50": _pct(t_filter, 50), "filter_ms_p99": _pct(t_filter, 99),
            "filter_ms_mean": round(statistics.mean(t_filter) * 1e3, 3) if t_filter else None,
            "bind_ms_p50": _pct(t_bind, 50), "bind_ms_p99": _pct(t_bind, 99),
            "gpus_touched": len(gpus_used), "gpus_total": total_gpus, "nodes_touched": len(nodes_used),
            "mean_hbm_fill_of_touched_gpus": round(statistics.mean(
                v / 294912 for v in mem_used.values()), 3) if mem_used else None}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=8)
    ap.add_argument("--pods", type=int, default=None, help="default: half the vGPUs (placement differs)")
    ap.add_argument("--full", action="store_true", help="also fill the cluster until rejection")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    pods = a.pods or a.nodes * 64 // 4
    rows = []
    for node_policy in ("binpack", "spread"):
        for gpu_policy in ("binpack", "spread"):
            r = run(a.nodes, pods, node_policy, gpu_policy)
            print(json.dumps(r), flush=True)
            rows.append(r)
    if a.full:
        r = run(a.nodes, a.nodes * 64 * 2, "binpack", "binpack")
        r["mode"] = "fill"
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.out:
        Path(a.out).parent.mkdir(parents=True, exist_ok=True)
        Path(a.out).write_text(json.dumps(rows, indent=1))
    return rows


if __name__ == "__main__":
    main()
