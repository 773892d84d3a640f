"""End to end across process and protocol boundaries (the reference's test/e2e
tier): the real scheduler, device plugin and monitor binaries
against an HTTP API server, driven the way kube-apiserver (webhook),
kube-scheduler (extender /filter, /bind) and the kubelet (device-plugin gRPC)
drive them.  The "container" is the shim-preloaded mock-HIP driver, so the
HBM limit, the shared region and the monitor's per-pod metrics are real.
The GPU variant of this test (tests/test_e2e_gpu.py) runs a PyTorch workload
on the MI355X instead."""

import json
import subprocess

import pytest

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.e2e.harness import E2ECluster, container_env, samples, wait_for
from k8s_vgpu_scheduler_amd.testing import amd_pod

MIB = 1 << 20


@pytest.fixture(scope="module")
def cluster(tmp_path_factory, native_build):
    with E2ECluster(str(tmp_path_factory.mktemp("e2e")), fake_gpus=2, split=4) as cl:
        yield cl


def test_binaries_register_the_node(cluster):
    anns = cluster.api.cluster.get("nodes", "node1")["metadata"]["annotations"]
    devs = codec.unmarshal_node_devices(anns["hami.io/node-amd-register"])
    assert len(devs) == 2 and all(d.count == 4 and d.devcore == 256 for d in devs)
    st = cluster.api.cluster.get("nodes", "node1")["status"]
    assert st["allocatable"]["amd.com/gpu"] == "8"          # kubelet saw 2 GPUs x 4 replicas
    assert {m for m, _ in cluster.api.requests} >= {"GET", "PATCH"}   # all through HTTP


def test_pod_lifecycle(cluster, native_build):
    cl = cluster
    pod = cl.submit(amd_pod("vgpu-a", mem=8192, cores=25))
    assert pod["spec"]["schedulerName"] == "hami-scheduler"        # set by the webhook
    assert cl.schedule("default", "vgpu-a") == "node1"
    allocs = cl.start_containers("default", "vgpu-a")
    envs = allocs[0]["envs"]
    assert envs["HIP_DEVICE_MEMORY_LIMIT_0"] == "8192m" and envs["GPU_MAX_HW_QUEUES"] == "2"
    assert codec.ranges_count(codec.parse_ranges(envs["HSA_CU_MASK"].split(":", 1)[1])) == 64
    anns = cl.api.cluster.get("pods", "vgpu-a", "default")["metadata"]["annotations"]
    assert anns["hami.io/bind-phase"] == "success"

    # the container: shim preloaded through the mounts, limit enforced, region visible to the monitor
    env = container_env(allocs[0])
    env["MOCKHIP_TOTAL_MIB"] = "65536"
    proc = subprocess.Popen([str(native_build["driver"]), "alloc", "3000", "meminfo", "alloc", "6000",
                             "sleep", "6000"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        def used():
            return [v for l, v in samples(cl.metrics("mon_metrics"), "hami_vgpu_memory_used_bytes")
                    if l.get("pod") == "vgpu-a"]
        vals = wait_for(used, 30, "monitor to report the container's HBM use")
        assert vals[0] == 3000 * MIB
        lim = [v for l, v in samples(cl.metrics("mon_metrics"), "hami_vgpu_memory_limit_bytes")
               if l.get("pod") == "vgpu-a"]
        assert lim == [8192 * MIB]
    finally:
        out, err = proc.communicate(timeout=30)
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert '"total_mib":8192' in lines[1] and '"rc":2' in lines[2], (out, err)   # 6000 more MiB: OOM

    alloc = [v for l, v in samples(cl.metrics("sched_metrics"), "hami_vgpu_memory_allocated_bytes")
             if l.get("pod") == "vgpu-a"]
    assert alloc == [8192 * MIB]
    # a pod that fits nowhere is filtered out, with the reason recorded
    cl.submit(amd_pod("too-big", mem=400000))
    assert cl.schedule("default", "too-big") is None
    # ...and stays Pending with a FilteringFailed event (test/e2e/pod/test_pod.go:108-122)
    evs = wait_for(lambda: [e for e in cl.api.cluster.list("events", "default")
                            if (e.get("involvedObject") or {}).get("name") == "too-big"
                            and e.get("reason") == "FilteringFailed"], 10, "FilteringFailed event")
    assert evs[0]["type"] == "Warning" and "node1" in evs[0]["message"], evs[0]
    assert not cl.api.cluster.get("pods", "too-big", "default")["spec"].get("nodeName")
    # deleting the pod releases its share in the scheduler
    cl.delete_pod("default", "vgpu-a")
    wait_for(lambda: not [1 for l, v in samples(cl.metrics("sched_metrics"), "hami_vgpu_memory_allocated_bytes")
                          if l.get("pod") == "vgpu-a"], 30, "scheduler to release the pod")
    assert all(v is None for v in cl.alive().values()), cl.alive()


def test_gputype_and_uuid_selection(cluster):
    """Type and uuid selectors through the real binaries (webhook, /filter,
    /bind, Allocate); the same cases run against the amd-smi registered card in
    tests/test_e2e_gpu.py."""
    cl = cluster
    devs = codec.unmarshal_node_devices(
        cl.api.cluster.get("nodes", "node1")["metadata"]["annotations"]["hami.io/node-amd-register"])
    cases = [("want-mi355", {"amd.com/use-gputype": "MI355"}, "node1"),
             ("avoid-mi355", {"amd.com/nouse-gputype": "MI355"}, None),
             ("want-mi300", {"amd.com/use-gputype": "MI300X"}, None),
             ("want-uuid", {"amd.com/use-gpu-uuid": devs[1].id}, "node1"),
             ("avoid-uuid", {"amd.com/nouse-gpu-uuid": ",".join(d.id for d in devs)}, None)]
    for name, annos, want in cases:
        cl.submit(amd_pod(name, mem=1024, cores=10, annotations=annos))
        assert cl.schedule("default", name) == want, (name, annos)
        if want:
            alloc = cl.start_containers("default", name)[0]
            if "use-gpu-uuid" in str(annos):
                assert devs[1].id in json.dumps(alloc), alloc
        cl.delete_pod("default", name)


def test_shimless_container_on_a_time_shared_node_is_evicted(tmp_path):
    """The shimless-eviction path end to end on the CPU (the GPU test's twin,
    tests/test_e2e_gpu.py): the real binaries on a time-sharing node
    (cuPartition: false), a fake KFD holding the container's VRAM under a host
    pid the monitor maps to the pod through the cgroup, no shim region: the
    monitor evicts the pod within --over-grant-passes (3) 5 s passes under the
    default block action."""
    import time
    kfd = tmp_path / "kfd"
    for i, (gid, bus) in enumerate(((4242, 0x11), (5151, 0x12)), start=1):
        n = kfd / "topology" / "nodes" / str(i)
        n.mkdir(parents=True)
        (n / "gpu_id").write_text(f"{gid}\n")
        (n / "properties").write_text(f"simd_count 1024\nlocation_id {bus << 8}\ndomain 0\n")
    procs = tmp_path / "proc"
    procs.mkdir()
    with E2ECluster(str(tmp_path / "cl"), fake_gpus=2, split=8, device_config={"amd": {"cuPartition": False}},
                    extra_env={"MIVGPU_KFD_SYSFS": str(kfd)}, monitor_args=["--proc-root", str(procs)]) as cl:
        cl.submit(amd_pod("rogue", mem=8192, cores=12))
        assert cl.schedule("default", "rogue") == "node1"
        alloc = cl.start_containers("default", "rogue")[0]
        env = container_env(alloc)
        uid = cl.api.cluster.get("pods", "rogue", "default")["metadata"]["uid"]
        gid = {"GPU-0000": 4242, "GPU-0001": 5151}[env["MIVGPU_DEVICE_UUIDS"].split(",")[0]]
        hp = 777777
        (kfd / "proc" / str(hp)).mkdir(parents=True)
        (kfd / "proc" / str(hp) / f"vram_{gid}").write_text(f"{2 << 30}\n")
        (procs / str(hp)).mkdir()
        (procs / str(hp) / "status").write_text(f"Name:\tpython\nNSpid:\t{hp}\t42\n")
        (procs / str(hp) / "cgroup").write_text(f"0::/kubepods.slice/pod{uid}/cri-rogue\n")
        t0 = time.monotonic()
        try:
            wait_for(lambda: ("default", "rogue") in cl.api.cluster.evictions, 60,
                     "the monitor to evict the shimless pod")
        except TimeoutError:
            pytest.fail("not evicted; monitor log:\n" + cl.logs("monitor")[-4000:])
        # three 5 s passes after the one that first sees it (slack for a loaded CPU)
        assert time.monotonic() - t0 <= 4 * 5 + 15
