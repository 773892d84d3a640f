"""libmivgpu.so under the real HIP runtime on an MI355X (PyTorch workloads in
child processes, the shim preloaded the way the device plugin injects it).

Mirrors the reference's libvgpu behaviour checks (HBM limit virtualisation and
OOM, shared-region accounting read by vGPUmonitor, SM-limit duty cycling) and
the CU-partition placement that replaces MPS/MIG on MI355X.
"""

import os
import tempfile

import pytest

from k8s_vgpu_scheduler_amd.shim.probe import run_child, run_parallel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tmp():
    from k8s_vgpu_scheduler_amd.utils import build
    if not build.SHIM_SO.exists() or not build.OPS_SO.exists():
        build.build_all()
    return tempfile.mkdtemp(prefix="mivgpu-gputest-")


def test_hbm_limit_virtualised_and_enforced(tmp):
    r = run_child("matmul", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "a.cache"),
                             "HIP_DEVICE_MEMORY_LIMIT_0": "4096m"}, True,
                  ["--n", "2048", "--iters", "5", "--oom-probe-mib", "5000"])
    assert r["rc"] == 0, r.get("stderr")
    assert r["mem_total_mib"] == 4096 and r["props_total_mib"] == 4096
    assert r["mem_free_mib"] <= 4096
    assert r["oom_probe"] == "oom"


def test_allocation_accounting_visible_to_monitor(tmp):
    cache = os.path.join(tmp, "b.cache")
    r = run_child("region", {"MIVGPU_SHARED_CACHE": cache, "HIP_DEVICE_MEMORY_LIMIT_0": "8192m",
                             "MIVGPU_DEVICE_UUIDS": "GPU-test"}, True, ["--oom-probe-mib", "1024"])
    assert r["rc"] == 0, r.get("stderr")
    assert r["self_found"] and r["limit_mib"] == 8192
    assert r["self_buffer_mib"] >= 1024 and r["dev_used_mib"] >= 1024
    assert r["launches"] >= 1
    assert r["uuid"] == "GPU-test"


def test_two_processes_share_one_container_limit(tmp):
    cache = os.path.join(tmp, "c.cache")
    env = {"MIVGPU_SHARED_CACHE": cache, "HIP_DEVICE_MEMORY_LIMIT_0": "3072m"}
    # each holds 2 GiB for 8 s after probing: the container-wide limit admits one
    outs = run_parallel("matmul", [env, env], True, ["--n", "1024", "--iters", "5",
                                                     "--oom-probe-mib", "2048", "--hold-s", "8"])
    assert all(o["rc"] == 0 for o in outs), outs
    assert sorted(o["oom_probe"] for o in outs) == ["allocated", "oom"]


def test_cu_mask_confines_to_balanced_cus():
    r = run_child("hwid", {"HSA_CU_MASK": "0:0-31"}, False, [])
    assert r["rc"] == 0, r.get("stderr")
    assert r["distinct"] == 32
    assert r["xccs"] == list(range(8))   # CU i lives on XCD i % 8


def test_governor_duty_cycle(tmp):
    base = run_child("matmul", {}, False, ["--n", "8192", "--iters", "200"])
    r = run_child("matmul", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "d.cache"), "HIP_DEVICE_CORE_LIMIT": "50",
                             "GPU_CORE_UTILIZATION_POLICY": "force"}, True, ["--n", "8192", "--iters", "200"])
    assert base["rc"] == 0 and r["rc"] == 0, (base.get("stderr"), r.get("stderr"))
    ratio = r["tflops"] / base["tflops"]
    assert 0.35 <= ratio <= 0.65, ratio
    assert r["gates"] > 0 and r["gate_held_ms"] > 0


def test_shim_overhead_unlimited(tmp):
    base = run_child("matmul", {}, False, ["--n", "8192", "--iters", "100"])
    r = run_child("matmul", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "e.cache")}, True,
                  ["--n", "8192", "--iters", "100"])
    assert base["rc"] == 0 and r["rc"] == 0
    assert r["tflops"] >= 0.97 * base["tflops"], (r["tflops"], base["tflops"])
