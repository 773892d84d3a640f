"""Request extraction tables for the MI355X backend
(AMDDevices.generate_resource_requests; reference
pkg/device/nvidia/device.go GenerateResourceRequests, the AMD backend's
pkg/device/amd/device.go:333-344): counts, HBM in MiB or %, defaults, the
memory factor and the core clamp."""

import pytest

from k8s_vgpu_scheduler_amd.device.amd.device import AMDConfig, init_amd_device
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
from k8s_vgpu_scheduler_amd.testing import amd_container


@pytest.fixture(scope="module", autouse=True)
def _client():
    init_global_client(FakeCluster())


def req(ctr, **cfg):
    return init_amd_device(AMDConfig(**cfg)).generate_resource_requests(ctr)


def key(r):
    return (r.nums, r.memreq, r.mem_percentage_req, r.coresreq)


@pytest.mark.parametrize("name,ctr,cfg,want", [
    ("no gpu request", amd_container(gpu=None, mem=100), {}, (0, 0, 101, 0)),
    ("whole card by default", amd_container(gpu=1), {}, (1, 0, 100, 0)),
    ("memory in MiB", amd_container(gpu=1, mem=36864), {}, (1, 36864, 101, 0)),
    ("memory as quantity string", {"name": "c", "resources": {"limits": {"amd.com/gpu": "2",
                                                                          "amd.com/gpumem": "1k"}}}, {},
     (2, 1000, 101, 0)),
    ("percentage", amd_container(gpu=1, mem_pct=25), {}, (1, 0, 25, 0)),
    ("percentage above 100 clamps", amd_container(gpu=1, mem_pct=250), {}, (1, 0, 100, 0)),
    ("percentage 0 falls back to the whole card", amd_container(gpu=1, mem_pct=0), {}, (1, 0, 100, 0)),
    ("default memory", amd_container(gpu=1), {"default_memory": 4096}, (1, 4096, 101, 0)),
    ("memory factor", amd_container(gpu=1, mem=10), {"memory_factor": 1024}, (1, 10240, 101, 0)),
    ("default cores", amd_container(gpu=1, mem=10), {"default_cores": 25}, (1, 10, 101, 25)),
    ("explicit cores override default", amd_container(gpu=1, mem=10, cores=50), {"default_cores": 25},
     (1, 10, 101, 50)),
    ("cores above 100 clamp to a whole card", amd_container(gpu=1, mem=10, cores=150), {}, (1, 10, 101, 100)),
    ("zero gpus is no request", amd_container(gpu=0, mem=10), {}, (0, 0, 101, 0)),
    ("negative gpus is no request", amd_container(gpu=-1), {}, (0, 0, 101, 0)),
    ("fractional gpus is no request", {"name": "c", "resources": {"limits": {"amd.com/gpu": "500m"}}}, {},
     (0, 0, 101, 0)),
    ("negative memory rejects the request", amd_container(gpu=1, mem=-5), {}, (0, 0, 101, 0)),
    ("memory overflowing int32 after the factor", amd_container(gpu=1, mem=2 ** 22), {"memory_factor": 1024},
     (0, 0, 101, 0)),
    ("negative cores rejects the request", amd_container(gpu=1, cores=-1), {}, (0, 0, 101, 0)),
])
def test_generate_resource_requests(name, ctr, cfg, want):
    assert key(req(ctr, **cfg)) == want, name


def test_requests_read_from_requests_when_limits_absent():
    ctr = {"name": "c", "resources": {"requests": {"amd.com/gpu": "1", "amd.com/gpumem": "512"}}}
    assert key(req(ctr)) == (1, 512, 101, 0)      # Limits first, then Requests (as the reference)


def test_custom_resource_names():
    ctr = {"name": "c", "resources": {"limits": {"example.com/vgpu": "1", "example.com/vmem": "64"}}}
    r = req(ctr, resource_count_name="example.com/vgpu", resource_memory_name="example.com/vmem")
    assert key(r) == (1, 64, 101, 0)
