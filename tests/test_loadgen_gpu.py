"""Hand-written load generators (csrc/ops/loadgen.hip) and the isolation
behaviour they are used to measure: CU partitions and the governor."""

import os
import tempfile

import pytest
import torch

from k8s_vgpu_scheduler_amd import ops
from k8s_vgpu_scheduler_amd.shim.probe import run_child

pytestmark = pytest.mark.gpu


def test_stream_copy_exact():
    src = torch.empty((64 << 20) // 4, dtype=torch.int32, device="cuda").random_()
    dst = torch.zeros_like(src)
    ops.stream_copy(src, dst)
    assert torch.equal(src, dst)
    tail = torch.arange(1000, dtype=torch.int32, device="cuda")      # 4000 B: tail loop only
    out = torch.zeros_like(tail)
    ops.stream_copy(tail, out)
    assert torch.equal(tail, out)
    with pytest.raises(RuntimeError):
        ops.stream_copy(src[:3], dst[:3])                             # 12 B: not 16-byte sized


def test_stream_read_checksum_exact():
    src = torch.empty((32 << 20) // 4, dtype=torch.int32, device="cuda").random_()
    got = ops.stream_read(src).item() & (2 ** 64 - 1)
    exp = int((src.cpu().numpy().view("uint32").astype("uint64")).sum()) & (2 ** 64 - 1)
    assert got == exp


def test_mfma_burn_runs_at_matrix_core_rate():
    r = run_child("mfma", {}, False, ["--iters", "20"])
    assert r["rc"] == 0, r.get("stderr")
    assert r["finite"]
    assert r["tflops"] > 500, r     # dense bf16 peak is ~2.5 PF/s


def test_cu_partition_scales_matrix_core_throughput():
    full = run_child("mfma", {}, False, ["--iters", "20"])
    quarter = run_child("mfma", {"HSA_CU_MASK": "0:0-63"}, False, ["--iters", "20"])
    assert full["rc"] == 0 and quarter["rc"] == 0
    ratio = quarter["tflops"] / full["tflops"]
    assert 0.18 <= ratio <= 0.32, ratio


def test_governor_duty_cycle_on_handwritten_load():
    tmp = tempfile.mkdtemp(prefix="mivgpu-lg-")
    probe = run_child("mfma", {}, False, ["--iters", "60"])
    assert probe["rc"] == 0, probe.get("stderr")
    # ~1.5 s of work unthrottled: the bucket's 100 ms burst is a small part of it
    iters = str(max(60, int(60 * 1.5 / max(probe["seconds"], 1e-3))))
    full = run_child("mfma", {}, False, ["--iters", iters])
    half = run_child("mfma", {"MIVGPU_SHARED_CACHE": os.path.join(tmp, "g.cache"), "HIP_DEVICE_CORE_LIMIT": "50",
                              "GPU_CORE_UTILIZATION_POLICY": "force"}, True, ["--iters", iters])
    assert full["rc"] == 0 and half["rc"] == 0, half.get("stderr")
    ratio = half["tflops"] / full["tflops"]
    assert 0.42 <= ratio <= 0.6, ratio
    assert half["gates"] > 0


def test_hipstream_under_shim_has_no_overhead():
    tmp = tempfile.mkdtemp(prefix="mivgpu-lg-")
    # ~0.1 s of copying per run (20 iterations were ~9 ms: one scheduling blip
    # moved the ratio by 5 %)
    # A B B A A B, best of three each: the copy rate is bimodal on this box
    # with or without the shim (~4670 or ~4370 GB/s per process, natively
    # too: scripts/probe/hipstream_ab.py), and two shim runs both landing low
    # failed a best-of-two comparison
    runs = {False: [], True: []}
    for i, with_shim in enumerate((False, True, True, False, False, True)):
        env = {"MIVGPU_SHARED_CACHE": os.path.join(tmp, f"s{i}.cache")} if with_shim else {}
        r = run_child("hipstream", env, with_shim, ["--n", "1024", "--iters", "200"])
        assert r["rc"] == 0 and r["exact"], r
        runs[with_shim].append(r["gbps"])
    base, shim = max(runs[False]), max(runs[True])
    assert shim >= 0.95 * base, runs
