"""The compute-partition manager against the real amd-smi backend (MI355X).

The reconfiguration itself (amdsmi_set_gpu_compute_partition) resets the GPU
and needs privileges this pool does not grant, so the setter is replaced by a
recorder; everything around it runs on the hardware: the current mode from
amd-smi, and the busy check from amd-smi's per-GPU process list -- a GPU with
a live process must never be reconfigured (plugin/migmgr.go:65-556 only
touches idle GPUs).
"""

import subprocess
import sys
import time

import pytest

from k8s_vgpu_scheduler_amd import smi
from k8s_vgpu_scheduler_amd.deviceplugin.partition import STATUS_ANNOS, PartitionManager
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster, make_node

pytestmark = pytest.mark.gpu

HOLDER = r"""
import time, torch
x = torch.ones(1 << 28, device="cuda")
torch.cuda.synchronize()
print("HOLDING", flush=True)
time.sleep(60)
"""


def test_manager_never_reconfigures_a_gpu_in_use(tmp_path):
    try:
        backend = smi.AmdSmiBackend()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"amd-smi unavailable: {e}")
    calls = []
    backend.set_compute_partition = lambda phys, mode: calls.append((phys, mode))   # never touch the card
    gpus = backend.gpus()
    phys = gpus[0].physical
    cur = PartitionManager(backend, "node1").current()
    assert cur[phys] in smi.PARTITION_MODES
    target = "CPX" if cur[phys] != "CPX" else "SPX"
    c = FakeCluster()
    init_global_client(c)
    c.create("nodes", make_node("node1", annotations={"mivgpu.io/partition-request": f"{phys}={target}"}))
    holder = subprocess.Popen([sys.executable, "-c", HOLDER], stdout=subprocess.PIPE, text=True)
    try:
        assert holder.stdout.readline().strip() == "HOLDING"
        deadline = time.time() + 20
        procs = []
        while time.time() < deadline and not procs:
            procs = [p for g in gpus if g.physical == phys for p in backend.processes(g)]
            time.sleep(0.5)
        assert procs, "amd-smi lists no process on a GPU that holds 1 GiB"
        mgr = PartitionManager(backend, "node1", lock_path=str(tmp_path / "apply.lock"))
        assert mgr.busy(phys, set()) == "processes"
        assert mgr.reconcile() is False
        assert calls == []
        status = c.get("nodes", "node1")["metadata"]["annotations"][STATUS_ANNOS]
        assert f"{phys}={cur[phys]}>{target}:busy" in status
    finally:
        holder.kill()
        holder.wait()
