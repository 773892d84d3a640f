"""GPU discovery backends against a real MI355X (amd-smi and sysfs/KFD).

The device plugin's view of the card (count, CUs, HBM, DRM minors, compute
partition, health, events) comes from these backends, so they are checked on
the hardware, and against each other.  The facts the box reported are written
to gpurun_out/smi_facts.json for the record.
"""

import json
import os

import pytest

from k8s_vgpu_scheduler_amd import smi

pytestmark = pytest.mark.gpu


def _facts(b):
    return [{"uuid": g.uuid, "name": g.name, "cus": g.cus, "memory_mib": g.memory_mib, "numa": g.numa,
             "bdf": g.bdf, "render_minor": g.render_minor, "card_minor": g.card_minor, "rocr_id": g.rocr_id,
             "compute_partition": g.compute_partition, "physical": g.physical} for g in b.gpus()]


@pytest.fixture(scope="module")
def backends():
    out = {}
    for cls in (smi.AmdSmiBackend, smi.SysfsBackend):
        try:
            out[cls.name] = cls()
        except Exception as e:  # noqa: BLE001
            out[cls.name] = e
    return out


def test_detect_finds_the_mi355x(backends):
    b = smi.detect()
    gs = b.gpus()
    assert len(gs) >= 1
    g = gs[0]
    assert g.cus == 256, g
    # 288 GB HBM3E; the driver reserves a little
    assert 270_000 <= g.memory_mib <= 294_912, g
    assert g.render_minor >= 128 and g.compute_partition.upper() in smi.PARTITION_MODES
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/smi_facts.json", "w") as f:
        json.dump({k: (_facts(v) if isinstance(v, smi.Backend) else repr(v)) for k, v in backends.items()},
                  f, indent=1)


def test_backends_agree(backends):
    ok = {k: v for k, v in backends.items() if isinstance(v, smi.Backend)}
    assert ok, backends
    views = {k: sorted((g.render_minor, g.cus, g.numa, g.bdf.lower(), g.compute_partition.upper(), g.uuid,
                        g.rocr_id, g.name, g.memory_mib // 1024) for g in v.gpus()) for k, v in ok.items()}
    for v in views.values():
        for g in v:
            # one identity scheme: GPU-<16 hex KFD unique id>, the board product name
            assert g[5].startswith("GPU-") and len(g[5]) == 20 and g[6] == g[5], g
            assert g[7].startswith("AMD Instinct MI35") and "Radeon" not in g[7], g
    if len(views) == 2:
        a, s = views["amdsmi"], views["sysfs"]
        # same render nodes, CU counts, NUMA nodes, PCI addresses, partition modes, ids and names
        assert [x[:8] for x in a] == [x[:8] for x in s], views
        assert all(abs(x[8] - y[8]) <= 2 for x, y in zip(a, s)), views


def test_health_usage_and_events(backends):
    b = smi.detect()
    gs = b.gpus()
    for g in gs:
        ok, why = b.health(g)
        assert ok, why
        assert b.memory_used_mib(g) >= 0
        u = b.utilization(g)
        assert set(u) >= {"gfx", "umc"}
    # the event source either registers (and times out quietly on an idle card)
    # or reports that it is unavailable; it must never raise
    ev = b.wait_health_events(gs, 0.5)
    assert ev is None or all(isinstance(e, smi.HealthEvent) for e in ev)


_SMI_PROBE = r"""
import json, amdsmi
amdsmi.amdsmi_init()
h = amdsmi.amdsmi_get_processor_handles()[0]
t = amdsmi.amdsmi_get_gpu_memory_total(h, amdsmi.AmdSmiMemoryType.VRAM)
u = amdsmi.amdsmi_get_gpu_memory_usage(h, amdsmi.AmdSmiMemoryType.VRAM)
v = amdsmi.amdsmi_get_gpu_vram_usage(h)
print(json.dumps({"total_mib": t >> 20, "used_mib": u >> 20, "vram_total": v["vram_total"],
                  "vram_used": v["vram_used"]}))
amdsmi.amdsmi_shut_down()
"""


def test_amdsmi_inside_a_slice_reports_the_grant(tmp_path):
    """`import amdsmi` in a 36 GiB slice (the shim
    preloaded, the grant naming this GPU) reports 36864 MiB total and the
    container's usage; the same query without the shim reports the card."""
    import subprocess
    import sys

    from k8s_vgpu_scheduler_amd.shim import shim_env

    g = smi.detect("amdsmi").gpus()[0]
    base = dict(os.environ)
    base.pop("LD_PRELOAD", None)

    def probe(env):
        r = subprocess.run([sys.executable, "-c", _SMI_PROBE], env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads(r.stdout.strip().splitlines()[-1])

    native = probe(base)
    sl = dict(base, **shim_env(""), HIP_DEVICE_MEMORY_LIMIT_0="36864m", MIVGPU_DEVICE_UUIDS=g.uuid,
              MIVGPU_SHARED_CACHE=str(tmp_path / "smi.cache"))
    inside = probe(sl)
    print(json.dumps({"native": native, "slice": inside, "uuid": g.uuid}))
    assert native["total_mib"] > 280_000 and native["vram_total"] > 280_000, native
    assert inside["total_mib"] == 36864 and inside["vram_total"] == 36864, inside
    assert inside["used_mib"] <= 36864 and inside["vram_used"] <= 36864, inside
