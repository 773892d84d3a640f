"""The shim obeys the host-owned control file and the grant, not its region
(ADVICE r3 medium #2), on the mock HIP runtime.

* a block in the read-only control file parks launches while its lease is
  live, whatever the tenant writes into its region; an expired lease (a dead
  monitor) parks nothing;
* ``host_excess`` (VRAM the monitor measured beyond the region's counter) is
  charged by the quota check and shows in hipMemGetInfo;
* under a grant file the limit is the grant's, so raising ``mem_limit`` in the
  region buys nothing;
* the charging A/B switches (gate mode, share estimator, context refresh)
  cannot be set by a container that runs under a grant file.
"""

from __future__ import annotations

import threading
import time

from k8s_vgpu_scheduler_amd.monitor import region as R
from k8s_vgpu_scheduler_amd.monitor.control import ControlFile, create, offsets

from test_shim_cpu import run

import ctypes


def _grant(tmp_path, ctl=None, **kv):
    lines = [f"{k}={v}" for k, v in kv.items()]
    if ctl is not None:
        lines.append(f"MIVGPU_CONTROL_FILE={ctl}")
    lines.append(f"MIVGPU_SHARED_CACHE={tmp_path / 'g.cache'}")
    p = tmp_path / "limits.conf"
    p.write_text("\n".join(lines) + "\n")
    return str(p)


def _ctl(tmp_path):
    path = str(tmp_path / "c.ctl")
    create(path)
    return path, ControlFile(path)


def test_control_offsets_match_c_layout(native_build):
    lib = ctypes.CDLL(str(native_build["shim"]))
    lib.mivgpu_abi_offsetof.restype = ctypes.c_long
    for fid, off in offsets().items():
        assert lib.mivgpu_abi_offsetof(fid) == off, f"field {fid}"


def test_control_block_parks_launches_until_released(native_build, tmp_path):
    path, cf = _ctl(tmp_path)
    cf.publish(block=True, switch=False, over=True, lease_s=30)

    def release():
        time.sleep(0.6)
        cf.publish(block=False, switch=False, over=False, lease_s=30)
    threading.Thread(target=release).start()
    t0 = time.time()
    out = run(native_build, tmp_path, "launch", 3, env={"MIVGPU_LIMITS_FILE": _grant(tmp_path, ctl=path)},
              cache="g.cache")
    assert out[0]["real_seen"] == 3 and time.time() - t0 >= 0.5


def test_tenant_cannot_clear_the_control_block(native_build, tmp_path):
    """The tenant's region says "not blocked", repeatedly: the control file wins."""
    path, cf = _ctl(tmp_path)
    cf.publish(block=True, switch=False, over=True, lease_s=30)
    grant = _grant(tmp_path, ctl=path)
    R.SharedRegion.create(str(tmp_path / "g.cache")).close()
    reg = R.SharedRegion(str(tmp_path / "g.cache"))
    stop = threading.Event()

    def tenant():
        while not stop.is_set():
            reg.set_recent_kernel(2)
            time.sleep(0.01)
    th = threading.Thread(target=tenant)
    th.start()

    def release():
        time.sleep(1.0)
        cf.publish(block=False, switch=False, over=False, lease_s=30)
    threading.Thread(target=release).start()
    t0 = time.time()
    try:
        out = run(native_build, tmp_path, "launch", 2, env={"MIVGPU_LIMITS_FILE": grant}, cache="g.cache")
    finally:
        stop.set()
        th.join()
    assert out[0]["real_seen"] == 2 and time.time() - t0 >= 0.9
    reg.close()


def test_expired_lease_blocks_nothing(native_build, tmp_path):
    path, cf = _ctl(tmp_path)
    cf.publish(block=True, switch=False, over=True, lease_s=-1)
    t0 = time.time()
    out = run(native_build, tmp_path, "launch", 3, env={"MIVGPU_LIMITS_FILE": _grant(tmp_path, ctl=path)},
              cache="g.cache")
    assert out[0]["real_seen"] == 3 and time.time() - t0 < 5


def test_host_excess_is_charged(native_build, tmp_path):
    path, cf = _ctl(tmp_path)
    ex = [0] * 16
    ex[0] = 3 << 30
    cf.publish(block=False, switch=False, over=False, excess=ex, lease_s=30)
    grant = _grant(tmp_path, ctl=path, HIP_DEVICE_MEMORY_LIMIT_0="4096m")
    out = run(native_build, tmp_path, "meminfo", "alloc", 1500, "alloc", 900,
              env={"MIVGPU_LIMITS_FILE": grant}, cache="g.cache")
    assert out[0]["total_mib"] == 4096 and out[0]["free_mib"] == 1024
    assert out[1]["rc"] == 2 and out[2]["rc"] == 0
    # the same with the lease gone: the excess no longer counts
    cf.publish(block=False, switch=False, over=False, excess=ex, lease_s=-1)
    out = run(native_build, tmp_path, "alloc", 3500, env={"MIVGPU_LIMITS_FILE": grant}, cache="g2.cache")
    assert out[0]["rc"] == 0


def test_over_grant_verdict_refuses_every_allocation(native_build, tmp_path):
    path, cf = _ctl(tmp_path)
    cf.publish(block=False, switch=False, over=True, lease_s=30)
    grant = _grant(tmp_path, ctl=path, HIP_DEVICE_MEMORY_LIMIT_0="4096m")
    out = run(native_build, tmp_path, "alloc", 1, env={"MIVGPU_LIMITS_FILE": grant}, cache="g.cache")
    assert out[0]["rc"] == 2
    cf.publish(block=False, switch=False, over=False, lease_s=30)
    out = run(native_build, tmp_path, "alloc", 1, env={"MIVGPU_LIMITS_FILE": grant}, cache="g.cache")
    assert out[0]["rc"] == 0


def test_region_limit_rewrite_buys_nothing_under_a_grant(native_build, tmp_path):
    grant = _grant(tmp_path, HIP_DEVICE_MEMORY_LIMIT_0="1024m")
    R.SharedRegion.create(str(tmp_path / "g.cache"), mem_limit=1 << 40).close()   # a pre-seeded, forged region
    out = run(native_build, tmp_path, "alloc", 2000, "meminfo", env={"MIVGPU_LIMITS_FILE": grant},
              cache="g.cache")
    assert out[0]["rc"] == 2 and out[1]["total_mib"] == 1024


def test_charging_switches_ignored_under_a_grant(native_build, tmp_path):
    ab = {"MIVGPU_GATE_MODE": "device", "MIVGPU_SHARE_EST": "instant", "MIVGPU_CONTEXT_REFRESH_MS": "999999"}
    free = run(native_build, tmp_path, "cfginfo", env=ab)[0]
    assert free["flags"] & 3 == 3 and free["ctx_refresh_ns"] == 999999 * 1000000
    granted = run(native_build, tmp_path, "cfginfo", env={**ab, "MIVGPU_LIMITS_FILE": _grant(tmp_path)})[0]
    assert granted["flags"] & 7 == 0 and granted["flags"] & 8
    assert granted["ctx_refresh_ns"] == 20000000


def test_control_file_named_only_by_the_grant(native_build, tmp_path):
    """With a grant file, MIVGPU_CONTROL_FILE in the environment (a tenant
    pointing the shim at a file it controls) is ignored."""
    path, cf = _ctl(tmp_path)
    out = run(native_build, tmp_path, "cfginfo",
              env={"MIVGPU_LIMITS_FILE": _grant(tmp_path), "MIVGPU_CONTROL_FILE": path})[0]
    assert not out["flags"] & 16
    out = run(native_build, tmp_path, "cfginfo", env={"MIVGPU_LIMITS_FILE": _grant(tmp_path, ctl=path)})[0]
    assert out["flags"] & 16
