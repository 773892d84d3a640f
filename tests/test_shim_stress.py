"""Concurrency and memory-safety of libmivgpu.so's host code.

Several processes x threads hammer one container's shared region through the
mock HIP runtime with random hipMalloc/hipFree and hipMemCreate/hipMemRelease
under a tight HBM limit; afterwards the region must account zero bytes and no
live slots.  The same stress runs under AddressSanitizer and ThreadSanitizer
builds of the shim + mock runtime + driver (host sanitizers only: GPU ASan is
not available on this pool).
"""

import json
import os
import subprocess

import pytest

from k8s_vgpu_scheduler_amd.monitor import region as R
from k8s_vgpu_scheduler_amd.utils import build


def _stress(driver, shim, cache, procs=4, threads=4, iters=400, max_mib=512, limit="3072m", preload_extra=(),
            extra_env=None, timeout=240):
    env = dict(os.environ)
    env.update({"MOCKHIP_TOTAL_MIB": "65536", "MIVGPU_SHARED_CACHE": str(cache),
                "HIP_DEVICE_MEMORY_LIMIT_0": limit,
                "LD_PRELOAD": " ".join([*preload_extra, str(shim)])})
    env.update(extra_env or {})
    ps = [subprocess.Popen([str(driver), "stress", str(threads), str(iters), str(max_mib)], env=env,
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for _ in range(procs)]
    outs = []
    for p in ps:
        so, se = p.communicate(timeout=timeout)
        line = next((x for x in so.splitlines() if x.startswith("{")), None)
        outs.append((p.returncode, json.loads(line) if line else None, se))
    return outs


def _check_region_clean(cache):
    reg = R.SharedRegion(str(cache), writable=False)
    try:
        assert reg.dev_used(0) == 0
        assert reg.active_procs() == []
    finally:
        reg.close()


def test_multiprocess_thread_stress_accounting(native_build, tmp_path):
    cache = tmp_path / "s.cache"
    outs = _stress(native_build["driver"], native_build["shim"], cache)
    for rc, res, err in outs:
        assert rc == 0, err[-2000:]
        assert res["errors"] == 0 and res["usage_after"] == 0, res
        assert res["allocs"] > 0
    assert sum(r["ooms"] for _, r, _ in outs) > 0          # the 3 GiB limit was actually hit
    _check_region_clean(cache)


@pytest.mark.parametrize("kind", ["address", "thread"])
def test_sanitized_stress(kind, tmp_path):
    try:
        b = build.build_sanitized(kind)
    except RuntimeError as e:       # toolchain without this sanitizer runtime
        pytest.skip(f"{kind} sanitizer build unavailable: {e}")
    cache = tmp_path / f"{kind}.cache"
    env = {"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1:halt_on_error=1",
           "TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1:report_signal_unsafe=0"}
    outs = _stress(b["driver"], b["shim"], cache, procs=2, threads=4, iters=200,
                   preload_extra=(b["runtime"],), extra_env=env)
    for rc, res, err in outs:
        assert "ERROR: AddressSanitizer" not in err, err[-4000:]
        assert "WARNING: ThreadSanitizer" not in err, err[-4000:]
        assert rc == 0 and res is not None, err[-2000:]
        assert res["errors"] == 0 and res["usage_after"] == 0, res
    _check_region_clean(cache)


@pytest.mark.parametrize("kind", ["plain", "thread"])
def test_stress_with_runtime_vram_accounting(kind, native_build, tmp_path):
    """Concurrent alloc/free and launches with the KFD context accounting and
    the occupancy sampler active (the mock runtime publishes its per-process
    VRAM and wave-count files, the other stress process is a peer on the same
    GPU), the governor's whole host path engaged (the mock runs the gate and
    clock kernels on the host: enqueue, idle stamper, sampler): no sanitizer
    reports, no
    errors, and the shared region is clean once every process has exited."""
    from tests.test_shim_cpu import _fake_kfd

    kfd = _fake_kfd(tmp_path / "kfd", [(4242, 0x75 << 8, 0)])
    env = {"MIVGPU_KFD_SYSFS": str(kfd), "MOCKHIP_KFD_SYSFS": str(kfd), "MOCKHIP_KFD_GPU_ID": "4242",
           "MIVGPU_CONTEXT_REFRESH_MS": "1", "HIP_DEVICE_CORE_LIMIT": "50", "GPU_CORE_UTILIZATION_POLICY": "force",
           "MOCKHIP_KFD_OCC": "1", "MOCKHIP_GOVERNOR": "1",
           "TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1:report_signal_unsafe=0"}
    if kind == "plain":
        driver, shim, extra = native_build["driver"], native_build["shim"], ()
    else:
        try:
            b = build.build_sanitized(kind)
        except RuntimeError as e:
            pytest.skip(f"{kind} sanitizer build unavailable: {e}")
        driver, shim, extra = b["driver"], b["shim"], (b["runtime"],)
    cache = tmp_path / "k.cache"
    outs = _stress(driver, shim, cache, procs=2, threads=4, iters=200, preload_extra=extra, extra_env=env)
    for rc, res, err in outs:
        assert "WARNING: ThreadSanitizer" not in err, err[-4000:]
        assert rc == 0 and res is not None, err[-2000:]
        assert res["errors"] == 0 and res["allocs"] > 0, res
    _check_region_clean(cache)
