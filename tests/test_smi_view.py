"""amd-smi / rocm-smi inside a vGPU container report the grant (CPU, mock SMI).

The reference's one hard-limit artifact is nvidia-smi showing the 3000 MiB
cap inside the container (README.md:67-74, imgs/hard_limit.jpg); its AMD
support gives this up (docs/develop/amd-vgpu.md:156-158).  The shim
interposes dlsym, through which the SMI CLIs and ``import amdsmi`` reach
libamd_smi.so / librocm_smi64.so: the memory queries of a GRANTED device
report the HBM limit as the total and the container's usage as used.  Here
the library is csrc/mockhip/mock_smi.cpp (one MI355X at 0000:75:00.0, 288
GiB, 5000 MiB in use) and the device is matched through a fake KFD
topology's unique_id to the grant's GPU-<16 hex> id.
"""

import os

from test_shim_cpu import run

UID = 0x1234ABCD5678EF01


def _kfd(root, uid=UID, loc=0x75 << 8):
    n = root / "topology" / "nodes" / "1"
    n.mkdir(parents=True)
    (n / "gpu_id").write_text("4242\n")
    (n / "properties").write_text(f"simd_count 1024\nsimd_per_cu 4\nlocation_id {loc}\ndomain 0\nunique_id {uid}\n")
    (root / "topology" / "nodes" / "0").mkdir(parents=True)
    (root / "topology" / "nodes" / "0" / "gpu_id").write_text("0\n")
    (root / "topology" / "nodes" / "0" / "properties").write_text("simd_count 0\nlocation_id 0\ndomain 0\n")
    return root


def _env(kfd, **kw):
    e = {"MIVGPU_KFD_SYSFS": str(kfd), "HIP_DEVICE_MEMORY_LIMIT_0": "36864m",
         "MIVGPU_DEVICE_UUIDS": f"GPU-{UID:016x}"}
    e.update(kw)
    return e


def test_granted_device_reports_the_grant(native_build, tmp_path):
    kfd = _kfd(tmp_path / "kfd")
    out = run(native_build, tmp_path, "alloc", 1000, "smi", native_build["mock_smi"], env=_env(kfd))
    s = out[-1]
    assert s["ok"] == 1, s
    assert s["total_mib"] == 36864 and s["rsmi_total_mib"] == 36864 and s["vram_total_mb"] == 36864, s
    assert s["vram_size_mb"] == 36864, s
    assert s["used_mib"] == 1000 and s["rsmi_used_mib"] == 1000 and s["vram_used_mb"] == 1000, s   # the container's
    assert s["gtt_mib"] == 512 << 10, s                                                            # GTT untouched


def test_other_devices_and_unlimited_containers_see_the_hardware(native_build, tmp_path):
    kfd = _kfd(tmp_path / "kfd", uid=0x42)          # not the granted GPU
    s = run(native_build, tmp_path, "smi", native_build["mock_smi"], env=_env(kfd))[-1]
    assert s["total_mib"] == 294912 and s["used_mib"] == 5000, s
    kfd2 = _kfd(tmp_path / "kfd2")
    e = _env(kfd2)
    e.pop("HIP_DEVICE_MEMORY_LIMIT_0")                # no HBM limit: nothing to report
    s = run(native_build, tmp_path, "smi", native_build["mock_smi"], env=e, cache="u.cache")[-1]
    assert s["total_mib"] == 294912 and s["rsmi_used_mib"] == 5000, s


def test_without_the_shim_the_library_answers(native_build, tmp_path):
    kfd = _kfd(tmp_path / "kfd")
    s = run(native_build, tmp_path, "smi", native_build["mock_smi"], env=_env(kfd), preload=False)[-1]
    assert s["total_mib"] == 294912 and s["vram_used_mb"] == 5000, s


def test_visible_devices_name_the_device_without_a_grant_list(native_build, tmp_path):
    kfd = _kfd(tmp_path / "kfd")
    e = _env(kfd, ROCR_VISIBLE_DEVICES=f"GPU-{UID:016x}")
    e.pop("MIVGPU_DEVICE_UUIDS")
    s = run(native_build, tmp_path, "smi", native_build["mock_smi"], env=e)[-1]
    assert s["total_mib"] == 36864, s
    assert os.path.exists(native_build["mock_smi"])
