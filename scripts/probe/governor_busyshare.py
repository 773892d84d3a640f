"""GPU-box probe: busy share of a governed tenant in a rocprofv3 kernel trace.

Scenarios:
  heavy25_light3  a 25 % (force) matmul tenant next to three light tenants
                  (one tiny kernel every 50 ms each)
  heavy25_alone   the same tenant alone
  heavy50_alone   at 50 %
The heavy tenant runs under rocprofv3 --kernel-trace; its busy share = union
of its kernel intervals / span (utils/busyshare.py).  Output: JSON lines.
"""

import json
import os
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from k8s_vgpu_scheduler_amd.shim import shim_env  # noqa: E402
from k8s_vgpu_scheduler_amd.utils.busyshare import busy_share  # noqa: E402

OUT = ROOT / "gpurun_out" / "busyshare"


def env_with(extra):
    e = dict(os.environ)
    e.update(shim_env())
    e["PYTHONPATH"] = str(ROOT) + os.pathsep + e.get("PYTHONPATH", "")
    e["TMPDIR"] = "/tmp"
    e.update(extra)
    return e


def scenario(name, pct, lights, iters):
    tmp = Path(tempfile.mkdtemp(prefix="busyshare-"))
    procs = []
    for i in range(lights):
        procs.append(subprocess.Popen([sys.executable, "-m", "k8s_vgpu_scheduler_amd.shim.probe", "--child", "light",
                                       "--hold-s", "40"], env=env_with({"MIVGPU_SHARED_CACHE": str(tmp / f"l{i}.c")}),
                                      stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, cwd=str(ROOT)))
    out_dir = OUT / name
    shutil.rmtree(out_dir, ignore_errors=True)
    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    e = env_with({"MIVGPU_SHARED_CACHE": str(tmp / "heavy.c"), "HIP_DEVICE_CORE_LIMIT": str(pct),
                  "GPU_CORE_UTILIZATION_POLICY": "force"})
    cmd = [rocprof, "--kernel-trace", "--output-format", "csv", "-d", str(out_dir), "--", sys.executable, "-m",
           "k8s_vgpu_scheduler_amd.shim.probe", "--child", "matmul", "--n", "8192", "--iters", str(iters)]
    print(f"[{name}] lights={len(procs)} profiling ...", file=sys.stderr, flush=True)
    try:
        r = subprocess.run(cmd, env=e, capture_output=True, text=True, timeout=150, cwd="/tmp")
    except subprocess.TimeoutExpired as ex:
        print(f"[{name}] TIMEOUT; child stdout so far: {ex.stdout!r:.2000}\nstderr: {ex.stderr!r:.3000}",
              file=sys.stderr, flush=True)
        raise
    finally:
        print(f"[{name}] profiled run ended; stopping lights", file=sys.stderr, flush=True)
        for p in procs:
            p.kill()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                print(f"[{name}] light {p.pid} did not exit", file=sys.stderr, flush=True)
    print(f"[{name}] analysing trace", file=sys.stderr, flush=True)
    line = next((x for x in r.stdout.splitlines() if x.startswith("{")), "{}")
    res = json.loads(line)
    shares = busy_share(str(out_dir), skip_first_s=0.5)   # skip startup (first GEMMs, bucket's burst)
    heavy = max(shares.values(), key=lambda d: d["kernels"]) if shares else {}
    if heavy.get("kernels"):
        heavy["kernel_us_mean"] = round(1e3 * heavy["busy_ms"] / heavy["kernels"], 2)
    print(json.dumps({"scenario": name, "limit_pct": pct, "lights": lights, "rc": r.returncode,
                      "tflops": round(res.get("tflops", 0), 1), "gate_held_ms": res.get("gate_held_ms"),
                      "received_ms": res.get("received_ms"), "seconds": res.get("seconds"),
                      "sampler_state_ms": res.get("sampler_state_ms"), "sampler_samples": res.get("sampler_samples"),
                      "trace": heavy}), flush=True)
    if r.returncode != 0:
        print(r.stderr[-2000:], file=sys.stderr)
        raise SystemExit(1)


if __name__ == "__main__":
    scenario("heavy100_alone", 100, 0, 1000)    # unthrottled: the kernel duration to compare against
    scenario("heavy25_light3", 25, 3, 2000)
    scenario("heavy25_alone", 25, 0, 2000)
    scenario("heavy50_alone", 50, 0, 1500)
