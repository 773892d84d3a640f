"""GPU-box probe: KFD cu_occupancy of Qwen3-8B decode slices (the bench workload).

Scenarios (each: spawn slices, LOAD, GO with --steps replays, sample every
--period-ms the cu_occupancy of every KFD process that appeared on our GPU
after the spawn):
  one      1 unmasked slice, native (decode owns the GPU)
  masked4  4 slices under the shim with 64-CU masks
  open4    4 unmasked native slices (time-shared)
  one_nosample  1 unmasked slice without sampling (does sampling perturb?)
Output: JSON lines.
"""

import glob
import json
import os
import sys
import tempfile
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from k8s_vgpu_scheduler_amd.bench.slices import plan_slices, run_round, spawn_round  # noqa: E402


def our_gpu_id():
    # KFD topology node of ROCR device 0: first node with simd_count > 0 in the
    # visible set is not knowable without HIP; use the render minor via amdsmi.
    import amdsmi
    amdsmi.amdsmi_init()
    h = amdsmi.amdsmi_get_processor_handles()[0]
    return str(amdsmi.amdsmi_get_gpu_kfd_info(h)["kfd_id"])


def stats_paths(gid):
    return {os.path.basename(os.path.dirname(p)): p + "/cu_occupancy"
            for p in glob.glob(f"/sys/class/kfd/kfd/proc/*/stats_{gid}")}


class Sampler(threading.Thread):
    def __init__(self, gid, exclude, period):
        super().__init__(daemon=True)
        self.gid, self.exclude, self.period = gid, exclude, period
        self.stop = False
        self.rows = {}

    def run(self):
        while not self.stop:
            for pid, p in stats_paths(self.gid).items():
                if pid in self.exclude:
                    continue
                try:
                    with open(p) as f:
                        v = int(f.read().strip())
                except (OSError, ValueError):
                    continue
                self.rows.setdefault(pid, []).append(v)
            time.sleep(self.period)

    def summary(self):
        out = {}
        for pid, vs in self.rows.items():
            if not any(vs):
                continue
            hist = {}
            for v in vs:
                hist[v] = hist.get(v, 0) + 1
            out[pid] = {"n": len(vs), "mean": round(sum(vs) / len(vs), 2), "max": max(vs),
                        "frac_nonzero": round(sum(1 for v in vs if v) / len(vs), 3),
                        "hist_top": sorted(hist.items(), key=lambda kv: -kv[1])[:8]}
        return out


def scenario(name, specs, steps, gid, sample, period):
    tmp = Path(tempfile.mkdtemp(prefix="kfdocc-"))
    before = set(stats_paths(gid))
    procs = spawn_round(specs, None, tmp, tmp, ["--steps", str(steps), "--warmup", "3"], name)
    sampler = None

    def sync():
        nonlocal sampler
        if sample and sampler is None:
            sampler = Sampler(gid, before, period)
            sampler.start()

    res = run_round(procs, sync=sync)
    if sampler:
        sampler.stop = True
        sampler.join()
    tok_s = res["tokens"] / res["wall_s"]
    print(json.dumps({"scenario": name, "tok_s": round(tok_s, 1),
                      "per_slice_tok_s": [round(d["tok_s"], 1) for d in res["done"]],
                      "occupancy": sampler.summary() if sampler else None}), flush=True)


def main():
    gid = our_gpu_id()
    steps = int(os.environ.get("PROBE_STEPS", "300"))
    period = float(os.environ.get("PROBE_PERIOD_MS", "1")) / 1e3
    print(json.dumps({"gpu_id": gid}), flush=True)
    scenario("one", plan_slices(1, shim=False, gpumem_mib=None), steps, gid, True, period)
    scenario("one_nosample", plan_slices(1, shim=False, gpumem_mib=None), steps, gid, False, period)
    scenario("masked4", plan_slices(4, shim=True, gpumem_mib=36864), steps, gid, True, period)
    scenario("open4", plan_slices(4, shim=False, gpumem_mib=None, hw_queues=2), steps, gid, True, period)


if __name__ == "__main__":
    main()
