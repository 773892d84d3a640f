"""GPU-box probe: what does KFD's per-process wave-occupancy counter report on MI355X?

Starts busy child processes (unmasked, and masked to 64 CUs), samples
/sys/class/kfd/kfd/proc/<pid>/stats_<gpu_id>/cu_occupancy for every KFD
process, and records read cost and values.  Also dumps amd-smi identity and
link enums.  Output: JSON lines on stdout.
"""

import glob
import json
import os
import subprocess
import sys
import time

CHILD = r"""
import sys, time, torch
mode = sys.argv[1]
n = 8192 if mode == 'mm' else 1024
a = torch.randn(n, n, device='cuda', dtype=torch.bfloat16)
b = torch.randn(n, n, device='cuda', dtype=torch.bfloat16)
torch.cuda.synchronize()
print('READY', flush=True)
t_end = time.time() + float(sys.argv[2])
while time.time() < t_end:
    for _ in range(20):
        c = a @ b
    if mode == 'light':
        torch.cuda.synchronize(); time.sleep(0.05)
torch.cuda.synchronize()
"""


def kfd_procs():
    out = {}
    for d in glob.glob("/sys/class/kfd/kfd/proc/*"):
        pid = os.path.basename(d)
        for s in glob.glob(d + "/stats_*"):
            out.setdefault(pid, []).append(s)
    return out


def read(p):
    t0 = time.perf_counter()
    try:
        with open(p) as f:
            v = f.read().strip()
    except OSError as e:
        v = f"ERR {e}"
    return v, (time.perf_counter() - t0) * 1e6


def sample(label, secs=2.0, period=0.01):
    rows = {}
    costs = []
    t_end = time.time() + secs
    while time.time() < t_end:
        for pid, stats in kfd_procs().items():
            for s in stats:
                v, us = read(s + "/cu_occupancy")
                costs.append(us)
                rows.setdefault(f"{pid}:{os.path.basename(s)}", []).append(v)
        time.sleep(period)
    summ = {}
    for k, vs in rows.items():
        nums = [int(v) for v in vs if v.lstrip("-").isdigit()]
        summ[k] = {"n": len(vs), "mean": (sum(nums) / len(nums)) if nums else None,
                   "max": max(nums) if nums else None, "min": min(nums) if nums else None,
                   "sample": vs[:5]}
    costs.sort()
    print(json.dumps({"probe": label, "per_proc": summ,
                      "read_us_p50": costs[len(costs) // 2] if costs else None,
                      "read_us_p99": costs[int(len(costs) * 0.99)] if costs else None}), flush=True)


def spawn(mode, secs, env_extra=None):
    env = dict(os.environ)
    env.update(env_extra or {})
    p = subprocess.Popen([sys.executable, "-c", CHILD, mode, str(secs)], env=env, stdout=subprocess.PIPE, text=True)
    assert p.stdout.readline().strip() == "READY"
    return p


def main():
    print(json.dumps({"probe": "listing", "procs": {k: [os.listdir(s) for s in v] for k, v in kfd_procs().items()},
                      "proc_dirs": {d: os.listdir(d) for d in glob.glob('/sys/class/kfd/kfd/proc/*')}}), flush=True)
    p = spawn("mm", 6)
    print(json.dumps({"probe": "child", "pid": p.pid, "listing": {d: os.listdir(d) for d in glob.glob('/sys/class/kfd/kfd/proc/*')}}), flush=True)
    sample("one_unmasked_mm")
    p.wait()
    p = spawn("mm", 6, {"HSA_CU_MASK": "0:0-63"})
    sample("one_masked64_mm")
    p.wait()
    ps = [spawn("mm", 6), spawn("mm", 6)]
    sample("two_unmasked_mm")
    for q in ps:
        q.wait()
    ps = [spawn("mm", 6), spawn("light", 6)]
    sample("heavy_plus_light")
    for q in ps:
        q.wait()
    sample("idle", secs=0.5)
    try:
        import amdsmi
        amdsmi.amdsmi_init()
        hs = amdsmi.amdsmi_get_processor_handles()
        facts = {"link_type_enum": [str(x) for x in amdsmi.AmdSmiLinkType],
                 "fns": [f for f in dir(amdsmi) if "topo" in f or "link" in f or "board" in f or "asic" in f]}
        h = hs[0]
        for fn in ("amdsmi_get_gpu_asic_info", "amdsmi_get_gpu_board_info", "amdsmi_get_gpu_device_uuid",
                   "amdsmi_get_gpu_kfd_info", "amdsmi_get_gpu_vbios_info", "amdsmi_get_gpu_enumeration_info"):
            try:
                facts[fn] = {k: str(v) for k, v in dict(getattr(amdsmi, fn)(h)).items()} \
                    if not isinstance(getattr(amdsmi, fn)(h), str) else getattr(amdsmi, fn)(h)
            except Exception as e:  # noqa: BLE001
                facts[fn] = f"ERR {e}"
        for fn in ("amdsmi_topo_get_link_type", "amdsmi_topo_get_link_weight",
                   "amdsmi_get_minmax_bandwidth_between_processors", "amdsmi_topo_get_p2p_status"):
            try:
                facts[fn + "(self)"] = str(getattr(amdsmi, fn)(h, h))
            except Exception as e:  # noqa: BLE001
                facts[fn + "(self)"] = f"ERR {e}"
        try:
            facts["xgmi_info"] = str(amdsmi.amdsmi_get_xgmi_info(h))
        except Exception as e:  # noqa: BLE001
            facts["xgmi_info"] = f"ERR {e}"
        try:
            facts["link_metrics"] = str(amdsmi.amdsmi_get_link_metrics(h))[:2000]
        except Exception as e:  # noqa: BLE001
            facts["link_metrics"] = f"ERR {e}"
        print(json.dumps({"probe": "amdsmi", **facts}), flush=True)
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"probe": "amdsmi", "error": str(e)}), flush=True)
    pn = glob.glob("/sys/class/drm/card*/device/product_name")
    print(json.dumps({"probe": "sysfs_names", "product_name": {p: open(p).read().strip() for p in pn}}), flush=True)


if __name__ == "__main__":
    main()
