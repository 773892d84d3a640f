"""GPU-box probe: which torch calls give a process KFD hardware queues?

Lists /sys/class/kfd/kfd/proc/*/queues before and after each step; the
process whose queue count changes is this one.  Output: JSON lines.
"""
import glob
import json
import os


def snap():
    out = {}
    for d in glob.glob("/sys/class/kfd/kfd/proc/*/queues"):
        try:
            out[d.split("/")[-2]] = len(os.listdir(d))
        except OSError:
            pass
    return out


def step(name, fn, prev):
    fn()
    cur = snap()
    diff = {k: (prev.get(k, 0), v) for k, v in cur.items() if prev.get(k, 0) != v}
    print(json.dumps({"step": name, "changed": diff}), flush=True)
    return cur


s = snap()
import torch  # noqa: E402

s = step("import torch", lambda: None, s)
s = step("set_device", lambda: torch.cuda.set_device(0), s)
s = step("synchronize", torch.cuda.synchronize, s)
s = step("Event record", lambda: torch.cuda.Event().record(), s)
s = step("tensor on gpu", lambda: torch.ones(4, device="cuda"), s)
s = step("synchronize again", torch.cuda.synchronize, s)
