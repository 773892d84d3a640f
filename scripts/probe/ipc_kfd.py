# Does KFD's per-process vram_<gpu> count memory imported through hipIpcOpenMemHandle?
import glob, json, os, time
import torch
import torch.multiprocessing as mp


def kfd_self():
    # find own entry: the single KFD process whose vram grows by a 96 MiB probe
    def snap():
        out = {}
        for f in glob.glob("/sys/class/kfd/kfd/proc/*/vram_*"):
            try:
                out[f] = int(open(f).read())
            except OSError:
                pass
        return out
    a = snap()
    x = torch.empty(96 << 20, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    b = snap()
    hits = [f for f in b if f in a and 96 << 20 <= b[f] - a[f] < 100 << 20]
    del x
    torch.cuda.empty_cache()
    return hits[0] if len(hits) == 1 else None


def consumer(q, done):
    torch.ones(1, device="cuda")
    f = kfd_self()
    before = int(open(f).read())
    t = q.get()
    torch.cuda.synchronize()
    time.sleep(0.2)
    after = int(open(f).read())
    done.put({"file": f, "before_mib": before >> 20, "after_mib": after >> 20, "imported_mib": t.numel() * 4 >> 20})
    del t


if __name__ == "__main__":
    mp.set_start_method("spawn")
    q, done = mp.Queue(), mp.Queue()
    p = mp.Process(target=consumer, args=(q, done))
    p.start()
    t = torch.ones(256 << 20, device="cuda", dtype=torch.float32)   # 1 GiB
    time.sleep(5)
    q.put(t)
    r = done.get(timeout=120)
    p.join(timeout=60)
    print("IPCKFD " + json.dumps(r), flush=True)
