"""HBM read bandwidth a CU partition can pull, alone and side by side.

Calibrates the decode kernels of a slice: a 64-CU slice cannot stream faster
than what 64 CUs can read, and N slices together cannot beyond what HBM gives
N disjoint partitions at once.

    python -m k8s_vgpu_scheduler_amd.bench.membw --out membw.json
      single: one process per partition size (256 / 128 / 64 / 32 CUs), block sweep
      shared: 2 / 4 / 8 processes on disjoint XCD-balanced partitions, started on
              a common wall-clock instant, aggregate bytes over a fixed window

Reads rotate over 4 x 1 GiB buffers so the 256 MB Infinity Cache cannot serve
repeats; the kernel is ops.stream_read (16-byte non-temporal loads, exact sum).
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

GIB = 1 << 30


LAYOUT = "balanced"


def _mask(cus: int, slot: int = 0, layout: str | None = None) -> str:
    """CU partition ``slot`` of ``cus`` CUs.  ``balanced``: consecutive mask bits
    = the same number of CUs on every XCD (CU i lives on XCD i % 8);
    ``xcd``: whole XCDs (cus / 32 of them), the CPX-like layout in which tenants
    would share no XCD.  Measured on MI355X in SPX mode (profiles/README.md
    §23): an ``xcd`` mask is silently dropped -- a queue dispatches to every
    XCD, so a mask that leaves an XCD without CUs is not applied and the
    process runs on all 256 CUs.  XCD-exclusive tenants need a compute
    partition mode (CPX/DPX/QPX), not a CU mask."""
    layout = layout or LAYOUT
    if layout == "xcd" and cus % 32 == 0:
        k = cus // 32
        xcds = range(slot * k, slot * k + k)
        ids = sorted(x + 8 * j for x in xcds for j in range(32))
        return "0:" + ",".join(f"{c}-{c}" for c in ids)
    lo = slot * cus
    return f"0:{lo}-{lo + cus - 1}"


def child(args) -> dict:
    import torch

    from k8s_vgpu_scheduler_amd import ops

    bufs = [torch.ones(GIB // 2, dtype=torch.int16, device="cuda") for _ in range(args.gib)]
    out = torch.zeros(1, dtype=torch.int64, device="cuda")
    cus = ops.visible_cus()
    res = {"cus": cus, "mask": os.environ.get("HSA_CU_MASK", "")}
    if args.shared:
        blocks = cus * args.blocks_per_cu
        for b in bufs:                                  # warm up before the common start
            ops.stream_read(b, out, blocks)
        torch.cuda.synchronize()
        print("READY", flush=True)
        start_at = float(sys.stdin.readline())         # the parent's common instant
        while time.time() < start_at:
            time.sleep(0.0005)
        t0 = time.time()
        n = 0
        while time.time() - t0 < args.window_s:
            for b in bufs:
                ops.stream_read(b, out, blocks)
            torch.cuda.synchronize()
            n += len(bufs)
        dt = time.time() - t0
        res.update({"bytes": n * GIB, "t0": t0, "t1": t0 + dt, "gbps": n * GIB / dt / 1e9, "blocks": blocks})
        return res
    best = {}
    for bpc in (2, 4, 8, 16, 32):
        blocks = cus * bpc
        for b in bufs:
            ops.stream_read(b, out, blocks)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            for b in bufs:
                ops.stream_read(b, out, blocks)
        e1.record()
        torch.cuda.synchronize()
        best[bpc] = round(5 * len(bufs) * GIB / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    res["gbps_by_blocks_per_cu"] = best
    res["gbps"] = max(best.values())
    return res


def _spawn(mask: str | None, extra: list[str]) -> subprocess.Popen:
    env = dict(os.environ)
    if mask:
        env["HSA_CU_MASK"] = mask
    env.setdefault("GPU_MAX_HW_QUEUES", "2")
    return subprocess.Popen([sys.executable, "-m", "k8s_vgpu_scheduler_amd.bench.membw", "--child", *extra],
                            env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                            text=True)


def _collect(p: subprocess.Popen) -> dict:
    out, err = p.communicate(timeout=600)
    if p.returncode != 0:
        raise RuntimeError(err[-2000:])
    return json.loads([l for l in out.splitlines() if l.startswith("{")][-1])


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--shared", action="store_true")
    ap.add_argument("--window-s", type=float, default=3.0)
    ap.add_argument("--blocks-per-cu", type=int, default=8)
    ap.add_argument("--gib", type=int, default=4,
                    help="working set per process in GiB (a decode slice streams ~20 GiB per step)")
    ap.add_argument("--shared-bpc", type=int, default=0,
                    help="blocks per CU in the shared rows (0 = the best single-process value)")
    ap.add_argument("--shared-only", default="", help="comma list of process counts: only these shared rows")
    ap.add_argument("--layout", default="balanced", choices=["balanced", "xcd"],
                    help="CU partition layout: XCD-balanced (default) or whole XCDs per partition")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    global LAYOUT
    LAYOUT = a.layout
    if a.child:
        print(json.dumps(child(a)), flush=True)
        return 0
    doc = {"single": {}, "shared": {}, "gib_per_process": a.gib, "layout": a.layout}
    counts = [int(x) for x in a.shared_only.split(",") if x] or [2, 4, 8]
    for cus in (256, 128, 64, 32):
        if a.shared_only and 256 // cus not in counts:
            continue
        r = _collect(_spawn(None if cus == 256 else _mask(cus), ["--gib", str(a.gib)]))
        doc["single"][cus] = r
        print(f"single {cus:3d} CUs: {r['gbps']:.0f} GB/s {r['gbps_by_blocks_per_cu']}", flush=True)
    for n in counts:
        cus = 256 // n
        bpc = a.shared_bpc or max(doc["single"][cus]["gbps_by_blocks_per_cu"],
                                  key=doc["single"][cus]["gbps_by_blocks_per_cu"].get)
        ps = [_spawn(_mask(cus, i), ["--shared", "--window-s", str(a.window_s), "--blocks-per-cu", str(bpc),
                                     "--gib", str(a.gib)])
              for i in range(n)]
        for p in ps:                          # every child initialised and warm
            line = p.stdout.readline()
            if line.strip() != "READY":
                raise RuntimeError(f"child not ready: {line!r} {p.stderr.read()[-2000:]}")
        start = time.time() + 0.5
        for p in ps:
            p.stdin.write(f"{start}\n")
            p.stdin.flush()
        rs = [_collect(p) for p in ps]
        span = max(r["t1"] for r in rs) - min(r["t0"] for r in rs)
        agg = sum(r["bytes"] for r in rs) / span / 1e9
        doc["shared"][n] = {"cus_each": cus, "blocks_per_cu": int(bpc), "per_process_gbps": [round(r["gbps"], 1) for r in rs],
                            "aggregate_gbps": round(agg, 1)}
        print(f"shared {n} x {cus} CUs: aggregate {agg:.0f} GB/s, each {[round(r['gbps']) for r in rs]}",
              flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
