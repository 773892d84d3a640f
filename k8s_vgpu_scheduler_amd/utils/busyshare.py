"""GPU busy share of one process from a rocprofv3 kernel trace.

``python -m k8s_vgpu_scheduler_amd.utils.busyshare <dir>`` reads every
``*kernel_trace.csv`` under ``<dir>`` (rocprofv3 --kernel-trace --output-format
csv) and reports, per process, the union of its kernels' [start, end]
intervals over the span from its first kernel start to its last kernel end --
the fraction of wall time the GPU was executing that tenant's work.  The
governor's own gate kernels (``mivgpu_gate``) are counted separately: they are
the holds, not the tenant's work.
"""

from __future__ import annotations

import csv
import glob
import json
import os
import sys


def _union(iv):
    iv.sort()
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def busy_share(trace_dir: str, skip_first_s: float = 0.0) -> dict:
    rows = []
    for f in glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    by_pid: dict[str, dict] = {}
    for r in rows:
        pid = r.get("Process_Id") or r.get("Pid") or "?"
        name = r.get("Kernel_Name", "")
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = by_pid.setdefault(pid, {"work": [], "gate": []})
        d["gate" if "mivgpu_gate" in name else "work"].append((s, e))
    out = {}
    for pid, d in by_pid.items():
        if not d["work"]:
            continue
        t0 = min(s for s, _ in d["work"]) + int(skip_first_s * 1e9)
        work = [(max(s, t0), e) for s, e in d["work"] if e > t0]
        if not work:
            continue
        span = max(e for _, e in work) - t0
        busy = _union(work)
        gate = [(max(s, t0), e) for s, e in d["gate"] if e > t0]
        # gates that did not hold (< 100 us): the governor's per-gate cost
        quick = sorted((e - s) / 1e3 for s, e in d["gate"] if e - s < 100_000)
        out[pid] = {"kernels": len(work), "span_ms": round(span / 1e6, 2), "busy_ms": round(busy / 1e6, 2),
                    "busy_share": round(busy / span, 4) if span else None, "gates": len(gate),
                    "gate_hold_ms": round(_union(gate) / 1e6, 2) if gate else 0.0,
                    "nonholding_gates": len(quick),
                    "nonholding_gate_us_p50": round(quick[len(quick) // 2], 2) if quick else None}
    return out


if __name__ == "__main__":
    skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    print(json.dumps(busy_share(sys.argv[1], skip), indent=1))
