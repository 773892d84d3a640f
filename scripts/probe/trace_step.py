"""Per-kernel durations and the gaps between them over the last decode steps
of a rocprofv3 kernel trace (``--kernel-trace --output-format csv``).

A step ends at the argmax kernel.  Each kernel of a step is keyed by its
position in the step (so qkv of layer 3 and of layer 4 average together), and
reported with its mean duration and the mean idle gap before it.

    python scripts/probe/trace_step.py <dir-or-run_kernel_trace.csv> [--steps 10]
"""

from __future__ import annotations

import argparse
import csv
import json
import os
import re
from collections import OrderedDict, defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^void ", "", n)
    return n.split("::")[-1][:60]


def load(path: str):
    if os.path.isdir(path):
        for root, _, files in os.walk(path):
            for f in files:
                if f.endswith("kernel_trace.csv"):
                    path = os.path.join(root, f)
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"])))
    rows.sort()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    rows = load(a.trace)
    ends = [i for i, r in enumerate(rows) if "ArgMaxOps" in r[2] or "decode_tail_kernel" in r[2]]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} steps in the trace")
    steps = [rows[ends[k - 1] + 1: ends[k] + 1] for k in range(len(ends) - a.steps, len(ends))]
    by_cls = OrderedDict()
    walls = []
    for st in steps:
        walls.append((st[-1][1] - st[0][0]) / 1e3)
        prev_end = None
        for s, e, name, grid, wg in st:
            key = f"{short(name)} g{grid // max(wg, 1)}x{wg}"
            d = by_cls.setdefault(key, defaultdict(float))
            d["n"] += 1
            d["dur"] += (e - s) / 1e3
            if prev_end is not None:
                d["gap"] += max(0, s - prev_end) / 1e3
            prev_end = e
    nsteps = len(steps)
    out = []
    for k, d in by_cls.items():
        out.append({"kernel": k, "per_step": d["n"] / nsteps, "mean_us": d["dur"] / d["n"],
                    "gap_before_us": d["gap"] / d["n"], "us_per_step": d["dur"] / nsteps,
                    "gap_us_per_step": d["gap"] / nsteps})
    wall = sum(walls) / nsteps
    busy = sum(o["us_per_step"] for o in out)
    gaps = sum(o["gap_us_per_step"] for o in out)
    summ = {"steps": nsteps, "wall_us": wall, "kernel_us": busy, "gap_us": gaps,
            "launches_per_step": sum(o["per_step"] for o in out)}
    if a.json:
        print(json.dumps({"summary": summ, "kernels": out}, indent=1))
        return
    print(f"{'kernel':70s} {'n/step':>6s} {'mean us':>8s} {'gap us':>7s} {'us/step':>8s}")
    for o in sorted(out, key=lambda o: -o["us_per_step"]):
        print(f"{o['kernel']:70s} {o['per_step']:6.0f} {o['mean_us']:8.2f} {o['gap_before_us']:7.2f} "
              f"{o['us_per_step']:8.1f}")
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
