"""Summarise a rocprofv3 kernel trace (rocpd SQLite ``*_results.db`` or the
``*_kernel_stats.csv`` of ``--output-format csv``) into a compact CSV/markdown
table for ``profiles/``:

    python -m k8s_vgpu_scheduler_amd.utils.profsum gpurun_out/r16/prof/run_results.db \
        --md profiles/decode_b32/kernel_stats_skinny.md --top 25
"""

from __future__ import annotations

import argparse
import csv
import re
import shutil
import sqlite3
import subprocess
from collections import defaultdict
from pathlib import Path


def _demangle(names: list[str]) -> dict:
    tool = shutil.which("c++filt") or shutil.which("llvm-cxxfilt")
    if not tool:
        return {}
    clean = [n[:-3] if n.endswith(".kd") else n for n in names]
    out = subprocess.run([tool], input="\n".join(clean), capture_output=True, text=True).stdout.splitlines()
    return dict(zip(names, out)) if len(out) == len(names) else {}


def _short(name: str, width: int = 70) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)                 # drop argument lists
    if name.startswith("Cijk_"):                       # hipBLASLt/Tensile: keep the macro tile
        m = re.search(r"MT(\d+x\d+x\d+)", name)
        name = f"hipBLASLt Cijk MT{m.group(1)}" if m else "hipBLASLt Cijk"
    return name[:width]


def from_db(path: str) -> list[dict]:
    c = sqlite3.connect(path)
    sym = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
    agg = defaultdict(lambda: {"calls": 0, "total_ns": 0, "grid": None, "wg": None})
    for kid, start, end, gx, wx in c.execute(
            "select kernel_id, start, end, grid_size_x, workgroup_size_x from rocpd_kernel_dispatch"):
        a = agg[sym.get(kid, str(kid))]
        a["calls"] += 1
        a["total_ns"] += end - start
        a["grid"], a["wg"] = gx, wx
    return [{"name": k, **v} for k, v in agg.items()]


def from_csv(path: str) -> list[dict]:
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append({"name": r["Name"], "calls": int(r["Calls"]), "total_ns": float(r["TotalDurationNs"]),
                         "grid": None, "wg": None})
    return rows


def summarise(rows: list[dict], min_calls: int = 1) -> list[dict]:
    rows = [r for r in rows if r["calls"] >= min_calls]
    dm = _demangle([r["name"] for r in rows])
    for r in rows:
        r["name"] = dm.get(r["name"], r["name"])
    total = sum(r["total_ns"] for r in rows) or 1
    out = []
    for r in sorted(rows, key=lambda r: -r["total_ns"]):
        out.append({"kernel": _short(r["name"]), "calls": r["calls"],
                    "avg_us": round(r["total_ns"] / r["calls"] / 1000, 2),
                    "share_pct": round(100 * r["total_ns"] / total, 2),
                    "grid": r["grid"], "wg": r["wg"]})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--md", default=None)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--min-calls", type=int, default=20, help="drop one-off (init) kernels")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = from_db(a.trace) if a.trace.endswith(".db") else from_csv(a.trace)
    s = summarise(rows, a.min_calls)[: a.top]
    lines = ["| kernel | calls | avg µs | share % | grid x | wg x |", "|---|---|---|---|---|---|"]
    lines += [f"| {r['kernel']} | {r['calls']} | {r['avg_us']} | {r['share_pct']} | {r['grid']} | {r['wg']} |"
              for r in s]
    text = "\n".join(lines)
    print(text)
    if a.md:
        Path(a.md).write_text(text + "\n")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(s[0]))
            w.writeheader()
            w.writerows(s)


if __name__ == "__main__":
    main()
