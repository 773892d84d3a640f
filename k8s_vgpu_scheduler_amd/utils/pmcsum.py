"""Summarise ``rocprofv3 --pmc ... --output-format csv`` counter files per kernel.

Each ``*_counter_collection.csv`` row is (dispatch, kernel, counter, value,
start, end).  Rows of several passes (one ``--pmc`` run per counter group,
the pool's rule) are merged by kernel name: per kernel the mean of every
counter per dispatch and the mean dispatch time; with ``FETCH_SIZE`` /
``WRITE_SIZE`` (KiB per dispatch, TCC->memory) the achieved HBM bandwidth.
On gfx950 FETCH_SIZE tallies 128-byte requests at 64 B, i.e. exactly half the
bytes of a wide coalesced stream (MI355X_MICROARCH.md, "FETCH_SIZE reports
exactly 1/2"): ``--fetch-scale`` (default 2) corrects read_MB / read_GBps.

    python -m k8s_vgpu_scheduler_amd.utils.profsum ... (kernel times)
    python -m k8s_vgpu_scheduler_amd.utils.pmcsum gpurun_out/pmc/a/run_counter_collection.csv \
        gpurun_out/pmc/b/run_counter_collection.csv --md profiles/pmc/decode_cu64.md
"""

from __future__ import annotations

import argparse
import csv
from collections import defaultdict

from k8s_vgpu_scheduler_amd.utils.profsum import _short

SKIP = ("at::native", "pack_weight", "rocclr", "distribution_")   # one-off init, not the step


def load(paths: list[str]) -> dict:
    """kernel -> {"dispatches": set, "ns": [..], counter: [values per dispatch]}."""
    ks: dict = defaultdict(lambda: {"dispatches": set(), "ns": {}, "c": defaultdict(dict)})
    for pi, path in enumerate(paths):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                name = _short(r["Kernel_Name"])
                if any(s in r["Kernel_Name"] for s in SKIP):
                    continue
                key = (pi, int(r["Dispatch_Id"]))
                k = ks[name]
                k["dispatches"].add(key)
                k["ns"][key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                k["c"][r["Counter_Name"]][key] = float(r["Counter_Value"])
    return ks


def summarise(ks: dict, fetch_scale: float = 2.0) -> list[dict]:
    rows = []
    for name, k in ks.items():
        row = {"kernel": name, "dispatches": len({d for _, d in k["dispatches"]})}
        ns = list(k["ns"].values())
        row["avg_us"] = round(sum(ns) / len(ns) / 1e3, 2)
        for cname, vals in sorted(k["c"].items()):
            v = list(vals.values())
            row[cname] = sum(v) / len(v)
        # bandwidth from the pass that collected the counter (its own dispatch times)
        for cname, col, scale in (("FETCH_SIZE", "read", fetch_scale), ("WRITE_SIZE", "write", 1.0)):
            if cname in k["c"]:
                tot_b = sum(k["c"][cname].values()) * 1024.0 * scale
                tot_ns = sum(k["ns"][d] for d in k["c"][cname])
                row[f"{col}_MB"] = round(tot_b / len(k["c"][cname]) / 1e6, 2)
                row[f"{col}_GBps"] = round(tot_b / tot_ns, 1) if tot_ns else 0.0
        rows.append(row)
    rows.sort(key=lambda r: -r["avg_us"] * r["dispatches"])
    return rows


def to_markdown(rows: list[dict], top: int = 20) -> str:
    cols = ["kernel", "dispatches", "avg_us"]
    extra = sorted({c for r in rows for c in r} - set(cols))
    cols += extra
    out = ["| " + " | ".join(cols) + " |", "|" + "---|" * len(cols)]
    for r in rows[:top]:
        cells = []
        for c in cols:
            v = r.get(c, "")
            if isinstance(v, float) and c not in ("avg_us", "read_GBps", "write_GBps", "read_MB", "write_MB"):
                v = f"{v:.4g}"
            cells.append(str(v))
        out.append("| " + " | ".join(cells) + " |")
    return "\n".join(out) + "\n"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+", help="*_counter_collection.csv of one or more --pmc passes")
    ap.add_argument("--md", default=None)
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--fetch-scale", type=float, default=2.0, help="bytes per FETCH_SIZE KiB x 1024 (gfx950: 2)")
    a = ap.parse_args(argv)
    md = to_markdown(summarise(load(a.csv), a.fetch_scale), a.top)
    print(md, end="")
    if a.md:
        with open(a.md, "w") as f:
            f.write(md)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
