"""Summarise rocprofv3 --pmc passes (scripts/gpu.sh pmc) into per-kernel JSON.

``python scripts/probe/pmc_summary.py <dir>`` reads every
``*counter_collection.csv`` under ``<dir>`` (one counter group per pass
subdirectory) and prints, per kernel name (first 90 characters), the number of
dispatches, the mean duration and the mean of each counter per dispatch, plus
FETCH_SIZE / duration as the achieved fetch bandwidth (FETCH_SIZE is in KiB).
The raw CSVs (tens of MB, mostly the random-init kernels' template names) are
not kept.
"""

from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(root: str) -> dict:
    per = defaultdict(lambda: {"dispatches": set(), "dur_ns": {}, "counters": defaultdict(float)})
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"][:90]
                d = per[name]
                key = (f, r["Dispatch_Id"])
                d["dispatches"].add(key)
                d["dur_ns"][key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                d["counters"][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for name, d in per.items():
        # every pass runs the same dispatches: per-dispatch means over the pass that holds the counter
        passes = {k[0] for k in d["dispatches"]}
        n = max(1, len(d["dispatches"]) // max(1, len(passes)))
        dur = sum(d["dur_ns"].values()) / max(1, len(d["dur_ns"]))
        row = {"dispatches": n, "mean_us": round(dur / 1e3, 2)}
        for c, v in d["counters"].items():
            row[c] = round(v / n, 1)
        if "FETCH_SIZE" in row and dur > 0:
            row["fetch_TBps"] = round(row["FETCH_SIZE"] * 1024 / dur / 1e3, 2)
        # EA read requests summed over every TCC instance, by size: 128-byte
        # (TCC_BUBBLE), 32-byte, the rest 64-byte -- rocprofv3's FETCH_SIZE
        # expression on gfx950, from the raw counters (memory-side read bytes,
        # all channels)
        rq, rq32, rq128 = (row.get("TCC_EA0_RDREQ_sum"), row.get("TCC_EA0_RDREQ_32B_sum"),
                           row.get("TCC_BUBBLE_sum", 0.0))
        if rq is not None and rq32 is not None and dur > 0:
            b = 128 * rq128 + 64 * (rq - rq128 - rq32) + 32 * rq32
            row["ea_read_MB"] = round(b / 1e6, 2)
            row["ea_read_TBps"] = round(b / dur / 1e3, 2)
        out[name] = row
    return dict(sorted(out.items(), key=lambda kv: -kv[1]["mean_us"] * kv[1]["dispatches"]))


if __name__ == "__main__":
    print(json.dumps(summarise(sys.argv[1]), indent=1))
