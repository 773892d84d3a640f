"""scripts/probe/trace_step.py: per-kernel durations and gaps of the last
decode steps of a rocprofv3 kernel trace (synthetic CSV, CPU)."""

import csv
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
FIELDS = ["Kind", "Agent_Id", "Queue_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X",
          "Workgroup_Size_X"]


def _trace(path: Path, steps: int):
    """Each step: gemm 10 us, 1 us gap, attention 5 us, 2 us gap, tail 3 us."""
    t = 1_000_000
    rows = []
    for _ in range(steps):
        for name, dur, gap, grid in (("void (anonymous namespace)::skinny_wide_kernel<1, 2, 2, 1>(int)", 10_000, 0,
                                      192 * 128),
                                     ("decode_attn_fused_kernel<4, 8, true, false, false>(int)", 5_000, 1_000, 5 * 512),
                                     ("decode_tail_kernel(int)", 3_000, 2_000, 8 * 256)):
            t += gap
            rows.append({"Kind": "KERNEL_DISPATCH", "Agent_Id": "Agent 2", "Queue_Id": 1, "Kernel_Name": name,
                         "Start_Timestamp": t, "End_Timestamp": t + dur, "Grid_Size_X": grid,
                         "Workgroup_Size_X": grid // {192 * 128: 192, 5 * 512: 5, 8 * 256: 8}[grid]})
            t += dur
        t += 500
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=FIELDS)
        w.writeheader()
        w.writerows(rows)


def test_trace_step_reports_durations_and_gaps(tmp_path):
    _trace(tmp_path / "run_kernel_trace.csv", 6)
    r = subprocess.run([sys.executable, str(ROOT / "scripts/probe/trace_step.py"), str(tmp_path), "--steps", "4",
                        "--json"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    ks = {k["kernel"].split(" ")[0]: k for k in out["kernels"]}
    assert ks["skinny_wide_kernel<1,"]["mean_us"] == 10.0
    assert ks["decode_attn_fused_kernel<4,"]["gap_before_us"] == 1.0
    assert ks["decode_tail_kernel"]["gap_before_us"] == 2.0
    assert out["summary"]["steps"] == 4 and out["summary"]["launches_per_step"] == 3
    assert out["summary"]["kernel_us"] == 18.0 and out["summary"]["gap_us"] == 3.0
    assert 21.0 <= out["summary"]["wall_us"] <= 21.5


def test_trace_step_needs_enough_steps(tmp_path):
    _trace(tmp_path / "run_kernel_trace.csv", 2)
    r = subprocess.run([sys.executable, str(ROOT / "scripts/probe/trace_step.py"), str(tmp_path), "--steps", "4"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "steps in the trace" in (r.stderr + r.stdout)
