"""bench.py's multi-rank harness rehearsed on the CPU (the driver runs it with
torchrun on 1/2/4/8 MI355X; here: gloo barriers and the CPU reference decoder in
the slice processes).  Checks the JSON contract: one line from rank 0, whole-job
aggregate value over all ranks, config fields, all three rounds."""

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _run(args, nproc):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(29600 + nproc), str(ROOT / "bench.py"), *args]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd="/tmp")
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout[-2000:]     # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("nproc", [1, 2])
def test_bench_json_contract_cpu_rehearsal(nproc):
    out = _run(["--gpus", str(nproc), "--device", "cpu", "--model", "qwen3-tiny", "--slices", "2", "--batch", "2",
                "--ctx", "32", "--steps", "3", "--warmup", "1"], nproc)
    assert out["n_gpus"] == nproc and out["steps"] == 3 and out["warmup"] == 1
    assert out["higher_is_better"] is True and out["scaling"] == "weak" and out["vs_baseline"] is None
    assert out["config"]["global_batch"] == nproc * 2 * 2
    assert out["config"]["parallelism"] == f"dp{nproc} x 2 vGPU slices/GPU"
    assert out["round"] == "shim" and out["value"] > 0
    assert "native_value" in out and "native_hip_default_queues_value" in out
    assert out["temporal_value"] > 0 and len(out["temporal_per_slice_tok_s_rank0"]) == 2   # the governor round
    # value is the whole-job aggregate: tokens of every slice on every rank / max wall
    tokens = nproc * 2 * 2 * 3
    assert out["value"] == pytest.approx(tokens / (out["ms_per_step"] * 3 / 1000), rel=0.02)
    assert len(out["per_slice_tok_s_rank0"]) == 2
    if nproc > 1:
        # the untimed all-reduce between ranks: exact, and reported beside the headline
        ar = out["allreduce_between_gpus"]
        assert [r["bytes"] for r in ar] == [64 << 10, 1 << 20] and all(r["correct"] for r in ar)
        assert out["allreduce_peak_busbw_gbps"] == max(r["busbw_gbps"] for r in ar) > 0
        # every rank's own view in the one line
        pr = out["per_rank"]
        assert [p["rank"] for p in pr] == list(range(nproc)) and all(p["tok_s"] > 0 for p in pr)
        assert sum(p["tok_s"] for p in pr) >= out["value"] * 0.98        # the aggregate uses the max wall
        assert all(len(p["per_slice_tok_s"]) == 2 for p in pr)
    else:
        assert "allreduce_between_gpus" not in out and "per_rank" not in out


@pytest.mark.parametrize("nproc", [4, 8])
def test_bench_json_contract_at_4_and_8_ranks(nproc):
    """The driver's 1/2/4/8 scaling curve, rehearsed at 4 and 8 ranks (one
    slice per rank, shim + native rounds, to fit the CPU container)."""
    out = _run(["--gpus", str(nproc), "--device", "cpu", "--model", "qwen3-tiny", "--slices", "1", "--batch", "2",
                "--ctx", "16", "--steps", "2", "--warmup", "1", "--mode", "both"], nproc)
    assert out["n_gpus"] == nproc and out["config"]["global_batch"] == nproc * 2
    assert out["config"]["parallelism"] == f"dp{nproc} x 1 vGPU slices/GPU"
    tokens = nproc * 2 * 2
    assert out["value"] == pytest.approx(tokens / (out["ms_per_step"] * 2 / 1000), rel=0.02)
    ar = out["allreduce_between_gpus"]
    assert all(r["correct"] for r in ar)
    assert [p["rank"] for p in out["per_rank"]] == list(range(nproc))
