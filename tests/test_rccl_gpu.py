"""The native RCCL validator (csrc/bench/rccl_check.cpp) on the box's GPU.

One rank is all a one-GPU box allows (RCCL refuses two ranks on one device);
the 8-GPU driver run executes it across ranks after the timed bench
(bench.py native_rccl_check).  Here: the binary builds its communicator,
runs all-reduce / all-gather / reduce-scatter, and checks every element --
natively and under libmivgpu.so with a grant (the shim must not break RCCL).
"""

import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu


def _run(tmp_path, env, tag):
    from k8s_vgpu_scheduler_amd.utils import build
    exe = build.build_rccl_check() if not build.RCCL_CHECK.exists() else build.RCCL_CHECK
    r = subprocess.run([str(exe), "--rank", "0", "--nranks", "1", "--uid", str(tmp_path / f"{tag}.uid"),
                        "--sizes", "1048576,67108864", "--iters", "5", "--warmup", "2"],
                       env=env, capture_output=True, text=True, timeout=180)
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    comm = [x["comm"] for x in lines if "comm" in x]
    # what RCCL saw, reported before the rows (bench.py carries it per rank)
    assert r.returncode != 0 or (comm and comm[0]["nranks"] == 1 and comm[0]["rank"] == 0), lines
    return r, [x for x in lines if "op" in x]


def test_native_rccl_check_one_rank(tmp_path):
    r, rows = _run(tmp_path, dict(os.environ), "native")
    print(json.dumps(rows))
    assert r.returncode == 0, r.stderr[-2000:]
    assert {x["op"] for x in rows} == {"all_reduce", "all_gather", "reduce_scatter"} and len(rows) == 6
    assert all(x["ok"] and x["bad_elements"] == 0 for x in rows), rows


def test_native_rccl_check_under_the_shim(tmp_path):
    from k8s_vgpu_scheduler_amd.shim import shim_env
    env = dict(os.environ, **shim_env(""), HIP_DEVICE_MEMORY_LIMIT_0="8192m",
               MIVGPU_SHARED_CACHE=str(tmp_path / "rccl.cache"))
    r, rows = _run(tmp_path, env, "shim")
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(rows) == 6 and all(x["ok"] for x in rows), rows
