"""Collective validator on the CPU: gloo, world_size 2 and 3, exact results,
bus-bandwidth bookkeeping and the placement verdict."""

import json
import os
import socket

import pytest
import torch.multiprocessing as mp

from k8s_vgpu_scheduler_amd.parallel import collectives as C


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, extra):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "MIVGPU_DIST_INIT": f"file://{out}.rdzv"})
    rc = C.main(["--backend", "gloo", "--max-bytes", str(64 << 10), "--iters", "3", "--warmup", "1",
                 "--out", out, *extra])
    if rc != 0:
        raise SystemExit(rc)


def _run(world, tmp_path, extra=()):
    out = str(tmp_path / f"coll{world}.json")
    mp.start_processes(_worker, args=(world, _free_port(), out, list(extra)), nprocs=world, join=True,
                       start_method="spawn")
    return json.loads(open(out).read())


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_collectives_exact_on_gloo(world, tmp_path):
    doc = _run(world, tmp_path)
    assert doc["world"] == world and doc["backend"] == "gloo"
    ops = {r["op"] for r in doc["results"]}
    assert ops == set(C.BUS_FACTOR)
    assert doc["all_correct"]
    for r in doc["results"]:
        assert r["bytes"] % (4 * world) == 0
        # both figures are rounded to 3 decimals: allow that rounding
        assert r["busbw_gbps"] == pytest.approx(r["algbw_gbps"] * C.BUS_FACTOR[r["op"]](world), rel=1e-2, abs=2.5e-3)


def test_placement_verdict_fails_below_expectation(tmp_path):
    with pytest.raises(Exception):
        _run(2, tmp_path, ["--expect-busbw-gbps", "1e9"])   # impossible bandwidth -> rc 1


def test_bus_factors_and_sizes():
    assert C.BUS_FACTOR["all_reduce"](8) == pytest.approx(1.75)
    assert C.BUS_FACTOR["all_gather"](2) == 0.5
    assert C.sizes(1024, 1 << 20) == [1024, 4096, 16384, 65536, 262144, 1048576]
    v = C.placement_verdict([{"op": "all_reduce", "busbw_gbps": 60.0, "correct": True}], 100.0, 0.5)
    assert v["placement_ok"] and v["all_correct"]
    assert not C.placement_verdict([{"op": "all_reduce", "busbw_gbps": 40.0, "correct": True}], 100.0,
                                   0.5)["placement_ok"]
