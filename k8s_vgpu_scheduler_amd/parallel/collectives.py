"""RCCL collective validator: correctness + bus bandwidth over xGMI.

Runs one process per GPU (``torch.distributed.run``); for each collective and
message size it checks the result exactly and times ``--iters`` back-to-back
calls between barriers + device synchronisation (max over ranks).  Bus
bandwidth uses the standard ring factors: all-reduce 2(n-1)/n, reduce-scatter
/ all-gather / all-to-all (n-1)/n, broadcast 1.

For a pod of N GPUs placed by the scheduler, ``--expect-busbw-gbps`` (or the
xGMI link data of the node's smi backend, ``--from-smi``) turns the peak
large-message all-reduce busBW into a placement verdict: on MI355X every GPU
pair has a direct xGMI link, so a pair that only reaches PCIe-class bandwidth
means the devices are not the ones the scheduler believes it allocated (or
that the shim broke the IPC path that RCCL's peer-to-peer transport uses —
the reference's known limitation, examples/nvidia/vllm_cross_vgpu.yaml:99-102).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        -m k8s_vgpu_scheduler_amd.parallel.collectives --out gpurun_out/rccl.json
"""

from __future__ import annotations

import argparse
import json
import time
from pathlib import Path

import torch
import torch.distributed as dist

from k8s_vgpu_scheduler_amd.parallel.dist import DistEnv, init_distributed, shutdown

BUS_FACTOR = {
    "all_reduce": lambda n: 2.0 * (n - 1) / n,
    "reduce_scatter": lambda n: (n - 1) / n,
    "all_gather": lambda n: (n - 1) / n,
    "all_to_all": lambda n: (n - 1) / n,
    "broadcast": lambda n: 1.0,
}


def sizes(min_bytes: int, max_bytes: int, factor: int = 4) -> list[int]:
    out, s = [], min_bytes
    while s <= max_bytes:
        out.append(s)
        s *= factor
    return out


class Collective:
    """One collective at one size: buffers, exact check, timed op."""

    def __init__(self, name: str, nbytes: int, env: DistEnv, dtype=torch.float32):
        self.name, self.env = name, env
        n, r = env.world, env.rank
        esize = torch.tensor([], dtype=dtype).element_size()
        count = max(n, nbytes // esize // n * n)     # divisible by world size
        self.nbytes = count * esize
        dev = env.device
        self.dtype = dtype
        if name == "all_reduce":
            self.buf = torch.empty(count, dtype=dtype, device=dev)
        elif name == "reduce_scatter":
            self.inp = torch.empty(count, dtype=dtype, device=dev)
            self.out = torch.empty(count // n, dtype=dtype, device=dev)
        elif name == "all_gather":
            self.inp = torch.empty(count // n, dtype=dtype, device=dev)
            self.out = torch.empty(count, dtype=dtype, device=dev)
        elif name == "all_to_all":
            self.inp = torch.empty(count, dtype=dtype, device=dev)
            self.out = torch.empty(count, dtype=dtype, device=dev)
        elif name == "broadcast":
            self.buf = torch.empty(count, dtype=dtype, device=dev)
        else:
            raise ValueError(name)
        self.count, self.n, self.r = count, n, r

    def fill(self):
        """Rank- and position-dependent small integers: sums stay exact in fp32."""
        n, r = self.n, self.r
        idx = torch.arange(self.count, device=self.env.device, dtype=torch.int64)
        if self.name in ("all_reduce", "broadcast"):
            self.buf.copy_(((idx % 7) + r + 1).to(self.dtype))
        elif self.name == "reduce_scatter":
            self.inp.copy_(((idx % 5) + r).to(self.dtype))
        elif self.name == "all_gather":
            self.inp.copy_(((idx[: self.count // n] % 3) + 10 * r).to(self.dtype))
        else:  # all_to_all: chunk j of rank r carries 100*r + j
            chunk = self.count // n
            self.inp.copy_((100 * r + idx // chunk).to(self.dtype))

    def run(self):
        if self.name == "all_reduce":
            dist.all_reduce(self.buf)
        elif self.name == "reduce_scatter":
            dist.reduce_scatter_tensor(self.out, self.inp)
        elif self.name == "all_gather":
            dist.all_gather_into_tensor(self.out, self.inp)
        elif self.name == "all_to_all":
            dist.all_to_all_single(self.out, self.inp)
        else:
            dist.broadcast(self.buf, src=0)

    def check(self) -> bool:
        n, r, dev = self.n, self.r, self.env.device
        idx = torch.arange(self.count, device=dev, dtype=torch.int64)
        if self.name == "all_reduce":
            exp = n * ((idx % 7) + 1) + n * (n - 1) // 2
            return torch.equal(self.buf, exp.to(self.dtype))
        if self.name == "broadcast":
            return torch.equal(self.buf, ((idx % 7) + 1).to(self.dtype))
        chunk = self.count // n
        if self.name == "reduce_scatter":
            j = idx[:chunk] + r * chunk
            exp = n * (j % 5) + n * (n - 1) // 2
            return torch.equal(self.out, exp.to(self.dtype))
        if self.name == "all_gather":
            src = idx // chunk
            exp = (idx % chunk) % 3 + 10 * src
            return torch.equal(self.out, exp.to(self.dtype))
        src = idx // chunk                     # all_to_all: chunk s came from rank s
        return torch.equal(self.out, (100 * src + r).to(self.dtype))


def _sync(env: DistEnv):
    if env.device.type == "cuda":
        torch.cuda.synchronize(env.device)


def measure(name: str, nbytes: int, env: DistEnv, iters: int, warmup: int) -> dict:
    c = Collective(name, nbytes, env)
    c.fill()
    c.run()
    _sync(env)
    ok = c.check()
    for _ in range(warmup):
        c.run()
    dist.barrier()
    _sync(env)
    t0 = time.perf_counter()
    for _ in range(iters):
        c.run()
    _sync(env)
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=env.device)
    okt = torch.tensor([1 if ok else 0], dtype=torch.int32, device=env.device)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    t = dt.item() / iters
    algbw = c.nbytes / t / 1e9
    return {"op": name, "bytes": c.nbytes, "us": round(t * 1e6, 2), "algbw_gbps": round(algbw, 3),
            "busbw_gbps": round(algbw * BUS_FACTOR[name](env.world), 3), "correct": bool(okt.item())}


def expected_busbw_from_smi(env: DistEnv) -> float | None:
    """Lowest pairwise xGMI bandwidth among the visible GPUs (smi backend)."""
    try:
        from k8s_vgpu_scheduler_amd.smi import detect
        be = detect(None)
        gpus = be.gpus()[: env.world]
        bws = [be.link(a, b).max_bw_gbps for i, a in enumerate(gpus) for b in gpus[i + 1:]]
        bws = [b for b in bws if b]
        return min(bws) if bws else None
    except Exception:
        return None


def placement_verdict(results: list[dict], expect_gbps: float | None, min_fraction: float) -> dict:
    ar = [r for r in results if r["op"] == "all_reduce"]
    peak = max((r["busbw_gbps"] for r in ar), default=0.0)
    out = {"peak_allreduce_busbw_gbps": peak, "expected_busbw_gbps": expect_gbps,
           "all_correct": all(r["correct"] for r in results)}
    if expect_gbps:
        out["placement_ok"] = peak >= min_fraction * expect_gbps
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="all_reduce,reduce_scatter,all_gather,all_to_all,broadcast")
    ap.add_argument("--min-bytes", type=int, default=1 << 10)
    ap.add_argument("--max-bytes", type=int, default=None, help="default 1 GiB on GPU, 4 MiB on CPU")
    ap.add_argument("--factor", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--backend", default=None, choices=[None, "nccl", "gloo"])
    ap.add_argument("--expect-busbw-gbps", type=float, default=None)
    ap.add_argument("--from-smi", action="store_true", help="expected busBW from the node's xGMI link data")
    ap.add_argument("--min-fraction", type=float, default=0.5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    env = init_distributed(a.backend)
    if env.world < 2:
        raise SystemExit("run under torch.distributed.run with >= 2 processes")
    max_bytes = a.max_bytes or ((1 << 30) if env.backend == "nccl" else (4 << 20))
    results = []
    for op in a.ops.split(","):
        for nb in sizes(a.min_bytes, max_bytes, a.factor):
            r = measure(op, nb, env, a.iters, a.warmup)
            results.append(r)
            if env.is_main:
                print(json.dumps(r), flush=True)
    expect = a.expect_busbw_gbps or (expected_busbw_from_smi(env) if a.from_smi else None)
    verdict = placement_verdict(results, expect, a.min_fraction)
    if env.is_main:
        doc = {"world": env.world, "backend": env.backend, "results": results, **verdict}
        print(json.dumps(verdict), flush=True)
        if a.out:
            Path(a.out).parent.mkdir(parents=True, exist_ok=True)
            Path(a.out).write_text(json.dumps(doc, indent=1))
    ok = verdict["all_correct"] and verdict.get("placement_ok", True)
    shutdown()
    return 0 if ok else 1


if __name__ == "__main__":
    raise SystemExit(main())
