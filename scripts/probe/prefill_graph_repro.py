"""Stage-by-stage repro of the serving engine's sequence on the GPU (one
thread, synchronised and reported after every stage): capture the decode
graph after a warm prefill, replay, prefill again, replay.
    python scripts/probe/prefill_graph_repro.py tiny|8b [thread]"""
import sys
import threading

import torch

from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_8B, QWEN3_TINY, Qwen3Decoder


def stage(name):
    torch.cuda.synchronize()
    print("OK", name, flush=True)


def run(cfg):
    d = Qwen3Decoder(cfg, batch=1, max_ctx=4096, device="cuda")
    d.reserve_prefill()
    d.prefill(list(range(3, 163)))
    stage("warm prefill")
    d.capture()
    stage("capture")
    d.graph.replay()
    stage(f"replay before prefill (token {int(d.tokens[0])}, pos {int(d.pos[0])})")
    d.prefill(list(range(5, 97)))
    stage(f"prefill after capture (token {int(d.tokens[0])}, pos {int(d.pos[0])})")
    d.graph.replay()
    stage(f"replay after prefill (token {int(d.tokens[0])}, pos {int(d.pos[0])})")
    for _ in range(20):
        d.graph.replay()
    stage(f"20 more replays (pos {int(d.pos[0])})")


cfg = QWEN3_8B if sys.argv[1] == "8b" else QWEN3_TINY
if len(sys.argv) > 2 and sys.argv[2] == "thread":
    t = threading.Thread(target=run, args=(cfg,))
    t.start()
    t.join()
else:
    run(cfg)
print("DONE", flush=True)
