"""Single-GPU generation engine behind the serving benchmark.

The reference measures its isolation cost as a user sees it: TTFT and
per-token latency of an OpenAI-compatible streaming server (vLLM, Qwen3-8B
bf16, TP=1) inside a HAMi slice vs on a whole GPU
(benchmarks/ai-benchmark/benchmark.py:11-62, gen_report.py:25-47,
benchmarks/deployments/job-on-hami.yml).  This engine is the MI355X-native
stand-in: the Qwen3 decoder of models/qwen3.py (random-init weights of the
exact architecture; no network for checkpoints) with

  * prefill of the prompt in one pass (``Qwen3Decoder.prefill``), replayed
    as one captured hipGraph per prompt-length bucket (32 ... 8192 tokens;
    causal flash attention, csrc/ops/prefill_attn.hip),
  * decode as replays of one captured hipGraph per token (the hand-written
    gfx950 kernels: skinny MFMA GEMMs, fused decode attention, norms),
  * one request at a time (the reference client is sequential), tokens
    yielded as they are produced so the server can stream them.

Text goes through a byte-level tokenizer: with random weights the output is
meaningless, only its timing is measured.
"""

from __future__ import annotations

import queue
import threading
import time
from dataclasses import dataclass

import torch

from k8s_vgpu_scheduler_amd.models.qwen3 import QWEN3_8B, QWEN3_TINY, Qwen3Config, Qwen3Decoder

MODELS = {"qwen3-8b": QWEN3_8B, "qwen3-tiny": QWEN3_TINY}


class ByteTokenizer:
    """UTF-8 bytes as token ids (offset past a few specials), a Qwen-style chat
    template, and printable ASCII for generated ids."""

    SPECIALS = {"<|endoftext|>": 0, "<|im_start|>": 1, "<|im_end|>": 2}
    OFFSET = 3

    def __init__(self, vocab: int):
        if vocab < 256 + self.OFFSET:
            raise ValueError("vocab too small for a byte tokenizer")
        self.vocab = vocab

    def encode(self, text: str) -> list[int]:
        return [b + self.OFFSET for b in text.encode("utf-8")]

    def chat(self, messages: list[dict]) -> list[int]:
        ids: list[int] = []
        for m in messages:
            ids += [self.SPECIALS["<|im_start|>"]] + self.encode(f"{m.get('role', 'user')}\n")
            ids += self.encode(str(m.get("content", ""))) + [self.SPECIALS["<|im_end|>"]] + self.encode("\n")
        return ids + [self.SPECIALS["<|im_start|>"]] + self.encode("assistant\n")

    @staticmethod
    def decode_one(tok: int) -> str:
        return chr(0x20 + tok % 95)


@dataclass
class Generation:
    prompt_tokens: int
    tokens: list


_END = object()


class Engine:
    """Owns the GPU from one thread: the decoder is built, warmed, captured and
    run only on the engine thread (hipBLASLt handles and workspaces, the
    captured graph and the caching allocator all see a single host thread);
    request threads hand it jobs and receive token ids through queues.  Jobs
    run in arrival order, one at a time, and the engine moves on to the next
    token while the previous one is being written to the client."""

    def __init__(self, model: str | Qwen3Config = "qwen3-8b", max_ctx: int = 4096, device: str | None = None,
                 graph: bool = True, seed: int = 0, max_prefill_graph: int = 8192,
                 gpu_memory_utilization: float | None = None):
        cfg = MODELS[model] if isinstance(model, str) else model
        self.cfg = cfg
        self.model_name = cfg.name
        self.tok = ByteTokenizer(cfg.vocab)
        self._jobs: queue.Queue = queue.Queue()
        self._ready = threading.Event()
        self._err: BaseException | None = None
        self.dec = None
        self.graph = False
        self.load_s = 0.0
        self.mem_total_mib = None
        self.gpu_memory_utilization = gpu_memory_utilization
        self._th = threading.Thread(target=self._loop, args=(cfg, max_ctx, device, graph, seed, max_prefill_graph),
                                    name="mivgpu-engine", daemon=True)
        self._th.start()
        self._ready.wait()
        if self._err is not None:
            raise self._err

    # ----------------------------------------------------------- engine thread
    @staticmethod
    def kv_bytes_per_token(cfg: Qwen3Config) -> int:
        return cfg.layers * 2 * cfg.kv_heads * cfg.head_dim * 2          # K and V, bf16

    def size_context(self, cfg, max_ctx, util):
        """vLLM-style --gpu-memory-utilization: the context (KV tokens) that
        fits in ``util`` of the device memory the process sees -- inside a
        slice that is the grant (libmivgpu.so virtualises hipMemGetInfo), not
        the card -- after the weights and a working margin."""
        free, total = torch.cuda.mem_get_info()
        self.mem_total_mib = total >> 20
        budget = int(total * util) - (total - free) - cfg.param_count() * 2 - (2 << 30)
        fit = max(0, budget) // self.kv_bytes_per_token(cfg) // 32 * 32
        if fit < 64:
            raise RuntimeError(f"{total >> 20} MiB visible: no room for a KV cache after the weights")
        return min(max_ctx, fit)

    def _build(self, cfg, max_ctx, device, graph, seed, max_prefill_graph):
        t0 = time.perf_counter()
        dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
        if dev != "cpu":
            free, total = torch.cuda.mem_get_info()
            self.mem_total_mib = total >> 20
            if self.gpu_memory_utilization:
                max_ctx = self.size_context(cfg, max_ctx, self.gpu_memory_utilization)
        self.dec = Qwen3Decoder(cfg, batch=1, max_ctx=max_ctx, device=dev, seed=seed)
        self.graph = graph and self.dec.device.type == "cuda"
        if self.dec.skinny:
            self.dec.reserve_prefill()
        if self.graph:
            # one graph per prompt-length bucket, then the decode step's
            self.dec.capture_prefill([b for b in self.dec.PREFILL_BUCKETS if b <= max_prefill_graph])
            self.dec.prefill(self._warm_prompt())
            self.dec.capture()
        else:
            self.dec.prefill(self._warm_prompt())
        self._sync()
        self.load_s = time.perf_counter() - t0

    def _warm_prompt(self) -> list[int]:
        return self.tok.encode("warm up " * 20)[:max(1, self.dec.T // 2)]

    def _loop(self, cfg, max_ctx, device, graph, seed, max_prefill_graph):
        try:
            self._build(cfg, max_ctx, device, graph, seed, max_prefill_graph)
        except BaseException as e:  # noqa: BLE001 -- reported to the constructor
            self._err = e
            self._ready.set()
            return
        self._ready.set()
        while True:
            job = self._jobs.get()
            if job is None:
                return
            prompt_ids, n, out, cancel = job
            try:
                with torch.no_grad():
                    self.dec.prefill(prompt_ids)
                    out.put(int(self.dec.tokens[0]))
                    for _ in range(n - 1):
                        if cancel.is_set():
                            break
                        out.put(self._step())
                out.put(_END)
            except Exception as e:  # noqa: BLE001 -- handed to the request
                out.put(e)

    def _sync(self):
        if self.dec.device.type == "cuda":
            torch.cuda.synchronize()

    def _step(self) -> int:
        if self.graph:
            self.dec.graph.replay()
        else:
            self.dec._step_impl()
        return int(self.dec.tokens[0])      # waits for this token

    # --------------------------------------------------------- request side
    @property
    def max_ctx(self) -> int:
        return self.dec.T

    def stream(self, prompt_ids: list[int], max_tokens: int):
        """Yield generated token ids one by one (the first right after prefill)."""
        n = max(0, min(max_tokens, self.dec.T - len(prompt_ids) - 1))
        if n == 0:
            return
        if not self._th.is_alive():
            raise RuntimeError("the engine thread is gone")
        out: queue.Queue = queue.Queue()
        cancel = threading.Event()
        self._jobs.put((list(prompt_ids), n, out, cancel))
        try:
            while True:
                try:
                    x = out.get(timeout=1.0)
                except queue.Empty:
                    if not self._th.is_alive():
                        raise RuntimeError("the engine thread is gone") from None
                    continue
                if x is _END:
                    return
                if isinstance(x, BaseException):
                    raise x
                yield x
        finally:
            cancel.set()        # a client that went away stops its job at the next token

    def generate(self, prompt_ids: list[int], max_tokens: int) -> Generation:
        return Generation(len(prompt_ids), list(self.stream(prompt_ids, max_tokens)))

    def close(self):
        if self._th.is_alive():
            self._jobs.put(None)
            self._th.join()
