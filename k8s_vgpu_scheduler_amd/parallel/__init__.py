"""Multi-GPU helpers: process-group setup and the RCCL/xGMI collective validator.

The reference has no collective code of its own: its only
multi-GPU concern is that a TP/DP pod lands on well-connected devices and that
the in-container shim does not break IPC-based collectives
(examples/nvidia/vllm_cross_vgpu.yaml:99-102).  The MI355X build proves both
with :mod:`.collectives` — one process per GPU, ``torch.distributed`` over RCCL
(backend ``"nccl"`` on ROCm), bus bandwidth per collective and message size,
compared against the xGMI link budget of the allocated GPU pair.
"""

from k8s_vgpu_scheduler_amd.parallel.dist import DistEnv, init_distributed, shutdown  # noqa: F401
