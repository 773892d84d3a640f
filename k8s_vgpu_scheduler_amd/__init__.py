"""MI355X-native GPU virtualisation middleware for Kubernetes.

Capability parity target: HAMi v2.10.0 (soitun/k8s-vgpu-scheduler, see
SURVEY.md).  Pods request ``amd.com/gpu``, ``amd.com/gpumem`` (MiB) and
``amd.com/gpucores`` (percent); the scheduler extender places them on xGMI-aware
GPU sets, the device plugin injects ``ROCR_VISIBLE_DEVICES`` / ``HSA_CU_MASK`` /
``HIP_DEVICE_MEMORY_LIMIT_i`` and the in-container shim ``libmivgpu.so``
enforces the slice.
"""

__version__ = "0.1.0"
