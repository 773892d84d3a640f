"""Locating and configuring the in-container shim ``libmivgpu.so``.

The env-var contract written by the device plugin's ``Allocate`` (AMD analogue
of the reference's CUDA_* contract, server.go:833-847):

* ``HIP_DEVICE_MEMORY_LIMIT_<i>=<MiB>m`` -- per container-local device HBM cap
* ``HIP_DEVICE_CORE_LIMIT=<pct>``         -- CU share (temporal governor)
* ``HSA_CU_MASK=<i>:<ranges>;...``        -- spatial CU partition (ROCr)
* ``GPU_CORE_UTILIZATION_POLICY``         -- default | force | disable
* ``HIP_TASK_PRIORITY``                   -- feedback-loop priority
* ``MIVGPU_SHARED_CACHE``                 -- shared-region file
* ``MIVGPU_OVERSUBSCRIBE`` / ``MIVGPU_LOG_LEVEL`` / ``MIVGPU_DISABLE_CONTROL``
"""

from __future__ import annotations

import os
from pathlib import Path

_PKG = Path(__file__).resolve().parents[1]
DEFAULT_SHIM = _PKG / "lib" / "libmivgpu.so"

ENV_MEM_LIMIT = "HIP_DEVICE_MEMORY_LIMIT"
ENV_CORE_LIMIT = "HIP_DEVICE_CORE_LIMIT"
ENV_CU_MASK = "HSA_CU_MASK"
ENV_POLICY = "GPU_CORE_UTILIZATION_POLICY"
ENV_PRIORITY = "HIP_TASK_PRIORITY"
ENV_CACHE = "MIVGPU_SHARED_CACHE"
ENV_OVERSUB = "MIVGPU_OVERSUBSCRIBE"
ENV_LOG = "MIVGPU_LOG_LEVEL"
ENV_DISABLE = "MIVGPU_DISABLE_CONTROL"
ENV_UUIDS = "MIVGPU_DEVICE_UUIDS"


def shim_path() -> Path:
    p = os.environ.get("MIVGPU_SHIM_PATH")
    return Path(p) if p else DEFAULT_SHIM


def shim_env(existing_preload: str | None = None) -> dict:
    """Environment that activates the shim in a child process."""
    p = str(shim_path())
    pre = existing_preload if existing_preload is not None else os.environ.get("LD_PRELOAD", "")
    parts = [x for x in pre.split(":") if x and x != p]
    return {"LD_PRELOAD": ":".join([p, *parts])}
