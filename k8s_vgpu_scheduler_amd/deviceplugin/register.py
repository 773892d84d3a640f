"""Node registration: publish this node's MI355X GPUs to the scheduler.

Reference: pkg/device-plugin/nvidiadevice/nvinternal/plugin/register.go:92-351
(``getAPIDevices``, ``RegisterInAnnotation``, ``WatchAndRegister``).  Writes
  hami.io/node-amd-register   JSON [DeviceInfo] (count = split count,
                              devmem = MiB x memory scaling, devcore = CUs x core scaling)
  hami.io/node-amd-score      xGMI pair scores (amd-smi link type / hops / bandwidth)
  hami.io/node-handshake-amd  "Reported_<time>" (answers the scheduler's Requesting_)
every 30 s (5 s after an error), skipping the patch when nothing changed.
Asymmetric pair scores are zeroed and reported as a node Warning event
(calculate_score.go:211-286 behaviour).
"""

from __future__ import annotations

import datetime as _dt
import logging
import os
import threading

from k8s_vgpu_scheduler_amd.device import codec
from k8s_vgpu_scheduler_amd.device.amd import topology
from k8s_vgpu_scheduler_amd.device.amd.device import HANDSHAKE_ANNOS, PAIR_SCORE_ANNOS, REGISTER_ANNOS
from k8s_vgpu_scheduler_amd.device.types import MODE_SHARED, DeviceInfo
from k8s_vgpu_scheduler_amd.smi import Backend, GPUInfo, pair_scores, sanitize_type
from k8s_vgpu_scheduler_amd.utils import util

from .allocate import PluginConfig

log = logging.getLogger(__name__)


def filtered(gpus: list[GPUInfo], cfg: PluginConfig) -> list[GPUInfo]:
    return [g for g in gpus if g.uuid not in cfg.filter_uuids and g.index not in cfg.filter_indexes]


def api_devices(backend: Backend, gpus: list[GPUInfo], cfg: PluginConfig) -> list[DeviceInfo]:
    out = []
    for g in filtered(gpus, cfg):
        healthy, _ = backend.health(g)
        out.append(DeviceInfo(id=g.uuid, index=g.index, count=cfg.device_split_count,
                              devmem=int(g.memory_mib * cfg.device_memory_scaling),
                              devcore=int(g.cus * cfg.device_core_scaling), type=sanitize_type(g.name),
                              numa=g.numa, mode=MODE_SHARED if g.compute_partition in ("SPX", "") else
                              g.compute_partition.lower(), health=healthy and g.healthy))
    return out


class Registrar:
    def __init__(self, backend: Backend, cfg: PluginConfig, node_name: str):
        self.backend, self.cfg, self.node = backend, cfg, node_name
        self._last: dict | None = None
        self._stop = threading.Event()

    def annotations(self, gpus: list[GPUInfo]) -> dict:
        devs = api_devices(self.backend, gpus, self.cfg)
        annos = {REGISTER_ANNOS: codec.marshal_node_devices(devs)}
        fg = filtered(gpus, self.cfg)
        # ENABLE_TOPOLOGY_SCORE (reference register.go:279): on by default for
        # MI355X, whose xGMI pair scores drive multi-GPU placement
        topo = os.environ.get("ENABLE_TOPOLOGY_SCORE", "true").strip().lower() not in ("0", "false", "no")
        if topo and len(fg) > 1:
            scores = pair_scores(self.backend, fg)
            bad = topology.is_asymmetric(scores)
            if bad:
                for a, b in bad:
                    scores[a][b] = scores[b][a] = 0
                try:
                    util.emit_node_warning_event(util.get_node(self.node), "AsymmetricXGMILinks",
                                                 f"asymmetric xGMI link data for pairs {bad}; scored 0")
                except Exception as e:  # noqa: BLE001
                    log.warning("could not emit asymmetric-link event: %s", e)
            annos[PAIR_SCORE_ANNOS] = codec.encode_pair_scores(scores)
        return annos

    def register_once(self, gpus: list[GPUInfo] | None = None) -> bool:
        from k8s_vgpu_scheduler_amd.deviceplugin.partition import is_applying

        if is_applying():          # GPUs are being re-partitioned: the device list is in flux
            return False
        gpus = gpus if gpus is not None else self.backend.gpus()
        annos = self.annotations(gpus)
        node = util.get_node(self.node)
        cur = (node.get("metadata") or {}).get("annotations") or {}
        hs = cur.get(HANDSHAKE_ANNOS, "")
        changed = self._last != annos or any(cur.get(k) != v for k, v in annos.items())
        if changed or hs.startswith("Requesting") or not hs:
            patch = dict(annos)
            patch[HANDSHAKE_ANNOS] = "Reported_" + _dt.datetime.now().strftime("%Y-%m-%d %H:%M:%S")
            util.patch_node_annotations(self.node, patch)
            self._last = annos
            return True
        return False

    def watch_and_register(self, period: float = 30.0, err_period: float = 5.0, pause: threading.Event | None = None):
        while not self._stop.is_set():
            wait = period
            if pause is not None and pause.is_set():
                self._stop.wait(1.0)
                continue
            try:
                self.register_once()
            except Exception as e:  # noqa: BLE001
                log.error("registration failed: %s", e)
                wait = err_period
            self._stop.wait(wait)

    def stop(self):
        self._stop.set()
