"""Container Device Interface (CDI) spec for MI355X GPUs.

Reference: pkg/device-plugin/nvidiadevice/nvinternal/cdi/cdi.go:60-279 (spec
generation, qualified names, a null handler when CDI is off) and the plugin's
device-list strategies (envvar / cdi-annotations / cdi-cri).  The AMD form is
simpler: a GPU is `/dev/kfd` (shared by all GPUs) plus its DRM nodes.  The
spec names each GPU by its registered UUID and by its index; the in-container
limiter (shim + preload) stays a per-container mount from Allocate because
its host directory is per container.

    kind:  amd.com/gpu      device: amd.com/gpu=<uuid>
"""

from __future__ import annotations

import json
import os
from pathlib import Path

CDI_VERSION = "0.6.0"
DEFAULT_KIND = "amd.com/gpu"
DEFAULT_DIR = "/var/run/cdi"
STRATEGIES = ("envvar", "cdi-annotations", "cdi-cri")
ANNOTATION_PREFIX = "cdi.k8s.io/"


def qualified_name(kind: str, device: str) -> str:
    return f"{kind}={device}"


def _nodes(g) -> list[dict]:
    out = []
    if g.render_minor >= 0:
        out.append({"path": f"/dev/dri/renderD{g.render_minor}"})
    if g.card_minor >= 0:
        out.append({"path": f"/dev/dri/card{g.card_minor}"})
    return out


def build_spec(gpus, kind: str = DEFAULT_KIND) -> dict:
    devices = []
    for g in gpus:
        edits = {"deviceNodes": _nodes(g)}
        devices.append({"name": g.uuid, "containerEdits": edits})
        devices.append({"name": str(g.index), "containerEdits": edits})
    return {
        "cdiVersion": CDI_VERSION,
        "kind": kind,
        "devices": devices,
        "containerEdits": {"deviceNodes": [{"path": "/dev/kfd"}]},
    }


def validate_spec(spec: dict):
    if spec.get("cdiVersion") != CDI_VERSION:
        raise ValueError("unsupported cdiVersion")
    vendor, _, cls = spec.get("kind", "").partition("/")
    if not vendor or not cls or "." not in vendor:
        raise ValueError(f"invalid CDI kind {spec.get('kind')!r}")
    names = [d["name"] for d in spec.get("devices", [])]
    if len(names) != len(set(names)):
        raise ValueError("duplicate CDI device names")
    for d in spec["devices"]:
        for n in d["containerEdits"].get("deviceNodes", []):
            if not n["path"].startswith("/dev/"):
                raise ValueError(f"bad device node {n['path']}")


def spec_path(spec_dir: str, kind: str = DEFAULT_KIND) -> Path:
    return Path(spec_dir) / (kind.replace("/", "-") + ".json")


def write_spec(spec: dict, spec_dir: str = DEFAULT_DIR) -> Path:
    validate_spec(spec)
    p = spec_path(spec_dir, spec["kind"])
    p.parent.mkdir(parents=True, exist_ok=True)
    tmp = p.with_suffix(".json.tmp")
    tmp.write_text(json.dumps(spec, indent=1))
    os.replace(tmp, p)
    return p


def annotation_key(ctr_name: str) -> str:
    return f"{ANNOTATION_PREFIX}mivgpu_{ctr_name}"
