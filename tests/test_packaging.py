"""Packaging: Helm chart consistency, init scripts, and the example pod specs
going through the webhook + scheduler against a fake MI355X node."""

import base64
import json
import os
import re
import subprocess
from pathlib import Path

import pytest
import yaml

from k8s_vgpu_scheduler_amd.device.quota import get_local_cache
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
from k8s_vgpu_scheduler_amd.scheduler.config import SchedulerConfig, init_devices_with_config
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.scheduler.webhook import Webhook
from k8s_vgpu_scheduler_amd.testing import amd_node, full_mesh_scores, mi355x_devices

ROOT = Path(__file__).resolve().parents[1]
CHART = ROOT / "charts" / "mivgpu"


def _values_paths(d, prefix=()):
    out = set()
    for k, v in d.items():
        p = prefix + (k,)
        out.add(p)
        if isinstance(v, dict):
            out |= _values_paths(v, p)
    return out


def test_chart_values_references_exist():
    values = yaml.safe_load((CHART / "values.yaml").read_text())
    known = _values_paths(values)
    missing = []
    for t in CHART.rglob("templates/**/*"):
        if t.is_dir():
            continue
        for m in re.finditer(r"\.Values((?:\.[A-Za-z0-9_]+)+)", t.read_text()):
            path = tuple(m.group(1).strip(".").split("."))
            if path not in known:
                missing.append((t.name, ".".join(path)))
    assert not missing, missing


def test_chart_blocks_balanced_and_yaml_like():
    chart = yaml.safe_load((CHART / "Chart.yaml").read_text())
    assert chart["apiVersion"] == "v2" and chart["name"] == "mivgpu"
    for t in CHART.rglob("templates/**/*.yaml"):
        s = t.read_text()
        opens = len(re.findall(r"{{-?\s*(?:if|with|range|define)\b", s))
        ends = len(re.findall(r"{{-?\s*end\s*-?}}", s))
        assert opens == ends, (t.name, opens, ends)


def test_chart_scheduler_args_match_cli():
    """Every --flag the chart passes exists in the binaries' argparse."""
    from k8s_vgpu_scheduler_amd.cmd import device_plugin, monitor  # noqa: F401
    src = {"scheduler": (ROOT / "k8s_vgpu_scheduler_amd/scheduler/config.py").read_text()
           + (ROOT / "k8s_vgpu_scheduler_amd/cmd/scheduler.py").read_text(),
           "device_plugin": (ROOT / "k8s_vgpu_scheduler_amd/cmd/device_plugin.py").read_text(),
           "monitor": (ROOT / "k8s_vgpu_scheduler_amd/cmd/monitor.py").read_text()}
    files = {"scheduler": CHART / "templates/scheduler/deployment.yaml",
             "device_plugin": CHART / "templates/device-plugin/daemonset.yaml",
             "monitor": CHART / "templates/device-plugin/daemonset.yaml"}
    for binary, f in files.items():
        text = f.read_text()
        if binary == "scheduler":
            text = text.split("- name: extender", 1)[1]
        elif binary == "device_plugin":
            text = text.split("- name: monitor", 1)[0]
        else:
            text = text.split("- name: monitor", 1)[1]
        for flag in set(re.findall(r"- (--[a-z][a-z0-9_-]*)", text)):
            assert f'"{flag}"' in src[binary], (binary, flag)


def test_vgpu_init_installs_atomically(tmp_path):
    src = tmp_path / "libmivgpu.so"
    src.write_bytes(b"\x7fELF-fake")
    dest = tmp_path / "hook"
    env = dict(os.environ, MIVGPU_LIB=str(src))
    subprocess.run(["bash", str(ROOT / "docker/vgpu-init.sh"), str(dest)], check=True, env=env)
    assert (dest / "libmivgpu.so").read_bytes() == b"\x7fELF-fake"
    assert (dest / "ld.so.preload").read_text() == "/usr/local/vgpu/libmivgpu.so\n"
    assert (dest / "containers").is_dir()
    r = subprocess.run(["bash", str(ROOT / "docker/vgpu-init.sh"), str(dest)], env=dict(env, MIVGPU_LIB="/nope"))
    assert r.returncode == 1


def _example_pods():
    for f in sorted((ROOT / "examples/amd").glob("*.yaml")):
        docs = [d for d in yaml.safe_load_all(f.read_text()) if d]
        for i, doc in enumerate(docs):
            if doc["kind"] == "Job":
                pod = {"apiVersion": "v1", "kind": "Pod",
                       "metadata": {"name": doc["metadata"]["name"], "namespace": "default"},
                       "spec": doc["spec"]["template"]["spec"]}
            else:
                pod = doc
                pod["metadata"].setdefault("namespace", "default")
            yield (f.name if len(docs) == 1 else f"{f.name}#{i}"), pod


@pytest.mark.parametrize("name,pod", list(_example_pods()), ids=lambda v: v if isinstance(v, str) else "")
def test_examples_admit_and_schedule(name, pod):
    c = FakeCluster()
    init_global_client(c)
    init_devices_with_config()
    get_local_cache().quotas.clear()
    devs = mi355x_devices("n1")
    c.create("nodes", amd_node("n1", scores=full_mesh_scores(devs)))
    s = Scheduler(c, SchedulerConfig())
    s.start()
    s.register()
    review = Webhook("hami-scheduler").handle_review(
        {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": {"uid": "u", "object": pod}})
    assert review["response"]["allowed"], (name, review["response"])
    ops = json.loads(base64.b64decode(review["response"]["patch"])) if "patch" in review["response"] else []
    assert any(o["path"] == "/spec/schedulerName" for o in ops), name
    c.create("pods", pod)
    got = s.filter({"Pod": c.get_pod("default", pod["metadata"]["name"]), "NodeNames": ["n1"]})
    if name == "select_card.yaml":   # asks for UUIDs this node does not have
        assert got["NodeNames"] in (None, []) and "n1" in got["FailedNodes"]
    else:
        assert got["NodeNames"] == ["n1"], (name, got)


def test_dashboard_queries_exported_series():
    dash = json.loads((ROOT / "dashboards/mivgpu-mi355x.json").read_text())
    src = ((ROOT / "k8s_vgpu_scheduler_amd/scheduler/metrics.py").read_text()
           + (ROOT / "k8s_vgpu_scheduler_amd/monitor/metrics.py").read_text())
    exported = set(re.findall(r'"((?:hami|mivgpu)_[a-z_]+)"', src))
    used = set()
    for p in dash["panels"]:
        for t in p["targets"]:
            used |= set(re.findall(r"\b((?:hami|mivgpu)_[a-z_]+)", t["expr"]))
    assert used and used <= exported, used - exported


# pip distribution that provides each importable top-level module
_DIST = {"grpc": "grpcio", "google": "protobuf", "yaml": "pyyaml", "prometheus_client": "prometheus_client",
         "requests": "requests", "amdsmi": "/opt/rocm/share/amd_smi"}


def _reachable_third_party(entry_points):
    """Top-level third-party modules imported (anywhere, transitively within the
    package) by the given entry-point modules."""
    import ast
    import sys

    pkg = "k8s_vgpu_scheduler_amd"
    std = set(sys.stdlib_module_names)
    seen, ext, todo = set(), {}, list(entry_points)

    def modfile(name):
        p = ROOT / name.replace(".", "/")
        return p / "__init__.py" if (p / "__init__.py").exists() else (p.with_suffix(".py") if p.with_suffix(
            ".py").exists() else None)
    while todo:
        m = todo.pop()
        if m in seen:
            continue
        seen.add(m)
        f = modfile(m)
        if f is None:
            continue
        base = m if f.name == "__init__.py" else m.rsplit(".", 1)[0]
        for node in ast.walk(ast.parse(f.read_text())):
            names = []
            if isinstance(node, ast.Import):
                names = [a.name for a in node.names]
            elif isinstance(node, ast.ImportFrom):
                mod = node.module or ""
                if node.level:
                    parts = base.split(".")
                    mod = ".".join(parts[:len(parts) - node.level + 1] + ([mod] if mod else []))
                names = [mod] + [f"{mod}.{a.name}" for a in node.names]
            for n in names:
                top = n.split(".")[0] if n else ""
                if top == pkg:
                    todo.append(n)
                elif top and top not in std:
                    ext.setdefault(top, set()).add(m)
    return ext


def test_runtime_image_installs_every_import():
    """the runtime stage must install every third-party
    module reachable from the scheduler, device-plugin and monitor binaries."""
    ext = _reachable_third_party([f"k8s_vgpu_scheduler_amd.cmd.{b}" for b in ("scheduler", "device_plugin", "monitor")])
    docker = (ROOT / "docker" / "Dockerfile").read_text()
    runtime = docker[docker.rindex("FROM "):]
    missing = {m: sorted(by) for m, by in ext.items() if _DIST.get(m, m) not in runtime}
    assert not missing, f"runtime image lacks {missing}"
    assert {"grpc", "prometheus_client", "requests", "yaml"} <= set(ext)


def test_grant_keys_match_the_shim():
    """The device plugin writes exactly the settings the shim takes from the
    grant file (is_grant_key in csrc/shim/mivgpu_shim.cpp)."""
    import re

    from k8s_vgpu_scheduler_amd.deviceplugin.allocate import GRANT_KEYS
    src = (ROOT / "csrc" / "shim" / "mivgpu_shim.cpp").read_text()
    body = src[src.index("bool is_grant_key(const char* key)"):]
    body = body[:body.index("for (const char* k : kKeys)")]
    shim_keys = set(re.findall(r'"([A-Z_]+)"', body))
    assert shim_keys == set(GRANT_KEYS), shim_keys ^ set(GRANT_KEYS)
