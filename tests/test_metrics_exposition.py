"""Prometheus exposition hygiene of the monitor's collector (both the current
and the --legacy-metrics names): the text parses, every family has HELP and
TYPE, no sample carries an empty or duplicated label set, and every series
the dashboard queries exists (dashboards/mivgpu-mi355x.json)."""

import json
import re
from pathlib import Path

import pytest
from prometheus_client import CollectorRegistry, generate_latest
from prometheus_client.parser import text_string_to_metric_families

from k8s_vgpu_scheduler_amd.monitor.lister import ContainerLister
from k8s_vgpu_scheduler_amd.monitor.metrics import MonitorCollector
from k8s_vgpu_scheduler_amd.smi import FakeBackend

from test_monitor import make_container, pod

ROOT = Path(__file__).resolve().parents[1]


def scrape(tmp_path, legacy):
    make_container(tmp_path, "u1", "main", uuid="GPU-0000", used=300 << 20, limit=2 << 30, recent=2).close()
    make_container(tmp_path, "u2", "side", uuid="GPU-0001", used=100 << 20, limit=1 << 30).close()
    lister = ContainerLister(str(tmp_path), lambda: [pod("u1", "p1", "ns1"), pod("u2", "p2", "ns2")])
    lister.update()
    reg = CollectorRegistry()
    reg.register(MonitorCollector(lister, FakeBackend(n=2), "node1", legacy=legacy))
    return generate_latest(reg).decode()


@pytest.mark.parametrize("legacy", [False, True])
def test_exposition_parses_and_is_well_formed(tmp_path, legacy):
    text = scrape(tmp_path, legacy)
    fams = list(text_string_to_metric_families(text))
    assert fams
    names = [f.name for f in fams]
    assert len(names) == len(set(names)), "a family is exported twice"
    for f in fams:
        assert f.documentation, f"{f.name} has no HELP"
        assert f.type in ("gauge", "counter", "info", "untyped", "summary", "histogram"), f.name
        seen = set()
        for s in f.samples:
            key = (s.name, tuple(sorted(s.labels.items())))
            assert key not in seen, f"duplicate sample {key}"
            seen.add(key)
            assert all(v != "" for k, v in s.labels.items() if k in ("node", "device_uuid")), s


def test_dashboard_queries_known_series(tmp_path):
    dash = json.loads((ROOT / "dashboards" / "mivgpu-mi355x.json").read_text())
    exprs = []

    def walk(o):
        if isinstance(o, dict):
            if isinstance(o.get("expr"), str):
                exprs.append(o["expr"])
            for v in o.values():
                walk(v)
        elif isinstance(o, list):
            for v in o:
                walk(v)
    walk(dash)
    assert exprs
    used = {m for e in exprs for m in re.findall(r"\b((?:hami|mivgpu)_[a-z_]+)", e)}
    import k8s_vgpu_scheduler_amd.monitor.metrics as mm
    import k8s_vgpu_scheduler_amd.scheduler.metrics as sm
    src = Path(mm.__file__).read_text() + Path(sm.__file__).read_text()
    missing = [m for m in sorted(used)
               if m not in src and not (m.endswith("_total") and m[:-len("_total")] in src)]
    assert not missing, f"dashboard queries series nobody exports: {missing}"
