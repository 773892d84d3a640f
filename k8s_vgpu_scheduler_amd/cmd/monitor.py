"""``mivgpu-monitor``: node vGPU monitor (metrics :9394 + priority feedback loop).

Reference: cmd/vGPUmonitor/main.go:57-172, feedback.go, metrics.go.  Validates
HOOK_PATH, lists this node's pods (field selector spec.nodeName) for the
container lister, serves Prometheus, and runs the 5 s feedback loop.
"""

from __future__ import annotations

import argparse
import logging
import os
import threading

from prometheus_client import CollectorRegistry, start_http_server

from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.informer import Informer
from k8s_vgpu_scheduler_amd.monitor.feedback import watch_and_feedback
from k8s_vgpu_scheduler_amd.monitor.lister import ContainerLister
from k8s_vgpu_scheduler_amd.monitor.metrics import MonitorCollector
from k8s_vgpu_scheduler_amd.smi import detect
from k8s_vgpu_scheduler_amd.utils.logsetup import setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("mivgpu-monitor")
    ap.add_argument("--metrics-bind-address", default=":9394")
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME", ""))
    ap.add_argument("--hook-path", default=os.environ.get("HOOK_PATH", "/usr/local/vgpu"))
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--smi-backend", default=None)
    ap.add_argument("-v", type=int, default=2)
    a = ap.parse_args(argv)
    setup_logging(a.v)
    log = logging.getLogger("mivgpu.monitor")
    if not os.path.isdir(a.hook_path):
        raise SystemExit(f"HOOK_PATH {a.hook_path} does not exist")
    from k8s_vgpu_scheduler_amd.k8s.rest import RestClient
    client = init_global_client(RestClient.from_env(a.kubeconfig))
    inf = Informer(client, "pods")
    inf.start()
    pods = (lambda: [p for p in inf.list() if (p.get("spec") or {}).get("nodeName") == a.node_name])
    lister = ContainerLister(a.hook_path, pods)
    try:
        backend = detect(a.smi_backend)
    except RuntimeError as e:
        log.warning("no amd-smi backend (%s): host metrics disabled", e)
        backend = None
    reg = CollectorRegistry()
    reg.register(MonitorCollector(lister, backend, a.node_name))
    host, _, port = a.metrics_bind_address.rpartition(":")
    start_http_server(int(port), addr=host or "0.0.0.0", registry=reg)
    stop = threading.Event()
    watch_and_feedback(lister, stop)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
