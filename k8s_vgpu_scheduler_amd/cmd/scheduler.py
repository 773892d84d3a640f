"""``mivgpu-scheduler``: scheduler extender + admission webhook + metrics.

Reference: cmd/scheduler/main.go:62-200.  Starts the informer-backed
Scheduler, the registration loop, the Prometheus endpoint (:9395) and the
HTTP(S) extender server with /filter /bind /webhook /healthz /readyz.

    python -m k8s_vgpu_scheduler_amd.cmd.scheduler --http_bind 0.0.0.0:443 \
        --cert_file /tls/tls.crt --key_file /tls/tls.key --scheduler-name hami-scheduler
"""

from __future__ import annotations

import argparse
import logging
import signal
import threading
import time

from prometheus_client import CollectorRegistry, start_http_server

from k8s_vgpu_scheduler_amd import __version__
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.rest import RestClient
from k8s_vgpu_scheduler_amd.scheduler import config as C
from k8s_vgpu_scheduler_amd.scheduler.metrics import SchedulerCollector
from k8s_vgpu_scheduler_amd.scheduler.routes import ExtenderServer
from k8s_vgpu_scheduler_amd.scheduler.scheduler import Scheduler
from k8s_vgpu_scheduler_amd.scheduler.webhook import Webhook
from k8s_vgpu_scheduler_amd.utils import nodelock
from k8s_vgpu_scheduler_amd.utils.logsetup import setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("mivgpu-scheduler")
    C.add_flags(ap)
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--version", action="store_true")
    a = ap.parse_args(argv)
    if a.version:
        print(__version__)
        return 0
    setup_logging(a.v, a.debug)
    log = logging.getLogger("mivgpu.scheduler")
    cfg = C.from_args(a)
    for k, v in sorted(vars(a).items()):
        log.info("FLAG: --%s=%r", k, v)
    nodelock.NODE_LOCK_TIMEOUT = cfg.node_lock_timeout
    client = init_global_client(RestClient.from_env(a.kubeconfig, qps=cfg.kube_qps, burst=cfg.kube_burst,
                                                    timeout=cfg.kube_timeout))
    C.init_devices_with_config(C.load_device_config(cfg.device_config_file), cfg.gpu_scheduler_policy)
    sched = Scheduler(client, cfg)
    sched.start()
    threading.Thread(target=sched.run_register_loop, name="register", daemon=True).start()

    reg = CollectorRegistry()
    reg.register(SchedulerCollector(sched, legacy=cfg.legacy_metrics))
    host, _, port = cfg.metrics_bind_address.rpartition(":")
    start_http_server(int(port), addr=host or "0.0.0.0", registry=reg)

    server = ExtenderServer(sched, Webhook(cfg.scheduler_name, cfg.force_overwrite_default_scheduler),
                            cfg.http_bind, cfg.cert_file, cfg.key_file, cfg.profiling).start()
    log.info("mivgpu-scheduler %s listening on %s", __version__, cfg.http_bind)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    while not stop.wait(5.0):
        try:
            if server.maybe_reload_cert():
                log.info("TLS certificate reloaded")
        except OSError as e:
            log.error("cert reload failed: %s", e)
    server.stop()
    sched.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
