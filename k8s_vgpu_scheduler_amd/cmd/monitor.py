"""``mivgpu-monitor``: node vGPU monitor (metrics :9394 + priority feedback loop).

Reference: cmd/vGPUmonitor/main.go:57-172, feedback.go, metrics.go.  Validates
HOOK_PATH, watches this node's pods only (server-side field selector
spec.nodeName, pkg/monitor/nvidia/cudevshr.go:308) for the container lister,
samples KFD wave occupancy, runs the node's share-board sampler (one
occupancy sampler per GPU whose shares the governed tenants are charged,
monitor/board.py), serves Prometheus (``--legacy-metrics`` adds the
pre-2.x series), and runs the 5 s feedback loop -- paused while the device
plugin holds the compute-partition apply lock (main.go:79-109).  Each pass
also enforces every granted container's HBM from KFD host truth, driven by
the host-owned grant files (monitor/hosttruth.py: over grant, shim not
loaded, excess), writes the verdicts into the read-only control files
(monitor/control.py), and escalates a container that stays over its grant
(``--over-grant-action``, monitor/escalate.py).
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
from k8s_vgpu_scheduler_amd.monitor.occupancy import OccupancySampler
from k8s_vgpu_scheduler_amd.smi import detect
from k8s_vgpu_scheduler_amd.utils.logsetup import setup_logging


def main(argv=None):
    ap = argparse.ArgumentParser("mivgpu-monitor")
    ap.add_argument("--metrics-bind-address", default=":9394")
    ap.add_argument("--node-name", default=os.environ.get("NODE_NAME", ""))
    ap.add_argument("--hook-path", default=os.environ.get("HOOK_PATH", "/usr/local/vgpu"))
    ap.add_argument("--kubeconfig", default=None)
    ap.add_argument("--smi-backend", default=None)
    ap.add_argument("--legacy-metrics", action="store_true",
                    help="also export the pre-2.x metric names (HostGPUMemoryUsage, vGPU_device_memory_*, ...)")
    ap.add_argument("--occupancy-period", type=float, default=0.05,
                    help="seconds between KFD wave-occupancy samples (0 = off)")
    ap.add_argument("--no-host-truth", action="store_true",
                    help="do not recompute container HBM usage from KFD each pass (trust the shared regions)")
    ap.add_argument("--over-grant-action", choices=("block", "evict", "kill"), default="block",
                    help="what happens to a container over its HBM grant (host truth) for --over-grant-passes "
                         "passes: block its launches (control file), evict its pod (Eviction API), or SIGKILL "
                         "its host processes holding VRAM")
    ap.add_argument("--shimless-action", choices=("none", "evict", "kill"), default=None,
                    help="a container holding VRAM with no live libmivgpu.so that is over its HBM grant or on a "
                         "GPU only the governor limits (time-sharing) is evicted / killed after --over-grant-passes "
                         "passes whatever --over-grant-action says (default: evict; kill under "
                         "--over-grant-action kill)")
    ap.add_argument("--proc-root", default="/proc",
                    help="process table the host-truth pass maps pods to host pids from (a directory laid out like "
                         "/proc: <pid>/status and <pid>/cgroup; the e2e tests point it at a copy naming pod cgroups)")
    ap.add_argument("--over-grant-passes", type=int, default=3,
                    help="consecutive over-grant passes before --over-grant-action evict/kill")
    ap.add_argument("--board-period-us", type=int, default=2000,
                    help="the node share-board sampler's period while any GPU has waves resident "
                         "(mivgpu-boardd: one wave-occupancy sampler per GPU for every tenant; 0 = off)")
    ap.add_argument("--state-file", default=os.environ.get("MIVGPU_MONITOR_STATE", ""),
                    help="write each feedback pass's host-truth state (uuid -> KFD gpu_id map and how it matched, "
                         "host pids per pod, vram per pid, grants, verdicts, escalation counters) to this JSON file")
    ap.add_argument("-v", type=int, default=2)
    a = ap.parse_args(argv)
    setup_logging(a.v)
    log = logging.getLogger("mivgpu.monitor")
    if not os.path.isdir(a.hook_path):
        raise SystemExit(f"HOOK_PATH {a.hook_path} does not exist")
    from k8s_vgpu_scheduler_amd.k8s.rest import RestClient
    client = init_global_client(RestClient.from_env(a.kubeconfig))
    inf = Informer(client, "pods", field_selector={"spec.nodeName": a.node_name})
    inf.start()
    lister = ContainerLister(a.hook_path, inf.list)
    try:
        # one lock around every amd-smi call: scrapes and the feedback pass
        # run on different threads
        from k8s_vgpu_scheduler_amd.smi import SerializedBackend
        backend = SerializedBackend(detect(a.smi_backend))
    except RuntimeError as e:
        log.warning("no amd-smi backend (%s): host metrics disabled", e)
        backend = None
    occ = OccupancySampler(period_s=a.occupancy_period).start() if a.occupancy_period > 0 else None
    board = None
    if a.board_period_us > 0:
        from k8s_vgpu_scheduler_amd.monitor.board import BoardSampler, board_host_dir
        board = BoardSampler(board_host_dir(a.hook_path), period_us=a.board_period_us).start()
    truth = escalation = None
    if not a.no_host_truth:
        from k8s_vgpu_scheduler_amd.monitor.escalate import OverGrantPolicy
        from k8s_vgpu_scheduler_amd.monitor.hosttruth import HostTruth, kfd_gpu_ids
        from k8s_vgpu_scheduler_amd.scheduler.events import EventRecorder
        events = EventRecorder(client, component="hami-vgpu-monitor")
        truth = HostTruth(kfd_gpu_ids(backend), events=events, proc_root=a.proc_root)
        escalation = OverGrantPolicy(a.over_grant_action, a.over_grant_passes, client=client, events=events,
                                     shimless_action=a.shimless_action)
    reg = CollectorRegistry()
    reg.register(MonitorCollector(lister, backend, a.node_name, occupancy=occ, legacy=a.legacy_metrics,
                                  truth=truth, escalation=escalation, board=board))
    host, _, port = a.metrics_bind_address.rpartition(":")
    start_http_server(int(port), addr=host or "0.0.0.0", registry=reg)
    stop = threading.Event()
    pause = threading.Event()
    threading.Thread(target=watch_partition_lock, args=(pause, stop), name="partition-lock", daemon=True).start()
    try:
        watch_and_feedback(lister, stop, pause=pause, truth=truth, escalation=escalation,
                           board_dir=board.dir if board is not None else None, state_file=a.state_file or None,
                           board=board)
    finally:
        if board is not None:
            board.stop()
    return 0


def watch_partition_lock(pause: threading.Event, stop: threading.Event, lock_path: str | None = None,
                         poll: float = 1.0):
    """Mirror the device plugin's partition apply lock into ``pause``."""
    from k8s_vgpu_scheduler_amd.deviceplugin.partition import APPLY_LOCK, is_applying
    log = logging.getLogger("mivgpu.monitor")
    path = lock_path or APPLY_LOCK
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
    except OSError:   # read-only mount of the device plugin's lock dir
        pass
    while True:
        busy = is_applying(path)
        if busy and not pause.is_set():
            log.info("partition apply lock %s present: feedback paused", path)
            pause.set()
        elif not busy and pause.is_set():
            log.info("partition apply lock released: feedback resumed")
            pause.clear()
        if stop.wait(poll):
            return


if __name__ == "__main__":
    raise SystemExit(main())
