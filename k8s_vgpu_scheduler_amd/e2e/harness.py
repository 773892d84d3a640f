"""End-to-end harness: the real binaries as processes, a real HTTP API server,
and stand-ins for the two Kubernetes components this system plugs into.

    FakeApiServer  (this process, HTTP)   <- RestClient in every binary
    mivgpu-scheduler      (process)       <- /webhook, /filter, /bind as kube-apiserver / kube-scheduler call them
    mivgpu-device-plugin  (process)       <- kubelet device-plugin gRPC (Register, ListAndWatch,
                                             GetPreferredAllocation, Allocate)
    mivgpu-monitor        (process)       -> /metrics, priority feedback
    FakeKubelet    (this process)         registration server + plugin client; starts the "container":
                                          a child process with the Allocate env, the shim preloaded the
                                          way /etc/ld.so.preload would, and mounts resolved to host paths

This is the call stack of SURVEY.md §3.1-3.5 crossing real process and
protocol boundaries; the reference exercises it with test/e2e on a cluster.
"""

from __future__ import annotations

import base64
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time
from concurrent import futures
from pathlib import Path

import grpc
import requests

from k8s_vgpu_scheduler_amd.deviceplugin import api
from k8s_vgpu_scheduler_amd.e2e.apiserver import FakeApiServer
from k8s_vgpu_scheduler_amd.k8s.fake import make_node

REPO = Path(__file__).resolve().parents[2]


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def wait_for(cond, timeout: float = 30.0, what: str = "condition", period: float = 0.05):
    t0 = time.time()
    last = None
    while time.time() - t0 < timeout:
        try:
            v = cond()
            if v:
                return v
        except Exception as e:  # noqa: BLE001 -- retried until the deadline
            last = e
        time.sleep(period)
    raise TimeoutError(f"timed out waiting for {what}" + (f" (last error: {last})" if last else ""))


def samples(text: str, name: str) -> list[tuple[dict, float]]:
    """(labels, value) of every sample of metric `name` in Prometheus text."""
    from prometheus_client.parser import text_string_to_metric_families
    return [(s.labels, s.value) for fam in text_string_to_metric_families(text) for s in fam.samples
            if s.name == name]


def apply_json_patch(doc: dict, ops: list[dict]) -> dict:
    """RFC 6902 add / replace / remove (what the admission webhook emits)."""
    doc = json.loads(json.dumps(doc))
    for op in ops:
        parts = [p.replace("~1", "/").replace("~0", "~") for p in op["path"].split("/")[1:]]
        parent = doc
        for p in parts[:-1]:
            parent = parent[int(p)] if isinstance(parent, list) else parent.setdefault(p, {})
        last = parts[-1]
        if isinstance(parent, list):
            idx = len(parent) if last == "-" else int(last)
            if op["op"] == "add":
                parent.insert(idx, op["value"])
            elif op["op"] == "replace":
                parent[idx] = op["value"]
            elif op["op"] == "remove":
                parent.pop(idx)
        else:
            if op["op"] in ("add", "replace"):
                parent[last] = op["value"]
            elif op["op"] == "remove":
                parent.pop(last, None)
    return doc


class FakeKubelet:
    """Registration server on `<dir>/kubelet.sock`; after a plugin registers it
    follows ListAndWatch (publishing the device count as node allocatable, as
    the kubelet does) and allocates for pods bound to its node."""

    def __init__(self, workdir: Path, apiserver: FakeApiServer, node: str):
        self.dir = workdir
        self.socket = str(workdir / "kubelet.sock")
        self.api, self.node = apiserver, node
        self.registrations: list = []
        self.devices: list = []
        self._stop = threading.Event()
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        api.add_registration_servicer(self.server, self)
        self.server.add_insecure_port(f"unix://{self.socket}")
        self.channel = None
        self.stub = None

    def start(self) -> "FakeKubelet":
        self.server.start()
        return self

    def stop(self):
        self._stop.set()
        if self.channel is not None:
            self.channel.close()
        self.server.stop(0)

    # ---------------------------------------------------- Registration API
    def Register(self, request, context):  # noqa: N802
        self.registrations.append(request)
        endpoint = str(self.dir / "plugins" / request.endpoint)
        if self.channel is not None:
            self.channel.close()
        self.channel = grpc.insecure_channel(f"unix://{endpoint}")
        self.stub = api.DevicePluginStub(self.channel)
        threading.Thread(target=self._list_and_watch, args=(self.stub, request.resource_name),
                         daemon=True).start()
        return api.Empty()

    def _list_and_watch(self, stub, resource: str):
        try:
            for resp in stub.ListAndWatch(api.Empty()):
                self.devices = list(resp.devices)
                healthy = sum(d.health == api.HEALTHY for d in resp.devices)
                self.api.cluster.patch("nodes", self.node, {"status": {
                    "capacity": {resource: str(len(resp.devices))},
                    "allocatable": {resource: str(healthy)}}})
                if self._stop.is_set():
                    return
        except grpc.RpcError:
            pass      # plugin restarted: it registers again

    # ------------------------------------------------------- pod admission
    def allocate(self, pod: dict, resource: str = "amd.com/gpu") -> list[dict]:
        """Kubelet's Allocate sequence for every container that asks for `resource`."""
        out = []
        healthy = [d.ID for d in self.devices if d.health == api.HEALTHY]
        for ctr in pod["spec"]["containers"]:
            n = int(((ctr.get("resources") or {}).get("limits") or {}).get(resource, 0))
            if n == 0:
                out.append({})
                continue
            pref = api.PreferredAllocationRequest()
            cr = pref.container_requests.add(allocation_size=n)
            cr.available_deviceIDs.extend(healthy)
            ids = list(self.stub.GetPreferredAllocation(pref, timeout=10).container_responses[0].deviceIDs)
            req = api.AllocateRequest()
            req.container_requests.add(devices_ids=ids)
            r = self.stub.Allocate(req, timeout=30).container_responses[0]
            out.append({"device_ids": ids, "envs": dict(r.envs),
                        "mounts": [{"container_path": m.container_path, "host_path": m.host_path,
                                    "read_only": m.read_only} for m in r.mounts],
                        "devices": [{"container_path": d.container_path, "host_path": d.host_path}
                                    for d in r.devices],
                        "annotations": dict(r.annotations)})
        return out


def host_path(path: str, mounts: list[dict]) -> str:
    """Resolve a container path through the bind mounts (longest prefix wins)."""
    best = None
    for m in mounts:
        cp = m["container_path"].rstrip("/")
        if path == cp or path.startswith(cp + "/"):
            if best is None or len(cp) > len(best["container_path"].rstrip("/")):
                best = m
    if best is None:
        return path
    return best["host_path"] + path[len(best["container_path"].rstrip("/")):]


def container_env(alloc: dict, base: dict | None = None) -> dict:
    """What a process in the container sees: the Allocate env, paths mapped to
    the host, and the preload that /etc/ld.so.preload would apply."""
    env = dict(base if base is not None else os.environ)
    env.update(alloc["envs"])
    mounts = alloc["mounts"]
    for k in ("MIVGPU_SHARED_CACHE", "MIVGPU_CONTROL_FILE", "MIVGPU_BOARD_DIR", "MIVGPU_BOARD_FLAGS_DIR"):
        if k in env:
            env[k] = host_path(env[k], mounts)
    from k8s_vgpu_scheduler_amd.deviceplugin.allocate import LIMITS_PATH, grant_text, parse_grant
    grant = next((m for m in mounts if m["container_path"] == LIMITS_PATH), None)
    if grant is not None:
        # the shim reads the grant from the read-only mount; on the host the
        # same file (with its region path mapped) is named by MIVGPU_LIMITS_FILE
        g = parse_grant(Path(grant["host_path"]).read_text())
        for k in ("MIVGPU_SHARED_CACHE", "MIVGPU_CONTROL_FILE", "MIVGPU_BOARD_DIR", "MIVGPU_BOARD_FLAGS_DIR"):
            if k in g:
                g[k] = host_path(g[k], mounts)
        hp = Path(grant["host_path"] + ".host")
        hp.write_text(grant_text(g))
        env["MIVGPU_LIMITS_FILE"] = str(hp)
    preload = next((m for m in mounts if m["container_path"] == "/etc/ld.so.preload"), None)
    if preload is not None:
        libs = [host_path(l.strip(), mounts) for l in Path(preload["host_path"]).read_text().splitlines()
                if l.strip()]
        env["LD_PRELOAD"] = ":".join(libs + [p for p in env.get("LD_PRELOAD", "").split(":") if p])
    return env


class E2ECluster:
    """One node, the three binaries, the API server and the kubelet."""

    def __init__(self, workdir: str | None = None, node: str = "node1", smi_backend: str = "fake",
                 fake_gpus: int = 2, split: int = 4, extra_env: dict | None = None, log_level: int = 3,
                 device_config: dict | None = None, monitor_args: list[str] | None = None):
        self.dir = Path(workdir or tempfile.mkdtemp(prefix="mivgpu-e2e-"))
        self.node, self.smi_backend, self.fake_gpus, self.split = node, smi_backend, fake_gpus, split
        self.extra_env = extra_env or {}
        self.log_level = log_level
        self.device_config = device_config   # the scheduler's --device-config-file contents ({"amd": {...}})
        self.monitor_args = list(monitor_args or [])   # extra mivgpu-monitor flags
        self.procs: dict[str, subprocess.Popen] = {}
        self.ports = {k: free_port() for k in ("http", "sched_metrics", "mon_metrics")}
        self.hook = self.dir / "hook"

    # -------------------------------------------------------------- start
    def _spawn(self, name: str, args: list[str]):
        env = dict(os.environ)
        env.update({"PYTHONPATH": str(REPO) + os.pathsep + env.get("PYTHONPATH", ""),
                    "MIVGPU_FAKE_GPUS": str(self.fake_gpus), "NODE_NAME": self.node,
                    "HAMI_RESYNC_INTERVAL": "1s"})
        env.update(self.extra_env)
        logf = open(self.dir / f"{name}.log", "w")
        self.procs[name] = subprocess.Popen([sys.executable, "-m", f"k8s_vgpu_scheduler_amd.cmd.{name}", *args],
                                            env=env, stdout=logf, stderr=subprocess.STDOUT,
                                            start_new_session=True, cwd=str(REPO))

    def __enter__(self) -> "E2ECluster":
        (self.dir / "plugins").mkdir(parents=True, exist_ok=True)
        self.hook.mkdir(parents=True, exist_ok=True)
        self.api = FakeApiServer(bookmark_s=1.0).start()
        self.kubeconfig = self.api.write_kubeconfig(str(self.dir / "kubeconfig"))
        self.api.cluster.create("nodes", make_node(self.node))
        self.kubelet = FakeKubelet(self.dir, self.api, self.node).start()
        kc = ["--kubeconfig", self.kubeconfig]
        dc = []
        if self.device_config:
            import yaml
            (self.dir / "device-config.yaml").write_text(yaml.safe_dump(self.device_config))
            dc = ["--device-config-file", str(self.dir / "device-config.yaml")]
        self._spawn("scheduler", [*kc, *dc, "--http_bind", f"127.0.0.1:{self.ports['http']}",
                                  "--metrics-bind-address", f"127.0.0.1:{self.ports['sched_metrics']}",
                                  "--scheduler-name", "hami-scheduler", "-v", str(self.log_level)])
        self._spawn("device_plugin", [*kc, "--node-name", self.node, "--kubelet-socket", self.kubelet.socket,
                                      "--socket-dir", str(self.dir / "plugins"), "--hook-path", str(self.hook),
                                      "--smi-backend", self.smi_backend, "--node-config", str(self.dir / "none.json"),
                                      "--device-split-count", str(self.split), "-v", str(self.log_level)])
        try:
            wait_for(lambda: (self.hook / "vgpu" / "ld.so.preload").exists(), 60, "device plugin install")
            self._spawn("monitor", [*kc, "--node-name", self.node, "--hook-path", str(self.hook),
                                    "--metrics-bind-address", f"127.0.0.1:{self.ports['mon_metrics']}",
                                    "--smi-backend", self.smi_backend, "-v", str(self.log_level),
                                    "--state-file", str(self.dir / "monitor_state.json"), *self.monitor_args])
            wait_for(lambda: requests.get(self.url("/healthz"), timeout=2).ok, 60, "scheduler /healthz")
            wait_for(lambda: self.kubelet.registrations, 60, "device plugin registration with the kubelet")
            wait_for(lambda: "hami.io/node-amd-register" in
                     (self.api.cluster.get("nodes", self.node)["metadata"].get("annotations") or {}), 60,
                     "node device registration")
            wait_for(lambda: samples(self.metrics("sched_metrics"), "hami_node_gpu_overview"), 60,
                     "scheduler to register the node's GPUs")
        except BaseException:
            self.__exit__(None, None, None)
            raise
        return self

    def __exit__(self, *exc):
        for name, p in self.procs.items():
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        for p in self.procs.values():
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait(timeout=10)
        self.kubelet.stop()
        self.api.stop()

    # --------------------------------------------------------- operations
    def url(self, path: str) -> str:
        return f"http://127.0.0.1:{self.ports['http']}{path}"

    def metrics(self, which: str) -> str:
        return requests.get(f"http://127.0.0.1:{self.ports[which]}/metrics", timeout=5).text

    def logs(self, name: str) -> str:
        return (self.dir / f"{name}.log").read_text(errors="replace")

    def monitor_state(self) -> dict:
        """The monitor's last feedback pass (``--state-file``): host truth's
        uuid -> gpu_id map, pids per pod, vram per pid, verdicts, counters."""
        try:
            return json.loads((self.dir / "monitor_state.json").read_text())
        except (OSError, ValueError):
            return {}

    def alive(self) -> dict:
        return {k: p.poll() for k, p in self.procs.items()}

    def submit(self, pod: dict) -> dict:
        """kube-apiserver admission: the mutating webhook, then persist."""
        pod = json.loads(json.dumps(pod))
        md = pod.setdefault("metadata", {})
        md.setdefault("namespace", "default")
        review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                  "request": {"uid": "e2e-" + md["name"], "kind": {"group": "", "version": "v1", "kind": "Pod"},
                              "operation": "CREATE", "namespace": md["namespace"], "object": pod}}
        resp = requests.post(self.url("/webhook"), json=review, timeout=10).json()["response"]
        if not resp.get("allowed"):
            raise PermissionError((resp.get("status") or {}).get("message", "denied"))
        if resp.get("patch"):
            pod = apply_json_patch(pod, json.loads(base64.b64decode(resp["patch"])))
        return self.api.cluster.create("pods", pod, md["namespace"])

    def schedule(self, namespace: str, name: str) -> str | None:
        """kube-scheduler with the extender: /filter over the node list, then /bind."""
        pod = self.api.cluster.get("pods", name, namespace)
        res = requests.post(self.url("/filter"), json={"Pod": pod, "NodeNames": [self.node]}, timeout=30).json()
        if res.get("Error"):
            raise RuntimeError(res["Error"])
        nodes = res.get("NodeNames") or []
        if not nodes:
            return None
        res = requests.post(self.url("/bind"), json={"PodName": name, "PodNamespace": namespace,
                                                     "PodUID": pod["metadata"]["uid"], "Node": nodes[0]},
                            timeout=30).json()
        if res.get("Error"):
            raise RuntimeError(res["Error"])
        return nodes[0]

    def start_containers(self, namespace: str, name: str) -> list[dict]:
        """Kubelet: Allocate for the bound pod and mark it Running."""
        pod = self.api.cluster.get("pods", name, namespace)
        assert pod["spec"].get("nodeName") == self.node, pod["spec"]
        allocs = self.kubelet.allocate(pod)
        self.api.cluster.patch("pods", name, {"status": {"phase": "Running"}}, namespace)
        return allocs

    def delete_pod(self, namespace: str, name: str):
        self.api.cluster.delete("pods", name, namespace)
