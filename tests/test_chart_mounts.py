"""The node DaemonSet gives the monitor every host path it reads (ADVICE r1:
the monitor once lacked the lock dir, so a series stayed empty in Helm
deployments while unit tests, pointed at a tmp dir, passed).

Paths the monitor reads, from its code:
  * the hook dir with the containers' shared regions (cmd/monitor.py --hook-path);
  * /tmp/vgpulock: the partition-apply lock it pauses on (MIVGPU_PARTITION_LOCK);
  * /sys: KFD per-process occupancy / VRAM (monitor/occupancy.py, hostpid.py);
  * /proc of the host: NSpid scan (monitor/hostpid.py) -> hostPID: true.
"""

import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
DS = (ROOT / "charts/mivgpu/templates/device-plugin/daemonset.yaml").read_text()


def _container_block(name):
    m = re.search(rf"^        - name: {name}\n(.*?)(?=^        - name: |^      volumes:)", DS, re.S | re.M)
    assert m, name
    return m.group(1)


def _mounts(block):
    return {(m.group(2) or m.group(3)).strip(): m.group(1)
            for m in re.finditer(r'\{name: ([\w-]+), mountPath: (?:"([^"]+)"|([^,}]+))', block)}


def test_monitor_mounts_every_path_it_reads():
    mon = _container_block("monitor")
    mounts = _mounts(mon)
    assert "{{ .Values.devicePlugin.hookPath }}/vgpu" in mounts
    assert "/tmp/vgpulock" in mounts and "/sys" in mounts
    lock = re.search(r"MIVGPU_PARTITION_LOCK\n\s+value: (\S+)", mon).group(1)
    assert any(lock.startswith(p.rstrip("/") + "/") for p in mounts), lock
    hook_arg = re.search(r"--hook-path=(.+)$", mon, re.M).group(1).strip()
    assert hook_arg in mounts


def test_device_plugin_and_monitor_share_the_lock_volume():
    dp, mon = _mounts(_container_block("device-plugin")), _mounts(_container_block("monitor"))
    assert dp.get("/tmp/vgpulock") == mon.get("/tmp/vgpulock") == "lock"


def test_host_pid_namespace_for_the_nspid_scan():
    assert re.search(r"^      hostPID: true$", DS, re.M)


def test_every_mounted_volume_is_declared():
    declared = set(re.findall(r"^        - name: ([\w-]+)\n          (?:hostPath|configMap)", DS, re.M))
    for name in ("device-plugin", "monitor"):
        for vol in _mounts(_container_block(name)).values():
            assert vol in declared, (name, vol)
