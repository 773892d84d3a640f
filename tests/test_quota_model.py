"""Model-based test of the namespace quota mirror (device/quota.py; reference
pkg/device/quota_test.go).  Hypothesis drives random interleavings of pod
usage add/remove/replace and ResourceQuota add/update/delete against a plain
dict model, checking ``fit_quota`` and the exported view after every step.

AMD usage is recorded in CUs and charged to the quota in percent of the
device's 256 CUs (``AMDDevices.quota_cores``: 64 CUs == 25 %)."""

import pytest
from hypothesis import settings, strategies as st
from hypothesis.stateful import RuleBasedStateMachine, invariant, rule

from k8s_vgpu_scheduler_amd.device.quota import QuotaManager
from k8s_vgpu_scheduler_amd.device.types import ContainerDevice
from k8s_vgpu_scheduler_amd.k8s.client import init_global_client
from k8s_vgpu_scheduler_amd.k8s.fake import FakeCluster
from k8s_vgpu_scheduler_amd.scheduler.config import init_devices_with_config

MEM, CORE = "amd.com/gpumem", "amd.com/gpucores"
NAMESPACES = ["a", "b"]


@pytest.fixture(autouse=True, scope="module")
def _devices():
    init_global_client(FakeCluster())
    init_devices_with_config()


def pod(ns):
    return {"metadata": {"name": "p", "namespace": ns}}


def pd(mem, cus):
    return {"AMD": [[ContainerDevice(uuid="GPU-0", type="AMD", usedmem=mem, usedcores=cus)]]}


def rq(ns, mem=None, core=None):
    hard = {}
    if mem is not None:
        hard[f"limits.{MEM}"] = str(mem)
    if core is not None:
        hard[f"limits.{CORE}"] = str(core)
    hard["limits.cpu"] = "4"          # unmanaged: ignored
    return {"metadata": {"name": "q", "namespace": ns}, "spec": {"hard": hard}}


class QuotaMachine(RuleBasedStateMachine):
    def __init__(self):
        super().__init__()
        self.q = QuotaManager()
        self.used = {ns: {MEM: 0, CORE: 0} for ns in NAMESPACES}
        self.limit = {ns: {} for ns in NAMESPACES}      # resource -> limit (explicit only)
        self.live = []                                   # (ns, mem, pct)
        self.current_rq = {ns: None for ns in NAMESPACES}

    @rule(ns=st.sampled_from(NAMESPACES), mem=st.integers(0, 4096), quarters=st.integers(0, 4))
    def add_usage(self, ns, mem, quarters):
        self.q.add_usage(pod(ns), pd(mem, 64 * quarters))
        self.used[ns][MEM] += mem
        self.used[ns][CORE] += 25 * quarters
        self.live.append((ns, mem, quarters))

    @rule(data=st.data())
    def rm_usage(self, data):
        if not self.live:
            return
        ns, mem, quarters = self.live.pop(data.draw(st.integers(0, len(self.live) - 1)))
        self.q.rm_usage(pod(ns), pd(mem, 64 * quarters))
        self.used[ns][MEM] -= mem
        self.used[ns][CORE] -= 25 * quarters

    @rule(data=st.data(), mem=st.integers(0, 4096), quarters=st.integers(0, 4))
    def replace_usage(self, data, mem, quarters):
        if not self.live:
            return
        i = data.draw(st.integers(0, len(self.live) - 1))
        ns, om, oq = self.live[i]
        self.q.replace_usage(pod(ns), pd(om, 64 * oq), pd(mem, 64 * quarters))
        self.used[ns][MEM] += mem - om
        self.used[ns][CORE] += 25 * (quarters - oq)
        self.live[i] = (ns, mem, quarters)

    @rule(ns=st.sampled_from(NAMESPACES), mem=st.one_of(st.none(), st.integers(0, 20000)),
          core=st.one_of(st.none(), st.integers(0, 400)))
    def set_quota(self, ns, mem, core):
        new = rq(ns, mem, core)
        self.q.update_quota(self.current_rq[ns], new)
        self.current_rq[ns] = new
        self.limit[ns] = {k: v for k, v in ((MEM, mem), (CORE, core)) if v is not None}

    @rule(ns=st.sampled_from(NAMESPACES))
    def delete_quota(self, ns):
        if self.current_rq[ns] is None:
            return
        self.q.del_quota(self.current_rq[ns])
        self.current_rq[ns] = None
        self.limit[ns] = {}

    @invariant()
    def fit_matches_model(self):
        for ns in NAMESPACES:
            for mem, core in ((0, 0), (1, 0), (0, 1), (512, 25), (10 ** 6, 0), (0, 500)):
                want = all(self.used[ns][k] + req <= self.limit[ns][k]
                           for k, req in ((MEM, mem), (CORE, core)) if k in self.limit[ns])
                assert self.q.fit_quota(ns, mem, 1, core, "AMD") == want, (ns, mem, core)

    @invariant()
    def view_matches_model(self):
        view = self.q.get_resource_quota()
        for ns in NAMESPACES:
            for k in (MEM, CORE):
                e = view.get(ns, {}).get(k)
                used = e.used if e else 0
                assert used == self.used[ns][k]
                assert (e is not None and e.limit_set) == (k in self.limit[ns])
            assert "cpu" not in view.get(ns, {})

    @invariant()
    def fit_key_tracks_limits(self):
        for ns in NAMESPACES:
            key = self.q.fit_key(ns)
            assert {k for k, _, _ in key} == set(self.limit[ns])


QuotaMachine.TestCase.settings = settings(max_examples=60, stateful_step_count=25, deadline=None)
test_quota_state_machine = QuotaMachine.TestCase


def test_unknown_device_always_fits():
    q = QuotaManager()
    q.add_quota(rq("a", mem=0))
    assert q.fit_quota("a", 10 ** 9, 1, 100, "NOT-A-DEVICE")


def test_memory_factor_scales_the_limit():
    q = QuotaManager()
    q.add_quota(rq("a", mem=100))
    assert not q.fit_quota("a", 150, 1, 0, "AMD")
    assert q.fit_quota("a", 150, 2, 0, "AMD")


def test_unparseable_quantity_ignored():
    q = QuotaManager()
    q.add_quota({"metadata": {"name": "q", "namespace": "a"}, "spec": {"hard": {f"limits.{MEM}": "lots"}}})
    assert q.fit_quota("a", 10 ** 9, 1, 0, "AMD")


def test_removal_never_goes_negative():
    q = QuotaManager()
    q.rm_usage(pod("a"), pd(100, 64))
    q.add_usage(pod("a"), pd(10, 0))
    q.rm_usage(pod("a"), pd(100, 64))
    assert q.get_resource_quota()["a"][MEM].used == 0
