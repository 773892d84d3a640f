"""Eight tenants on one MI355X, in a file of its own that sorts first.

The eight-slice rounds spawn 8 + 8 slice processes of Qwen3-8B (12 of its 36
layers: the same kernels and shapes, a third of the load time).  They run
before any test that initialises HIP inside the pytest process: a test
runner holding its own GPU context and queues next to eight slices pushed
the hardware scheduler past its queue slots (profiles/README.md section 27)
and, with the bench parent, over the box's 16-processes-per-GPU bound.
"""

import json

import pytest

from test_shim_gpu import _bench

pytestmark = pytest.mark.gpu


def test_eight_temporal_tenants_run_like_native():
    """eight 12.5 % tenants under the temporal
    governor (policy force, no CU masks) fill the GPU: the share board's
    fair-share mode counts a tenant present over its 20 ms presence window,
    so a tenant caught between two kernels at a pass is not under-charged
    and its neighbours are not held for it.  Round 5 (presence at the
    instant): 0.955 / fairness 0.941 on one box, 0.87 on another; round 6:
    0.989 / 0.984."""
    # 12 of the 36 layers: the same kernels and shapes, a third of the load
    # time -- eight governed slices load at 12.5 % each
    r = _bench(["--slices", "8", "--rounds", "temporal,native", "--steps", "100", "--warmup", "5", "--layers", "12"],
               timeout=170)
    gov = r["temporal_governor_rank0"]
    print(json.dumps({"temporal": r["temporal_value"], "native": r["native_value"],
                      "fairness": r["temporal_fairness_min_over_max"],
                      "held_ms": [g["held_ms"] for g in gov], "busy_share_pct": [g["busy_share_pct"] for g in gov]}))
    assert r["temporal_value"] >= 0.96 * r["native_value"], r
    assert r["temporal_fairness_min_over_max"] >= 0.95, r
    for g in gov:
        assert g["lifetime"]["gates"] > 0, gov                           # the governor ran
        # each near 12.5 % of the GPU time (9.99-14.36 seen on one box in round 6;
        # the throughput fairness above is the tight check)
        assert g["busy_share_pct"] is not None and 8.0 <= g["busy_share_pct"] <= 17.0, gov


def test_eight_pooled_slices_with_the_monitor_switch():
    """The default layout for sub-quarter pods (one whole-GPU CU range for all
    of them) with the node monitor's feedback pass engaging the governor for
    contending tenants, as production runs it (the reference turns the
    utilisation switch on for every busy tenant of equal priority,
    cmd/vGPUmonitor/feedback.go:56-72): within 3 % of native, fair."""
    r = _bench(["--slices", "8", "--rounds", "shim,native", "--steps", "100", "--warmup", "5", "--layers", "12"],
               timeout=170)
    mon = r.get("shim_monitor") or {}
    print(json.dumps({"shim": r["value"], "native": r["native_value"], "fairness": r["slice_fairness_min_over_max"],
                      "monitor": mon}))
    assert mon.get("passes", 0) >= 1 and mon.get("switch_on_slice_passes", 0) >= 8, mon   # the switch engaged
    assert r["value"] >= 0.97 * r["native_value"], r
    assert r["slice_fairness_min_over_max"] >= 0.95, r
