"""hack/verify.py in the CPU suite (the reference runs hack/verify-all.sh in CI):
chart version, RBAC coverage of every API call the binaries make, CDNA4-only
native sources, static checks.  The RBAC checker must also catch a missing verb."""

import importlib.util
import shutil
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
_spec = importlib.util.spec_from_file_location("hack_verify", ROOT / "hack" / "verify.py")
V = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(V)


@pytest.mark.parametrize("check", sorted(V.CHECKS))
def test_verifier_passes(check):
    assert V.CHECKS[check]() == []


def test_rbac_checker_catches_a_missing_verb(tmp_path, monkeypatch):
    chart = tmp_path / "mivgpu"
    shutil.copytree(V.CHART, chart)
    rb = chart / "templates" / "device-plugin" / "rbac.yaml"
    rb.write_text(rb.read_text().replace("verbs: [get, list, create, patch, update]", "verbs: [create, patch]"))
    monkeypatch.setattr(V, "CHART", chart)
    errs = V.check_rbac()
    assert any(e.startswith("device-plugin: list core/events") for e in errs), errs
    assert not any(e.startswith("scheduler:") for e in errs)


def test_api_call_extraction():
    calls = V.api_calls(ROOT / "k8s_vgpu_scheduler_amd" / "scheduler" / "scheduler.py")
    assert ("", "pods", "watch") in calls and ("", "nodes", "list") in calls
    assert ("coordination.k8s.io", "leases", "watch") in calls


def test_native_check_flags_cuda_isms(tmp_path, monkeypatch):
    (tmp_path / "csrc").mkdir()
    (tmp_path / "csrc" / "k.hip").write_text(
        '// cudaMalloc in a comment is fine\n#ifdef __HIP_PLATFORM_AMD__\nx = __shfl_xor_sync(m, v, 1);\n#endif\n'
        'log("cudaMemcpy");\n')
    monkeypatch.setattr(V, "ROOT", tmp_path)
    errs = V.check_native()
    assert len(errs) == 2 and "platform branch" in errs[0] and "warp-32" in errs[1], errs
