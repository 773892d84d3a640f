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


def test_pmcsum_merges_passes_and_scales_fetch(tmp_path):
    """utils/pmcsum: per-kernel means over --pmc passes, FETCH_SIZE doubled
    (gfx950 tallies 128-B requests at 64 B), bandwidth from each pass's times."""
    from k8s_vgpu_scheduler_amd.utils import pmcsum

    hdr = ('"Correlation_Id","Dispatch_Id","Agent_Id","Queue_Id","Process_Id","Thread_Id","Grid_Size","Kernel_Id",'
           '"Kernel_Name","Workgroup_Size","LDS_Block_Size","Scratch_Size","VGPR_Count","Accum_VGPR_Count",'
           '"SGPR_Count","Counter_Name","Counter_Value","Start_Timestamp","End_Timestamp"\n')

    def row(d, name, cn, v, t0, t1):
        return f'{d},{d},"Agent 2",1,1,1,64,1,"{name}",64,0,0,8,0,8,"{cn}",{v},{t0},{t1}\n'

    a = tmp_path / "a.csv"
    a.write_text(hdr + row(1, "void gemm_kernel<1>(float*)", "FETCH_SIZE", 1000.0, 0, 1000)
                 + row(2, "void gemm_kernel<1>(float*)", "FETCH_SIZE", 1000.0, 5000, 6000)
                 + row(3, "void at::native::fill(float*)", "FETCH_SIZE", 9.0, 0, 10))
    b = tmp_path / "b.csv"
    b.write_text(hdr + row(1, "void gemm_kernel<1>(float*)", "SQ_WAVES", 64.0, 0, 3000)
                 + row(2, "void gemm_kernel<1>(float*)", "SQ_WAVES", 32.0, 0, 1000))
    rows = pmcsum.summarise(pmcsum.load([str(a), str(b)]))
    assert [r["kernel"] for r in rows] == ["gemm_kernel<1>"]          # one-off init kernels dropped
    r = rows[0]
    assert r["dispatches"] == 2 and r["SQ_WAVES"] == 48.0 and r["FETCH_SIZE"] == 1000.0
    assert r["read_MB"] == round(2 * 1000 * 1024 / 1e6, 2)
    assert r["read_GBps"] == round(2 * 2000 * 1024 / 2000, 1)          # bytes / ns over pass a only
    assert "| gemm_kernel<1> | 2 |" in pmcsum.to_markdown(rows)
