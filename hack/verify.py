#!/usr/bin/env python3
"""Repository verifiers (the reference's hack/verify-*.sh + hack/tools, redone
for this tree).

  chart-version  charts/mivgpu/Chart.yaml version/appVersion == package __version__
  rbac           every Kubernetes API call a binary can make (found statically in
                 the modules its entry point imports) is granted by the ClusterRole
                 its ServiceAccount is bound to in the chart (hack/tools/rbaccheck)
  native         csrc/ is CDNA4-only: no CUDA headers/identifiers, no NVIDIA
                 platform branches, no warp-32 intrinsics, no hipify leftovers
  static         every Python file compiles; the C++ shim/mock sources pass
                 g++ -fsyntax-only -Wall -Wextra -Werror

    python hack/verify.py [all|chart-version|rbac|native|static] [-v]

Exit status 0 when every selected check passes.
"""

from __future__ import annotations

import ast
import re
import shutil
import subprocess
import sys
from pathlib import Path

import yaml

ROOT = Path(__file__).resolve().parent.parent
PKG = "k8s_vgpu_scheduler_amd"
CHART = ROOT / "charts" / "mivgpu"

# entry point -> (RBAC template, ClusterRole name suffix).  The monitor runs in
# the device-plugin DaemonSet under the device plugin's ServiceAccount.
BINARIES = {
    "scheduler": (["cmd/scheduler.py"], "scheduler/rbac.yaml"),
    "device-plugin": (["cmd/device_plugin.py", "cmd/monitor.py"], "device-plugin/rbac.yaml"),
}

# Kubernetes kinds our client addresses by plural name -> API group
KINDS = {"nodes": "", "pods": "", "events": "", "resourcequotas": "", "configmaps": "", "namespaces": "",
         "leases": "coordination.k8s.io", "secrets": "", "services": ""}
VERBS = {"get", "list", "create", "update", "patch", "delete", "watch"}
# typed helpers of k8s/client.py:KubeClient -> (resource, verb)
HELPERS = {"get_node": ("nodes", "get"), "list_nodes": ("nodes", "list"), "get_pod": ("pods", "get"),
           "list_pods": ("pods", "list"), "patch_node": ("nodes", "patch"), "patch_pod": ("pods", "patch"),
           "bind": ("pods/binding", "create"), "evict": ("pods/eviction", "create")}


# ----------------------------------------------------------------- helpers
def _module_path(mod: str) -> Path | None:
    rel = mod.split(".")
    if rel[0] != PKG:
        return None
    base = ROOT.joinpath(*rel)
    if base.with_suffix(".py").exists():
        return base.with_suffix(".py")
    if (base / "__init__.py").exists():
        return base / "__init__.py"
    return None


def _imports(path: Path, mod: str) -> set[str]:
    tree = ast.parse(path.read_text(), str(path))
    pkg = mod if path.name == "__init__.py" else mod.rsplit(".", 1)[0]
    out = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            out.update(a.name for a in node.names)
        elif isinstance(node, ast.ImportFrom):
            if node.level:
                parts = pkg.split(".")
                base = ".".join(parts[: len(parts) - node.level + 1])
                src = f"{base}.{node.module}" if node.module else base
            else:
                src = node.module or ""
            out.add(src)
            out.update(f"{src}.{a.name}" for a in node.names)     # `from pkg import module`
    # every parent package's __init__ runs on import
    full = set()
    for m in out:
        parts = m.split(".")
        full.update(".".join(parts[:i]) for i in range(1, len(parts) + 1))
    return {m for m in full if _module_path(m) is not None}


def reachable(entries: list[str]) -> dict[str, Path]:
    todo = [f"{PKG}." + e[:-3].replace("/", ".") for e in entries]
    seen: dict[str, Path] = {}
    while todo:
        m = todo.pop()
        if m in seen:
            continue
        p = _module_path(m)
        if p is None:
            continue
        seen[m] = p
        todo.extend(_imports(p, m) - set(seen))
    return seen


def api_calls(path: Path) -> set[tuple[str, str, str]]:
    """(group, resource, verb) for every API request the module can make."""
    tree = ast.parse(path.read_text(), str(path))
    out = set()
    for node in ast.walk(tree):
        if not isinstance(node, ast.Call):
            continue
        f = node.func
        name = f.attr if isinstance(f, ast.Attribute) else (f.id if isinstance(f, ast.Name) else "")
        first = node.args[0] if node.args else None
        kind = first.value if isinstance(first, ast.Constant) and isinstance(first.value, str) else None
        if name == "Informer" and len(node.args) >= 2:
            k = node.args[1]
            if isinstance(k, ast.Constant) and k.value in KINDS:
                out |= {(KINDS[k.value], k.value, "list"), (KINDS[k.value], k.value, "watch")}
        elif isinstance(f, ast.Attribute) and name in HELPERS:
            res, verb = HELPERS[name]
            out.add(("", res, verb))
        elif isinstance(f, ast.Attribute) and name in VERBS and kind in KINDS:
            out.add((KINDS[kind], kind, name))
    return out


def _render(text: str) -> str:
    # enough Helm for RBAC templates: every action becomes a scalar
    return re.sub(r"\{\{-?.*?-?\}\}", "x", text)


def granted(template: str) -> set[tuple[str, str, str]]:
    out = set()
    for doc in yaml.safe_load_all(_render((CHART / "templates" / template).read_text())):
        if not doc or doc.get("kind") not in ("ClusterRole", "Role"):
            continue
        for r in doc.get("rules", []):
            for g in r.get("apiGroups", []):
                for res in r.get("resources", []):
                    for v in r.get("verbs", []):
                        out.add((g, res, v))
    return out


def _allowed(need, have) -> bool:
    g, res, verb = need
    return any(hg in (g, "*") and hr in (res, "*") and hv in (verb, "*") for hg, hr, hv in have)


# ------------------------------------------------------------------ checks
def check_chart_version(verbose=False) -> list[str]:
    chart = yaml.safe_load((CHART / "Chart.yaml").read_text())
    src = (ROOT / PKG / "__init__.py").read_text()
    m = re.search(r'^__version__\s*=\s*"([^"]+)"', src, re.M)
    version = m.group(1) if m else None
    errs = []
    if str(chart.get("version")) != version:
        errs.append(f"Chart.yaml version {chart.get('version')} != package {version}")
    if str(chart.get("appVersion")) != version:
        errs.append(f"Chart.yaml appVersion {chart.get('appVersion')} != package {version}")
    return errs


def check_rbac(verbose=False) -> list[str]:
    errs = []
    for binary, (entries, template) in BINARIES.items():
        mods = reachable(entries)
        need: dict[tuple, set] = {}
        for m, p in mods.items():
            for call in api_calls(p):
                need.setdefault(call, set()).add(m)
        have = granted(template)
        for call in sorted(need):
            if not _allowed(call, have):
                g, res, verb = call
                errs.append(f"{binary}: {verb} {g or 'core'}/{res} used by {sorted(need[call])} "
                            f"is not granted in templates/{template}")
        if verbose:
            print(f"  {binary}: {len(mods)} modules, {len(need)} API permissions used")
    return errs


_CUDA = [
    (re.compile(r"#\s*include\s*[<\"](cuda|cublas|cudnn|nccl|cutlass|cub/)"), "CUDA header"),
    (re.compile(r"\bcuda[A-Z]\w*|\bCU[A-Z_]{3,}\b|\bcu(Launch|Mem|Ctx|Stream)\w*"), "CUDA identifier"),
    (re.compile(r"#\s*(if|ifdef|ifndef|elif)\b.*__(HIP_PLATFORM_(AMD|NVIDIA|NVCC|HCC)|CUDA_ARCH|CUDACC)__"),
     "platform branch (write CDNA4 code directly)"),
    (re.compile(r"__shfl(_\w+)?_sync|__ballot_sync|__activemask|\bwarpSize\s*==\s*32"), "warp-32 intrinsic"),
    (re.compile(r"hipify|HIPIFY"), "hipify leftover"),
]


def _strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", lambda m: "\n" * m.group(0).count("\n"), src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return re.sub(r'"(\\.|[^"\\\n])*"', '""', src)    # string literals (log text) are not code


def check_native(verbose=False) -> list[str]:
    errs = []
    files = [p for p in (ROOT / "csrc").rglob("*") if p.suffix in (".hip", ".cpp", ".h", ".hpp", ".inc")]
    for p in files:
        raw = p.read_text(errors="replace")
        code = _strip_comments(raw)
        for i, (line, rline) in enumerate(zip(code.splitlines(), raw.splitlines()), 1):
            for j, (rx, what) in enumerate(_CUDA):
                # includes are matched on the raw line: string stripping would blank "cuda.h"
                if rx.search(rline if j == 0 else line):
                    errs.append(f"{p.relative_to(ROOT)}:{i}: {what}: {rline.strip()[:100]}")
    if verbose:
        print(f"  native: {len(files)} sources scanned")
    return errs


def check_static(verbose=False) -> list[str]:
    errs = []
    pys = [p for p in ROOT.rglob("*.py") if not any(x in p.parts for x in (".git", "build", "gpurun_out"))]
    for p in pys:
        try:
            compile(p.read_text(), str(p), "exec", dont_inherit=True)
        except SyntaxError as e:
            errs.append(f"{p.relative_to(ROOT)}:{e.lineno}: {e.msg}")
    cxx = shutil.which("g++")
    rocm = Path("/opt/rocm/include")
    srcs = [ROOT / "csrc/shim/mivgpu_shim.cpp", ROOT / "csrc/mockhip/mock_amdhip.cpp",
            ROOT / "csrc/mockhip/shim_driver.cpp", ROOT / "csrc/mockhip/mock_roctx.cpp"]
    gen = ROOT / "build" / "gen"
    if cxx and rocm.exists():
        for s in srcs:
            cmd = [cxx, "-std=c++17", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                   "-Wno-deprecated-declarations", "-D__HIP_PLATFORM_AMD__", f"-isystem{rocm}",
                   f"-I{ROOT / 'csrc/include'}", f"-I{gen}", str(s)]
            if s.name == "mivgpu_shim.cpp":    # built with its glibc floor (utils/build.py)
                cmd[-1:-1] = ["-DMIVGPU_GLIBC_FLOOR", "-include", str(ROOT / "csrc/shim/glibc_floor.h")]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode:
                errs.append(f"{s.relative_to(ROOT)}: g++ -Wall -Wextra -Werror:\n{r.stderr[-1500:]}")
    if verbose:
        print(f"  static: {len(pys)} Python files, {len(srcs)} C++ sources")
    return errs


CHECKS = {"chart-version": check_chart_version, "rbac": check_rbac, "native": check_native,
          "static": check_static}


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    verbose = "-v" in argv
    names = [a for a in argv if a != "-v"] or ["all"]
    if names == ["all"]:
        names = list(CHECKS)
    bad = 0
    for n in names:
        errs = CHECKS[n](verbose)
        print(f"{'FAIL' if errs else 'ok  '} {n}")
        for e in errs:
            print(f"     {e}")
        bad += bool(errs)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
