"""Latency report over client JSONL runs (the analysis of the reference's
benchmarks/ai-benchmark/gen_report.py:25-201: raw TTFT percentiles, then
means after a percentile trim and a MAD outlier filter; histograms / CDFs
when matplotlib is importable).  Adds what the reference leaves to the reader:
each dataset's overhead against the first one (the native baseline).

    python -m k8s_vgpu_scheduler_amd.serve.report --dataset native n.jsonl \\
        --dataset vgpu v.jsonl --output-dir report
"""

from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

TRIM_PCT = 5.0
MAD_Z = 3.5


def load(path) -> list[dict]:
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]


def latencies(rows: list[dict]) -> tuple[np.ndarray, np.ndarray]:
    """TTFT per request and every inter-token gap (seconds)."""
    ttft, gaps = [], []
    for r in rows:
        if r.get("t_first") is None:
            continue
        ttft.append(r["t_first"] - r["t0"])
        ts = r.get("t_tokens") or []
        if len(ts) > 1:
            gaps.extend(np.diff(np.asarray(ts, dtype=np.float64)).tolist())
    return np.asarray(ttft, dtype=np.float64), np.asarray(gaps, dtype=np.float64)


def clean(x: np.ndarray, trim_pct: float = TRIM_PCT, mad_z: float = MAD_Z) -> np.ndarray:
    """Keep [trim_pct, 100-trim_pct] percentiles, then drop |robust z| >= mad_z."""
    if x.size == 0:
        return x
    lo, hi = np.percentile(x, [trim_pct, 100.0 - trim_pct])
    x = x[(x >= lo) & (x <= hi)]
    if x.size == 0:
        return x
    med = np.median(x)
    mad = np.median(np.abs(x - med)) * 1.4826
    return x[np.abs(x - med) / (mad + 1e-12) < mad_z]


def summarize(rows: list[dict], trim_pct: float = TRIM_PCT, mad_z: float = MAD_Z) -> dict:
    ttft, gaps = latencies(rows)
    tc, gc = clean(ttft, trim_pct, mad_z), clean(gaps, trim_pct, mad_z)

    def pct(x, q):
        return float(np.percentile(x, q)) if x.size else None

    toks = [len(r.get("t_tokens") or []) for r in rows]
    spans = [r["t_end"] - r["t0"] for r in rows if r.get("t_end")]
    return {"requests": len(rows), "tokens_per_request": float(np.mean(toks)) if toks else 0.0,
            "ttft_p50_s": pct(ttft, 50), "ttft_p95_s": pct(ttft, 95), "ttft_p99_s": pct(ttft, 99),
            "ttft_clean_mean_s": float(tc.mean()) if tc.size else None,
            "per_token_p50_s": pct(gaps, 50), "per_token_p99_s": pct(gaps, 99),
            "per_token_clean_mean_s": float(gc.mean()) if gc.size else None,
            "decode_tok_s": (sum(toks) / sum(spans)) if spans and sum(spans) > 0 else None}


def compare(named: dict) -> dict:
    """Summaries plus each dataset's overhead vs the first (percent, + = slower)."""
    out = {n: summarize(rows) for n, rows in named.items()}
    base = next(iter(out.values()), None)
    for n, s in out.items():
        for k in ("ttft_clean_mean_s", "per_token_clean_mean_s", "ttft_p50_s"):
            if base and base.get(k) and s.get(k) is not None:
                s[k.replace("_s", "") + "_overhead_pct"] = round(100.0 * (s[k] / base[k] - 1.0), 2)
    return out


def _plots(named_arrays: dict, outdir: Path, label: str, stem: str) -> list[str]:
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:  # noqa: BLE001  -- plots are optional
        return []
    files = []
    arrays = {n: a for n, a in named_arrays.items() if a.size}
    if not arrays:
        return files
    fig, ax = plt.subplots()
    for n, a in arrays.items():
        ax.hist(a * 1e3, bins=50, alpha=0.55, label=n)
    ax.set_xlabel(f"{label} (ms)")
    ax.legend()
    fig.savefig(outdir / f"{stem}_hist.png")
    plt.close(fig)
    fig, ax = plt.subplots()
    for n, a in arrays.items():
        s = np.sort(a) * 1e3
        ax.plot(s, np.linspace(0.0, 1.0, s.size), label=n)
    ax.set_xlabel(f"{label} (ms)")
    ax.set_ylabel("CDF")
    ax.grid(True, linestyle="--", alpha=0.3)
    ax.legend()
    fig.savefig(outdir / f"{stem}_cdf.png")
    plt.close(fig)
    return [f"{stem}_hist.png", f"{stem}_cdf.png"]


def write_report(named: dict, outdir, title: str = "Serving latency: vGPU slices vs native") -> dict:
    outdir = Path(outdir)
    outdir.mkdir(parents=True, exist_ok=True)
    summary = compare(named)

    def ms(v):
        return f"{v * 1e3:.2f}" if v is not None else "-"

    lines = [f"# {title}", "", "| dataset | requests | TTFT p50 | p95 | p99 | TTFT clean mean | per-token clean mean "
             "| TTFT overhead | per-token overhead |", "|---|---|---|---|---|---|---|---|---|"]
    for n, s in summary.items():
        lines.append(f"| {n} | {s['requests']} | {ms(s['ttft_p50_s'])} | {ms(s['ttft_p95_s'])} | "
                     f"{ms(s['ttft_p99_s'])} | {ms(s['ttft_clean_mean_s'])} | {ms(s['per_token_clean_mean_s'])} | "
                     f"{s.get('ttft_clean_mean_overhead_pct', 0.0):+.2f} % | "
                     f"{s.get('per_token_clean_mean_overhead_pct', 0.0):+.2f} % |")
    lines += ["", "Times in ms; clean = after a 5 % percentile trim and a MAD (z < 3.5) filter; "
              "overheads against the first dataset."]
    arrays = {n: latencies(r) for n, r in named.items()}
    figs = _plots({n: clean(a[0]) for n, a in arrays.items()}, outdir, "TTFT", "ttft")
    figs += _plots({n: clean(a[1]) for n, a in arrays.items()}, outdir, "per-token latency", "per_token")
    if figs:
        lines += ["", "## Figures", ""] + [f"![{f}]({f})" for f in figs]
    (outdir / "report.md").write_text("\n".join(lines) + "\n")
    (outdir / "summary.json").write_text(json.dumps(summary, indent=1))
    return summary


def main(argv=None):
    ap = argparse.ArgumentParser(description="TTFT / per-token latency report")
    ap.add_argument("--dataset", action="append", nargs=2, metavar=("NAME", "FILE"), required=True)
    ap.add_argument("--output-dir", default="report")
    a = ap.parse_args(argv)
    summary = write_report({n: load(f) for n, f in a.dataset}, a.output_dir)
    print(json.dumps(summary, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
