"""Static HTML report: the reference browser UI's views without a server (survey C45).

The reference UI (client/web/index.html, web/scripts/*.js) shows one scatter plot per label pair
(oracle predictions, consensus), first/second-pass reliability bars scaled x100
(client/web_interface.py:196-203), the oracle table and a console.  Here the same views are rendered
into one self-contained HTML file (inline SVG, no CDN: the GPU boxes have no network), optionally
with benchmark records (JSON lines from ``bench.py --log``).
"""
from __future__ import annotations

import html
import json
from typing import List, Optional, Sequence

import torch

_COLORS = {"reliable": "#2b7bba", "masked": "#d1495b", "consensus": "#111"}


def _scatter_svg(xs, ys, rel, cx, cy, title, size=220) -> str:
    pad = 18
    lo_x, hi_x = min(list(xs) + [cx]), max(list(xs) + [cx])
    lo_y, hi_y = min(list(ys) + [cy]), max(list(ys) + [cy])
    sx = (size - 2 * pad) / ((hi_x - lo_x) or 1.0)
    sy = (size - 2 * pad) / ((hi_y - lo_y) or 1.0)
    px = lambda v: pad + (v - lo_x) * sx  # noqa: E731
    py = lambda v: size - pad - (v - lo_y) * sy  # noqa: E731
    dots = "".join(
        f'<circle cx="{px(x):.1f}" cy="{py(y):.1f}" r="3.5" fill="{_COLORS["reliable" if r else "masked"]}"/>'
        for x, y, r in zip(xs, ys, rel))
    cross = (f'<path d="M{px(cx)-6:.1f},{py(cy):.1f}h12M{px(cx):.1f},{py(cy)-6:.1f}v12" '
             f'stroke="{_COLORS["consensus"]}" stroke-width="2"/>')
    return (f'<figure><svg width="{size}" height="{size}" style="border:1px solid #ccc">{dots}{cross}</svg>'
            f'<figcaption>{html.escape(title)}</figcaption></figure>')


def _bar(label: str, v: float) -> str:
    pct = max(0.0, min(100.0, 100.0 * v))
    return (f'<div>{html.escape(label)}: {pct:.1f}%<div style="background:#eee;width:300px">'
            f'<div style="background:#2b7bba;width:{3 * pct:.0f}px;height:10px"></div></div></div>')


def instance_html(engine, b: int = 0, labels: Optional[Sequence[str]] = None, addresses=None) -> str:
    """Views of instance ``b`` of a :class:`svoc.engine.ConsensusEngine`."""
    scale = 1e-6 if engine.mode == "exact" else 1.0
    D = engine.D
    vals = engine.values[b, :, :D].double().cpu() * scale
    rel = engine.reliable[b].bool().cpu().tolist()
    cons = (engine.consensus[b].double().cpu() * scale).tolist()
    r1, r2 = (engine.rel[b].double().cpu() * scale).tolist()
    labels = list(labels) if labels else [f"dim {d}" for d in range(D)]
    parts = [f"<h2>instance {b}</h2>", _bar("reliability (first pass)", r1), _bar("reliability (second pass)", r2)]
    figs = []
    for d in range(0, D - 1, 2):  # one plot per label pair, as the reference UI
        figs.append(_scatter_svg(vals[:, d].tolist(), vals[:, d + 1].tolist(), rel, cons[d], cons[d + 1],
                                 f"{labels[d]} / {labels[d + 1]}"))
    if D == 1:
        figs.append(_scatter_svg(vals[:, 0].tolist(), [0.0] * len(rel), rel, cons[0], 0.0, labels[0]))
    parts.append('<div style="display:flex;flex-wrap:wrap;gap:8px">' + "".join(figs) + "</div>")
    rows = []
    for i in range(engine.N):
        a = hex(addresses[i]) if addresses else str(i)
        v = ", ".join(f"{x:.3f}" for x in vals[i].tolist())
        rows.append(f"<tr><td>{html.escape(a)}</td><td>{v}</td><td>{'yes' if rel[i] else '<b>masked</b>'}</td></tr>")
    parts.append("<table border=1 cellpadding=3><tr><th>oracle</th><th>prediction</th><th>reliable</th></tr>"
                 + "".join(rows) + "</table>")
    parts.append("<p>consensus: [" + ", ".join(f"{x:.4f}" for x in cons) + "]</p>")
    return "\n".join(parts)


def bench_html(records: List[dict]) -> str:
    if not records:
        return ""
    head = "<tr><th>config</th><th>n_gpus</th><th>value</th><th>unit</th><th>ms/step</th></tr>"
    rows = "".join(
        f"<tr><td>{html.escape(str(r.get('config', {}).get('model', '')))}</td><td>{r.get('n_gpus')}</td>"
        f"<td>{r.get('value', 0):.4g}</td><td>{html.escape(str(r.get('unit', '')))}</td>"
        f"<td>{r.get('ms_per_step', 0):.3f}</td></tr>" for r in records)
    return f"<h2>benchmarks</h2><table border=1 cellpadding=3>{head}{rows}</table>"


def write_report(path: str, engine=None, instances: Sequence[int] = (0,), labels=None, addresses=None,
                 bench_jsonl: Optional[str] = None, title: str = "svoc consensus report") -> str:
    body = [f"<h1>{html.escape(title)}</h1>"]
    if engine is not None:
        for b in instances:
            body.append(instance_html(engine, b, labels, addresses))
    if bench_jsonl:
        with open(bench_jsonl, encoding="utf-8") as f:
            recs = [json.loads(l) for l in f if l.strip()]
        body.append(bench_html(recs))
    doc = ("<!doctype html><html><head><meta charset='utf-8'><title>" + html.escape(title) +
           "</title></head><body style='font-family:sans-serif'>" + "\n".join(body) + "</body></html>")
    with open(path, "w", encoding="utf-8") as f:
        f.write(doc)
    return path
