"""Kernel table of bench.py's TIMED region only: the kernels of a rocprofv3 kernel trace
that run between the two `svoc_bench_marker_kernel` launches of one timed region (bench.py --markers), so the
setup (stream-pool RNG, warm-up, graph capture) never appears.  Per kernel: calls, total / average µs, and the
share of the timed window; per step: µs of each kernel per step and the window per step.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rk_c3 -o run -- python3 bench.py --config c3 --markers
    python tools/replay_kernels.py gpurun_out/rk_c3 "title" [region=1] [steps=20] > profiles/r6_c3_replay_kernels.md

Region k is the k-th timed region of the run (bench.py measures the headline first, then alt_storage /
exact_stream / alt_precision / cls_pool in that order, each with its own markers).
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict

MARK = "svoc_bench_marker_kernel"


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f, encoding="utf-8")):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(name: str) -> str:
    n = name.split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    return n if len(n) <= 90 else n[:87] + "..."


def window(rows, region: int):
    marks = [r for r in rows if MARK in r[2]]
    if len(marks) < 2 * region:
        raise SystemExit(f"only {len(marks)} marker kernels in the trace (bench.py --markers?)")
    return marks[2 * region - 2][1], marks[2 * region - 1][0]


def render(d: str, title: str, region: int = 1, steps: int = 20) -> str:
    rows = load(d)
    lo, hi = window(rows, region)
    per = defaultdict(lambda: [0, 0])
    busy = []
    for s, e, n in rows:
        if s >= lo and e <= hi and MARK not in n:
            per[short(n)][0] += 1
            per[short(n)][1] += e - s
            busy.append((s, e))
    busy.sort()
    union, cur = 0, None
    for s, e in busy:
        if cur and s <= cur[1]:
            cur[1] = max(cur[1], e)
        else:
            if cur:
                union += cur[1] - cur[0]
            cur = [s, e]
    if cur:
        union += cur[1] - cur[0]
    span = hi - lo
    tot = sum(t for _, t in per.values())
    out = [f"# {title}", "",
           f"Timed region {region} of `bench.py --markers` (rocprofv3 --kernel-trace): {span / 1e3:.1f} us for {steps} steps "
           f"= {span / 1e3 / steps:.1f} us/step under the profiler; some kernel running {100 * union / span:.1f} % of it. "
           "Kernel time sums overlapping kernels (pipelined streams), so the % column can exceed 100 in total.", "",
           "| kernel | calls | calls/step | total us | avg us | us/step | % of window |", "|---|---:|---:|---:|---:|---:|---:|"]
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        out.append(f"| `{n}` | {c} | {c / steps:g} | {t / 1e3:.1f} | {t / 1e3 / c:.1f} | {t / 1e3 / steps:.1f} | "
                   f"{100 * t / span:.1f} |")
    out.append(f"| (sum) | {sum(c for c, _ in per.values())} | | {tot / 1e3:.1f} | | {tot / 1e3 / steps:.1f} | "
               f"{100 * tot / span:.1f} |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    a = sys.argv
    sys.stdout.write(render(a[1], a[2], int(a[3]) if len(a) > 3 else 1, int(a[4]) if len(a) > 4 else 20))
