"""rocprofv3 `--stats` kernel table (run_kernel_stats.csv) -> the markdown tables under profiles/.

    python tools/kernel_stats_md.py gpurun_out/prof_c3/run_kernel_stats.csv "title" [note] > profiles/X.md
"""
from __future__ import annotations

import csv
import sys


def render(path: str, title: str, note: str = "", top: int = 12) -> str:
    rows = list(csv.DictReader(open(path, encoding="utf-8")))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    out = [f"# {title}", ""]
    if note:
        out += [note, ""]
    out += ["| kernel | calls | avg us | min us | max us | % |", "|---|---|---|---|---|---|"]
    for r in rows[:top]:
        name = r["Name"] if len(r["Name"]) <= 100 else r["Name"][:97] + "..."
        out.append(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} | "
                   f"{float(r['MaxNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    sys.stdout.write(render(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else ""))
