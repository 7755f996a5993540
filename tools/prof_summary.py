"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into a compact markdown table."""
import csv
import glob
import os
import re
import sys


def short(name: str) -> str:
    name = re.sub(r"at::native::|at::cuda::|\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*", "", name)
    return name[:90]


def main(d, out=None, top=15):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    lines = ["| kernel | calls | avg us | total ms | % |", "|---|---:|---:|---:|---:|"]
    for r in rows[:top]:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                     f"{float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.1f} |")
    txt = "\n".join(lines)
    if out:
        open(out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
