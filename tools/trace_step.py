"""Per-step kernel breakdown from a rocprofv3 --kernel-trace CSV: kernels between consecutive launches
of an anchor kernel (default: the consensus round), averaged over the steady-state steps."""
import csv
import glob
import re
import sys
from collections import defaultdict


def main(d, anchor="consensus_fast", skip=2):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
    if len(idx) < skip + 2:
        print("not enough anchor launches", len(idx))
        return
    acc = defaultdict(float)
    cnt = defaultdict(int)
    steps = 0
    span = 0.0
    for a, b in zip(idx[skip:-1], idx[skip + 1:]):
        steps += 1
        span += (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
        for r in rows[a:b]:
            k = re.sub(r"\(.*", "", r["Kernel_Name"])[:80]
            acc[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cnt[k] += 1
    print(f"| kernel | launches/step | us/step |\n|---|---:|---:|")
    for k in sorted(acc, key=lambda k: -acc[k]):
        print(f"| `{k}` | {cnt[k] / steps:.1f} | {acc[k] / steps:.1f} |")
    print(f"\nsteady-state step span (anchor to anchor): {span / steps:.1f} us over {steps} steps; "
          f"kernel busy {sum(acc.values()) / steps:.1f} us/step")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []))
