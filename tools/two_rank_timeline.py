"""Merge two processes' rocprofv3 kernel traces (one GPU) into a timeline summary: per rank the busy time of
its kernels in the timed window, how much of it overlaps the other rank's kernels, and the idle gaps.

    python tools/two_rank_timeline.py gpurun_out/tr_fp32_r0 gpurun_out/tr_fp32_r1
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:70]))
    rows.sort()
    return rows


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def inter(a, b):
    i = j = t = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        t += max(0, e - s)
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return t


ks = [load(d) for d in sys.argv[1:3]]
# the timed window: the last 40 % of each trace (after warm-up, graph capture, the stream pool generation)
lo = max(k[int(len(k) * 0.6)][0] for k in ks)
hi = min(k[-1][1] for k in ks)
print(f"window: {(hi - lo) / 1e6:.2f} ms")
bus = []
for r, k in enumerate(ks):
    iv = union([(max(s, lo), min(e, hi)) for s, e, _ in k if e > lo and s < hi])
    busy = sum(e - s for s, e in iv)
    bus.append(iv)
    per = defaultdict(lambda: [0, 0])
    for s, e, n in k:
        if e > lo and s < hi:
            per[n][0] += 1
            per[n][1] += min(e, hi) - max(s, lo)
    print(f"rank {r}: kernels busy {busy / 1e6:.2f} ms of the window ({100 * busy / (hi - lo):.0f} %)")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:6]:
        print(f"    {t / 1e6:8.2f} ms  {c:5d}x  {n}")
both = inter(bus[0], bus[1])
anyb = sum(e - s for s, e in union(bus[0] + bus[1]))
print(f"both ranks' kernels running at once: {both / 1e6:.2f} ms; GPU busy with either: {anyb / 1e6:.2f} ms "
      f"({100 * anyb / (hi - lo):.0f} % of the window); idle: {(hi - lo - anyb) / 1e6:.2f} ms")
