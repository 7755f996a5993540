"""Aggregate rocprofv3 --pmc counter_collection CSVs per kernel (sum over dispatches / dispatch count)."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def load(dirs):
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = re.sub(r"\(.*", "", r["Kernel_Name"])[:60]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
                agg[k]["_VGPR"] = float(r.get("VGPR_Count", r.get("Arch_VGPR_Count", 0)) or 0)
    return agg, disp


if __name__ == "__main__":
    agg, disp = load(sys.argv[1:])
    for k, c in agg.items():
        n = len(disp[k])
        print(f"## {k}  (dispatches={n})")
        for name in sorted(c):
            print(f"  {name:28s} {c[name] / (1 if name.startswith('_') else n):>16.4g}")
        w = c.get("SQ_WAVES", 0)
        if w and "SQ_INSTS_VALU" in c:
            print(f"  VALU insts / wave          {c['SQ_INSTS_VALU'] / w:>16.1f}")
            print(f"  LDS insts / wave           {c.get('SQ_INSTS_LDS', 0) / w:>16.1f}")
            print(f"  SALU insts / wave          {c.get('SQ_INSTS_SALU', 0) / w:>16.1f}")
        if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_INST_ANY" in c:
            print(f"  wait_inst / wave_cycles    {c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:>16.3f}")
            print(f"  active_valu / wave_cycles  {c['SQ_ACTIVE_INST_VALU'] / c['SQ_WAVE_CYCLES']:>16.3f}")
