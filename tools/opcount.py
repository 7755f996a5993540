"""Per-kernel instruction-class counts from a hipcc -save-temps .s file: opcount.py file.s [filter]."""
import re
import sys
from collections import Counter

path = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
cur, counts = None, {}
for line in open(path):
    m = re.match(r"^(_Z\w+):", line)
    if m:
        cur = m.group(1)
        counts[cur] = Counter()
        continue
    if line.startswith(".Lfunc_end"):
        cur = None
    if cur is None:
        continue
    t = line.strip().split()
    if not t or t[0].startswith((";", ".")) or t[0].endswith(":"):
        continue
    op = t[0]
    cls = ("pkminmax" if re.match(r"v_pk_m(in|ax)_u16", op) else "bperm" if "bpermute" in op else
           "permlane" if "permlane" in op else "bufload" if op.startswith("buffer_load") else
           "salu" if op.startswith("s_") else "valu" if op.startswith("v_") else "ds" if op.startswith("ds_") else "other")
    counts[cur][cls] += 1
    counts[cur]["total"] += 1
for k, c in counts.items():
    if filt in k:
        print(k[:64], dict(sorted(c.items())))
