"""VGPR high-water profile of one kernel in a hipcc -save-temps .s file: vprof.py file.s kernel-substr [window]."""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
win = int(sys.argv[3]) if len(sys.argv) > 3 else 100
L = open(path).read().split("\n")
start = next(i for i, l in enumerate(L) if l.startswith(name + ":") or (name in l and l.split(":")[0].endswith(name)))
end = next(i for i in range(start, len(L)) if L[i].startswith(".Lfunc_end"))
body = L[start:end]
for i in range(0, len(body), win):
    mx = 0
    for l in body[i:i + win]:
        if "lane" in l:
            continue
        for a in re.findall(r"\bv(\d+)\b", l):
            mx = max(mx, int(a))
        for a, b in re.findall(r"v\[(\d+):(\d+)\]", l):
            mx = max(mx, int(b))
    print(f"{start + i}:{mx}", end="  ")
print()
