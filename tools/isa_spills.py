"""Spill report of one kernel in a .hip file: v_readlane / v_writelane / scratch ops per loop depth,
and the large loop blocks (the hot loop bodies) that hold any of them.

    python tools/isa_spills.py csrc/kernels/consensus_fast_win.hip <mangled-kernel-substring> [-I dir]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile


def file_flags(src):
    """The kernel source's own extra hipcc flags (``// svoc-hipcc-flags: ...``, csrc/build.py)."""
    for line in open(src, encoding="utf-8").readlines()[:60]:
        if "svoc-hipcc-flags:" in line:
            return line.split("svoc-hipcc-flags:", 1)[1].split()
    return []


def isa(src, incs):
    d = tempfile.mkdtemp()
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-O3", *[f"-I{i}" for i in incs],
           *file_flags(src), "-c", os.path.abspath(src), "-o", os.path.join(d, "x.o"), "-save-temps"]
    subprocess.run(cmd, cwd=d, check=True, capture_output=True)
    return open(os.path.join(d, [f for f in os.listdir(d) if f.endswith(".s") and "gfx950" in f][0])).read()


def report(s, kname):
    names = re.findall(r"^(_Z\S*" + re.escape(kname) + r"\S*):", s, re.M)
    for k in names:
        i = s.index(k + ":")
        j = s.index(".Lfunc_end", i)
        blocks = [["entry", 0, collections.Counter()]]
        for line in s[i:j].splitlines():
            m = re.match(r"^(\.LBB\S+):", line)
            if m:
                blocks.append([m.group(1), 0, collections.Counter()])
                continue
            mm = re.search(r"Depth=(\d+)", line)
            if mm:
                blocks[-1][1] = max(blocks[-1][1], int(mm.group(1)))
            t = line.strip().split()
            if t and not t[0].startswith((".", ";")):
                blocks[-1][2][t[0]] += 1
        per = collections.defaultdict(collections.Counter)
        for _, dep, c in blocks:
            per[dep]["instrs"] += sum(c.values())
            per[dep]["readlane"] += c["v_readlane_b32"]
            per[dep]["writelane"] += c["v_writelane_b32"]
            per[dep]["scratch"] += sum(v for op, v in c.items() if "scratch" in op)
        hot = sum(c["v_readlane_b32"] + c["v_writelane_b32"] for _, dep, c in blocks if dep >= 1 and sum(c.values()) > 500)
        print(k[:90], {d: dict(v) for d, v in sorted(per.items())}, "hot-loop spill ops:", hot)


if __name__ == "__main__":
    incs = [os.path.abspath(a[2:]) for a in sys.argv[3:] if a.startswith("-I")] or [os.path.abspath("csrc/include"), os.path.abspath("csrc")]
    report(isa(sys.argv[1], incs), sys.argv[2])
