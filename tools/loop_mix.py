"""Instruction mix of a kernel's hottest loop (the largest block range between a loop header and its
back-edge) from the gfx950 ISA: counts per mnemonic, VALU / SALU / LDS / VMEM totals.

    python tools/loop_mix.py csrc/kernels/consensus_fast_winf.hip <mangled-kernel-substring> [top]
"""
import collections
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_loads import isa  # noqa: E402


def main():
    src, kname = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    s = isa(src)
    k = re.findall(r"^(_Z\S*" + re.escape(kname) + r"\S*):", s, re.M)[0]
    i = s.index(k + ":")
    j = s.index(".Lfunc_end", i)
    lines = s[i:j].splitlines()
    # blocks of each depth-1 loop: the header ("Loop Header: Depth=1") and every block whose comment
    # names it ("in Loop: Header=BBx_y Depth=...", inner loops included); the biggest loop wins
    loops = collections.defaultdict(collections.Counter)
    cur = None
    for ln in lines:
        m = re.match(r"^\.L(BB\S+):(.*)", ln)
        if m:
            cur = None
            if "Loop Header: Depth=1" in m.group(2):
                cur = m.group(1)
            else:
                mm = re.search(r"Header=(BB\S+) Depth=1", m.group(2))
                if mm:
                    cur = mm.group(1)
                else:
                    mm = re.search(r"Parent Loop (BB\S+) Depth=1", m.group(2))
                    cur = mm.group(1) if mm else None
            continue
        t = ln.strip().split()
        if cur and t and not t[0].startswith((".", ";")):
            loops[cur][t[0]] += 1
    for lb, cc in sorted(loops.items(), key=lambda kv: -sum(kv[1].values())):
        print(f"  loop {lb}: {sum(cc.values())} instructions")
    want = sys.argv[4] if len(sys.argv) > 4 else None
    lab, c = (want, loops[want]) if want else max(loops.items(), key=lambda kv: sum(kv[1].values()))
    cls = collections.Counter()
    for name, n in c.items():
        key = ("VALU" if name.startswith("v_") else "SALU" if name.startswith("s_") and not name.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_cbranch", "s_branch")) else
               "LDS" if name.startswith("ds_") else "VMEM" if name.startswith(("buffer_", "global_", "scratch_")) else "other")
        cls[key] += n
    print(f"{k[:80]} loop {lab}: {dict(cls)}")
    for name, n in c.most_common(top):
        print(f"  {n:6d} {name}")


if __name__ == "__main__":
    main()
