"""Memory-level parallelism of a kernel's load batches: for each run of buffer loads in the ISA, how many
loads the run issues and the deepest `s_waitcnt vmcnt(k)` seen before the run's values are consumed.
A batch of 64 loads that waits with vmcnt(63..0) one by one keeps them all in flight; vmcnt(0) after
every load (a v_readlane'd SGPR offset per load) means one in flight.

    python tools/isa_loads.py csrc/kernels/consensus_fast_winf.hip <mangled-kernel-substring>
"""
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


def isa(src):
    d = tempfile.mkdtemp()
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-O3", f"-I{inc}/include", f"-I{inc}",
           *file_flags(src), "-c", os.path.abspath(src), "-o", os.path.join(d, "x.o"), "-save-temps"]
    subprocess.run(cmd, cwd=d, check=True, capture_output=True)
    return open(os.path.join(d, [f for f in os.listdir(d) if f.endswith(".s") and "gfx950" in f][0])).read()


def batches(lines):
    """Runs of >= 8 buffer loads (other instructions allowed in between, until a vmcnt(0) wait)."""
    out, cur, max_inflight, zero_waits = [], 0, 0, 0
    inflight = 0
    for ln in lines:
        t = ln.strip()
        if t.startswith("buffer_load"):
            cur += 1
            inflight += 1
            max_inflight = max(max_inflight, inflight)
        m = re.match(r"s_waitcnt vmcnt\((\d+)\)", t)
        if m:
            k = int(m.group(1))
            inflight = min(inflight, k)
            if k == 0 and cur:
                if cur >= 8:
                    out.append((cur, max_inflight))
                cur, max_inflight, inflight = 0, 0, 0
    return out


def main():
    src, kname = sys.argv[1], sys.argv[2]
    s = isa(src)
    for k in re.findall(r"^(_Z\S*" + re.escape(kname) + r"\S*):", s, re.M):
        i = s.index(k + ":")
        j = s.index(".Lfunc_end", i)
        lines = s[i:j].splitlines()
        b = batches(lines)
        rl = sum(1 for ln in lines if ln.strip().startswith("v_readlane"))
        print(k[:90])
        print(f"  readlane {rl}  load batches (loads, max in flight): {b}")


if __name__ == "__main__":
    main()
