"""Print per-kernel register / spill / LDS stats from a hipcc -save-temps .s file."""
import re
import sys

for path in sys.argv[1:]:
    txt = open(path).read()
    for blk in re.split(r"\n  - ", txt.split("amdhsa.kernels:")[-1])[1:]:
        def g(k):
            m = re.search(r"\." + k + r":\s+(\S+)", blk)
            return m.group(1) if m else "-"
        print(f"{g('name')[:70]:70s} vgpr={g('vgpr_count'):>4} agpr={g('agpr_count'):>3} "
              f"sgpr={g('sgpr_count'):>4} vspill={g('vgpr_spill_count'):>3} sspill={g('sgpr_spill_count'):>4} "
              f"scratch={g('private_segment_fixed_size'):>4} lds={g('group_segment_fixed_size')}")
