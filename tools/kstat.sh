#!/bin/bash
# Register/spill report for one kernel source: tools/kstat.sh csrc/kernels/X.hip [grep-filter]
set -euo pipefail
src=$(realpath "$1"); filt="${2:-.}"
d=$(mktemp -d /tmp/kstat.XXXX); cd "$d"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -O3 -I/root/repo/csrc/include -I/root/repo/csrc $(grep -m1 -o "svoc-hipcc-flags:.*" "$src" | cut -d: -f2-) -save-temps -c "$src" -o k.o 2>&1 | grep -v "warning: argument unused" || true
python3 /root/repo/csrc/tools_kstat.py *gfx950.s | grep -E "$filt"
echo "asm: $d/$(ls *gfx950.s)"
