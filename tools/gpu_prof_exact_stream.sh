#!/bin/bash
# Kernel table of one exact transaction wave at the c3 shape (tools/dbg_exact_stream.py, 16 instances).
set -u
R=$(pwd); mkdir -p gpurun_out
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
   -d $R/gpurun_out/prof_xs -o run -- python3 $R/tools/dbg_exact_stream.py 16 1 > $R/gpurun_out/prof_xs.log 2>&1) || { tail -5 gpurun_out/prof_xs.log; exit 1; }
tail -4 gpurun_out/prof_xs.log
python3 tools/prof_summary.py gpurun_out/prof_xs
