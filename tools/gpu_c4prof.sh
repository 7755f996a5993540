#!/bin/bash
set -u
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 > gpurun_out/bench_c4.log 2>&1 || { tail -5 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d $R/gpurun_out/prof_c4 -o run -- python3 $R/bench.py --config c4 --steps 4 --warmup 1 --graph 0 > $R/gpurun_out/prof_c4.log 2>&1) || exit 1
timeout -k 10 300 python bench.py --config c2 --mode exact --steps 10 --warmup 2 > gpurun_out/bench_exact_default.log 2>&1 || exit 1
tail -1 gpurun_out/bench_exact_default.log
timeout -k 10 300 python bench.py --config c3 --mode exact --steps 5 --warmup 1 > gpurun_out/bench_exact_c3.log 2>&1 || exit 1
tail -1 gpurun_out/bench_exact_c3.log
