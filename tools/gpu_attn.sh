#!/bin/bash
set -u
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_encoder_ops_gpu.py tests/test_sentiment.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/attn_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c4 --steps 10 --warmup 2 > gpurun_out/bench_c4.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c4.log | cut -c1-200
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d $R/gpurun_out/prof_c4 -o run -- python3 $R/bench.py --config c4 --steps 4 --warmup 1 --graph 0 > $R/gpurun_out/prof_c4.log 2>&1) || exit 1
grep attn gpurun_out/prof_c4/run_kernel_stats.csv | cut -c1-60,150-260
