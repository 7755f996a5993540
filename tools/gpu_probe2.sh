#!/bin/bash
# r2 probes: MFMA vs VALU qr A/B (+ rocprof kernel table), wide-N bench, exact c3-shape bench
set -u
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python tools/qr_mfma_ab.py --out gpurun_out/qr_mfma_ab.json > gpurun_out/qr_mfma_ab.log 2>&1 || { tail -20 gpurun_out/qr_mfma_ab.log; exit 1; }
tail -2 gpurun_out/qr_mfma_ab.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d $R/gpurun_out/prof_qr -o run -- python3 $R/tools/qr_mfma_ab.py > $R/gpurun_out/prof_qr.log 2>&1) || exit 1
timeout -k 10 300 python bench.py --config-file configs/wide512.yaml --steps 10 --warmup 2 > gpurun_out/bench_wide512.log 2>&1 || exit 1
tail -1 gpurun_out/bench_wide512.log
timeout -k 10 300 python bench.py --config c3 --mode exact --storage int32 --steps 5 --warmup 1 > gpurun_out/bench_exact_c3_int32.log 2>&1 || exit 1
tail -1 gpurun_out/bench_exact_c3_int32.log
