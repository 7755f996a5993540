#!/bin/bash
# c4 QKV-on-rocBLAS check: its GPU test, then the alternating c4 A/B (tools/gpu_c4_ab.sh).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_encoder_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qkv_test.log 2>&1 || { tail -30 gpurun_out/qkv_test.log; exit 1; }
tail -1 gpurun_out/qkv_test.log
bash tools/gpu_c4_ab.sh || exit 1
echo all done
