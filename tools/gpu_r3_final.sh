#!/bin/bash
# Re-entry check of the rebuilt tree: GPU tests + headline benches (tools/gpu_quick3.sh), the c4
# residual-in-GEMM A/B, the exact stream at the YAML batch, then the c4 per-shape GEMM probe.
set -u
mkdir -p gpurun_out
bash tools/gpu_quick3.sh || exit 1
bash tools/gpu_c4_ab.sh || exit 1
bash tools/gpu_exact_stream.sh || exit 1
timeout -k 10 200 python -u tools/probe_gemm_shapes.py > gpurun_out/gemm_shapes.log 2>&1 || { tail -5 gpurun_out/gemm_shapes.log; exit 1; }
cat gpurun_out/gemm_shapes.log
echo all done
