#!/bin/bash
# Re-entry check of the rebuilt tree: GPU tests + headline benches (tools/gpu_quick3.sh), then the c4
# per-shape GEMM probe (tools/probe_gemm_shapes.py).
set -u
mkdir -p gpurun_out
bash tools/gpu_quick3.sh || exit 1
timeout -k 10 200 python -u tools/probe_gemm_shapes.py > gpurun_out/gemm_shapes.log 2>&1 || { tail -5 gpurun_out/gemm_shapes.log; exit 1; }
cat gpurun_out/gemm_shapes.log
bash tools/gpu_resgemm_ab.sh || exit 1
bash tools/gpu_exact_stream.sh || exit 1
echo all done
