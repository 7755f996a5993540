#!/bin/bash
# c4 encoder: GPU kernel tests (bf16 + fp32), then the c4 bench (bf16 headline + fp32 alt_precision field)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encoder_ops_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_enc.log 2>&1; rc=$?; tail -15 gpurun_out/pt_enc.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --config c4 --steps 10 --warmup 2 > gpurun_out/b_c4.log 2>&1 || { tail -5 gpurun_out/b_c4.log; exit 1; }
grep '^{' gpurun_out/b_c4.log
