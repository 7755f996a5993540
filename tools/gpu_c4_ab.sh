#!/bin/bash
# c4 A/B: QKV projection on rocBLAS (SVOC_ENC_QKV_ROCBLAS=1) vs the default,
# alternating, 2 reps each.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 0 1; do
    SVOC_ENC_QKV_ROCBLAS=$v timeout -k 10 200 python bench.py --config c4 --steps 10 --warmup 2 > gpurun_out/rg_$v.log 2>&1 \
        || { tail -5 gpurun_out/rg_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/rg_$v.log') if l.startswith('{')][-1]); print('QKV_ROCBLAS=$v rep $rep', round(d['value'],1), d['ms_per_step'])"
  done
done
