#!/bin/bash
# c3-shape exact transactional stream at the YAML's own batch (1024 instances x 64 transactions per
# step) and at 256: the 64-instance record under-fills the 256 CUs (each wave is one batched round).
set -u
mkdir -p gpurun_out
for b in 256 1024; do
  timeout -k 10 300 python bench.py --config-file configs/c3_exact_stream.yaml --batch $b --steps 2 --warmup 1 \
      > gpurun_out/xs_$b.log 2>&1 || { tail -5 gpurun_out/xs_$b.log; exit 1; }
  grep '^{' gpurun_out/xs_$b.log | tail -1 | cut -c1-300
done
