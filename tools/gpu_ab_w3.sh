#!/bin/bash
# A/B: fp32 window kernel, default 4-wave workgroups vs wave_hint 3 (three-wave workgroups, 3 waves per
# SIMD), alternating, c3 and c2 fp32; after the new GPU test of the variant.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_f32_gpu.py -x -q --timeout 120 --timeout-method thread -k "three_wave or window_matches" > gpurun_out/ab_test.log 2>&1 || { tail -30 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
b() { timeout -k 10 200 python bench.py "$@" > gpurun_out/ab_b.log 2>&1 || { tail -5 gpurun_out/ab_b.log; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_b.log') if l.startswith('{')][-1]); print(' '.join(sys.argv[1:]), round(d['value']), round(d['ms_per_step'],4))" "$@" | tee -a gpurun_out/ab_w3.txt; }
for rep in 1 2; do
  for wh in 0 3; do
    b --config c3 --storage fp32 --steps 20 --warmup 3 --wave-hint $wh
    b --config c2 --storage fp32 --steps 20 --warmup 3 --wave-hint $wh
  done
done
echo done
