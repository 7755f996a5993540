#!/bin/bash
# fp32 window kernel after the phase-B / pre-check load batching: its GPU tests, then c3 / c2 fp32 with
# odd workgroups started k x ~4 us late (wave_hint 100 + k), alternating; then the exact transactional
# stream at the c3 shape (64 instances).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_f32_gpu.py tests/test_revert_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_test.log 2>&1 || { tail -30 gpurun_out/ab_test.log; exit 1; }
tail -1 gpurun_out/ab_test.log
: > gpurun_out/ab_stagger.txt
b() { timeout -k 10 200 python bench.py "$@" > gpurun_out/ab_b.log 2>&1 || { tail -5 gpurun_out/ab_b.log; exit 1; }
      python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_b.log') if l.startswith('{')][-1]); print(' '.join(sys.argv[1:]), round(d['value']), round(d['ms_per_step'],4), d['config'].get('ok_fraction'))" "$@" | tee -a gpurun_out/ab_stagger.txt; }
for rep in 1 2; do
  for wh in 0 105 115; do
    b --config c3 --storage fp32 --steps 20 --warmup 3 --wave-hint $wh
  done
  b --config c2 --storage fp32 --steps 20 --warmup 3
done
b --config-file configs/c3_exact_stream.yaml --batch 64 --steps 2 --warmup 1
echo done
