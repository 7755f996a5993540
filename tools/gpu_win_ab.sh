#!/bin/bash
# A/B of the window kernel vs the two-network kernel: window tests, c3/c2 benches (default vs
# --wave-hint -7), per-phase kernel timings.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_win_gpu.py tests/test_win_gpu_extra.py -x -q --timeout 120 --timeout-method thread > gpurun_out/win_tests.log 2>&1
rc=$?; tail -5 gpurun_out/win_tests.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for cfg in c3 c2; do
  for h in 0 -7; do
    timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --wave-hint $h > gpurun_out/b_${cfg}_$h.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/b_${cfg}_$h.log').read().strip().splitlines()[-1]); print('$cfg hint $h', round(d['value']), d['ms_per_step'])"
  done
done
timeout -k 10 200 python tools/win_phases.py > gpurun_out/phases_c3.log 2>&1 && cat gpurun_out/phases_c3.log
timeout -k 10 300 python tools/win_phases.py 64 1024 8 2500 > gpurun_out/phases_c2.log 2>&1; cat gpurun_out/phases_c2.log
