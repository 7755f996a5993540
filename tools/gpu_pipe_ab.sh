#!/bin/bash
# Pipelined streaming step (update scatter of range k+1 overlapped with the round of range k): tests + A/B.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_tests.log 2>&1
rc=$?; tail -3 gpurun_out/pipe_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in c3 c5; do
  for k in 1 2 3 4; do
    timeout -k 10 200 python bench.py --config $cfg --steps 30 --warmup 5 --pipeline $k > gpurun_out/b_${cfg}_pipe$k.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/b_${cfg}_pipe$k.log').read().strip().splitlines()[-1]); print('$cfg pipeline $k', round(d['value']), round(d['ms_per_step'], 4))"
  done
done
