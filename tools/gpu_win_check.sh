#!/bin/bash
# Window-kernel change check: its GPU tests, per-phase timings (c3, c2 shapes), c3 bench.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_win_gpu.py tests/test_win_gpu_extra.py tests/test_ops_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/win_tests.log 2>&1
rc=$?; tail -3 gpurun_out/win_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/win_phases.py > gpurun_out/phases_check.log 2>&1 || exit 1
timeout -k 10 200 python tools/win_phases.py 200 2000 24 1024 > gpurun_out/phases_check_n200.log 2>&1 || exit 1
grep "win " gpurun_out/phases_check_n200.log | head -2
grep "win " gpurun_out/phases_check.log | head -3
timeout -k 10 200 python bench.py --config c3 --steps 30 --warmup 5 > gpurun_out/b_c3_check.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('gpurun_out/b_c3_check.log').read().strip().splitlines()[-1]); print('c3', round(d['value']), round(d['ms_per_step'], 4))"
