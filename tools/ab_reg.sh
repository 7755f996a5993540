#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -q -p no:cacheprovider -k "fast_hip_vs_torch" > gpurun_out/pytest_reg.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_reg.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in c2 c3; do for h in ${HINTS:-0 -1}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --wave-hint $h > gpurun_out/ab_${cfg}_$h.log 2>&1 || exit $?
  echo "$cfg hint=$h $(grep -o '"value": [0-9.]*' gpurun_out/ab_${cfg}_$h.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${cfg}_$h.log)"
done; done
