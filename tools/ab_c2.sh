#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for h in 8 4 2; do
  timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --wave-hint $h > gpurun_out/ab_c2_$h.log 2>&1 || exit $?
  echo "hint=$h $(grep -o '"value": [0-9.]*' gpurun_out/ab_c2_$h.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_c2_$h.log)"
done
