#!/bin/bash
# Quick GPU check: selected test files (QUICK_TESTS) + bench lines (QUICK_BENCH, '|'-separated arg sets).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${QUICK_TESTS:-tests/test_f32_gpu.py} -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -ne 0 ] && exit $rc
IFS='|' read -ra BS <<< "${QUICK_BENCH:-}"
for b in "${BS[@]}"; do
  timeout -k 10 200 python bench.py $b > gpurun_out/quick_bench.log 2>&1 || { tail -5 gpurun_out/quick_bench.log; exit 1; }
  echo "$b: $(tail -1 gpurun_out/quick_bench.log | cut -c1-170)"
done
